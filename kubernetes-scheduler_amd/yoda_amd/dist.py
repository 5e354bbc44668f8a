"""Node-sharded evaluation across GPUs: the two exchange steps of SURVEY.md §8e.

Each rank (one process per GPU) holds a contiguous node block and the full pod batch.
Per batch:
  1. K1 on the shard -> per-pod partial maxima (MAX) and n_feasible / n_zero_total (SUM):
     CollectMaxValues is a reduction over ALL nodes (collection.go:30-55), so the maxima
     must be global before any score is final.
  2. K2 on the shard with the global maxima -> per-pod (best raw score MAX, then the lowest
     node index among shards reaching it and the lowest raw score in ONE MIN, tie counts
     SUM).
Collectives are torch.distributed all-reduces on device tensors (backend "nccl" = RCCL over
xGMI on MI355X; "gloo" in the CPU tests).  libyoda launches on torch's current stream so
the collectives are ordered after the kernels without host synchronisation.

uint64/uint32 buffers are reduced through their signed views with the sign bit flipped,
which maps unsigned order onto signed order (MAX/MIN stay exact for all 64-bit values).

An evaluation batch can instead be POD-sharded (`pod_partition`): every rank holds the whole
node snapshot (100k nodes are ~70 MB of 288 GB) and a slice of the pods, and no collective
is needed at all (bench.py --shard pods).  Node sharding stays the default: its per-rank
kernels are faster on one MI355X at 2-8 ranks (each rank's K1/K2 keep all 100k pods' wave
classes; profiles/r01/current/shard_timing.txt), and it is the path for node sets split
across GPUs and for the greedy batch (whose picks change node state).
"""
from __future__ import annotations

from typing import Callable, List, Sequence

import numpy as np
import torch

from .soa import EvalResult

I64_SIGN = -(1 << 63)
I32_SIGN = -(1 << 31)


class ShardBuffers:
    """Per-rank exchange buffers (device tensors) for P pods, laid out as include/yoda.h's
    yoda_shard_* entry points expect."""

    def __init__(self, n_pods: int, device):
        P = max(n_pods, 1)
        self.n_pods = n_pods
        self.maxima = torch.empty(6 * P, dtype=torch.int64, device=device)  # u64 [6][P]
        self.counts = torch.empty(2 * P, dtype=torch.int32, device=device)  # u32 [2][P]
        self.best = torch.empty(P, dtype=torch.int64, device=device)
        self.best_g = torch.empty(P, dtype=torch.int64, device=device)
        self.idx = torch.empty(P, dtype=torch.int32, device=device)         # u32
        self.ties = torch.empty(P, dtype=torch.int32, device=device)        # u32
        # [lowest i64 | idx widened to i64]: both merge by MIN, so one all-reduce serves both
        self.mins = torch.empty(2 * P, dtype=torch.int64, device=device)
        self.lowest = self.mins[:P]
        # maxima need the sign flip only when a field can exceed 2^63 (U64 path); the fast
        # record paths bound every field by 2^44
        self.unsigned_maxima = True

    def ensure_witness(self):
        """Capacity greedy: witness buffers, [2][6][P] u32 (counts | lowest nodes), the local
        maxima kept across the MAX all-reduce, and the nodes widened for the unsigned MIN."""
        if getattr(self, "wit", None) is None:
            P = max(self.n_pods, 1)
            dev = self.maxima.device
            self.wit = torch.empty(12 * P, dtype=torch.int32, device=dev)
            self.maxima_local = torch.empty(6 * P, dtype=torch.int64, device=dev)
            self.wit_node64 = torch.empty(6 * P, dtype=torch.int64, device=dev)

    @staticmethod
    def ptr(t: torch.Tensor) -> int:
        return t.data_ptr()


def _flip(t: torch.Tensor, sign: int):
    t.bitwise_xor_(sign)


class Reducer:
    """All-reduce over the shards: either torch.distributed (one tensor per rank) or a local
    list of tensors (several shards in one process, for single-GPU testing)."""

    def __init__(self, group=None, local: bool = False):
        self.group = group
        self.local = local

    def __call__(self, ts: Sequence[torch.Tensor], op: str):
        if self.local:
            stacked = torch.stack(list(ts))
            if op == "max":
                r = stacked.max(dim=0).values
            elif op == "min":
                r = stacked.min(dim=0).values
            else:
                r = stacked.sum(dim=0, dtype=ts[0].dtype)
            for t in ts:
                t.copy_(r)
            return
        import torch.distributed as dist
        rop = {"max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN, "sum": dist.ReduceOp.SUM}[op]
        for t in ts:
            dist.all_reduce(t, op=rop, group=self.group)

    def gather_tensors(self, ts: Sequence[torch.Tensor]) -> List[torch.Tensor]:
        """All-gather of one device tensor per local shard -> for each local shard, the
        concatenation of every shard's tensor in rank order."""
        if self.local:
            cat = torch.cat(list(ts))
            return [cat for _ in ts]
        import torch.distributed as dist
        t = ts[0]
        out = torch.empty(dist.get_world_size(self.group) * t.numel(), dtype=t.dtype,
                          device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        return [out]

    def gather(self, arrays: Sequence[np.ndarray]) -> List[np.ndarray]:
        """All-gather of one float64 array per local shard -> every shard's array (rank order).
        Local mode: the arrays themselves.  RCCL needs device tensors, gloo host tensors."""
        if self.local:
            return [np.asarray(a, np.float64) for a in arrays]
        import torch.distributed as dist
        backend = dist.get_backend(self.group)
        dev = (torch.device("cuda", torch.cuda.current_device()) if backend == "nccl"
               else torch.device("cpu"))
        t = torch.from_numpy(np.ascontiguousarray(arrays[0], np.float64)).to(dev)
        out = [torch.empty_like(t) for _ in range(dist.get_world_size(self.group))]
        dist.all_gather(out, t, group=self.group)
        return [o.cpu().numpy() for o in out]


def merge_phase1(reduce: Reducer, bufs: List[ShardBuffers], narrow: bool = False):
    """Global maxima (MAX, unsigned) and feasible / zero-total counts (SUM).

    narrow: every maxima value is below 2^32 (the N32 record path: card fields <= 2^32 - 2),
    so the MAX runs on int32 values offset by 2^31 -- half the bytes on the wire."""
    if narrow:
        for b in bufs:
            b.max32 = (b.maxima - (1 << 31)).to(torch.int32)
        reduce([b.max32 for b in bufs], "max")
        for b in bufs:
            b.maxima.copy_(b.max32.to(torch.int64) + (1 << 31))
        reduce([b.counts for b in bufs], "sum")
        return
    flip = any(b.unsigned_maxima for b in bufs)
    if flip:
        for b in bufs:
            _flip(b.maxima, I64_SIGN)
    reduce([b.maxima for b in bufs], "max")
    if flip:
        for b in bufs:
            _flip(b.maxima, I64_SIGN)
    reduce([b.counts for b in bufs], "sum")


def merge_phase2(reduce: Reducer, bufs: List[ShardBuffers],
                 prepare: Callable[[ShardBuffers], None]):
    """best: MAX; then each shard masks idx/ties unless it reaches the global best
    (prepare), idx: MIN (unsigned), ties: SUM, lowest: MIN."""
    for b in bufs:
        b.best_g.copy_(b.best)
    reduce([b.best_g for b in bufs], "max")
    for b in bufs:
        prepare(b)
        hi = b.mins[b.lowest.numel():]
        hi.copy_(b.idx).bitwise_and_(0xFFFFFFFF)  # u32 order as non-negative i64
    reduce([b.mins for b in bufs], "min")         # lowest and idx together
    for b in bufs:
        b.idx.copy_(b.mins[b.lowest.numel():])    # back to the u32 bit pattern
    reduce([b.ties for b in bufs], "sum")


def merge_phase2_packed(reduce: Reducer, bufs: List[ShardBuffers], ib: int):
    """The fast record paths' phase-2 merge (north_star: "per-shard winners merged by an RCCL
    all-reduce(max) on the packed key"): each shard's (best raw score, lowest node reaching
    it) becomes ONE int64 key  score << ib | (2^ib - 1 - node)  -- a larger key is a higher
    score or, on equal scores, a lower node (the selectHost tie rule of DESIGN.md §2) -- and a
    MAX all-reduce of the keys gives the global winner; the shards holding it then SUM their
    tie counts.  Requires every node id < 2^ib - 1 and every score < 2^(63 - ib) (checked by
    the caller from yoda_score_bound).  `lowest` (only the U64 path's normalize check reads
    it) is set to the winning score."""
    imax = (1 << ib) - 1
    for b in bufs:
        idx64 = b.idx.to(torch.int64) & 0xFFFFFFFF
        key = (b.best << ib) | (imax - idx64)
        b.best_g.copy_(torch.where(b.best >= 0, key, torch.zeros_like(key)))
    reduce([b.best_g for b in bufs], "max")
    for b in bufs:
        key = b.best_g
        won = key > 0
        best_g = torch.where(won, key >> ib, torch.full_like(key, -1))
        idx_g = torch.where(won, imax - (key & imax), torch.full_like(key, 0xFFFFFFFF))
        keep = won & (b.best == best_g)
        b.ties.copy_(torch.where(keep, b.ties, torch.zeros_like(b.ties)))
        b.best_g.copy_(best_g)
        b.idx.copy_(idx_g.to(torch.int32))  # the u32 bit pattern
        b.lowest.copy_(best_g)
    reduce([b.ties for b in bufs], "sum")


def merge_witness(reduce: Reducer, bufs: List[ShardBuffers], prepare: Callable):
    """Capacity greedy phase 1: global maxima (MAX) and counts (SUM) as merge_phase1, then the
    witnesses: a shard below a field's global maximum clears its witness of it (prepare),
    the counts are SUM-reduced and the lowest nodes MIN-reduced (unsigned)."""
    for b in bufs:
        b.maxima_local.copy_(b.maxima)
    merge_phase1(reduce, bufs)
    for b in bufs:
        prepare(b)
    n = 6 * max(bufs[0].n_pods, 1)
    reduce([b.wit[:n] for b in bufs], "sum")
    for b in bufs:
        b.wit_node64.copy_(b.wit[n:]).bitwise_and_(0xFFFFFFFF)  # u32 order as non-negative i64
    reduce([b.wit_node64 for b in bufs], "min")
    for b in bufs:
        b.wit[n:].copy_(b.wit_node64)


F32_SMALL_MAX = 55738  # N32's f32 small-field quotients hold up to here (yoda_layout.h)


def agree_on_path(reduce: Reducer, handles, shards, offsets, device):
    """Every shard must run the SAME record path: the exactness bounds of the fast paths
    involve maxima contributed by other shards.  First the N32 quotient
    type: when any shard holds a bandwidth / clock / core / power beyond F32_SMALL_MAX, the
    others re-upload with f64 quotients (yoda_small_field_max; a shard with mixed-model nodes
    then takes F64).  Then the widest path any shard needs (N32 < F64 < U64): the shards that
    chose a narrower one re-upload."""
    small = [torch.tensor([h.small_field_max], dtype=torch.int64, device=device)
             for h in handles]
    reduce(small, "max")
    wide = int(small[0].item()) > F32_SMALL_MAX
    for h, nodes, off in zip(handles, shards, offsets):
        if wide and h.path_code == 0 and h.small_field_max <= F32_SMALL_MAX:
            h.upload_nodes(nodes, node_offset=off, f64_quotients=True)
    codes = [torch.tensor([h.path_code], dtype=torch.int64, device=device) for h in handles]
    reduce(codes, "max")
    target = int(codes[0].item())
    for h, nodes, off in zip(handles, shards, offsets):
        if h.path_code != target:
            h.upload_nodes(nodes, node_offset=off, force_generic=target == 2,
                           force_f64=target == 1, f64_quotients=wide)
    return target


class ShardExchange:
    """Drives libyoda handles (one per shard) through the sharded entry points."""

    def __init__(self, handles, reducer: Reducer, device, path_code=None, compact: bool = True,
                 caller_order: bool = True):
        self.handles = list(handles)
        self.reduce = reducer
        self.device = device
        self.bufs = [ShardBuffers(h.n_pods, device) for h in self.handles]
        if path_code is not None and path_code != 2:  # agreed fast path: maxima < 2^63
            for b in self.bufs:
                b.unsigned_maxima = False
        # compact exchange (agreed fast path): int32 maxima on N32, and the packed-key phase-2
        # merge when the global node count and score bound fit one int64 key
        self.narrow, self.ib = False, None
        if compact and path_code in (0, 1):
            lim = [torch.tensor([min(h.score_bound, (1 << 63) - 1), h.node_offset + h.n_nodes,
                                 int(h.memory_ranks)],
                                dtype=torch.int64, device=device) for h in self.handles]
            reducer(lim, "max")
            bound, n_total, ranks = (int(x) for x in lim[0].tolist())
            ib = max(1, (n_total + 1).bit_length())  # node ids < 2^ib - 1
            if ib <= 40 and bound < (1 << (63 - ib)):
                self.ib = ib
            # int32 maxima need every field < 2^32: not with memory ranks (values beyond 32 bits)
            self.narrow = path_code == 0 and ranks == 0
        stream = torch.cuda.current_stream(device).cuda_stream if device.type == "cuda" else 0
        for h in self.handles:
            h.set_stream(stream)
            # the exchanged buffers in the caller's pod order: each shard sorts its pods and
            # nodes privately, as yoda_run does (the U64 path keeps the shared radix order)
            h.shard_exchange_order(caller_order)

    @classmethod
    def local(cls, handles, device, shards=None, offsets=None, compact: bool = True,
              caller_order: bool = True):
        """Several shards in one process (single-GPU testing).  Pass the node shards to
        enforce a common record path."""
        red = Reducer(local=True)
        path = None
        if shards is not None:
            path = agree_on_path(red, handles, shards, offsets, device)
        return cls(handles, red, device, path, compact=compact, caller_order=caller_order)

    @classmethod
    def distributed(cls, handle, device, shard=None, offset=0, group=None):
        """One shard per rank over torch.distributed (RCCL)."""
        red = Reducer(group=group)
        path = None
        if shard is not None:
            path = agree_on_path(red, [handle], [shard], [offset], device)
        return cls([handle], red, device, path)

    def _prepare(self, h, b: ShardBuffers):
        p = ShardBuffers.ptr
        h.shard_prepare_merge(p(b.best_g), p(b.best), p(b.idx), p(b.ties))

    def step(self, mode: int):
        """One batch: phase1, merge, phase2, merge, finalize — all asynchronous."""
        p = ShardBuffers.ptr
        for h, b in zip(self.handles, self.bufs):
            h.shard_phase1(mode, p(b.maxima), p(b.counts))
        scv = mode == 0
        merge_phase1(self.reduce, self.bufs, narrow=self.narrow and scv)
        for h, b in zip(self.handles, self.bufs):
            h.shard_phase2(mode, p(b.maxima), p(b.counts), p(b.best), p(b.idx), p(b.ties),
                           p(b.lowest))
        if self.ib is not None and scv:
            merge_phase2_packed(self.reduce, self.bufs, self.ib)
        else:
            hb = dict(zip(map(id, self.bufs), self.handles))
            merge_phase2(self.reduce, self.bufs, lambda b: self._prepare(hb[id(b)], b))
        for h, b in zip(self.handles, self.bufs):
            h.shard_finalize(mode, p(b.counts), p(b.best_g), p(b.idx), p(b.ties), p(b.lowest))
        if scv and self.handles[0].generic and self.handles[0].shard_overflow_count():
            # U64 pods whose NormalizeScore can overflow int64 (scheduler.go:176-179): every
            # shard's exact-normalize records all-gathered, then merged (the same pods are
            # flagged on every shard: the flags read only the reduced buffers)
            recs = [torch.empty(24 * max(h.n_pods, 1), dtype=torch.uint8, device=self.device)
                    for h in self.handles]
            for h, r in zip(self.handles, recs):
                h.shard_exact_records(r.data_ptr())
            world = (len(self.handles) if self.reduce.local
                     else torch.distributed.get_world_size(self.reduce.group))
            for h, a in zip(self.handles, self.reduce.gather_tensors(recs)):
                h.shard_exact_merge(a.data_ptr(), world)

    def run(self, mode: int) -> EvalResult:
        self.step(mode)
        torch.cuda.synchronize(self.device) if self.device.type == "cuda" else None
        return self.handles[0].download()


class LibExchange:
    """Node sharding with libyoda's OWN exchanges (yoda_comm_run, include/yoda.h, DESIGN.md
    §7), issued by libyoda through RCCL on the handle's stream -- the path a cgo / C caller
    without torch uses.  Per step: after K1 one grouped all-reduce, MAX over [maxima 6P |
    2 agreement words] and SUM over the counts [2P]; after K2, on the fast record paths, the
    packed (score << ib | ~node) key MAX then the tie-count SUM of the shards holding the
    winner.  Only the U64 path in Mode A all-gathers the per-shard (best, index, ties,
    lowest) records instead (its NormalizeScore check needs the lowest score), plus the
    exact-normalize records when K3 flags pods.  torch.distributed here only agrees on the
    record path and broadcasts the communicator id."""

    def __init__(self, handle, device, shard=None, offset: int = 0, group=None):
        import torch.distributed as dist
        from .capi import comm_unique_id
        if shard is not None:
            agree_on_path(Reducer(group=group), [handle], [shard], [offset], device)
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        on_dev = dist.get_backend(group) == "nccl"
        # one GPU per rank, or RCCL's init fails with a bare "invalid usage" (keys: host hash
        # and PCI bus id, so identical servers of a multi-node job do not collide)
        agree_on_devices(handle.device_key(), device if on_dev else torch.device("cpu"), group)
        t = torch.zeros(128, dtype=torch.uint8, device=device if on_dev else "cpu")
        if rank == 0:
            t.copy_(torch.tensor(list(comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(t, src=0, group=group)
        handle.comm_init(bytes(t.cpu().numpy().tobytes()), rank, world)
        if device.type == "cuda":
            handle.set_stream(torch.cuda.current_stream(device).cuda_stream)
        self.handle = handle

    def step(self, mode: int):
        self.handle.comm_run(mode)


def agree_on_devices(key: str, device, group=None) -> list:
    """All-gather every rank's device key (Yoda.device_key: host hash / PCI bus id) and raise
    YodaError (YODA_ERR_SAME_DEVICE, naming the ranks) when two ranks share a GPU -- before
    yoda_comm_init, whose RCCL init would fail on it with "invalid usage".  Returns the keys in
    rank order."""
    import torch.distributed as dist
    from .capi import DEVICE_KEY_BYTES, comm_check_devices
    world = dist.get_world_size(group)
    raw = key.encode()[:DEVICE_KEY_BYTES - 1].ljust(DEVICE_KEY_BYTES, b"\0")
    mine = torch.tensor(list(raw), dtype=torch.uint8, device=device)
    every = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(every, mine, group=group)
    ids = [bytes(t.cpu().numpy().tobytes()).rstrip(b"\0").decode() for t in every]
    comm_check_devices(ids)
    return ids


def shard_bounds(n_nodes: int, world: int) -> np.ndarray:
    """Contiguous node blocks, one per rank."""
    return np.linspace(0, n_nodes, world + 1).astype(np.int64)


POD_BLOCK = 256  # pods per K1/K2 workgroup (4 waves of 64), yoda_kernels.hip


def balanced_bounds(bounds, costs) -> np.ndarray:
    """New contiguous node bounds with equal estimated cost per rank: the cost of each old
    shard (e.g. its measured K1 + K2 time) is spread evenly over its nodes, and the new bounds
    are the equal-cost quantiles of that piecewise-linear cumulative cost.  Every shard keeps
    at least one node (when there are as many nodes as ranks).  Any contiguous split is exact;
    this one only evens out the ranks' step times."""
    b = np.asarray(bounds, np.float64)
    c = np.maximum(np.asarray(costs, np.float64), 0.0)
    W = len(c)
    n = int(b[-1])
    if W <= 1 or c.sum() <= 0 or n < W:
        return np.asarray(bounds, np.int64)
    cum = np.concatenate([[0.0], np.cumsum(c)])
    targets = cum[-1] * np.arange(1, W) / W
    new = np.interp(targets, cum, b)
    out = np.concatenate([[0], np.rint(new), [n]]).astype(np.int64)
    for k in range(1, W):  # strictly increasing, room for the later shards
        out[k] = min(max(out[k], out[k - 1] + 1), n - (W - k))
    return out


def pod_partition(pods, world: int, by_key: bool = True,
                  block: int = POD_BLOCK, snake: bool = False) -> List[np.ndarray]:
    """Pod sharding of an evaluation batch: rank r evaluates pods part[r] (input indices)
    against the WHOLE node snapshot.  Every pod's Filter / PreScore maxima / Score / select
    reads only the node snapshot (collection.go:30-55, algorithm.go:96, scheduler.go:158-183;
    the batch has no assume between its pods), so the ranks exchange nothing: the union of
    their results is the unsharded result.  Any partition is exact.

    by_key (default): sort the batch by the request key (scv/clock, scv/number, scv/memory —
    the device sort's key, yoda_order.hip), cut it into blocks of `block` pods and deal the
    blocks round-robin.  Each block is a workgroup's worth of near-identical requests, as in
    one global sort, so the block classes of K1/K2 work as well per rank as on
    one GPU; dealing them cyclically gives every rank the same mix of cheap and expensive
    requests (contiguous key ranges are 2x out of balance at 8 ranks: a low scv/clock
    request is feasible on many more nodes).  Part sizes differ by at most `block`.
    by_key=False: contiguous slices of the input order (sizes differ by at most 1)."""
    P = pods.n_pods
    if world < 1:
        raise ValueError("world must be >= 1")
    if not by_key or not P:
        return [np.ascontiguousarray(x)
                for x in np.array_split(np.arange(P, dtype=np.int64), world)]
    c = np.where(pods.has_clock != 0, pods.clock, 0).astype(np.uint64)
    n = np.where(pods.has_number != 0, pods.number, 0).astype(np.uint64)
    m = np.where(pods.has_memory != 0, pods.memory, 0).astype(np.uint64)
    order = np.lexsort((np.arange(P), m, n, c)).astype(np.int64)
    blocks = [order[i:i + block] for i in range(0, P, block)]
    owner = np.arange(len(blocks)) % world
    if snake:  # boustrophedon deal: 0..W-1, W-1..0, ...
        rev = (np.arange(len(blocks)) // world) % 2 == 1
        owner = np.where(rev, world - 1 - owner, owner)
    mine = [[b for b, o in zip(blocks, owner) if o == r] for r in range(world)]
    return [np.ascontiguousarray(np.concatenate(x) if x else np.zeros(0, np.int64))
            for x in mine]


# ---- sharded greedy batch (config 5 across GPUs) ------------------------------------------
GREEDY_CARD_CAPACITY = 1  # include/yoda.h YODA_GREEDY_CARD_CAPACITY


class HandleShard:
    """A libyoda handle (one node shard) as seen by sharded_greedy."""

    def __init__(self, handle, device):
        self.h = handle
        self.device = device
        self.bufs = None
        if device.type == "cuda":
            handle.set_stream(torch.cuda.current_stream(device).cuda_stream)

    @property
    def generic(self) -> bool:
        return self.h.generic

    def upload_pods(self, pods):
        self.h.upload_pods(pods)

    def phase1(self) -> ShardBuffers:
        from .soa import MODE_SCV
        if self.bufs is None or self.bufs.n_pods != self.h.n_pods:
            self.bufs = ShardBuffers(self.h.n_pods, self.device)
        self.h.shard_phase1(MODE_SCV, self.bufs.maxima.data_ptr(), self.bufs.counts.data_ptr())
        return self.bufs

    def phase1_witness(self) -> ShardBuffers:
        """Capacity windows: phase 1 with the maxima witnesses (yoda_shard_phase1_witness)."""
        if self.bufs is None or self.bufs.n_pods != self.h.n_pods:
            self.bufs = ShardBuffers(self.h.n_pods, self.device)
        b = self.bufs
        b.ensure_witness()
        self.h.shard_phase1_witness(b.maxima.data_ptr(), b.counts.data_ptr(), b.wit.data_ptr())
        return b

    def witness_prepare(self, b: ShardBuffers):
        self.h.shard_witness_prepare(b.maxima.data_ptr(), b.maxima_local.data_ptr(),
                                     b.wit.data_ptr())

    def witness(self):
        """(maxima [6, P], wit [12, P]) after the merge and topk(), caller's pod order."""
        return self.h.shard_witness_download(self.bufs.maxima.data_ptr(), self.bufs.wit.data_ptr())

    def topk(self, k: int | None = None, deep: int = 0):
        return self.h.shard_topk(self.bufs.maxima.data_ptr(), self.bufs.counts.data_ptr(), k,
                                 deep)

    def best_one(self, i: int):
        return self.h.shard_best_one(i)

    def set_node_state(self, nodes, alloc, card_number):
        self.h.set_node_state(nodes, alloc, card_number)


def merge_topk(ts_list: Sequence[np.ndarray], ti_list: Sequence[np.ndarray], k: int):
    """The first k of the union of the shards' candidate lists ([k, P] each), in the lists'
    order (score desc, node asc; padding -1.0 / 0xFFFFFFFF sorts last).  The global top-k is
    contained in the union of the shards' top-k, so this is exact.  (A numpy restatement of
    libyoda's merge for exact lists; the drivers call merge_gathered.)"""
    S = np.concatenate([np.asarray(t, np.float64) for t in ts_list], axis=0)
    I = np.concatenate([np.asarray(t).astype(np.uint64) for t in ti_list], axis=0)
    o = np.lexsort((I, -S), axis=0)[:k]
    return (np.take_along_axis(S, o, axis=0),
            np.take_along_axis(I, o, axis=0).astype(np.uint32))


def merge_gathered(gathered) -> tuple:
    """The world's gathered [2, d, P] lists (scores; nodes as f64) merged by libyoda's
    yoda_merge_shard_lists -- the merge yoda_comm_greedy runs, so both drivers take the same
    lists (deep capacity lists cut where an unlisted node could enter)."""
    from .capi import merge_shard_lists
    S = np.stack([np.asarray(x[0], np.float64) for x in gathered])
    I = np.stack([np.asarray(x[1]).astype(np.uint32) for x in gathered])
    return merge_shard_lists(S, I)


def sharded_greedy(shards, reduce: Reducer, nodes, pods, flags: int = 0, window: int = 6144,
                   stats: dict | None = None) -> np.ndarray:
    """Greedy batch assignment (yoda_greedy's semantics: sort.go:8-10 queue order, each pick
    adding the pod's scv/memory to the node, algorithm.go:299-303) over node shards.

    Per window: K1 on every shard, maxima MAX / counts SUM all-reduced, per-shard top-k lists
    all-gathered and merged, then the host session (identical on every rank) resolves the
    window in queue order; a pod it cannot certify is scored exactly on every shard against
    the current node state and the (score, node) candidates are all-gathered.  With
    YODA_GREEDY_CARD_CAPACITY phase 1 also merges the maxima witnesses, the session applies
    the capacity certificate, and a pod it cannot certify opens the next window (sized after
    how far the last one got), as the single-handle yoda_greedy does.
    `shards`: this process's shards (HandleShard); `nodes`: the FULL snapshot.  The shards'
    node state is restored at the end."""
    from .capi import GreedySession, greedy_cap_depth, next_window, topk_k, topk_k_capacity
    k = topk_k()
    k_cap = topk_k_capacity()  # the capacity windows' phase-1 depth
    k_deep = greedy_cap_depth()  # their lists merged deeper (yoda_comm_greedy's window sequence)
    gs = GreedySession(nodes, pods, flags)
    order = gs.queue_order()
    P = pods.n_pods
    W = max(1, int(window))
    capacity = bool(flags & GREEDY_CARD_CAPACITY)

    def push():
        n, a, c = gs.take_dirty()
        if n.size:
            for s in shards:
                s.set_node_state(n, a, c)

    windows = exact = restarts = refreshes = 0

    def merged_lists():
        lists = [s.topk() for s in shards]
        g = reduce.gather([np.stack([ts, ti.astype(np.float64)]) for _, ts, ti in lists])
        ts, ti = merge_gathered(g)
        return lists[0][0], ts, ti
    generic = any(s.generic for s in shards)
    try:
        if generic:
            # the U64 record path has no candidate lists: every pod in queue order is one exact
            # sharded step (ShardExchange) against the current node state
            ex = ShardExchange([s.h for s in shards], reduce, shards[0].device, path_code=2)
            from .soa import MODE_SCV
            ex.bufs = [ShardBuffers(1, shards[0].device) for _ in shards]
            for q in range(P):
                push()
                one = pods.take(order[q:q + 1])
                for s in shards:
                    s.upload_pods(one)
                ex.step(MODE_SCV)
                gs.assign(q, int(shards[0].h.download_picks()[0][0]))
                exact += 1
            push()
        if capacity and not generic:
            ws, Wc = 0, W
            while ws < P:
                wn = min(Wc, P - ws)
                push()
                win = pods.take(order[ws:ws + wn])
                for s in shards:
                    s.upload_pods(win)
                bufs = [s.phase1_witness() for s in shards]
                sb = dict(zip(map(id, bufs), shards))
                merge_witness(reduce, bufs, lambda b: sb[id(b)].witness_prepare(b))
                lists = [s.topk(k_cap, k_deep) for s in shards]
                g = reduce.gather([np.stack([ts, ti.astype(np.float64)]) for _, ts, ti in lists])
                ts, ti = merge_gathered(g)
                mx, wit = shards[0].witness()
                gs.begin_window(ws, ts.shape[0], lists[0][0], ts, ti)
                gs.set_witness(mx, wit[:6], wit[6:])
                nxt = gs.resolve()
                windows += 1
                if nxt < wn:  # the uncertified pod opens the next window (yoda_greedy's rule)
                    restarts += 1
                    ws += nxt
                    Wc = next_window(nxt, W)
                else:
                    ws += wn
                    Wc = min(W, 2 * Wc)
        for ws in (range(0, P, W) if not capacity and not generic else ()):
            wn = min(W, P - ws)
            push()
            win = pods.take(order[ws:ws + wn])
            for s in shards:
                s.upload_pods(win)
            merge_phase1(reduce, [s.phase1() for s in shards])
            counts, ts, ti = merged_lists()
            gs.begin_window(ws, k, counts, ts, ti)
            # mid-window list refresh (yoda_greedy's): every 8 exact pods, when
            # >= 16 of the next 256 window pods are uncertified, every shard's top-k runs again
            # against the current state (phase 1's masks and maxima stay valid)
            fb_since = 0
            while True:
                i = gs.resolve()
                if i >= wn:
                    break
                fb_since += 1
                if fb_since >= 8 and wn - i >= 512:
                    fb_since = 0
                    if gs.uncertified(i + 1, 256) >= 16:
                        push()
                        _, ts, ti = merged_lists()
                        gs.refresh(i, ts, ti)
                        refreshes += 1
                        i = gs.resolve()
                        if i >= wn:
                            break
                push()
                cands = reduce.gather([np.array(s.best_one(i), np.float64) for s in shards])
                bs, bn = -1.0, -1
                for sc, nd in cands:
                    nd = int(nd)
                    if nd >= 0 and (sc > bs or (sc == bs and nd < bn)):
                        bs, bn = float(sc), nd
                if bn < 0:
                    raise RuntimeError(f"greedy: no feasible node for window pod {i}")
                gs.assign(ws + i, bn)
                exact += 1
            windows += 1
        push()
    finally:
        n, a, c = gs.touched_original()
        if n.size:
            for s in shards:
                s.set_node_state(n, a, c)
    pick, resolved, assigned = gs.picks()
    if stats is not None:
        stats.update(windows=windows, exact_pods=exact, certified_pods=resolved,
                     restarts=restarts, refreshes=refreshes)
    gs.close()
    return pick
