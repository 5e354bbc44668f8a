"""Node-sharded evaluation across GPUs: the two exchange steps of SURVEY.md §8e.

Each rank (one process per GPU) holds a contiguous node block and the full pod batch.
Per batch:
  1. K1 on the shard -> per-pod partial maxima (MAX) and n_feasible / n_zero_total (SUM):
     CollectMaxValues is a reduction over ALL nodes (collection.go:30-55), so the maxima
     must be global before any score is final.
  2. K2 on the shard with the global maxima -> per-pod (best raw score MAX, then the lowest
     node index among shards reaching it MIN, tie counts SUM, lowest raw score MIN).
Collectives are torch.distributed all-reduces on device tensors (backend "nccl" = RCCL over
xGMI on MI355X; "gloo" in the CPU tests).  libyoda launches on torch's current stream so
the collectives are ordered after the kernels without host synchronisation.

uint64/uint32 buffers are reduced through their signed views with the sign bit flipped,
which maps unsigned order onto signed order (MAX/MIN stay exact for all 64-bit values).
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
        self.lowest = torch.empty(P, dtype=torch.int64, device=device)

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


def merge_phase1(reduce: Reducer, bufs: List[ShardBuffers]):
    """Global maxima (MAX, unsigned) and feasible / zero-total counts (SUM)."""
    for b in bufs:
        _flip(b.maxima, I64_SIGN)
    reduce([b.maxima for b in bufs], "max")
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
        _flip(b.idx, I32_SIGN)
    reduce([b.idx for b in bufs], "min")
    for b in bufs:
        _flip(b.idx, I32_SIGN)
    reduce([b.ties for b in bufs], "sum")
    reduce([b.lowest for b in bufs], "min")


def agree_on_path(reduce: Reducer, handles, shards, offsets, device):
    """Every shard must run the SAME record path: the exactness bounds of the fast paths
    involve maxima contributed by other shards.  Take the widest path any
    shard needs (N32 < F64 < U64) and re-upload the shards that chose a narrower one."""
    codes = [torch.tensor([h.path_code], dtype=torch.int64, device=device) for h in handles]
    reduce(codes, "max")
    target = int(codes[0].item())
    for h, nodes, off in zip(handles, shards, offsets):
        if h.path_code != target:
            h.upload_nodes(nodes, node_offset=off, force_generic=target == 2,
                           force_f64=target == 1)
    return target


class ShardExchange:
    """Drives libyoda handles (one per shard) through the sharded entry points."""

    def __init__(self, handles, reducer: Reducer, device):
        self.handles = list(handles)
        self.reduce = reducer
        self.device = device
        self.bufs = [ShardBuffers(h.n_pods, device) for h in self.handles]
        stream = torch.cuda.current_stream(device).cuda_stream if device.type == "cuda" else 0
        for h in self.handles:
            h.set_stream(stream)

    @classmethod
    def local(cls, handles, device, shards=None, offsets=None):
        """Several shards in one process (single-GPU testing).  Pass the node shards to
        enforce a common record path."""
        red = Reducer(local=True)
        if shards is not None:
            agree_on_path(red, handles, shards, offsets, device)
        return cls(handles, red, device)

    @classmethod
    def distributed(cls, handle, device, shard=None, offset=0, group=None):
        """One shard per rank over torch.distributed (RCCL)."""
        red = Reducer(group=group)
        if shard is not None:
            agree_on_path(red, [handle], [shard], [offset], device)
        return cls([handle], red, device)

    def _prepare(self, h, b: ShardBuffers):
        p = ShardBuffers.ptr
        h.shard_prepare_merge(p(b.best_g), p(b.best), p(b.idx), p(b.ties))

    def step(self, mode: int):
        """One batch: phase1, merge, phase2, merge, finalize — all asynchronous."""
        p = ShardBuffers.ptr
        for h, b in zip(self.handles, self.bufs):
            h.shard_phase1(mode, p(b.maxima), p(b.counts))
        merge_phase1(self.reduce, self.bufs)
        for h, b in zip(self.handles, self.bufs):
            h.shard_phase2(mode, p(b.maxima), p(b.counts), p(b.best), p(b.idx), p(b.ties),
                           p(b.lowest))
        hb = dict(zip(map(id, self.bufs), self.handles))
        merge_phase2(self.reduce, self.bufs, lambda b: self._prepare(hb[id(b)], b))
        for h, b in zip(self.handles, self.bufs):
            h.shard_finalize(mode, p(b.counts), p(b.best_g), p(b.idx), p(b.ties), p(b.lowest))

    def run(self, mode: int) -> EvalResult:
        self.step(mode)
        torch.cuda.synchronize(self.device) if self.device.type == "cuda" else None
        return self.handles[0].download()


def shard_bounds(n_nodes: int, world: int) -> np.ndarray:
    """Contiguous node blocks, one per rank."""
    return np.linspace(0, n_nodes, world + 1).astype(np.int64)
