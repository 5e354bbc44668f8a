"""N>1 path on CPU: two gloo ranks, each holding a node shard, merge their exchange buffers
with the collectives of yoda_amd/dist.py.  The per-shard buffers are what libyoda's
yoda_shard_phase1/phase2 produce (computed here from the oracle, which has global
knowledge); after the merge every rank must hold the single-shard (whole cluster) values."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from yoda_amd import synth
from yoda_amd.dist import (Reducer, ShardBuffers, merge_phase1, merge_phase2,
                           merge_phase2_packed, shard_bounds)
from yoda_amd.soa import MODE_SCV

P, N = 24, 90


def _cluster(compact=False):
    nodes = synth.make_nodes(N, seed=314)
    pods = synth.make_pods(P, seed=271)
    if not compact:
        # unsigned values above 2^63 exercise the sign-flip MAX
        nodes.card_bandwidth[5, :] = np.uint64((1 << 64) - 3)
    else:
        # N32 range (the narrow int32 MAX): fields up to 2^32 - 2 and equal-score nodes
        nodes.card_free_memory[3, 0] = np.uint64(0xFFFFFFFE)
        nodes.card_total_memory[3, 0] = np.uint64(0xFFFFFFFE)
        for f in ("card_free_memory", "card_total_memory", "card_clock", "card_bandwidth",
                  "card_core", "card_power", "card_healthy", "card_number", "card_count",
                  "free_memory_sum", "total_memory_sum", "alloc_memory"):
            getattr(nodes, f)[60] = getattr(nodes, f)[10]  # a tie across the shards
    nodes.total_memory_sum[7] = 0
    return nodes.normalized(), pods


def _expected(nodes, pods):
    """Per-pod global exchange values over the whole cluster."""
    res = oracle.schedule(nodes, pods, MODE_SCV)
    exp = {"maxima": res.maxima.T.copy(), "nf": res.n_feasible.astype(np.int64)}
    best, idx, ties, low, nz = [], [], [], [], []
    for p in range(P):
        _, feas, raw, _ = oracle.pod_detail(nodes, pods, p)
        f = np.nonzero(feas)[0]
        nz.append(int((nodes.total_memory_sum[f] == 0).sum()))
        if f.size == 0:
            best.append(-1), idx.append(0xFFFFFFFF), ties.append(0), low.append((1 << 63) - 1)
            continue
        b = raw[f].max()
        best.append(int(b)), idx.append(int(f[raw[f] == b][0]))
        ties.append(int((raw[f] == b).sum())), low.append(int(raw[f].min()))
    exp.update(best=np.array(best), idx=np.array(idx, np.uint64), ties=np.array(ties),
               low=np.array(low), nz=np.array(nz))
    return exp


def _shard_buffers(nodes, pods, lo, hi):
    """What yoda_shard_phase1/phase2 would write for nodes [lo, hi)."""
    shard = nodes.slice(lo, hi)
    res = oracle.schedule(shard, pods, MODE_SCV)
    b = ShardBuffers(P, torch.device("cpu"))
    b.maxima.copy_(torch.from_numpy(res.maxima.T.copy().reshape(-1).view(np.int64)))
    nz = []
    best, idx, ties, low = [], [], [], []
    for p in range(P):
        _, feas, raw, _ = oracle.pod_detail(nodes, pods, p)  # raw uses GLOBAL maxima
        f = np.nonzero(feas[lo:hi])[0] + lo
        nz.append(int((nodes.total_memory_sum[f] == 0).sum()))
        if f.size == 0:
            best.append(-1), idx.append(-1), ties.append(0), low.append((1 << 63) - 1)
            continue
        bb = raw[f].max()
        best.append(int(bb)), idx.append(int(f[raw[f] == bb][0]))
        ties.append(int((raw[f] == bb).sum())), low.append(int(raw[f].min()))
    b.counts.copy_(torch.tensor(list(res.n_feasible.astype(np.int64)) + nz, dtype=torch.int32))
    b.best.copy_(torch.tensor(best))
    b.idx.copy_(torch.tensor(idx, dtype=torch.int32))   # u32 0xFFFFFFFF viewed as int32 -1
    b.ties.copy_(torch.tensor(ties, dtype=torch.int32))
    b.lowest.copy_(torch.tensor(low))
    return b


def _prepare_cpu(b: ShardBuffers):
    """CPU stand-in of libyoda's k_merge_prepare."""
    keep = (b.best == b.best_g) & (b.best_g >= 0)
    b.idx.copy_(torch.where(keep, b.idx, torch.full_like(b.idx, -1)))
    b.ties.copy_(torch.where(keep, b.ties, torch.zeros_like(b.ties)))


def _worker(rank, world, port, q, compact=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nodes, pods = _cluster(compact)
        bnd = shard_bounds(N, world)
        b = _shard_buffers(nodes, pods, int(bnd[rank]), int(bnd[rank + 1]))
        red = Reducer()
        if compact:  # int32 maxima + the packed (score, node) key merge
            merge_phase1(red, [b], narrow=True)
            merge_phase2_packed(red, [b], ib=(N + 1).bit_length())
        else:
            merge_phase1(red, [b])
            merge_phase2(red, [b], _prepare_cpu)
        q.put((rank, b.maxima.numpy().view(np.uint64).copy(), b.counts.numpy().copy(),
               b.best_g.numpy().copy(), b.idx.numpy().view(np.uint32).copy(),
               b.ties.numpy().copy(), b.lowest.numpy().copy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world,compact", [(2, False), (3, False), (2, True), (3, True)])
def test_gloo_shard_merge(world, compact):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, PORTS[(world, compact)], q, compact))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nodes, pods = _cluster(compact)
    exp = _expected(nodes, pods)
    if compact:  # the packed merge leaves lowest = the winning score (fast paths only)
        exp["low"] = exp["best"]
    for rank, mx, cnt, best, idx, ties, low in outs:
        np.testing.assert_array_equal(mx.reshape(6, P), exp["maxima"], err_msg=f"rank {rank}")
        np.testing.assert_array_equal(cnt[:P], exp["nf"])
        np.testing.assert_array_equal(cnt[P:], exp["nz"])
        np.testing.assert_array_equal(best, exp["best"])
        np.testing.assert_array_equal(idx, exp["idx"])
        np.testing.assert_array_equal(ties, exp["ties"])
        np.testing.assert_array_equal(low, exp["low"])


PORTS = {(w, c): _free_port() for w in (2, 3) for c in (False, True)}


@pytest.mark.parametrize("by_key", [True, False])
def test_pod_partition_covers_batch(by_key):
    """dist.pod_partition (bench.py's default --gpus N sharding): disjoint, balanced, covers
    every pod, deterministic; and evaluating each part separately against the whole node
    snapshot gives the unsharded result (the oracle is the checker; pods exchange nothing)."""
    from yoda_amd.dist import pod_partition
    nodes, pods = synth.make_config(2, pods=301, nodes=400)
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=4)
    for world in (1, 2, 3, 8):
        parts = pod_partition(pods, world, by_key=by_key, block=16)
        assert len(parts) == world
        sizes = [len(p) for p in parts]
        assert max(sizes) - min(sizes) <= (16 if by_key else 1)
        allp = np.concatenate(parts)
        assert np.array_equal(np.sort(allp), np.arange(pods.n_pods))
        if by_key:  # whole key-sorted blocks, dealt round-robin
            key = np.lexsort((np.arange(pods.n_pods), pods.memory * pods.has_memory,
                              pods.number * pods.has_number, pods.clock * pods.has_clock))
            assert np.array_equal(parts[0][:16], key[:16])
            if world > 1:
                assert np.array_equal(parts[1][:16], key[16:32])
        again = pod_partition(pods, world, by_key=by_key, block=16)
        assert all(np.array_equal(a, b) for a, b in zip(parts, again))
        for idx in parts[:2]:
            got = oracle.schedule(nodes, pods.take(idx), MODE_SCV, threads=4)
            for f in ("pick", "status", "n_feasible", "n_ties", "top_score"):
                assert np.array_equal(getattr(got, f), getattr(want, f)[idx]), f
    assert [len(p) for p in pod_partition(pods.slice(0, 0), 3)] == [0, 0, 0]


def test_balanced_bounds():
    """dist.balanced_bounds (bench.py re-cuts node blocks by measured K1 + K2 time)."""
    from yoda_amd.dist import balanced_bounds
    b = shard_bounds(100_000, 8)
    assert np.array_equal(balanced_bounds(b, [1.0] * 8), b)  # already even
    costs = [0.86] + [0.71] * 7
    nb = balanced_bounds(b, costs)
    assert nb[0] == 0 and nb[-1] == 100_000 and np.all(np.diff(nb) > 0)
    assert nb[1] < b[1]  # the expensive first shard shrinks
    # estimated cost per new shard (cost spread evenly within each old shard) is equal
    dens = np.repeat(np.array(costs) / np.diff(b), np.diff(b))
    per = [dens[nb[k]:nb[k + 1]].sum() for k in range(8)]
    assert max(per) - min(per) < 1e-3 * sum(per)
    # degenerate inputs: zero costs, one rank, as many nodes as ranks
    assert np.array_equal(balanced_bounds(b, [0.0] * 8), b)
    assert np.array_equal(balanced_bounds([0, 10], [3.0]), [0, 10])
    tight = balanced_bounds([0, 1, 2, 3], [100.0, 0.0, 0.0])
    assert np.array_equal(tight, [0, 1, 2, 3])


def _devices_worker(rank, world, port, q, ids):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from yoda_amd.capi import YodaError
        from yoda_amd.dist import agree_on_devices
        try:
            q.put((rank, agree_on_devices(ids[rank], torch.device("cpu"))))
        except YodaError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shared", ["no", "yes", "other_host"])
def test_gloo_agree_on_devices(shared):
    """dist.agree_on_devices (LibExchange runs it before yoda_comm_init): the ranks all-gather
    their device keys (host hash / PCI bus id); two ranks on one GPU make EVERY rank raise
    YODA_ERR_SAME_DEVICE naming them (so no rank goes on into RCCL's init alone), while the
    same bus id on another host (identical servers of a multi-node job) passes."""
    world = 3
    h0, h1 = "00000000000000aa/", "00000000000000bb/"
    third = {"no": h0 + "0000:25:00.0", "yes": h0 + "0000:05:00.0",
             "other_host": h1 + "0000:05:00.0"}[shared]
    ids = [h0 + "0000:05:00.0", h0 + "0000:15:00.0", third]
    shared = shared == "yes"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_devices_worker, args=(r, world, port, q, ids))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        if shared:
            assert "SAME_DEVICE: ranks 0 and 2" in outs[r], outs[r]
        else:
            assert outs[r] == ids


def _pod_worker(rank, world, port, q):
    """bench.py --gpus N's default (pod sharding): rank r evaluates dist.pod_partition's part r
    against the WHOLE snapshot (the oracle standing in for libyoda on CPU), with nothing
    exchanged but bench.py's max-over-ranks elapsed time; rank 0 gathers the picks only to
    check them."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from yoda_amd.dist import pod_partition
        nodes, pods = synth.make_config(2, pods=300, nodes=400)
        part = pod_partition(pods, world, block=16)[rank]
        res = oracle.schedule(nodes, pods.take(part), MODE_SCV)
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py: elapsed = max over ranks
        q.put((rank, part, res.pick.copy(), res.status.copy(), res.n_ties.copy(), float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_pod_shards_union(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pod_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nodes, pods = synth.make_config(2, pods=300, nodes=400)
    want = oracle.schedule(nodes, pods, MODE_SCV)
    seen = np.zeros(pods.n_pods, int)
    for rank, part, pick, status, ties, tmax in outs:
        assert tmax == float(world)
        seen[part] += 1
        np.testing.assert_array_equal(pick, want.pick[part])
        np.testing.assert_array_equal(status, want.status[part])
        np.testing.assert_array_equal(ties, want.n_ties[part])
    assert (seen == 1).all()
