"""Sharded greedy batch (config 5 across GPUs) on CPU: the real driver (yoda_amd/dist.py
sharded_greedy) and the real host session (libyoda yoda_gs_*, pure host code), with each
shard's device work (K1 counts/maxima, top-k lists, exact single-pod best) computed by the
oracle for that shard's nodes.  The picks must equal the sequential oracle's
(oracle_greedy: sort.go:8-10 order, algorithm.go:299-303 assume), including the
YODA_GREEDY_CARD_CAPACITY extension.  World 1 (three shards in one process) and world 2 over
gloo."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from yoda_amd import synth
from yoda_amd.capi import merge_shard_lists, topk_k, topk_k_capacity
from yoda_amd.dist import Reducer, ShardBuffers, merge_topk, shard_bounds, sharded_greedy
from yoda_amd.soa import MODE_SCV

P, N = 60, 40


# contended clusters hold more nodes per shard than the capacity windows' deep lists
# (yoda_greedy_cap_depth, 64), so those lists end before the feasible set and windows restart
N_CONTENDED, P_CONTENDED = 240, 200


def _cluster(contended=False, seed=5):
    nodes = synth.make_nodes(N_CONTENDED if contended else N, seed=seed)
    pods = synth.make_pods(P_CONTENDED if contended else P, seed=seed + 1, priorities=True)
    if not contended:
        nodes.total_memory_sum[3] = 0  # a zero-total node: the Error status
        return nodes.normalized(), pods.normalized()
    # identical nodes and pods: every candidate list is a tie, each pick drops its node below
    # the list's threshold, and after k picks the resolve must fall back to exact scoring
    for f in ("card_number", "card_count", "free_memory_sum", "total_memory_sum",
              "alloc_memory"):
        getattr(nodes, f)[:] = getattr(nodes, f)[0]
    for f in ("card_free_memory", "card_total_memory", "card_clock", "card_bandwidth",
              "card_core", "card_power", "card_healthy"):
        getattr(nodes, f)[:] = getattr(nodes, f)[0]
    pods.has_number[:], pods.number[:] = 1, 1
    pods.has_memory[:], pods.memory[:] = 1, 2000
    pods.has_clock[:] = 0
    return nodes.normalized(), pods.normalized()


class OracleShard:
    """Nodes [lo, hi) of a mutable copy of the snapshot; device work done by the oracle."""
    generic = False

    def __init__(self, nodes, lo, hi):
        self.nodes = nodes.slice(0, nodes.n_nodes)  # a copy
        self.nodes.alloc_memory = np.array(nodes.alloc_memory, np.uint64)
        self.nodes.card_number = np.array(nodes.card_number, np.uint64)
        self.lo, self.hi = lo, hi
        self.bufs = None

    def upload_pods(self, pods):
        self.pods = pods

    def _detail(self, p):
        _, feas, raw, _ = oracle.pod_detail(self.nodes, self.pods, p)
        f = np.nonzero(feas[self.lo:self.hi])[0] + self.lo
        return f, raw

    def phase1(self):
        n = self.pods.n_pods
        res = oracle.schedule(self.nodes.slice(self.lo, self.hi), self.pods, MODE_SCV)
        self.bufs = ShardBuffers(n, torch.device("cpu"))
        self.bufs.maxima.copy_(torch.from_numpy(res.maxima.T.copy().reshape(-1).view(np.int64)))
        nz = [int((self.nodes.total_memory_sum[self._detail(p)[0]] == 0).sum()) for p in range(n)]
        self.bufs.counts.copy_(torch.tensor(list(res.n_feasible.astype(np.int64)) + nz,
                                            dtype=torch.int32))
        return self.bufs

    def topk(self, k=None, deep=0):
        # deep lists (capacity windows): the exact first `deep` -- exact down to their end, as
        # libyoda's merged ones are
        k, n = max(topk_k() if k is None else k, deep), self.pods.n_pods
        ts = np.full((k, n), -1.0)
        ti = np.full((k, n), 0xFFFFFFFF, np.uint32)
        for p in range(n):
            f, raw = self._detail(p)
            sc = np.where(self.nodes.total_memory_sum[f] == 0, 0, raw[f])
            o = np.lexsort((f, -sc))[:k]
            ts[:len(o), p], ti[:len(o), p] = sc[o], f[o]
        counts = self.bufs.counts.numpy().view(np.uint32).reshape(2, n).copy()
        return counts, ts, ti

    def phase1_witness(self):
        """Phase 1 plus, per maxima field, the shard's witnesses: feasible nodes whose
        qualifying cards (collection.go:46) reach the shard's maximum, and the lowest one."""
        b = self.phase1()
        b.ensure_witness()
        n, nd = self.pods.n_pods, self.nodes
        mx = b.maxima.numpy().view(np.uint64).reshape(6, n)
        wc = np.zeros((6, n), np.uint32)
        wn = np.full((6, n), 0xFFFFFFFF, np.uint32)
        K = nd.card_free_memory.shape[1]
        for p in range(n):
            f, _ = self._detail(p)
            if f.size == 0:
                continue
            m = int(self.pods.memory[p]) if self.pods.has_memory[p] else 0
            c = int(self.pods.clock[p]) if self.pods.has_clock[p] else 0
            real = np.arange(K)[None, :] < nd.card_count[f][:, None]
            q = real & (nd.card_free_memory[f] >= m) & (nd.card_clock[f] >= c)
            anyq = q.any(axis=1)
            fields = (nd.card_bandwidth, nd.card_clock, nd.card_core, nd.card_free_memory,
                      nd.card_power, nd.card_total_memory)  # MaxValue order
            for fi, arr in enumerate(fields):
                contrib = np.where(q, arr[f], 0).max(axis=1)
                hit = anyq & (contrib == mx[fi, p])
                wc[fi, p] = hit.sum()
                if hit.any():
                    wn[fi, p] = f[hit].min()
        b.wit.copy_(torch.from_numpy(np.concatenate([wc, wn]).reshape(-1).view(np.int32)))
        return b

    def witness_prepare(self, b):
        n = self.pods.n_pods
        off = (b.maxima_local != b.maxima).numpy()
        w = b.wit.numpy()
        w[:6 * n][off] = 0
        w[6 * n:][off] = -1

    def witness(self):
        n = self.pods.n_pods
        return (self.bufs.maxima.numpy().view(np.uint64).reshape(6, n).copy(),
                self.bufs.wit.numpy().view(np.uint32).reshape(12, n).copy())

    def best_one(self, i):
        f, raw = self._detail(i)
        if f.size == 0:
            return -1.0, -1
        b = raw[f].max()
        return float(b), int(f[raw[f] == b][0])

    def set_node_state(self, nodes, alloc, card_number):
        self.nodes.alloc_memory[nodes] = alloc
        self.nodes.card_number[nodes] = card_number


def _want(nodes, pods, flags):
    pick, _ = oracle.greedy(nodes, pods, MODE_SCV, flags)
    return pick


@pytest.mark.parametrize("contended", [False, True])
@pytest.mark.parametrize("flags,window", [(0, 7), (0, 4096), (1, 4096), (1, 5)])
def test_sharded_greedy_local(flags, window, contended):
    nodes, pods = _cluster(contended)
    b = shard_bounds(nodes.n_nodes, 3)
    shards = [OracleShard(nodes, int(b[r]), int(b[r + 1])) for r in range(3)]
    stats = {}
    got = sharded_greedy(shards, Reducer(local=True), nodes, pods, flags, window, stats)
    np.testing.assert_array_equal(got, _want(nodes, pods, flags))
    if contended and flags == 0 and window == 4096:
        assert stats["exact_pods"] > 0  # the fallback path ran
    if contended and flags == 1 and window == 4096:
        assert stats["restarts"] > 0    # the capacity certificate failed and windows restarted
    for s in shards:  # node state restored
        np.testing.assert_array_equal(s.nodes.alloc_memory, nodes.alloc_memory)
        np.testing.assert_array_equal(s.nodes.card_number, nodes.card_number)


def _worker(rank, world, port, flags, contended, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nodes, pods = _cluster(contended)
        b = shard_bounds(nodes.n_nodes, world)
        shard = OracleShard(nodes, int(b[rank]), int(b[rank + 1]))
        q.put((rank, sharded_greedy([shard], Reducer(), nodes, pods, flags, 16)))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("flags,contended", [(0, False), (0, True), (1, False), (1, True)])
def test_sharded_greedy_gloo(flags, contended):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, flags, contended, q))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nodes, pods = _cluster(contended)
    want = _want(nodes, pods, flags)
    for rank, got in outs:
        np.testing.assert_array_equal(got, want, err_msg=f"rank {rank}")


def test_sharded_greedy_refresh():
    """A 1,100-pod window of a contended fleet (identical pods and nodes: each list's nodes are
    used up by the pods before it): the driver's mid-window list refresh (yoda_gs_uncertified /
    yoda_gs_refresh, as yoda_greedy's) runs, and the picks are still the sequential oracle's."""
    big = 1100
    nodes = synth.make_nodes(N, seed=5)
    pods = synth.make_pods(big, seed=6, priorities=True)
    for f in ("card_number", "card_count", "free_memory_sum", "total_memory_sum",
              "alloc_memory"):
        getattr(nodes, f)[:] = getattr(nodes, f)[0]
    for f in ("card_free_memory", "card_total_memory", "card_clock", "card_bandwidth",
              "card_core", "card_power", "card_healthy"):
        getattr(nodes, f)[:] = getattr(nodes, f)[0]
    pods.has_number[:], pods.number[:] = 1, 1
    pods.has_memory[:], pods.memory[:] = 1, 300
    pods.has_clock[:] = 0
    nodes, pods = nodes.normalized(), pods.normalized()
    b = shard_bounds(N, 2)
    shards = [OracleShard(nodes, int(b[r]), int(b[r + 1])) for r in range(2)]
    stats = {}
    got = sharded_greedy(shards, Reducer(local=True), nodes, pods, 0, 4096, stats)
    np.testing.assert_array_equal(got, _want(nodes, pods, 0))
    assert stats["refreshes"] > 0 and stats["exact_pods"] > 0, stats


def _merge_restated(S, I, k_exact):
    """yoda_merge_shard_lists restated: the union in (score desc, node asc) order, cut -- for
    deep lists -- after the first k_exact at the first entry not above every shard's last."""
    world, kl, wn = S.shape
    ts = np.full((kl, wn), -1.0)
    ti = np.full((kl, wn), 0xFFFFFFFF, np.uint32)
    deep = kl > topk_k_capacity()
    for p in range(wn):
        ent, lasts = [], []
        for r in range(world):
            ln = 0
            while ln < kl and I[r, ln, p] != 0xFFFFFFFF:
                ln += 1
            ent += [(-S[r, j, p], int(I[r, j, p])) for j in range(ln)]
            if ln:
                lasts.append((-S[r, ln - 1, p], int(I[r, ln - 1, p])))
        ent.sort()
        cut = max(lasts) if deep and lasts else None
        for j, e in enumerate(ent[:kl]):
            if cut is not None and j >= topk_k() and not e < cut:
                break
            ts[j, p], ti[j, p] = -e[0], e[1]
    return ts, ti


@pytest.mark.parametrize("kl", [8, 16, 64])
def test_merge_shard_lists(kl):
    """The list merge both sharded greedy drivers call (yoda_merge_shard_lists): exact lists
    equal merge_topk's union; deep lists (kl > topk_k_capacity) end where a node a shard left
    unlisted could enter."""
    rng = np.random.default_rng(kl)
    world, wn = 3, 40
    S = np.full((world, kl, wn), -1.0)
    I = np.full((world, kl, wn), 0xFFFFFFFF, np.uint32)
    for r in range(world):
        for p in range(wn):
            ln = int(rng.integers(0, kl + 1))  # short (ended) and full lists
            sc = np.sort(rng.integers(0, 30, ln).astype(np.float64))[::-1]  # ties across shards
            nd = np.sort(rng.choice(np.arange(r * 1000, r * 1000 + 500), ln, replace=False))
            o = np.lexsort((nd, -sc))
            S[r, :ln, p], I[r, :ln, p] = sc[o], nd[o]
    ts, ti = merge_shard_lists(S, I)
    want_s, want_i = _merge_restated(S, I, topk_k())
    np.testing.assert_array_equal(ts, want_s)
    np.testing.assert_array_equal(ti, want_i)
    if kl <= topk_k_capacity():  # exact lists: the plain union
        ms, mi = merge_topk(list(S), list(I), kl)
        np.testing.assert_array_equal(ti, mi)
        np.testing.assert_array_equal(ts, np.where(mi == 0xFFFFFFFF, -1.0, ms))
    # pods before `from` are left as initialised
    ts2, ti2 = merge_shard_lists(S, I, from_=wn // 2)
    np.testing.assert_array_equal(ti2[:, :wn // 2], 0xFFFFFFFF)
    np.testing.assert_array_equal(ti2[:, wn // 2:], ti[:, wn // 2:])
