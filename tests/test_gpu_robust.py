"""GPU parity off the homogeneous happy path: mixed-model nodes (per-card GPU models) and memory
fields beyond 32 bits (memory ranks on the N32 path), against the C oracle.

The block kernels decide mixed-model nodes with lane = node loops over their free-ordered cards
(k1_block_n32: PodFitsClock count + smallest/largest qualifying-set maxima; k2_block_n32: the
row B'[q] with the clock test folded in), and a snapshot whose memory does not fit 32 bits keeps
the N32 kernels with ranks in the u32 fields (yoda_layout.h MemTab).  Bar: bit-exact picks,
statuses, feasible counts, ties, top scores and maxima (the same as tests/test_gpu_parity.py)."""
import numpy as np
import pytest

import oracle
from yoda_amd import synth
from yoda_amd.capi import Yoda
from yoda_amd.soa import MODE_DISKIO, MODE_SCV

from test_gpu_parity import _boundary_cluster, assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    y = Yoda(0)
    yield y
    y.close()


@pytest.mark.parametrize("frac", [0.5, 1.0])
def test_mixed_model_nodes_config2(dev, frac):
    nodes, pods = synth.make_config(2)
    nodes = synth.mixed_models(nodes, frac, seed=31)
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    for per_node in (False, True):
        dev.upload_nodes(nodes, per_node_k1=per_node, per_node_k2=per_node)
        assert dev.path == "n32"
        assert_same(dev.eval(pods, MODE_SCV), want)


@pytest.mark.parametrize("seed", range(3))
def test_mixed_boundary_clusters(dev, seed):
    """Every node mixed-model, card frees on the pods' thresholds, clocks of the pods' labels:
    the lane = node clock counts and qualifying-set maxima must never decide a pair wrongly."""
    rng = np.random.default_rng(9100 + seed)
    pods = synth.make_pods(800, int(rng.integers(1 << 30)))
    pods.memory[rng.random(800) < 0.05] = 0
    pods = pods.normalized()
    nodes = _boundary_cluster(rng, 2000, 8, pods)
    nodes = synth.mixed_models(nodes, 0.8, seed=int(rng.integers(1 << 30)))
    # per-card TotalMemory too (the one-model nodes become "one model, several totals")
    tot = synth.TOTALS[rng.integers(0, 3, size=nodes.card_total_memory.shape)]
    real = np.arange(8)[None, :] < nodes.card_count[:, None]
    nodes.card_total_memory[:] = np.where(real, np.maximum(tot, nodes.card_free_memory), 0)
    nodes = nodes.normalized()
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    for order in (True, False):
        dev.set_pod_order(order)
        for no_gtab in (False, True):
            dev.upload_nodes(nodes, no_gtab=no_gtab)
            assert_same(dev.eval(pods, MODE_SCV), want)
    dev.set_pod_order(True)


def test_no_uniform_flag_takes_the_mixed_rows(dev):
    """YODA_UPLOAD_NO_UNIFORM: every node is treated as mixed-model (per-card loops)."""
    nodes, pods = synth.make_config(2, pods=600, nodes=3000)
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    dev.upload_nodes(nodes, no_uniform=True)
    assert_same(dev.eval(pods, MODE_SCV), want)


@pytest.mark.parametrize("cfg", [2, 4])
def test_forced_memory_ranks_identical(dev, cfg):
    """Ranks on a snapshot whose memory fits 32 bits: every output identical to the plain
    N32 run and to the oracle (rows, normalized rows and the bitmask too)."""
    nodes, pods = synth.make_config(cfg, pods=900, nodes=3000)
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    outs = []
    for ranks in (False, True):
        dev.upload_nodes(nodes, mem_ranks=ranks)
        assert dev.memory_ranks == ranks and dev.path == "n32"
        got = dev.eval(pods, MODE_SCV)
        assert_same(got, want)
        dev.upload_pods(pods)
        dev.run(MODE_SCV, bitmask=True)
        words = dev.download_bitmask()
        dev.upload_pods(pods.slice(0, 48))
        feas, rows, norm = dev.score_rows(MODE_SCV, norm=True)
        outs.append((words, feas, rows, norm))
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


def test_memory_in_bytes_takes_ranks(dev):
    """Memory in bytes (fields beyond 32 bits): the N32 path with memory ranks, the same
    picks as the F64 per-pair kernels and the oracle; maxima are values (bytes)."""
    nodes, pods = synth.make_config(2)
    nb, pb = synth.memory_in_bytes(nodes, pods)
    want = oracle.schedule(nb, pb, MODE_SCV, threads=8)
    dev.upload_nodes(nb)
    assert dev.path == "n32" and dev.memory_ranks
    got = dev.eval(pb, MODE_SCV)
    assert_same(got, want)
    assert got.maxima[:, 3].max() > (1 << 32)  # FreeMemory maxima in bytes
    dev.upload_nodes(nb, force_f64=True)
    assert dev.path == "f64" and not dev.memory_ranks
    assert_same(dev.eval(pb, MODE_SCV), want)
    # a pod upload BEFORE the snapshot: its thresholds follow the snapshot uploaded later
    z = Yoda(0)
    z.upload_pods(pb)
    z.upload_nodes(nb)
    z.run(MODE_SCV)
    assert_same(z.download(), want)
    z.upload_nodes(nodes)  # back to plain values: the thresholds are re-derived
    z.upload_pods(pods)
    z.run(MODE_SCV)
    assert_same(z.download(), oracle.schedule(nodes, pods, MODE_SCV, threads=8))
    z.close()


@pytest.mark.parametrize("flags", [0, 1])
def test_memory_ranks_greedy(dev, flags):
    """The greedy windows (top-k block K2, capacity witnesses, exact fallbacks) with memory
    ranks: the sequential oracle's picks."""
    nodes, pods = synth.make_config(5, pods=3000, nodes=2500)
    nb, pb = synth.memory_in_bytes(nodes, pods)
    dev.upload_nodes(nb)
    assert dev.memory_ranks
    got = dev.greedy(pb, MODE_SCV, flags)
    want, _ = oracle.greedy(nb, pb, MODE_SCV, flags)
    np.testing.assert_array_equal(got, want)


def test_memory_ranks_sharded(dev):
    """Node shards with memory ranks (each shard its own rank space): the exchanged maxima are
    values, so the merge equals the single handle and the oracle."""
    import torch
    from yoda_amd.dist import ShardExchange
    nodes, pods = synth.make_config(2, pods=500, nodes=3000)
    nb, pb = synth.memory_in_bytes(nodes, pods)
    want = oracle.schedule(nb, pb, MODE_SCV, threads=8)
    bounds = [0, 1400, 3000]
    handles, shards = [], []
    for g in range(2):
        y = Yoda(0)
        shards.append(nb.slice(bounds[g], bounds[g + 1]))
        y.upload_nodes(shards[-1], node_offset=bounds[g])
        y.upload_pods(pb)
        handles.append(y)
    ex = ShardExchange.local(handles, torch.device("cuda:0"), shards, bounds[:2])
    assert all(h.memory_ranks for h in handles) and not ex.narrow
    assert_same(ex.run(MODE_SCV), want)
    for y in handles:
        y.close()


# The 100k x 100k variants (mixed50, bytes, het100k) are checked pod for pod against the
# oracle's digests in tests/test_gpu_fullsize.py.


@pytest.mark.parametrize("mode", [MODE_SCV, MODE_DISKIO])
def test_config4_declared_size(dev, mode):
    """BASELINE config 4 at its declared size (10k pods x 20k nodes), every pod."""
    nodes, pods = synth.make_config(4)
    dev.upload_nodes(nodes)
    got = dev.eval(pods, mode)
    want = oracle.schedule(nodes, pods, mode, threads=16)
    assert_same(got, want, mode)


@pytest.mark.parametrize("seed", range(2))
def test_mixed_block_rules(dev, seed):
    """The whole-block rules for blocks of mixed-model nodes (k1_block_class: ALL past the
    prefix-maxima saturation, NONE / ALL from the per-clock healthy counts; the decoupled K2
    bounds from each node's largest card values) on the cases that must keep them off:
    blocks with more than 4 healthy-card clocks (no table), clocks beyond 16 bits on one-model
    nodes, nodes without cards, scv/number "0" with a clock label no card has, pods without
    scv/memory (every card qualifies), every pod against the oracle."""
    rng = np.random.default_rng(7300 + seed)
    n, p = 4096, 2400
    nodes = synth.make_nodes(n, int(rng.integers(1 << 30)))
    nodes = synth.mixed_models(nodes, 0.7, seed=int(rng.integers(1 << 30)))
    clocks6 = np.array([1200, 1300, 1410, 1500, 1600, 1755], dtype=np.uint64)
    real = np.arange(8)[None, :] < nodes.card_count[:, None]
    six = np.arange(n) < 1024  # the first 16 blocks: six clocks among their cards
    nodes.card_clock[six] = np.where(real[six], clocks6[rng.integers(0, 6, size=(1024, 8))], 0)
    empty = rng.random(n) < 0.02  # CardList empty, CardNumber kept
    for a in (nodes.card_free_memory, nodes.card_total_memory, nodes.card_clock,
              nodes.card_bandwidth, nodes.card_core, nodes.card_power, nodes.card_healthy):
        a[empty] = 0
    nodes.card_count[empty] = 0
    nodes = nodes.normalized()
    pods = synth.make_pods(p, int(rng.integers(1 << 30)))
    pods.has_memory[rng.random(p) < 0.4] = 0
    pods.memory[pods.has_memory == 0] = 0
    zero = rng.random(p) < 0.1  # scv/number "0"
    pods.has_number[zero] = 1
    pods.number[zero] = 0
    odd = rng.random(p) < 0.1  # a clock label no card has
    pods.has_clock[odd] = 1
    pods.clock[odd] = 1999
    pods = pods.normalized()
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    dev.upload_nodes(nodes)
    assert dev.path == "n32"
    assert_same(dev.eval(pods, MODE_SCV), want)
    # a one-model fleet whose clocks exceed 16 bits (no per-clock table) beside it
    big, bpods = synth.make_config(2, pods=1200, nodes=3000)
    big.card_clock[:] = np.where(big.card_clock > 0, big.card_clock * 100, 0)
    bpods.clock[:] = np.where(bpods.has_clock == 1, bpods.clock * 100, 0)
    big, bpods = big.normalized(), bpods.normalized()
    dev.upload_nodes(big)
    assert_same(dev.eval(bpods, MODE_SCV), oracle.schedule(big, bpods, MODE_SCV, threads=8))


def test_consecutive_runs_deferred_pod_arrays(dev):
    """yoda_run's fast path uploads only the pod arrays its kernels read first and copies the
    rest after them (pods_complete): consecutive runs on different batches, a bitmask run and a
    Mode-B run in between (both read the deferred arrays) and a repeated batch must each match
    the oracle (no stale deferred arrays)."""
    nodes, _ = synth.make_config(2, pods=10, nodes=4000)
    dev.upload_nodes(nodes)
    batches = [synth.make_pods(n, s) for n, s in ((3000, 41), (1700, 42), (4100, 43))]
    want = [oracle.schedule(nodes, b, MODE_SCV, threads=8) for b in batches]
    for i in (0, 1, 2, 0, 2):
        dev.upload_pods(batches[i])
        dev.run(MODE_SCV)
        assert_same(dev.download(), want[i])
        if i == 1:  # paths that read the deferred arrays, between two fast runs
            dev.run(MODE_SCV, bitmask=True)
            assert_same(dev.download(), want[i])
            dev.run(MODE_DISKIO)
            assert_same(dev.download(), oracle.schedule(nodes, batches[i], MODE_DISKIO, threads=8),
                        MODE_DISKIO)
