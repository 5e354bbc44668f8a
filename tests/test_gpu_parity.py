"""GPU parity: libyoda (HIP, gfx950) against the C oracle on identical seeded inputs.

Bar: bit-exact picks, statuses, feasible counts, tie counts, top scores and PreScore maxima
(integer work; the Mode-B float math is compared through its integer scores).  Ties are
broken by lowest node index in both, and the tie count is the size of the set k8s
selectHost would draw from."""
import numpy as np
import pytest

import oracle
import pyoracle as po
from yoda_amd import synth
from yoda_amd.capi import Yoda
from yoda_amd.soa import MODE_DISKIO, MODE_SCV, NodeSoA

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    y = Yoda(0)
    yield y
    y.close()


def assert_same(got, want, mode=MODE_SCV, pods=None):
    sel = slice(None) if pods is None else pods
    np.testing.assert_array_equal(got.status[sel], want.status[sel], err_msg="status")
    np.testing.assert_array_equal(got.pick[sel], want.pick[sel], err_msg="pick")
    np.testing.assert_array_equal(got.n_feasible[sel], want.n_feasible[sel], err_msg="n_feasible")
    ok = want.status[sel] == 0
    np.testing.assert_array_equal(got.n_ties[sel][ok], want.n_ties[sel][ok], err_msg="n_ties")
    np.testing.assert_array_equal(got.top_score[sel][ok], want.top_score[sel][ok],
                                  err_msg="top_score")
    if mode == MODE_SCV:
        np.testing.assert_array_equal(got.maxima[sel], want.maxima[sel], err_msg="maxima")


def run_both(dev, nodes, pods, mode=MODE_SCV, force_generic=False, threads=8, force_f64=False):
    dev.upload_nodes(nodes, force_generic=force_generic, force_f64=force_f64)
    got = dev.eval(pods, mode)
    want = oracle.schedule(nodes, pods, mode, threads=threads)
    return got, want


def test_kat1(dev):
    from test_oracle import kat1_cluster
    scvs, pod = kat1_cluster()
    nodes, pods = oracle.from_py(scvs, [pod])
    for generic in (False, True):
        got, want = run_both(dev, nodes, pods, force_generic=generic)
        assert int(got.pick[0]) == 1 and int(got.top_score[0]) == 4061
        assert list(map(int, got.maxima[0])) == [1200, 1500, 108, 16000, 400, 32000]
        assert_same(got, want)


@pytest.mark.parametrize("mode", [MODE_SCV, MODE_DISKIO])
def test_config1(dev, mode):
    nodes, pods = synth.make_config(1)
    got, want = run_both(dev, nodes, pods, mode)
    assert_same(got, want, mode)


@pytest.mark.parametrize("mode", [MODE_SCV, MODE_DISKIO])
def test_config2_full(dev, mode):
    nodes, pods = synth.make_config(2)   # 1k pods x 5k nodes, seed 42
    got, want = run_both(dev, nodes, pods, mode)
    assert dev.path == "n32"
    assert_same(got, want, mode)
    assert (got.status == 0).mean() > 0.5


@pytest.mark.parametrize("mode", [MODE_SCV, MODE_DISKIO])
def test_config4_heterogeneous(dev, mode):
    nodes, pods = synth.make_config(4, pods=2000, nodes=6000)
    got, want = run_both(dev, nodes, pods, mode)
    assert_same(got, want, mode)
    if mode == MODE_SCV:
        # >= 90% of pairs infeasible
        frac = want.n_feasible.astype(np.float64).sum() / (2000 * 6000)
        assert frac < 0.10


@pytest.mark.parametrize("path", ["n32", "f64", "u64"])
def test_every_record_path(dev, path):
    nodes, pods = synth.make_config(2, pods=300, nodes=2000)
    got, want = run_both(dev, nodes, pods, force_generic=path == "u64", force_f64=path == "f64")
    assert dev.path == path
    assert_same(got, want)


def test_wide_memory_fields(dev):
    # free memory in bytes (> 2^32): the N32 kernels with memory ranks (yoda_layout.h MemTab);
    # a wide small field on a mixed-model node (bandwidth > 65535, one card) takes the F64
    # per-pair kernels instead (tests/test_gpu_wide.py: one-model nodes stay on N32)
    nodes, pods = synth.make_config(2, pods=200, nodes=1500)
    nodes.card_free_memory[:] *= np.uint64(1 << 20)
    nodes.card_total_memory[:] *= np.uint64(1 << 20)
    pods.memory[:] *= np.uint64(1 << 20)
    got, want = run_both(dev, nodes, pods)
    assert dev.path == "n32" and dev.memory_ranks
    assert_same(got, want)
    nodes.card_bandwidth[7, 0] = np.uint64(70000)
    got, want = run_both(dev, nodes, pods)
    assert dev.path == "f64" and not dev.memory_ranks
    assert_same(got, want)


@pytest.mark.parametrize("k", [1, 2, 4, 8, 16])
def test_card_slot_variants(dev, k):
    nodes = synth.make_nodes(700, seed=100 + k, cards=k)
    pods = synth.make_pods(200, seed=200 + k)
    got, want = run_both(dev, nodes, pods)
    assert_same(got, want)


def _edge_cluster(rng, n, k):
    nodes = synth.make_nodes(n, int(rng.integers(1 << 30)), cards=k)
    nodes.card_number[rng.random(n) < 0.1] = 0
    nodes.card_clock[rng.random(nodes.card_clock.shape) < 0.2] = 1500
    nodes.card_count[rng.random(n) < 0.1] = rng.integers(0, k + 1)
    return nodes.normalized()


@pytest.mark.parametrize("seed", range(4))
def test_randomized_edges(dev, seed):
    rng = np.random.default_rng(1000 + seed)
    nodes = _edge_cluster(rng, 1500, 8)
    pods = synth.make_pods(400, int(rng.integers(1 << 30)))
    pods.number[rng.random(400) < 0.05] = np.uint64((1 << 64) - 1)
    pods.number[rng.random(400) < 0.05] = 0
    pods.memory[rng.random(400) < 0.05] = np.uint64((1 << 64) - 5)
    pods.clock[rng.random(400) < 0.05] = np.uint64(1 << 60)
    for path in ("n32", "n32-per-node", "f64", "u64"):
        dev.upload_nodes(nodes, force_generic=path == "u64", force_f64=path == "f64",
                         per_node_k1=path == "n32-per-node", per_node_k2=path == "n32-per-node")
        assert dev.path == path.split("-")[0]
        assert_same(dev.eval(pods, MODE_SCV), oracle.schedule(nodes, pods, MODE_SCV, threads=8))


def _boundary_cluster(rng, n, k, pods):
    """Nodes whose card fields sit exactly on the pods' thresholds (free == m, free == m - 1,
    clock == c), mixed one-model / mixed-model nodes, empty and short CardLists, CardNumber
    edge values: the cases where K1's wave bounds must not decide a node wrongly."""
    nodes = synth.make_nodes(n, int(rng.integers(1 << 30)), cards=k)
    mem = pods.memory[pods.has_memory == 1]
    pick = rng.integers(0, max(len(mem), 1), size=nodes.card_free_memory.shape)
    on = rng.random(nodes.card_free_memory.shape) < 0.3
    if len(mem):
        edge = mem[pick].astype(np.int64) - rng.integers(0, 2, size=pick.shape)
        edge = np.clip(edge, 0, None).astype(np.uint64)
        nodes.card_free_memory[on] = np.minimum(edge[on], nodes.card_total_memory[on])
    mixed = rng.random(n) < 0.25
    nodes.card_clock[mixed] = synth.CLOCKS[rng.integers(0, 3, size=(int(mixed.sum()), k))]
    nodes.card_healthy[rng.random(nodes.card_healthy.shape) < 0.2] = 0
    cn = nodes.card_number
    cn[rng.random(n) < 0.05] = np.uint64((1 << 64) - 1)
    cn[rng.random(n) < 0.05] = np.uint64((1 << 32) + 3)
    cn[rng.random(n) < 0.05] = 0
    nodes.card_count[rng.random(n) < 0.1] = rng.integers(0, k + 1)
    return nodes.normalized()


@pytest.mark.parametrize("seed", range(3))
def test_k1_block_classification(dev, seed):
    """The block-classified K1 (N32) against the per-node K1 and the oracle, on sorted and
    unsorted batches (waves of similar or of unrelated pods), including the bitmask."""
    rng = np.random.default_rng(7000 + seed)
    pods = synth.make_pods(900, int(rng.integers(1 << 30)))
    pods.number[rng.random(900) < 0.05] = np.uint64((1 << 32) + 1)
    pods.number[rng.random(900) < 0.05] = np.uint64((1 << 64) - 1)
    pods.number[rng.random(900) < 0.05] = 0
    pods.number[rng.random(900) < 0.05] = 17
    pods.memory[rng.random(900) < 0.05] = 0
    pods = pods.normalized()
    nodes = _boundary_cluster(rng, 2200, 8, pods)
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    words = {}
    for order in (True, False):
        dev.set_pod_order(order)
        for per_node in (False, True):
            dev.upload_nodes(nodes, per_node_k1=per_node, per_node_k2=per_node)
            assert dev.path == "n32"
            assert_same(dev.eval(pods, MODE_SCV), want)
            dev.upload_pods(pods)
            dev.run(MODE_SCV, bitmask=True)
            words[(order, per_node)] = dev.download_bitmask()
    dev.set_pod_order(True)
    ref = words[(False, True)]
    for w in words.values():
        np.testing.assert_array_equal(w, ref)
    bits = np.unpackbits(ref.view(np.uint8), bitorder="little", axis=1)[:, :nodes.n_nodes]
    for p in range(0, 900, 97):
        _, feas, _, _ = oracle.pod_detail(nodes, pods, p)
        np.testing.assert_array_equal(bits[p].astype(bool), feas)


def test_tie_heavy(dev):
    # identical nodes: every feasible node ties; lowest index wins, tie count = n_feasible
    base = synth.make_nodes(1, seed=5)
    n = 3000
    nodes = NodeSoA(**{f: np.repeat(getattr(base, f), n, axis=0)
                       for f in base.__dataclass_fields__})
    pods = synth.make_pods(300, seed=6)
    got, want = run_both(dev, nodes, pods)
    assert_same(got, want)
    ok = want.status == 0
    assert (got.n_ties[ok] == got.n_feasible[ok]).all()


def test_empty_inputs(dev):
    nodes, pods = synth.make_config(2, pods=10, nodes=100)
    zero_nodes = nodes.slice(0, 0)
    got, want = run_both(dev, zero_nodes, pods)
    assert (got.pick == -1).all() and (got.status == 1).all()
    assert_same(got, want)
    dev.upload_nodes(nodes)
    r = dev.eval(pods.slice(0, 0))
    assert r.pick.size == 0


def test_div_zero_and_single_feasible(dev):
    from test_oracle import H
    n0 = po.Scv(card_number=1, card_list=[H(5000)], free_memory_sum=5000, total_memory_sum=0)
    n1 = po.Scv(card_number=1, card_list=[H(5000)], free_memory_sum=5000, total_memory_sum=100)
    n2 = po.Scv(card_number=0, card_list=[], free_memory_sum=0, total_memory_sum=100)
    for scvs in ([n0, n1], [n0, n2], [n2, n2]):
        nodes, pods = oracle.from_py(scvs, [po.Pod(), po.Pod(number=1)], max_cards=2)
        got, want = run_both(dev, nodes, pods)
        assert_same(got, want)


@pytest.mark.parametrize("clock0", [10 ** 15 + 1, (1 << 62) // 100])
def test_normalize_overflow_generic_path(dev, clock0):
    from test_oracle import _overflow_pair
    nodes, pods = oracle.from_py(_overflow_pair(clock0), [po.Pod()])
    got, want = run_both(dev, nodes, pods)
    assert dev.generic  # clock > 2^44 leaves the fast path
    assert_same(got, want)


def test_huge_values_generic(dev):
    rng = np.random.default_rng(77)
    nodes = synth.make_nodes(500, seed=78)
    big = rng.integers(0, 1 << 63, size=nodes.card_free_memory.shape, dtype=np.int64)
    nodes.card_free_memory[:] = big.astype(np.uint64)
    nodes.card_total_memory[:] = (big.astype(np.uint64) * np.uint64(3))
    nodes.total_memory_sum[:] = rng.integers(1, 1 << 62, size=500).astype(np.uint64)
    nodes = nodes.normalized()
    pods = synth.make_pods(100, seed=79)
    got, want = run_both(dev, nodes, pods)
    assert dev.generic
    assert_same(got, want)


def test_bitmask_matches_oracle(dev):
    nodes, pods = synth.make_config(2, pods=64, nodes=1000)
    dev.upload_nodes(nodes)
    dev.upload_pods(pods)
    dev.run(MODE_SCV, bitmask=True)
    words = dev.download_bitmask()
    bits = np.unpackbits(words.view(np.uint8), bitorder="little", axis=1)[:, :1000].astype(bool)
    for p in range(0, 64, 7):
        _, feas, _, _ = oracle.pod_detail(nodes, pods, p)
        np.testing.assert_array_equal(bits[p], feas)


@pytest.mark.parametrize("path", ["n32", "f64", "u64"])
def test_pod_order_is_invisible(dev, path):
    """The device-side batch sort (yoda_order.hip) changes only the visiting order: picks,
    statuses, ties, top scores, maxima, feasible counts, the bitmask and the score rows must
    be identical with it on and off, and equal to the oracle."""
    nodes, pods = synth.make_config(2, pods=700, nodes=2500)
    kw = {"n32": {}, "f64": {"force_f64": True}, "u64": {"force_generic": True}}[path]
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    outs = []
    for order in (True, False):
        dev.set_pod_order(order)
        dev.upload_nodes(nodes, **kw)
        got = dev.eval(pods, MODE_SCV)
        assert_same(got, want)
        dev.upload_pods(pods)
        dev.run(MODE_SCV, bitmask=True)
        words = dev.download_bitmask()
        dev.upload_pods(pods.slice(0, 200))
        feas, rows = dev.score_rows(MODE_SCV)
        outs.append((got, words, feas, rows))
    dev.set_pod_order(True)
    (a, wa, fa, ra), (b, wb, fb, rb) = outs
    for f in ("pick", "status", "n_ties", "top_score", "maxima", "n_feasible"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    np.testing.assert_array_equal(wa, wb)
    np.testing.assert_array_equal(fa, fb)
    np.testing.assert_array_equal(ra, rb)
    for p in (0, 77, 199):
        _, f, raw, _ = oracle.pod_detail(nodes, pods, p)
        np.testing.assert_array_equal(ra[p][f], raw[f])


def test_mode_b_kats(dev):
    from test_oracle import KAT2
    pod = po.Pod(rio=10.0, rcpu=100)
    scvs = [po.Scv(card_number=0, card_list=[], free_memory_sum=0, total_memory_sum=1,
                   cpu=float(c), disk_io=float(d)) for (c, d), _ in KAT2]
    nodes, pods = oracle.from_py(scvs, [pod], max_cards=1)
    got, want = run_both(dev, nodes, pods, MODE_DISKIO)
    assert int(got.pick[0]) == 4 and int(got.top_score[0]) == 10
    assert_same(got, want, MODE_DISKIO)


def test_sharded_merge_on_one_gpu(dev):
    """Simulate G node shards with G handles and the exchange done by torch on the device."""
    import torch
    from yoda_amd.dist import ShardExchange
    nodes, pods = synth.make_config(2, pods=500, nodes=3000)
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    for G in (2, 3):
        bounds = np.linspace(0, nodes.n_nodes, G + 1).astype(int)
        handles, shards = [], []
        for g in range(G):
            y = Yoda(0)
            shards.append(nodes.slice(bounds[g], bounds[g + 1]))
            y.upload_nodes(shards[-1], node_offset=int(bounds[g]))
            y.upload_pods(pods)
            handles.append(y)
        ex = ShardExchange.local(handles, torch.device("cuda:0"), shards,
                                 [int(b) for b in bounds[:-1]], compact=G == 2)
        # G = 2: int32 maxima + the packed (score, node) key merge; G = 3: the 64-bit merge
        assert (ex.ib is not None and ex.narrow) == (G == 2)
        for mode in (MODE_SCV, MODE_DISKIO):
            res = ex.run(mode)
            w = want if mode == MODE_SCV else oracle.schedule(nodes, pods, mode, threads=8)
            assert_same(res, w, mode)
        for y in handles:
            y.close()


@pytest.mark.parametrize("by_key", [True, False])
def test_pod_sharded_on_one_gpu(dev, by_key):
    """Pod sharding (bench.py --gpus N default): G handles, each with the WHOLE node snapshot
    and the pods of dist.pod_partition; the union of their results is the oracle's, with
    nothing exchanged.  More than 128 pods per shard so the device pod sort runs per shard."""
    from yoda_amd.dist import pod_partition
    nodes, pods = synth.make_config(2, pods=1500, nodes=3000)
    for mode in (MODE_SCV, MODE_DISKIO):
        want = oracle.schedule(nodes, pods, mode, threads=8)
        for G in (1, 2, 3, 8):
            parts = pod_partition(pods, G, by_key=by_key)
            dev.upload_nodes(nodes)
            for idx in parts:
                got = dev.eval(pods.take(idx), mode)
                for f in ("status", "pick", "n_feasible"):
                    np.testing.assert_array_equal(getattr(got, f), getattr(want, f)[idx],
                                                  err_msg=f"{f} G={G}")
                ok = want.status[idx] == 0
                np.testing.assert_array_equal(got.n_ties[ok], want.n_ties[idx][ok])
                np.testing.assert_array_equal(got.top_score[ok], want.top_score[idx][ok])
                if mode == MODE_SCV:
                    np.testing.assert_array_equal(got.maxima, want.maxima[idx])


def test_sharded_paths_agree(dev):
    """One shard needs the F64 path (a wide field), the other would pick N32: both must
    end on F64, and the merged result must equal the single-handle result."""
    import torch
    from yoda_amd.dist import ShardExchange
    nodes, pods = synth.make_config(2, pods=300, nodes=2000)
    nodes.card_bandwidth[1500, 0] = np.uint64(70000)   # > 16 bits, mixed model: F64 on shard 1 only
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    shards = [nodes.slice(0, 1000), nodes.slice(1000, 2000)]
    handles = []
    for i, sh in enumerate(shards):
        y = Yoda(0)
        y.upload_nodes(sh, node_offset=1000 * i)
        y.upload_pods(pods)
        handles.append(y)
    assert [h.path for h in handles] == ["n32", "f64"]
    ex = ShardExchange.local(handles, torch.device("cuda:0"), shards, [0, 1000])
    assert [h.path for h in handles] == ["f64", "f64"]
    assert_same(ex.run(MODE_SCV), want)
    for y in handles:
        y.close()


def test_full_size_config3_every_pod(dev):
    """100k pods x 100k nodes on one GPU: EVERY pod's (pick, status, n_feasible, n_ties,
    top score) against the C oracle, through the per-1,024-pod digests of
    tests/golden/fullsize.json (the oracle's 10^10 pairs run in the build container), plus a
    direct oracle sample and size-independent invariants."""
    import fullsize_check as fc
    fx = fc.load("config3")
    nodes, pods = synth.make_config(3)
    fc.check_inputs(fx, nodes, pods)
    dev.upload_nodes(nodes)
    got = dev.eval(pods, MODE_SCV)
    bad = fc.config3_mismatch(fx, got, nodes, pods, oracle)
    assert bad is None, bad
    rng = np.random.default_rng(3)
    # and a direct oracle sample (~0.1 s of the 16-thread C oracle on the GPU box)
    sample = np.sort(rng.choice(pods.n_pods, size=256, replace=False))
    want = oracle.schedule(nodes, pods.take(sample), MODE_SCV, threads=16)
    sub = type(got)(**{f: getattr(got, f)[sample] for f in got.__dataclass_fields__})
    assert_same(sub, want)
    ok = got.status == 0
    assert ((got.pick >= 0) == ok).all()
    assert (got.pick[ok] < nodes.n_nodes).all()
    assert (got.n_ties[ok] >= 1).all() and (got.n_ties[ok] <= got.n_feasible[ok]).all()
    assert (got.n_feasible[got.status == 1] == 0).all()


@pytest.mark.parametrize("mode", [MODE_SCV, MODE_DISKIO])
@pytest.mark.parametrize("path", ["n32", "f64", "u64"])
def test_score_rows_match_oracle(dev, mode, path):
    """yoda_score_rows: the Filter bit and raw Score of every node (plugin row mode)."""
    nodes, pods = synth.make_config(2, pods=24, nodes=900)
    nodes.total_memory_sum[3] = 0
    dev.upload_nodes(nodes, force_f64=path == "f64", force_generic=path == "u64")
    dev.upload_pods(pods)
    feas, rows = dev.score_rows(mode)
    for p in range(pods.n_pods):
        _, f, raw, _ = oracle.pod_detail(nodes, pods, p, mode)
        np.testing.assert_array_equal(feas[p], f)
        ok = f & (nodes.total_memory_sum != 0) if mode == MODE_SCV else f
        np.testing.assert_array_equal(rows[p][ok], raw[ok])
        assert (rows[p][~f] == -1).all()
    want = oracle.schedule(nodes, pods, mode, threads=8)
    assert_same(dev.download(), want, mode)


@pytest.mark.parametrize("mode", [MODE_SCV, MODE_DISKIO])
@pytest.mark.parametrize("path", ["n32", "f64", "u64"])
def test_normalized_rows_match_oracle(dev, mode, path):
    """yoda_score_rows_norm: the device NormalizeScore (scheduler.go:158-183) of every node
    equals the oracle's (oracle_pod_detail norm), -1 where Filter fails.  Includes a pod with
    a single feasible node (highest == lowest: lowest--), one with none, and zero-total
    nodes (their raw score has no Allocate/Actual term in both)."""
    nodes, pods = synth.make_config(2, pods=40, nodes=900)
    nodes.total_memory_sum[3] = 0
    nodes.card_number[5] = 16                       # the only node with 16 cards
    pods.has_number[0], pods.number[0] = 1, 16
    pods.has_memory[0] = pods.has_clock[0] = 0
    pods.has_number[1], pods.number[1] = 1, 17      # no feasible node
    nodes, pods = nodes.normalized(), pods.normalized()
    dev.upload_nodes(nodes, force_f64=path == "f64", force_generic=path == "u64")
    dev.upload_pods(pods)
    feas, rows, norm = dev.score_rows(mode, norm=True)
    for p in range(pods.n_pods):
        _, f, raw, nrm = oracle.pod_detail(nodes, pods, p, mode)
        np.testing.assert_array_equal(feas[p], f)
        np.testing.assert_array_equal(norm[p], nrm, err_msg=f"pod {p}")
        np.testing.assert_array_equal(rows[p][f], raw[f], err_msg=f"pod {p}")
    if mode == MODE_SCV:
        assert feas[0].sum() == 1 and norm[0][5] == 100 and feas[1].sum() == 0
    assert ((norm[feas] >= 0) & (norm[feas] <= 100)).all()


def test_plugin_over_libyoda(dev):
    from yoda_amd.pack import pods_to_dicts
    from yoda_amd.plugin import YodaPlugin, schedule_one
    nodes, pods = synth.make_config(2, pods=30, nodes=700)
    names = [f"node-{i}" for i in range(nodes.n_nodes)]
    dev.upload_nodes(nodes)
    plugin = YodaPlugin(dev, names, nodes)
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    for p, pod in enumerate(pods_to_dicts(pods)):
        node, st = schedule_one(plugin, pod)
        assert (node == names[want.pick[p]]) if want.status[p] == 0 else node is None


@pytest.mark.parametrize("flags", [0, 1])
@pytest.mark.parametrize("path", ["n32", "f64", "u64"])
def test_greedy_matches_sequential_oracle(dev, flags, path):
    """Batched greedy (config 5 semantics, scaled down) == the sequential oracle."""
    nodes, pods = synth.make_config(5, pods=2500, nodes=600)
    dev.upload_nodes(nodes, force_f64=path == "f64", force_generic=path == "u64")
    got = dev.greedy(pods, MODE_SCV, flags)
    want, _ = oracle.greedy(nodes, pods, MODE_SCV, flags)
    np.testing.assert_array_equal(got, want)
    windows, fallbacks = dev.greedy_stats()
    if flags == 0 and path != "u64":
        assert windows >= 1 and fallbacks < pods.n_pods
    # the uploaded snapshot is unchanged afterwards
    assert_same(dev.eval(pods, MODE_SCV), oracle.schedule(nodes, pods, MODE_SCV, threads=8))


@pytest.mark.parametrize("path", ["n32", "f64"])
def test_greedy_several_sorted_windows(dev, path):
    """Several 6144-pod windows (each sorted on the device, outputs read through the
    permutation) with exact single-pod fallbacks (k_greedy_one) == the sequential oracle."""
    nodes, pods = synth.make_config(5, pods=13000, nodes=300)
    dev.upload_nodes(nodes, force_f64=path == "f64")
    got = dev.greedy(pods, MODE_SCV, 0)
    want, _ = oracle.greedy(nodes, pods, MODE_SCV, 0)
    np.testing.assert_array_equal(got, want)
    windows, fallbacks = dev.greedy_stats()
    assert windows == 3 and fallbacks < pods.n_pods


def test_greedy_small_windows_and_mode_b(dev):
    nodes, pods = synth.make_config(5, pods=400, nodes=300)
    pods.priority[:] = 0
    dev.upload_nodes(nodes)
    np.testing.assert_array_equal(dev.greedy(pods, MODE_DISKIO),
                                  oracle.greedy(nodes, pods, MODE_DISKIO)[0])
    # heavy contention: every pod wants the same few nodes
    pods.memory[:] = 1
    pods.has_memory[:] = 1
    np.testing.assert_array_equal(dev.greedy(pods, MODE_SCV), oracle.greedy(nodes, pods)[0])


@pytest.mark.parametrize("path", ["n32", "f64"])
@pytest.mark.parametrize("shape", ["config5", "contended", "zero_total", "wrap"])
def test_greedy_card_capacity_batched(dev, path, shape):
    """YODA_GREEDY_CARD_CAPACITY, batched (windows restart at the first pod the capacity
    certificate cannot clear) == the sequential oracle, on inputs that stress each branch:
    nodes running out of cards (lists exhausted, maxima witnesses lost), identical nodes
    (every list a tie), zero-total nodes (Error status changing with feasibility), and an
    allocated-memory sum wrapping past 2^64."""
    nodes, pods = synth.make_config(5, pods=6000, nodes=500)
    if shape == "contended":
        for f in ("card_number", "card_count", "free_memory_sum", "total_memory_sum",
                  "alloc_memory", "card_free_memory", "card_total_memory", "card_clock",
                  "card_bandwidth", "card_core", "card_power", "card_healthy"):
            getattr(nodes, f)[:] = getattr(nodes, f)[0]
        pods.has_memory[:] = 1
        pods.memory[:] = 100
    elif shape == "zero_total":
        nodes.total_memory_sum[::7] = 0
    elif shape == "wrap":
        pods.has_memory[:5] = 1
        pods.memory[:5] = np.uint64((1 << 64) - 3)
        pods.priority[:5] = 100
    nodes, pods = nodes.normalized(), pods.normalized()
    dev.upload_nodes(nodes, force_f64=path == "f64")
    got = dev.greedy(pods, MODE_SCV, 1)
    want, _ = oracle.greedy(nodes, pods, MODE_SCV, 1)
    np.testing.assert_array_equal(got, want)
    windows, restarts = dev.greedy_stats()
    assert windows >= 2 and restarts < pods.n_pods
    assert_same(dev.eval(pods.slice(0, 300), MODE_SCV),
                oracle.schedule(nodes, pods.slice(0, 300), MODE_SCV, threads=8))


def test_uniform_node_factoring(dev):
    """Nodes with one GPU model take the factored K1/K2 branch; mixed nodes the per-card
    one.  Both must equal the oracle, and equal each other with the factoring disabled."""
    nodes, pods = synth.make_config(2, pods=400, nodes=3000)
    rng = np.random.default_rng(12)
    mixed = rng.random(nodes.n_nodes) < 0.5
    k = nodes.card_clock.shape[1]
    nodes.card_clock[mixed] = synth.CLOCKS[rng.integers(0, 3, size=(mixed.sum(), k))]
    nodes.card_bandwidth[mixed[:, None] & (rng.random(nodes.card_bandwidth.shape) < 0.3)] = 1200
    # one model but mixed TotalMemory: the uniform branch without the per-node total
    mixed_total = ~mixed & (rng.random(nodes.n_nodes) < 0.4)
    nodes.card_total_memory[mixed_total, 0] += 4096
    nodes = nodes.normalized()
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    for no_uniform, force_f64, per_node in ((False, False, False), (True, False, False),
                                            (False, True, False), (False, False, True)):
        dev.upload_nodes(nodes, no_uniform=no_uniform, force_f64=force_f64, per_node_k1=per_node,
                         per_node_k2=per_node)
        assert dev.path == ("f64" if force_f64 else "n32")
        assert_same(dev.eval(pods, MODE_SCV), want)
        dev.upload_pods(pods.slice(0, 16))
        feas, rows = dev.score_rows(MODE_SCV)
        for p in range(16):
            _, f, raw, _ = oracle.pod_detail(nodes, pods, p)
            np.testing.assert_array_equal(rows[p][f], raw[f])


def test_large_batch_few_nodes(dev):
    """One rank of a node-sharded batch: many pods over few nodes, where the chunk plan keeps
    chunks of >= 1536 nodes (plan_chunks_for); a pod sample against the oracle and the
    invariants for every pod."""
    nodes, pods = synth.make_config(3, pods=24000, nodes=7000)
    got = dev.eval(pods, MODE_SCV) if dev.upload_nodes(nodes) is None else None
    rng = np.random.default_rng(9)
    sample = np.sort(rng.choice(pods.n_pods, size=600, replace=False))
    want = oracle.schedule(nodes, pods.take(sample), MODE_SCV, threads=16)
    sub = type(got)(**{f: getattr(got, f)[sample] for f in got.__dataclass_fields__})
    assert_same(sub, want)
    ok = got.status == 0
    assert ((got.pick >= 0) == ok).all() and (got.pick[ok] < nodes.n_nodes).all()
    assert (got.n_ties[ok] >= 1).all() and (got.n_ties[ok] <= got.n_feasible[ok]).all()


@pytest.mark.parametrize("cfg", [2, 3])
def test_g_table_on_off(dev, cfg):
    """The K2 G table (per-node basic scores under the snapshot-wide maxima, read by waves
    whose reciprocals are G's) against the K2 computing them, and the oracle on a sample:
    every output identical.  Config 3 sizes keep most waves on the table; extra pods with
    restrictive requests and the mixed clocks give waves whose maxima are not G."""
    nodes, pods = synth.make_config(cfg, pods=6000, nodes=20000)
    rng = np.random.default_rng(40 + cfg)
    few = rng.random(pods.n_pods) < 0.2  # big requests: maxima below G on many waves
    pods.has_memory[few] = 1
    pods.memory[few] = rng.integers(70000, 81921, size=int(few.sum())).astype(np.uint64)
    pods = pods.normalized()
    dev.upload_nodes(nodes)
    with_g = dev.eval(pods, MODE_SCV)
    dev.upload_nodes(nodes, no_gtab=True)
    without = dev.eval(pods, MODE_SCV)
    assert_same(with_g, without)
    np.testing.assert_array_equal(with_g.n_ties, without.n_ties)
    sample = np.sort(rng.choice(pods.n_pods, size=300, replace=False))
    want = oracle.schedule(nodes, pods.take(sample), MODE_SCV, threads=16)
    sub = type(with_g)(**{f: getattr(with_g, f)[sample] for f in with_g.__dataclass_fields__})
    assert_same(sub, want)


@pytest.mark.parametrize("seed", range(3))
def test_k2_block_scoring(dev, seed):
    """The block-classified K2 (N32: node-lane scores for U nodes, LDS prefix sums for FAST
    nodes) against the per-pod K2 and the oracle: waves of near-identical pods (sorted, many
    U nodes), waves of unrelated pods (unsorted, non-uniform maxima), free memory on the
    pods' thresholds (qualifying sets that differ inside a wave), mixed-model nodes."""
    rng = np.random.default_rng(8100 + seed)
    pods = synth.make_pods(1100, int(rng.integers(1 << 30)))
    # clusters of identical requests: whole waves with one qualifying set
    same = rng.random(1100) < 0.4
    pods.memory[same] = rng.choice(np.array([0, 1000, 16000, 40000], dtype=np.uint64),
                                   size=int(same.sum()))
    pods = pods.normalized()
    nodes = _boundary_cluster(rng, 2600, 8, pods)
    # keep alloc varied: many distinct static scores, and ties through equal records
    dup = rng.random(nodes.n_nodes) < 0.1
    src = rng.integers(0, nodes.n_nodes, size=int(dup.sum()))
    for f in ("card_free_memory", "card_total_memory", "card_clock", "card_bandwidth",
              "card_core", "card_power", "card_healthy"):
        getattr(nodes, f)[dup] = getattr(nodes, f)[src]
    for f in ("card_number", "card_count", "free_memory_sum", "total_memory_sum", "alloc_memory"):
        getattr(nodes, f)[dup] = getattr(nodes, f)[src]
    nodes = nodes.normalized()
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    for order in (True, False):
        dev.set_pod_order(order)
        for k1, k2 in ((False, False), (True, False), (False, True)):
            dev.upload_nodes(nodes, per_node_k1=k1, per_node_k2=k2)
            assert_same(dev.eval(pods, MODE_SCV), want)
    dev.set_pod_order(True)


@pytest.mark.parametrize("mode", [MODE_SCV, MODE_DISKIO])
@pytest.mark.parametrize("path", ["n32", "f64", "u64"])
def test_comm_local_matches_unsharded(dev, mode, path):
    """libyoda's own sharded step (yoda_comm_run_local: the grouped MAX/SUM exchange of phase 1,
    then the packed-key merge on the fast paths or the record all-gather on the U64 path in
    Mode A; device copies as the transport) on 1-4 node shards == the unsharded evaluation:
    picks, statuses, feasible counts, ties, top scores, maxima."""
    from yoda_amd.capi import comm_run_local
    nodes, pods = synth.make_config(2, pods=700, nodes=3001)
    nodes.total_memory_sum[17] = 0
    nodes = nodes.normalized()
    want = oracle.schedule(nodes, pods, mode, threads=8)
    for world in (1, 2, 3, 4):
        b = np.linspace(0, nodes.n_nodes, world + 1).astype(int)
        hs = [Yoda(0) for _ in range(world)]
        for r, h in enumerate(hs):
            h.upload_nodes(nodes.slice(b[r], b[r + 1]), node_offset=int(b[r]),
                           force_f64=path == "f64", force_generic=path == "u64")
            h.upload_pods(pods)
        comm_run_local(hs, mode)
        for h in hs:
            assert_same(h.download(), want, mode)
            h.close()


def test_comm_rccl_world1(dev):
    """The RCCL path of yoda_comm_run (a one-rank communicator on this GPU) == yoda_run."""
    from yoda_amd.capi import comm_unique_id
    nodes, pods = synth.make_config(2, pods=500, nodes=4000)
    y = Yoda(0)
    y.upload_nodes(nodes)
    y.upload_pods(pods)
    y.comm_init(comm_unique_id(), 0, 1)
    for mode in (MODE_SCV, MODE_DISKIO):
        y.comm_run(mode)
        assert_same(y.download(), oracle.schedule(nodes, pods, mode, threads=8), mode)
    y.close()
