"""Pin the oracle: hand-derived known-answer tests from the Go text and a
randomized cross-check of the C oracle against the independent Python restatement.

The reference has no golden vectors and cannot run here (no Go toolchain), so these KATs
are the pin: each expected number below is worked from the cited Go lines by hand."""
import numpy as np
import pytest

import oracle
import pyoracle as po
from yoda_amd import synth
from yoda_amd.soa import MODE_DISKIO, MODE_SCV


def H(free, total=16000, clock=1500, bw=900, core=80, power=300, health="Healthy"):
    return po.Card(free_memory=free, total_memory=total, clock=clock, bandwidth=bw, core=core,
                   power=power, health=health)


def kat1_cluster():
    n0 = po.Scv(card_number=2, card_list=[H(10000), H(9000)], free_memory_sum=19000,
                total_memory_sum=32000, alloc_memory=0)
    big = dict(total=32000, clock=1500, bw=1200, core=108, power=400)
    n1 = po.Scv(card_number=4,
                card_list=[H(16000, **big), H(16000, **big), H(16000, **big),
                           H(16000, health="Unhealthy", **big)],
                free_memory_sum=64000, total_memory_sum=128000, alloc_memory=16000)
    n2 = po.Scv(card_number=1, card_list=[H(20000, total=20000)], free_memory_sum=20000,
                total_memory_sum=20000)
    pod = po.Pod(number=2, memory=8000, clock=1500)
    return [n0, n1, n2], pod


def test_kat1_mode_a_python():
    scvs, pod = kat1_cluster()
    assert [po.fits(pod, s)[0] for s in scvs] == [True, True, False]
    mv = po.collect_max_values(pod, scvs)
    # collection.go:57-76 — the Unhealthy card counts (no health check at :46)
    assert mv.as_list() == [1200, 1500, 108, 16000, 400, 32000]
    assert po.basic_score(mv, pod, scvs[0]) == 1300      # 659 + 641 (card 2: free 56*3)
    assert po.allocate_score(scvs[0]) == 300             # 32000*100/32000*3
    assert po.actual_score(scvs[0]) == 118               # 19000*100/32000 = 59, *2
    assert po.basic_score(mv, pod, scvs[1]) == 3700      # 4 cards x 925
    assert po.allocate_score(scvs[1]) == 261             # 112000*100/128000 = 87, *3
    assert po.actual_score(scvs[1]) == 100               # 50*2
    r = po.schedule_one(pod, scvs)
    assert (r.pick, r.status, r.n_feasible, r.top_score) == (1, 0, 2, 4061)
    assert r.tie_set == [1]


def test_kat1_mode_a_c_oracle():
    scvs, pod = kat1_cluster()
    nodes, pods = oracle.from_py(scvs, [pod])
    res = oracle.schedule(nodes, pods, MODE_SCV)
    assert res.pick[0] == 1 and res.status[0] == 0
    assert res.n_feasible[0] == 2 and res.n_ties[0] == 1 and res.top_score[0] == 4061
    assert list(res.maxima[0]) == [1200, 1500, 108, 16000, 400, 32000]
    rc, feas, raw, norm = oracle.pod_detail(nodes, pods, 0, MODE_SCV)
    assert rc == 0 and list(feas) == [True, True, False]
    assert list(raw[:2]) == [1718, 4061]
    assert list(norm[:2]) == [0, 100]


# KAT 2: Mode B, test-pod.yaml (Rcpu 100, Rio 10 -> beta = 1/11); (cpu%, disk MB/s) -> score
KAT2 = [((50, 10), 5), ((5, 0.5), 9), ((120, 0), 0), ((0, 400), 2), ((0, 0), 10)]
# KAT 3: test-pod-multi.yaml (Rcpu 500, diskIO "10m" -> Rio 0 -> beta 0, alpha 1)
KAT3 = [((50, 10), 5), ((0, 0), 10)]


@pytest.mark.parametrize("rcpu,rio,cases", [(100, 10.0, KAT2), (500, 0.0, KAT3)])
def test_kat_mode_b(rcpu, rio, cases):
    pod = po.Pod(rio=rio, rcpu=rcpu)
    scvs = [po.Scv(card_number=0, card_list=[], free_memory_sum=0, total_memory_sum=1,
                   cpu=float(c), disk_io=float(d)) for (c, d), _ in cases]
    want = [s for _, s in cases]
    assert [po.diskio_score(pod, s) for s in scvs] == want
    nodes, pods = oracle.from_py(scvs, [pod], max_cards=1)
    rc, feas, raw, norm = oracle.pod_detail(nodes, pods, 0, MODE_DISKIO)
    assert list(raw) == want and feas.all()
    res = oracle.schedule(nodes, pods, MODE_DISKIO)
    best = max(want)
    assert res.pick[0] == want.index(best) and res.n_ties[0] == want.count(best)


# KAT B3 (memo quirk, documentation mode): Rcpu 100, Rio 100 -> beta = alpha = 1/2.
# (cpu%, disk MB/s) -> S = 10 - 10|V/2 - U/2|: 9.5, 9.0, 5.0, 2.5, -5.0.  The node scored first
# gets trunc(S); the others read FormatFloat(S) back through Atoi: 9.5 -> 0, 2.5 -> 0,
# -5 -> uint64 wrap -> Uint64ToInt64 -> 0.
B3_NODES = [(10, 0), (20, 0), (100, 0), (50, 100), (0, 150)]
B3_CASES = [  # first -> (scores, pick, ties)
    (None, [9, 9, 5, 2, 0], 0, 2),   # uncached B1 (the product semantics)
    (0, [9, 9, 5, 0, 0], 0, 2),
    (1, [0, 9, 5, 0, 0], 1, 1),      # the quirk moves the pick
    (3, [0, 9, 5, 2, 0], 1, 1),
    (4, [0, 9, 5, 0, 0], 1, 1),
]


@pytest.mark.parametrize("first,scores,pick,ties", B3_CASES)
def test_kat_b3_memo_quirk(first, scores, pick, ties):
    pod = po.Pod(rio=100.0, rcpu=100)
    scvs = [po.Scv(card_number=0, card_list=[], free_memory_sum=0, total_memory_sum=1,
                   cpu=float(c), disk_io=float(d)) for c, d in B3_NODES]
    got = [po._score(pod, s, None, MODE_DISKIO, first, n) for n, s in enumerate(scvs)]
    assert got == scores
    r = po.schedule_one(pod, scvs, MODE_DISKIO, memo_first=first)
    assert (r.pick, r.n_ties) == (pick, ties)
    nodes, pods = oracle.from_py(scvs, [pod], max_cards=1)
    res = (oracle.schedule(nodes, pods, MODE_DISKIO) if first is None
           else oracle.schedule_memo(nodes, pods, first))
    assert (res.pick[0], res.n_ties[0], res.top_score[0]) == (pick, ties, scores[pick])


@pytest.mark.parametrize("seed", [0, 1])
def test_b3_memo_c_matches_python(seed):
    nodes = synth.make_nodes(40, 100 + seed)
    pods = synth.make_pods(48, 200 + seed)
    # integral S values are what the quirk keeps: give a quarter of the nodes cpu = disk = 0
    nodes.cpu[::4] = 0.0
    nodes.disk_io[::4] = 0.0
    scvs, plist = oracle.to_py(nodes, pods)
    for first in (0, 7):
        res = oracle.schedule_memo(nodes, pods, first)
        for p, pod in enumerate(plist):
            r = po.schedule_one(pod, scvs, MODE_DISKIO, memo_first=first)
            assert (res.pick[p], res.n_ties[p], res.top_score[p]) == (r.pick, r.n_ties,
                                                                      r.top_score)
    with pytest.raises(RuntimeError):
        oracle.schedule_memo(nodes, pods, nodes.n_nodes)


def test_go_float_to_uint64_edges():
    assert po.go_float64_to_uint64(5.9) == 5
    assert po.go_float64_to_uint64(-0.5) == 0
    assert po.uint64_to_int64(po.go_float64_to_uint64(-5.5)) == 0   # wraps >= 2^63 -> 0
    assert po.uint64_to_int64(po.go_float64_to_uint64(float("nan"))) == 0
    assert po.uint64_to_int64(po.go_float64_to_uint64(float("inf"))) == 0


def test_nan_beta_scores_zero():
    # Rio = 0 and Rcpu = 0: 0/0 = NaN -> beta NaN -> every score 0
    pod = po.Pod(rio=0.0, rcpu=0)
    s = po.Scv(card_number=0, card_list=[], free_memory_sum=0, total_memory_sum=1, cpu=10,
               disk_io=10)
    assert po.diskio_score(pod, s) == 0


def test_single_feasible_node_skips_score():
    # Only one feasible node with TotalMemorySum 0: k8s returns it without calling Score,
    # so the reference's divide-by-zero never happens.
    n0 = po.Scv(card_number=1, card_list=[H(5000)], free_memory_sum=5000, total_memory_sum=0)
    n1 = po.Scv(card_number=0, card_list=[], free_memory_sum=0, total_memory_sum=100)
    r = po.schedule_one(po.Pod(), [n0, n1])
    assert (r.pick, r.status) == (0, po.STATUS_OK)
    nodes, pods = oracle.from_py([n0, n1], [po.Pod()])
    res = oracle.schedule(nodes, pods)
    assert res.pick[0] == 0 and res.status[0] == 0


def test_div_zero_two_feasible():
    n0 = po.Scv(card_number=1, card_list=[H(5000)], free_memory_sum=5000, total_memory_sum=0)
    n1 = po.Scv(card_number=1, card_list=[H(5000)], free_memory_sum=5000, total_memory_sum=100)
    r = po.schedule_one(po.Pod(), [n0, n1])
    assert (r.pick, r.status) == (po.PICK_ERROR, po.STATUS_DIV_ZERO)
    nodes, pods = oracle.from_py([n0, n1], [po.Pod()])
    res = oracle.schedule(nodes, pods)
    assert res.pick[0] == po.PICK_ERROR and res.status[0] == po.STATUS_DIV_ZERO


def _overflow_pair(clock0):
    # clock/MaxBandwidth (algorithm.go:283) with MaxBandwidth 1: raw = 100*clock + const
    n0 = po.Scv(card_number=1, card_list=[H(10, clock=clock0, bw=1)], free_memory_sum=10,
                total_memory_sum=16000)
    n1 = po.Scv(card_number=1, card_list=[H(10, clock=1, bw=1)], free_memory_sum=10,
                total_memory_sum=16000)
    return [n0, n1]


@pytest.mark.parametrize("clock0,want", [
    # (h - l) * 100 = 1e19 wraps negative: normalized score < 0, k8s rejects (Error)
    (10 ** 15 + 1, (po.PICK_ERROR, po.STATUS_SCORE_RANGE, None)),
    # (h - l) ~ 2^62: the product wraps to a small value, both nodes normalize to 0 — in
    # range, so the pod IS scheduled, from a 2-node tie that raw argmax would not give
    ((1 << 62) // 100, (0, po.STATUS_OK, 2)),
])
def test_normalize_int64_overflow(clock0, want):
    scvs, pod = _overflow_pair(clock0), po.Pod()
    r = po.schedule_one(pod, scvs)
    assert (r.pick, r.status) == want[:2]
    if want[2] is not None:
        assert r.n_ties == want[2]
    nodes, pods = oracle.from_py(scvs, [pod])
    res = oracle.schedule(nodes, pods)
    assert (int(res.pick[0]), int(res.status[0])) == (r.pick, r.status)
    if want[2] is not None:
        assert int(res.n_ties[0]) == want[2]


def test_equal_scores_all_tie():
    s = po.Scv(card_number=1, card_list=[H(5000)], free_memory_sum=5000, total_memory_sum=16000)
    r = po.schedule_one(po.Pod(), [s, s, s])
    assert r.pick == 0 and r.n_ties == 3 and r.tie_set == [0, 1, 2]


def test_label_edge_semantics():
    # scv/number "-1" -> strToUint wraps to 2^64-1: never fits; "abc" -> 0: always fits
    s = po.Scv(card_number=0, card_list=[], free_memory_sum=0, total_memory_sum=1)
    assert po.fits(po.Pod(number=(1 << 64) - 1), s)[0] is False
    assert po.fits(po.Pod(number=0), s)[0] is True
    assert po.fits(po.Pod(), s)[0] is False        # absent: CardNumber > 0 required


def _random_cluster(rng, n_nodes, n_pods, k):
    nodes = synth.make_nodes(n_nodes, int(rng.integers(1 << 30)), cards=k)
    pods = synth.make_pods(n_pods, int(rng.integers(1 << 30)))
    # sprinkle edge values
    nodes.card_number[rng.random(n_nodes) < 0.1] = 0
    nodes.card_clock[rng.random(nodes.card_clock.shape) < 0.1] = 1500
    nodes.alloc_memory[rng.random(n_nodes) < 0.1] = np.uint64(10 ** 7)
    pods.number[rng.random(n_pods) < 0.05] = np.uint64((1 << 64) - 1)
    return nodes.normalized(), pods.normalized()


@pytest.mark.parametrize("seed", range(6))
def test_c_oracle_matches_python_restatement(seed):
    rng = np.random.default_rng(seed)
    for mode in (MODE_SCV, MODE_DISKIO):
        nodes, pods = _random_cluster(rng, 40, 12, k=int(rng.choice([1, 4, 8])))
        res = oracle.schedule(nodes, pods, mode)
        scvs, plist = oracle.to_py(nodes, pods)
        for p, pod in enumerate(plist):
            r = po.schedule_one(pod, scvs, mode)
            got = (int(res.pick[p]), int(res.status[p]), int(res.n_feasible[p]))
            assert got == (r.pick, r.status, r.n_feasible), (seed, mode, p)
            if r.status == po.STATUS_OK:
                assert int(res.n_ties[p]) == r.n_ties and int(res.top_score[p]) == r.top_score
                assert r.pick in r.tie_set
            if mode == MODE_SCV:
                assert list(map(int, res.maxima[p])) == r.maxima


def test_greedy_c_matches_python():
    rng = np.random.default_rng(99)
    nodes, pods = _random_cluster(rng, 25, 30, k=4)
    pods.priority[:] = rng.integers(0, 3, size=pods.n_pods)
    scvs, plist = oracle.to_py(nodes, pods)
    for flags in (0, 1):
        pick, _ = oracle.greedy(nodes, pods, MODE_SCV, flags)
        want = po.greedy(plist, scvs, 0, card_capacity=bool(flags))
        assert list(map(int, pick)) == want
