"""Mode B (BalancedCpuDiskIOPriority, algorithm.go:99-119) batch path on the GPU against the C
oracle: pod classes (distinct (alpha, beta) pairs), both launch forms (lane = node for few
classes, lane = class for many), the score-level thresholds at their boundaries, all-zero and
NaN scores, ragged node counts, and config 3 at full size (sampled)."""
import numpy as np
import pytest

import oracle
from yoda_amd import synth
from yoda_amd.capi import Yoda
from yoda_amd.soa import MODE_DISKIO

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    y = Yoda(0)
    yield y
    y.close()


def check(dev, nodes, pods, sample=None):
    dev.upload_nodes(nodes)
    got = dev.eval(pods, MODE_DISKIO)
    idx = np.arange(pods.n_pods) if sample is None else sample
    want = oracle.schedule(nodes, pods.take(idx), MODE_DISKIO, threads=8)
    for f in ("status", "pick", "n_feasible", "n_ties", "top_score"):
        np.testing.assert_array_equal(getattr(got, f)[idx], getattr(want, f), err_msg=f)
    return got


def levels_py():
    """Independent restatement of the level thresholds: the largest |d| whose score
    trunc(10 - 10|d|) is >= k, by bisection over float64 bit patterns (numpy, no FMA)."""
    def score(x):
        s = np.float64(10.0) - np.float64(10.0) * np.float64(x)
        return np.trunc(s) if s >= 1.0 else 0.0
    out = {}
    for k in range(1, 11):
        lo, hi = 0, 0x7FF0000000000000
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if score(np.array([mid], np.uint64).view(np.float64)[0]) >= k:
                lo = mid
            else:
                hi = mid
        out[k] = np.array([lo], np.uint64).view(np.float64)[0]
    return out


def boundary_nodes(k, n_extra=0, seed=0):
    """Nodes whose V = Cpu/100 straddles level k's threshold by up to 6 ulps (with alpha = 1,
    beta = 0, d = V exactly), the rest strictly below level k: such a pod's best level is k,
    and its tie count is the number of nodes on the low side."""
    t = levels_py()[k]
    c0 = np.float64(t) * 100.0
    cpus, lo, hi = [c0], c0, c0
    for _ in range(6):
        lo, hi = np.nextafter(lo, -np.inf), np.nextafter(hi, np.inf)
        cpus += [lo, hi]
    rng = np.random.default_rng(seed + k)
    cpus += list(np.float64(t) * 100.0 + 5.0 + rng.random(20 + n_extra) * 100.0)
    cpus = np.array(cpus, np.float64)
    rng.shuffle(cpus)
    nodes, _ = synth.make_config(2, pods=1, nodes=len(cpus))
    nodes.cpu = cpus
    nodes.disk_io = rng.random(len(cpus)) * 100.0
    return nodes.normalized()


def pods_with(rio, rcpu):
    _, pods = synth.make_config(2, pods=len(rio), nodes=8)
    pods.rio = np.asarray(rio, np.float64)
    pods.rcpu = np.asarray(rcpu, np.int64)
    return pods.normalized()


@pytest.mark.parametrize("k", range(1, 11))
def test_level_boundaries(dev, k):
    nodes = boundary_nodes(k)
    # alpha = 1, beta = 0 (Rio 0), a NaN pod (0/0), test-pod.yaml, test-pod-multi.yaml
    pods = pods_with([0.0, 0.0, 10.0, 0.0, 10.0], [100, 0, 100, 500, 100])
    got = check(dev, nodes, pods)
    assert got.top_score[0] == k
    assert got.n_ties[1] == nodes.n_nodes and got.pick[1] == 0  # NaN: every node scores 0
    rng = np.random.default_rng(k)
    rio = np.concatenate([[0.0, 0.0], rng.random(400) * 50.0])
    rcpu = np.concatenate([[100, 0], rng.integers(1, 4000, 400)])
    got = check(dev, boundary_nodes(k, n_extra=3000), pods_with(rio, rcpu))
    assert got.top_score[0] == k


@pytest.mark.parametrize("n_nodes", [1, 2, 63, 2047, 2048, 2049, 5000])
def test_ragged_node_counts(dev, n_nodes):
    nodes, _ = synth.make_config(2, pods=1, nodes=n_nodes)
    rng = np.random.default_rng(n_nodes)
    for n_cls in (3, 700):
        rio = rng.random(n_cls) * 20.0
        rcpu = rng.integers(1, 2000, n_cls)
        check(dev, nodes, pods_with(rio, rcpu))


def test_every_node_scores_zero(dev):
    nodes, _ = synth.make_config(2, pods=1, nodes=3000)
    nodes.cpu = np.full(nodes.n_nodes, 1000.0)  # V = 10: 10 - 100 < 1
    nodes = nodes.normalized()
    for rio, rcpu in (([0.0] * 4, [100] * 4), (np.zeros(200), np.arange(1, 201))):
        got = check(dev, nodes, pods_with(rio, rcpu))
        assert (got.n_ties == nodes.n_nodes).all() and (got.pick == 0).all()


def test_repeated_classes_shuffled(dev):
    """Few distinct specs dealt in random order over many pods (lane = node form), then the
    same pods re-uploaded with one more distinct pod each (lane = class form)."""
    nodes, _ = synth.make_config(2, pods=1, nodes=6000)
    rng = np.random.default_rng(9)
    spec = rng.integers(0, 7, 5000)
    rio = np.array([10.0, 0.0, 2.5, 33.3, 1e-3, 7.0, 10.0])[spec]
    rcpu = np.array([100, 500, 250, 100, 4000, 1, 300])[spec]
    got = check(dev, nodes, pods_with(rio, rcpu), sample=np.arange(0, 5000, 7))
    rio2 = rio.copy()
    rio2[::50] = rng.random(rio2[::50].size) * 40
    got2 = check(dev, nodes, pods_with(rio2, rcpu), sample=np.arange(0, 5000, 7))
    same = np.ones(5000, bool)
    same[::50] = False
    np.testing.assert_array_equal(got.pick[same], got2.pick[same])


# Config 3 in Mode B at 100k x 100k (one pod class, and a distinct request per pod): every
# pod in tests/test_gpu_fullsize.py (variants diskio, diskio_distinct).
