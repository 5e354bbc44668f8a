"""GPU: the batch order (yoda_order.hip) never changes results -- the padded counting sort of a
private run, its unpadded form when padding would cost more than 1/8 of the batch, the radix
fallback for batches with more (clock, number, has-memory) groups than the counting sort
holds, and no order at all -- each against the C oracle, bit-exact."""
import numpy as np
import pytest

import oracle
from yoda_amd import synth
from yoda_amd.capi import Yoda
from yoda_amd.soa import MODE_SCV, PodSoA

from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    y = Yoda(0)
    yield y
    y.close()


def _pods(p, seed, clocks, numbers, mem_frac=0.8):
    rng = np.random.default_rng(seed)
    has_number = (rng.random(p) < 0.9).astype(np.uint8)
    number = rng.choice(np.asarray(numbers, np.uint64), size=p)
    has_memory = (rng.random(p) < mem_frac).astype(np.uint8)
    memory = np.where(has_memory == 1, rng.integers(0, 81921, size=p), 0).astype(np.uint64)
    has_clock = (rng.random(p) < 0.6).astype(np.uint8)
    clock = np.where(has_clock == 1, rng.choice(np.asarray(clocks, np.uint64), size=p), 0)
    z = np.zeros(p)
    return PodSoA(has_number=has_number, number=number, has_memory=has_memory, memory=memory,
                  has_clock=has_clock, clock=clock.astype(np.uint64), priority=z,
                  rio=np.full(p, 10.0), rcpu=np.full(p, 100)).normalized()


def test_padded_order_config3_shape(dev):
    """Config-3-shaped batch: few large groups, padded (< 1/8 extra), counting order."""
    nodes, pods = synth.make_config(3, pods=20000, nodes=2000)
    dev.upload_nodes(nodes)
    got = dev.eval(pods, MODE_SCV)
    info = dev.order_info()
    assert info["kind"] == 2 and info["work"] == info["padded"] > pods.n_pods
    assert info["padded"] % 64 == 0 and info["groups"] > 0
    assert_same(got, oracle.schedule(nodes, pods, MODE_SCV, threads=8))


def test_many_small_groups_unpadded(dev):
    """~600 groups of a few pods: padding would multiply the work, so the counting order
    runs unpadded."""
    nodes = synth.make_nodes(2500, seed=5)
    clocks = list(range(1000, 1040)) + [1410, 1500, 1755]
    pods = _pods(1500, 6, clocks, [1, 2, 3, 4, 5, 6, 7, 8])
    dev.upload_nodes(nodes)
    got = dev.eval(pods, MODE_SCV)
    info = dev.order_info()
    assert info["kind"] == 2 and info["work"] == pods.n_pods < info["padded"]
    assert_same(got, oracle.schedule(nodes, pods, MODE_SCV, threads=8))


def test_too_many_groups_radix(dev):
    """Every pod its own clock value: more groups than the counting sort's histogram holds
    -> the radix order."""
    nodes = synth.make_nodes(1500, seed=7)
    pods = _pods(30000, 8, np.arange(1, 30001), [1, 2, 4])
    pods.clock[:] = np.arange(1, 30001, dtype=np.uint64)
    pods.has_clock[:] = 1
    pods.clock[::3] = 1500  # a third of them on a real clock value
    dev.upload_nodes(nodes)
    got = dev.eval(pods, MODE_SCV)
    info = dev.order_info()
    assert info["groups"] == 0 and info["kind"] == 1
    assert_same(got, oracle.schedule(nodes, pods, MODE_SCV, threads=8))


@pytest.mark.parametrize("pad", [False, True])
def test_order_modes_agree(dev, pad):
    """Padded and unpadded counting order, and no order: identical outputs."""
    nodes, pods = synth.make_config(2, pods=20000, nodes=1500)
    dev.upload_nodes(nodes)
    dev.set_pod_order(True, pad=pad)
    a = dev.eval(pods, MODE_SCV)
    info = dev.order_info()
    assert info["kind"] == 2
    assert (info["work"] > pods.n_pods) == pad
    dev.set_pod_order(False)
    b = dev.eval(pods, MODE_SCV)
    dev.set_pod_order(True)
    assert dev.order_info()["kind"] == 0
    for f in ("pick", "status", "n_feasible", "n_ties", "top_score", "maxima"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)


def test_repeated_runs_identical(dev):
    """The counting order inside a bucket follows atomics; outputs must not."""
    nodes, pods = synth.make_config(3, pods=8000, nodes=2000)
    dev.upload_nodes(nodes)
    first = dev.eval(pods, MODE_SCV)
    for _ in range(3):
        again = dev.eval(pods, MODE_SCV)
        for f in ("pick", "status", "n_feasible", "n_ties", "top_score", "maxima"):
            np.testing.assert_array_equal(getattr(first, f), getattr(again, f), err_msg=f)


def test_deferred_upload_alternating_batches(dev):
    """a fast private run reads only the 5 core pod arrays; the rest of the batch
    (f64 / u64 thresholds, Mode-B weights) reaches the device after its kernels.  Alternate two
    different batches through yoda_run, then read the deferred arrays through entry points that
    need them (Mode B, the U64-path score rows): every result == the oracle's for its batch."""
    nodes, pods_a = synth.make_config(3, pods=6000, nodes=3000)
    pods_b = synth.distinct_diskio(synth.make_pods(5000, seed=77))
    dev.upload_nodes(nodes)
    want = {k: oracle.schedule(nodes, p, MODE_SCV, threads=8)
            for k, p in (("a", pods_a), ("b", pods_b))}
    for k in ("a", "b", "a", "b"):
        pods = pods_a if k == "a" else pods_b
        assert_same(dev.eval(pods, MODE_SCV), want[k])
    # batch b uploaded once: a fast Mode-A run, then on the same upload a Mode-B run (alpha /
    # beta) and a bitmask run (not a fast run: the F64 thresholds), each against the oracle
    dev.upload_pods(pods_b)
    dev.run(MODE_SCV)
    assert_same(dev.download(), want["b"])
    dev.run(1)
    assert_same(dev.download(), oracle.schedule(nodes, pods_b, 1, threads=8), 1)
    dev.run(MODE_SCV, bitmask=True)
    assert_same(dev.download(), want["b"])
    assert_same(dev.eval(pods_a, MODE_SCV), want["a"])
