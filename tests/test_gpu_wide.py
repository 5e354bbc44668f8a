"""GPU parity with wide small card fields: bandwidth, clock, core and power beyond the old
16-bit N32 bound (the reference reads them as plain `uint`, collection.go:14-20).  N32 keeps
them in u32 with every quotient in f64 and, beyond 16 bits, unpacked K1
partial words; such snapshots must be one GPU model per node (else F64), and a clock quotient
that could overflow the u32 card score sends them to F64 too.  Everything is compared with
the C oracle (oracle/yoda_oracle.c)."""

import numpy as np
import pytest

import oracle
from test_gpu_parity import assert_same
from yoda_amd import synth
from yoda_amd.capi import Yoda
from yoda_amd.soa import MODE_SCV

pytestmark = pytest.mark.gpu
CAP = 1  # YODA_GREEDY_CARD_CAPACITY


@pytest.fixture(scope="module")
def dev():
    y = Yoda(0)
    yield y
    y.close()


def scaled(fields, factor, cfg=3, pods=1500, nodes=5000):
    """Config `cfg` (one GPU model per node) with `fields` multiplied by `factor` (the pods'
    scv/clock labels too when the clock is scaled, so the Filter keeps its outcome)."""
    nd, pd = synth.make_config(cfg, pods=pods, nodes=nodes)
    for f in fields:
        arr = getattr(nd, "card_" + f)
        arr[:] = arr * np.uint64(factor)
    if "clock" in fields:
        pd.clock[:] = pd.clock * np.uint64(factor)
    return nd, pd


@pytest.mark.parametrize("fields", [("bandwidth",), ("core", "power"),
                                    ("bandwidth", "clock", "core", "power")])
def test_wide_fields_eval(dev, fields):
    nodes, pods = scaled(fields, 1000)
    dev.upload_nodes(nodes)
    assert dev.path == "n32"
    got = dev.eval(pods, MODE_SCV)
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    assert_same(got, want)
    assert (want.status == 0).mean() > 0.3


def test_sixteen_bit_fields_stay_packed(dev):
    """60,000 (above the old 55,738 bound, within 16 bits) on every card of some nodes."""
    nodes, pods = synth.make_config(3, pods=1200, nodes=4000)
    nodes.card_bandwidth[::7] = np.uint64(60000)
    nodes.card_power[::5] = np.uint64(65535)
    dev.upload_nodes(nodes)
    assert dev.path == "n32"
    assert_same(dev.eval(pods, MODE_SCV), oracle.schedule(nodes, pods, MODE_SCV, threads=8))


def test_wide_mixed_model_node_takes_f64(dev):
    nodes, pods = scaled(("bandwidth",), 1000, pods=600, nodes=3000)
    nodes.card_bandwidth[11, 0] += np.uint64(1)      # node 11 no longer one model
    dev.upload_nodes(nodes)
    assert dev.path == "f64"
    assert_same(dev.eval(pods, MODE_SCV), oracle.schedule(nodes, pods, MODE_SCV, threads=8))


def test_clock_quotient_bound_takes_f64(dev):
    """clock / MaxBandwidth is not bounded by 100: a node with bandwidth 1 and a 30-bit clock
    could push the u32 card score past 2^32, so the snapshot is not N32."""
    nodes, pods = synth.make_config(3, pods=400, nodes=2000)
    nodes.card_bandwidth[17] = np.uint64(1)
    nodes.card_clock[17] = np.uint64(1 << 30)
    dev.upload_nodes(nodes)
    assert dev.path == "f64"
    assert_same(dev.eval(pods, MODE_SCV), oracle.schedule(nodes, pods, MODE_SCV, threads=8))


def test_wide_fields_score_rows(dev):
    nodes, pods = scaled(("bandwidth", "clock", "core", "power"), 1000, pods=24, nodes=900)
    dev.upload_nodes(nodes)
    assert dev.path == "n32"
    dev.upload_pods(pods)
    feas, rows = dev.score_rows(MODE_SCV)
    for p in range(pods.n_pods):
        _, f, raw, _ = oracle.pod_detail(nodes, pods, p, MODE_SCV)
        np.testing.assert_array_equal(feas[p], f)
        ok = f & (nodes.total_memory_sum != 0)
        np.testing.assert_array_equal(rows[p][ok], raw[ok])


@pytest.mark.parametrize("flags", [0, CAP])
def test_wide_fields_greedy(flags):
    """The greedy batch (top-k windows, exact fallbacks / capacity restarts) on the config-5
    generator with bandwidth x 1000, every pick against the sequential oracle."""
    nodes, pods = synth.make_config(5, pods=7000, nodes=5000)
    nodes.card_bandwidth[:] = nodes.card_bandwidth * np.uint64(1000)
    y = Yoda(0)
    y.upload_nodes(nodes)
    assert y.path == "n32"
    pick = y.greedy(pods, MODE_SCV, flags)
    want, _ = oracle.greedy(nodes, pods, MODE_SCV, flags)
    np.testing.assert_array_equal(pick, want)
    y.close()


# bandwidth x 1000 at 100k x 100k: every pod in tests/test_gpu_fullsize.py (variant bw1000)


@pytest.mark.parametrize("mixed_narrow_shard", [False, True])
def test_sharded_quotient_agreement(mixed_narrow_shard):
    """Node shards exchange maxima: a narrow shard next to a wide one must not keep f32
    quotients (their lemma needs every maximum <= 55,738).  dist.agree_on_path re-uploads it
    with f64 quotients -- or, holding mixed-model nodes, on F64, and then every shard."""
    import torch
    from yoda_amd.dist import ShardExchange
    nodes, pods = synth.make_config(3, pods=300, nodes=2000)
    if mixed_narrow_shard:
        part = synth.mixed_models(nodes.slice(0, 1000), 0.3)
        for f in ("card_clock", "card_bandwidth", "card_core", "card_power"):
            getattr(nodes, f)[:1000] = getattr(part, f)
    nodes.card_bandwidth[1000:] = nodes.card_bandwidth[1000:] * np.uint64(1000)
    want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
    shards = [nodes.slice(0, 1000), nodes.slice(1000, 2000)]
    handles = []
    for i, sh in enumerate(shards):
        y = Yoda(0)
        y.upload_nodes(sh, node_offset=1000 * i)
        y.upload_pods(pods)
        handles.append(y)
    assert handles[0].small_field_max <= 55738 < handles[1].small_field_max
    assert [h.path for h in handles] == ["n32", "n32"]
    ex = ShardExchange.local(handles, torch.device("cuda:0"), shards, [0, 1000])
    assert [h.path for h in handles] == (["f64", "f64"] if mixed_narrow_shard else ["n32", "n32"])
    assert_same(ex.run(MODE_SCV), want)
    for y in handles:
        y.close()
