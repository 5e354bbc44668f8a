"""Committed golden fixtures (tests/golden/, made by make_golden.py from the oracle and the
independent Python restatement): the oracle must reproduce them (CPU) and so must libyoda
(GPU), on every record path."""
import glob
import os

import numpy as np
import pytest

import oracle
from yoda_amd.soa import EvalResult, NodeSoA, PodSoA

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = sorted(glob.glob(os.path.join(HERE, "*.npz")))
OUT = ["pick", "status", "n_feasible", "n_ties", "top_score", "maxima"]


def load(path):
    z = np.load(path, allow_pickle=False)
    nodes = NodeSoA(**{k[5:]: z[k] for k in z.files if k.startswith("node_")})
    pods = PodSoA(**{k[4:]: z[k] for k in z.files if k.startswith("pod_")})
    return nodes, pods, z


def check(res, z, mode):
    ok = z[f"mode{mode}_status"] == 0
    for f in OUT:
        want, got = z[f"mode{mode}_{f}"], getattr(res, f)
        if f in ("n_ties", "top_score"):
            want, got = want[ok], got[ok]
        if f == "maxima" and mode == 1:
            continue
        np.testing.assert_array_equal(got, want, err_msg=f)


def test_fixtures_present():
    assert len(FIXTURES) >= 6


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_oracle_reproduces_golden(path):
    nodes, pods, z = load(path)
    for mode in (0, 1):
        check(oracle.schedule(nodes, pods, mode), z, mode)
    for flags in (0, 1):
        pick, _ = oracle.greedy(nodes, pods, 0, flags)
        np.testing.assert_array_equal(pick, z[f"greedy{flags}_pick"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_gpu_reproduces_golden(path):
    from yoda_amd.capi import Yoda
    nodes, pods, z = load(path)
    with Yoda(0) as y:
        for rec in ("auto", "f64", "u64"):
            y.upload_nodes(nodes, force_f64=rec == "f64", force_generic=rec == "u64")
            for mode in (0, 1):
                check(y.eval(pods, mode), z, mode)


def test_fullsize_fixture_pins_the_oracle():
    """tests/golden/fullsize.json (the every-pod digests the GPU suite checks at full size):
    the generator still makes the inputs it was computed on, and the C oracle reproduces its
    first and last config-3 blocks here (2 x 1,024 pods x 100k nodes)."""
    import fullsize_check as fc
    from yoda_amd import synth
    fx = fc.load("config3")
    nodes, pods = synth.make_config(3)
    fc.check_inputs(fx, nodes, pods)
    B, nb = fx["block"], len(fx["digests"])
    for b in (0, nb - 1):
        sel = np.arange(b * B, min(pods.n_pods, (b + 1) * B))
        res = oracle.schedule(nodes, pods.take(sel), 0, threads=8)
        assert fc.mf.eval_digests(res, B, 0)[0] == fx["digests"][b], b
    for key in ("config5_0", "config5_1"):
        import json
        if key not in json.load(open(fc.FIXTURE)):
            continue
        g = fc.load(key)
        fc.check_inputs(g, *synth.make_config(5))
        assert len(g["digests"]) == -(-g["pods"] // g["window"])


@pytest.mark.parametrize("name", ["mixed50", "bytes", "bw1000", "het100k", "diskio",
                                  "diskio_distinct"])
def test_variant_fixtures_pin_the_oracle(name):
    """The every-pod digests of the bench's variant workloads (tests/golden/fullsize.json
    variant_*): the generator still makes the same inputs, and the C oracle reproduces the
    first 1,024-pod block here (maxima included in Mode A)."""
    import fullsize_check as fc
    fx = fc.load(f"variant_{name}")
    nodes, pods, mode = fc.mf.variant_inputs(name)
    fc.check_variant_inputs(fx, nodes, pods)
    assert fx["mode"] == mode and len(fx["digests"]) == -(-pods.n_pods // fx["block"])
    B = fx["block"]
    res = oracle.schedule(nodes, pods.slice(0, B), mode, threads=8)
    assert fc.mf.eval_digests(res, B, mode)[0] == fx["digests"][0]
