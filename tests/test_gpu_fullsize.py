"""Every-pod parity at 100k pods x 100k nodes on every workload bench.py reports.

tests/golden/fullsize.json holds the C oracle's per-1,024-pod digests (make_fullsize.py, run
in the build container) of (pick, status, n_feasible, n_ties, top_score and, in Mode A, the six
CollectMaxValues maxima) for:
* config 3 itself -- which the forced F64 / U64 record paths and the per-pair kernels must
  also reproduce (the same workload on other kernels);
* the variant workloads of bench.py `extra.variants` (synth.VARIANTS): 50 % mixed-model nodes,
  memory in bytes (memory ranks), bandwidth x 1000 (wide small fields: f64 quotients), the
  config-4 generator at 100k x 100k (K = 16), and Mode B as generated (one pod class) and with
  a distinct diskIO / CPU request per pod.
Reference: collection.go:30-76 (maxima), algorithm.go:99-119 (Mode B), 264-310 (Mode A
score), scheduler.go:158-183 (NormalizeScore; argmax with the lowest-index tie-break).
"""
import numpy as np
import pytest

import fullsize_check as fc
import make_fullsize as mf
import oracle
from yoda_amd import synth
from yoda_amd.capi import Yoda
from yoda_amd.soa import MODE_SCV

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    y = Yoda(0)
    yield y
    y.close()


def _invariants(got, nodes):
    ok = got.status == 0
    assert ((got.pick >= 0) == ok).all()
    assert (got.pick[ok] < nodes.n_nodes).all()
    assert (got.n_ties[ok] >= 1).all() and (got.n_ties[ok] <= got.n_feasible[ok]).all()
    assert (got.n_feasible[got.status == 1] == 0).all()


# the record path / flags each variant must take
EXPECT = {"mixed50": ("n32", False), "bytes": ("n32", True), "bw1000": ("n32", False),
          "het100k": ("n32", False), "diskio": (None, False), "diskio_distinct": (None, False)}


@pytest.mark.parametrize("name", mf.VARIANTS)
def test_variant_every_pod(dev, name):
    fx = fc.load(f"variant_{name}")
    nodes, pods, mode = mf.variant_inputs(name)
    fc.check_variant_inputs(fx, nodes, pods)
    assert fx["mode"] == mode
    dev.upload_nodes(nodes)
    path, ranks = EXPECT[name]
    if path is not None:
        assert dev.path == path
    assert dev.memory_ranks == ranks
    got = dev.eval(pods, mode)
    bad = fc.eval_mismatch(fx, got, nodes, pods, oracle)
    assert bad is None, f"{name}: {bad}"
    _invariants(got, nodes)
    assert int(got.n_feasible.astype(np.int64).sum()) == fx["feasible_pairs"]


@pytest.mark.parametrize("kernels", ["f64", "u64", "per_pair"])
def test_config3_other_kernels_every_pod(dev, kernels):
    """Config 3 on the forced F64 and U64 record paths and on the per-pair N32 kernels (the
    bench's `f64`, `u64` and `per_pair_kernels` lines): every pod's digest, maxima included."""
    fx = fc.load("config3")
    nodes, pods = synth.make_config(3)
    fc.check_inputs(fx, nodes, pods)
    kw = {"f64": dict(force_f64=True), "u64": dict(force_generic=True),
          "per_pair": dict(per_node_k1=True, per_node_k2=True)}[kernels]
    dev.upload_nodes(nodes, **kw)
    assert dev.path == {"f64": "f64", "u64": "u64", "per_pair": "n32"}[kernels]
    got = dev.eval(pods, MODE_SCV)
    bad = fc.eval_mismatch(fx, got, nodes, pods, oracle)
    assert bad is None, f"{kernels}: {bad}"
