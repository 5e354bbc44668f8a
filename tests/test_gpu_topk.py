"""Greedy candidate lists (yoda_shard_topk on one handle): each pod's best k (score, node)
pairs, (score desc, node asc), against the oracle's per-node raw scores (oracle_pod_detail,
algorithm.go:96 + scheduler.go:154).  N32 batches run the block-classified K2 with packed keys
(k2_block_n32 TKO, k_topk_merge_keys); K = 16 and the F64 path the per-pair k2_score."""
import numpy as np
import pytest

import oracle
from yoda_amd import synth
from yoda_amd.capi import Yoda, topk_k
from yoda_amd.soa import MODE_SCV

pytestmark = pytest.mark.gpu


def _lists(nodes, pods, force_f64=False, alloc=None):
    import torch
    y = Yoda(0)
    y.upload_nodes(nodes, force_f64=force_f64)
    if alloc is not None:
        y.update_alloc(alloc)
    y.upload_pods(pods)
    P = pods.n_pods
    dmax = torch.zeros(6 * P, dtype=torch.int64, device="cuda:0")
    dcnt = torch.zeros(2 * P, dtype=torch.int32, device="cuda:0")
    y.shard_phase1(MODE_SCV, dmax.data_ptr(), dcnt.data_ptr())
    out = y.shard_topk(dmax.data_ptr(), dcnt.data_ptr())
    torch.cuda.synchronize()
    path = y.path
    y.close()
    return out, path


def _check(nodes, pods, counts, ts, ti, sample):
    k = topk_k()
    for p in sample:
        rc, feas, raw, _ = oracle.pod_detail(nodes, pods, int(p), MODE_SCV)
        idx = np.flatnonzero(feas)
        assert counts[0, p] == idx.size
        top = idx[np.lexsort((idx, -raw[idx]))][:k]
        m = top.size
        np.testing.assert_array_equal(ti[:m, p], top.astype(np.uint32), err_msg=f"pod {p}")
        np.testing.assert_array_equal(ts[:m, p], raw[top].astype(np.float64), err_msg=f"pod {p}")
        assert (ts[m:, p] == -1.0).all() and (ti[m:, p] == 0xFFFFFFFF).all()


@pytest.mark.parametrize("cfg,P,N,want_path", [(2, 700, 3000, "n32"), (3, 1200, 5000, "n32"),
                                               (4, 300, 2500, "n32")])
def test_topk_lists_match_oracle(cfg, P, N, want_path):
    nodes, pods = synth.make_config(cfg, pods=P, nodes=N)
    (counts, ts, ti), path = _lists(nodes, pods)
    assert path == want_path
    rng = np.random.default_rng(cfg)
    _check(nodes, pods, counts, ts, ti, rng.choice(P, 120, replace=False))


def test_topk_lists_mixed_models_and_alloc():
    """Mixed-model nodes (per-pod exact scores), several reciprocal sets and allocations that
    reorder the static part: the same lists as the oracle; F64 records agree with N32."""
    nodes, pods = synth.make_config(2, pods=640, nodes=2600)
    rng = np.random.default_rng(5)
    mix = rng.random(nodes.n_nodes) < 0.5
    k = nodes.card_clock.shape[1]
    half = k // 2
    nodes.card_clock[mix, half:] = np.where(nodes.card_clock[mix, half:] > 0, 1500, 0)
    nodes.card_bandwidth[mix, half:] = np.where(nodes.card_bandwidth[mix, half:] > 0, 1200, 0)
    alloc = (rng.random(nodes.n_nodes) * nodes.total_memory_sum.astype(np.float64)).astype(np.uint64)
    nodes.alloc_memory = alloc
    (counts, ts, ti), path = _lists(nodes, pods)
    assert path == "n32"
    _check(nodes, pods, counts, ts, ti, rng.choice(pods.n_pods, 120, replace=False))
    (c2, ts2, ti2), path2 = _lists(nodes, pods, force_f64=True)
    assert path2 == "f64"
    np.testing.assert_array_equal(ts2, ts)
    np.testing.assert_array_equal(ti2, ti)
    np.testing.assert_array_equal(c2, counts)


def test_topk_lists_ties_and_empty():
    """Identical nodes (every score ties: lowest ids first), pods feasible nowhere, one node."""
    nodes, pods = synth.make_config(2, pods=200, nodes=1)
    one = nodes.slice(0, 1)
    many = nodes.slice(0, 1)
    for name in ("card_number", "card_count", "free_memory_sum", "total_memory_sum",
                 "alloc_memory", "cpu", "disk_io"):
        setattr(many, name, np.repeat(getattr(one, name), 300, axis=0))
    for name in ("card_free_memory", "card_total_memory", "card_clock", "card_bandwidth",
                 "card_core", "card_power", "card_healthy"):
        setattr(many, name, np.repeat(getattr(one, name), 300, axis=0))
    pods.number[:50] = 64  # no node has 64 cards
    pods.has_number[:50] = 1
    (counts, ts, ti), _ = _lists(many, pods)
    _check(many, pods, counts, ts, ti, range(pods.n_pods))


def test_topk_lists_many_chunks():
    """A small batch over many nodes: hundreds of chunk lists per pod, so every thread of the
    merge (k_topk_merge_keys: one workgroup per pod) folds several lists before the wave and
    workgroup extraction rounds."""
    nodes, pods = synth.make_config(3, pods=128, nodes=40000)
    (counts, ts, ti), path = _lists(nodes, pods)
    assert path == "n32"
    rng = np.random.default_rng(11)
    _check(nodes, pods, counts, ts, ti, rng.choice(pods.n_pods, 40, replace=False))
