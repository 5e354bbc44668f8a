#!/usr/bin/env python3
"""Estimate, on the CPU, how the block-classified kernels split a workload: for every
(pod wave, node) pair of the sorted batch, K1's class (ALL / NONE / PART) and K2's
(skipped / U / FAST / EXACT).  Mirrors the bounds of k1_block_n32 / k2_block_n32 for
one-model nodes (every synthetic node of configs 2/3/5 is one-model).  Diagnostic only.

    python tools/class_stats.py [--config 3] [--pods 20000] [--nodes 20000]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "kubernetes-scheduler_amd"), os.path.join(REPO, "oracle")]
from yoda_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--pods", type=int, default=20000)
    ap.add_argument("--nodes", type=int, default=20000)
    a = ap.parse_args()
    nodes, pods = synth.make_config(a.config, pods=a.pods, nodes=a.nodes)
    P, N = pods.n_pods, nodes.n_nodes
    number = np.where(pods.has_number == 1, pods.number, 1).astype(np.uint64)
    m = np.where(pods.has_memory == 1, pods.memory, 0).astype(np.int64)
    c = np.where(pods.has_clock == 1, pods.clock, 0).astype(np.int64)
    need_m = np.where(pods.has_memory == 1, number, 0).astype(np.int64)
    need_c = np.where(pods.has_clock == 1, number, 0).astype(np.int64)
    key = (np.minimum(c, 0xffffff) << 40) | (np.minimum(number, 0xff).astype(np.int64) << 32) | m
    order = np.argsort(key, kind="stable")
    number, m, c, need_m, need_c = (x[order] for x in (number, m, c, need_m, need_c))
    K = nodes.card_free_memory.shape[1]
    free = nodes.card_free_memory.astype(np.int64)
    healthy = nodes.card_healthy.astype(bool)
    hfs = -np.sort(-np.where(healthy, free + 1, 0), axis=1)
    hfs = np.concatenate([hfs, np.zeros((N, 1), np.int64)], axis=1)  # slot K: no such card
    ck = nodes.card_clock[:, 0].astype(np.int64)
    nh = healthy.sum(axis=1)
    cn = nodes.card_number.astype(np.uint64)
    mrf1 = free.max(axis=1) + 1
    fs = -np.sort(-free, axis=1)
    k1 = {"all": 0, "none": 0, "part": 0}
    for w0 in range(0, P, 64):
        sl = slice(w0, min(w0 + 64, P))
        nm, mm, cc, nc, nu = need_m[sl], m[sl], c[sl], need_c[sl], number[sl]
        pm, pc = nm > 0, nc > 0
        mem_all = np.ones(N, bool)
        if pm.any():
            i = min(int(nm[pm].max()), K + 1) - 1
            mem_all = hfs[:, min(i, K)] > mm[pm].max()
        mem_none = np.zeros(N, bool)
        if pm.all():
            i = min(int(nm.min()), K + 1) - 1
            mem_none = hfs[:, min(i, K)] <= mm.min()
        cuni = pc.any() and cc[pc].min() == cc[pc].max()
        clk_all = np.ones(N, bool) if not pc.any() else (
            (ck == cc[pc].max()) & (nh >= nc[pc].max()) if cuni else np.zeros(N, bool))
        clk_none = np.zeros(N, bool)
        if pc.all() and cuni:
            clk_none = (ck != cc.max()) | (nh < nc.min())
        feas_all = (nu.max() <= cn) & mem_all & clk_all
        feas_none = (nu.min() > cn) | mem_none | clk_none
        q_all = (ck >= cc.max()) & (mrf1 > mm.max())
        q_none = (ck < cc.min()) | (mrf1 <= mm.min())
        is_all = ~feas_none & feas_all & (q_all | q_none)
        k1["none"] += int(feas_none.sum())
        k1["all"] += int(is_all.sum())
        k1["part"] += int((~feas_none & ~is_all).sum())
    tot = sum(k1.values())
    print("K1 (wave, node) pairs:", {k: f"{v / tot:.4f}" for k, v in k1.items()})
    # K2: needs every pod's feasibility and maxima (the C oracle, sorted order)
    import oracle
    res = oracle.schedule(nodes, pods.take(order), 0, threads=8)
    mx = res.maxima  # [P][6] in collection.go order: bw, clock, core, free, power, total
    key_m = mx[:, [0, 2, 3, 4, 5]]
    k2 = {"skip": 0, "u": 0, "fast": 0, "exact": 0}
    extra = {"fast_rec": 0, "nonuni_feasible": 0}
    per_wave = []
    uni_waves = 0
    for w0 in range(0, P, 64):
        sl = slice(w0, min(w0 + 64, P))
        mm, cc = m[sl], c[sl]
        nu, nm, nc = number[sl], need_m[sl], need_c[sl]
        hidx = np.clip(nm, 1, K + 1) - 1
        feas = ((nu[:, None] <= cn[None, :])
                & ((nm[:, None] == 0) | (hfs[:, hidx].T > mm[:, None]))
                & ((nc[:, None] == 0) | ((ck[None, :] == cc[:, None]) & (nh[None, :] >= nc[:, None]))))
        anyf = feas.any(axis=0)
        allf = feas.all(axis=0)
        uni = (key_m[sl] == key_m[sl][0]).all()
        uni_waves += uni
        k2["skip"] += int((~anyf).sum())
        if not uni:
            k2["exact"] += int(anyf.sum())
            extra["nonuni_feasible"] += int(anyf.sum())
            per_wave.append(int(anyf.sum()))
            continue
        nq_lo = (fs >= mm.max()).sum(axis=1)
        nq_hi = (fs >= mm.min()).sum(axis=1)
        qall, qnone = ck >= cc.max(), ck < cc.min()
        u = allf & (nq_lo == nq_hi) & (qall | qnone)
        k2["u"] += int(u.sum())
        k2["fast"] += int((anyf & ~u).sum())
        extra["fast_rec"] += int((anyf & ~u & (nq_hi - nq_lo <= 1)).sum())
        per_wave.append(int((anyf & ~u).sum()))
    tot = sum(k2.values())
    print("K2 (wave, node) pairs:", {k: f"{v / tot:.4f}" for k, v in k2.items()},
          f"uniform-maxima waves {uni_waves}/{(P + 63) // 64}",
          {k: f"{v / tot:.4f}" for k, v in extra.items()})
    pw = np.array(per_wave)
    print("per-pod nodes per wave: mean %.0f p50 %.0f p90 %.0f p99 %.0f max %d (of %d nodes)" % (
        pw.mean(), np.percentile(pw, 50), np.percentile(pw, 90), np.percentile(pw, 99), pw.max(), N))


if __name__ == "__main__":
    main()
