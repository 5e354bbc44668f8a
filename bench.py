#!/usr/bin/env python3
"""bench.py — pod-node pair evals/s of the Yoda Filter/Score/select hot path on MI355X.

Metric (BASELINE.json): pod-node pair evals/sec (filter+score+select) at 100k x 100k,
bit-exact picks.  One step = feasibility + PreScore maxima + score + NormalizeScore/select of
ALL P pods over ALL N nodes (percentageOfNodesToScore 100), node snapshot and pods already
resident in HBM, picks left in device memory.  Workload: BASELINE config 3 (100k pods x 100k
nodes, K=8, seed 7; synthetic data).  --gpus N (strong scaling: total work fixed): by
default each rank evaluates a pod slice against the whole node snapshot, with no collective
(dist.pod_partition); --shard nodes shards the nodes instead and merges the per-pod results
with RCCL all-reduces (libyoda's yoda_comm_run, or yoda_amd/dist.py over torch).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  Besides the contract fields it carries `roofline` (dominant
kernel: algorithmic bytes / HIP-event-timed launch duration vs 8 TB/s) and `cpu_baseline`
(the C oracle, reference-shaped, on a bounded pod sample, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "kubernetes-scheduler_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from yoda_amd import synth  # noqa: E402
from yoda_amd.capi import Yoda  # noqa: E402
from yoda_amd.soa import MODE_DISKIO, MODE_SCV  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def bytes_per_pair(k: int, mode: int) -> int:
    """SURVEY.md §8d / BASELINE.md: one consult of the compact node record per pair,
    B_node = 32*K + 40 B (Mode B: 16 B).  Kept for reference only: the kernels consult a
    node's facts once per 64-pod wave (and decide most pairs for a whole wave), so this
    per-pair model overstates the bytes ~100x and is not the roofline."""
    return 16 if mode == MODE_DISKIO else 32 * k + 40


def k2_unique_bytes(P: int, N: int, k: int, path: str, mode: int) -> int:
    """Algorithmic bytes of ONE K2 launch: every byte it must read or write
    at least once -- per node its K2 summary (32 + 8K B) and its record (N32: 32 + 56K B,
    F64/U64: 32 + 48K B), per pod its thresholds and reciprocals (36 B) and its argmax
    outputs (best, index, ties, lowest: 24 B).  The feasibility relation between K1 and K2
    is an intermediate (sparse form in HBM, visible in the counter traffic)."""
    if mode == MODE_DISKIO:
        return N * 16 + P * (16 + 24)
    rec = 32 + (56 if path == "n32" else 48) * k
    summ = (32 + 8 * k) if path == "n32" else 0
    return N * (rec + summ) + P * (36 + 24)


def k1_unique_bytes(P: int, N: int, k: int, path: str, mode: int) -> int:
    """Algorithmic bytes of ONE K1 launch (Filter + PreScore maxima): per node
    its K1 summary (N32: 48 + 4K B rounded to 16; F64/U64: the record, 32 + 48K B), per
    64-node block its bound summary (N32: 4 (36 + 2K) B), per pod the five Filter inputs it
    reads (scv/memory and scv/clock as u32, scv/number u64, need-memory and need-clock flags
    u32: 24 B) and the stage's outputs (6 u64 maxima + feasible and zero-total counts: 56 B).
    The chunk partials, masks and block lists K1 writes for k_reduce1 / K2 are intermediates
    (they show in the counter traffic, not here)."""
    if mode == MODE_DISKIO:  # the all-feasible state: outputs only
        return P * 56
    if path == "n32":
        per_node = (48 + 4 * k + 15) // 16 * 16
        blocks = (N + 63) // 64 * 4 * (36 + 2 * k)
    else:
        per_node, blocks = 32 + 48 * k, 0
    return N * per_node + blocks + P * (24 + 56)


def step_unique_bytes(P: int, N: int, k: int, path: str, mode: int) -> int:
    """Algorithmic bytes of one whole step: node records + both summaries (K1: 48 + 4K B,
    K2: 32 + 8K B), the pod blob (68 B) and the per-pod outputs (pick, status, ties,
    n_feasible, n_zero_total, best, 6 maxima: 76 B)."""
    if mode == MODE_DISKIO:
        return N * 16 + P * (68 + 76)
    rec = 32 + (56 if path == "n32" else 48) * k
    summ = ((48 + 4 * k + 15) // 16 * 16 + 32 + 8 * k) if path == "n32" else 0
    return N * (rec + summ) + P * (68 + 76)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def kernel_names(path: str, mode: int):
    """(K1, K2) kernel names of a record path, as rocprofv3 / tools/pmc_summary.py name them."""
    if mode == MODE_DISKIO:  # the batch path (lane = class; lane = node for <= 64 classes)
        return "k_fill_diskio_state", "k2b_class_lanes"
    return {"n32": ("k1_block_n32", "k2_block_n32"),
            "f64": ("k1_filter_maxima", "k2_score"),
            "u64": ("k1_filter_maxima", "k2_score_generic")}[path]


def committed_step_traffic(P: int, N: int, world: int):
    """Counter HBM bytes of one whole step (every kernel, FETCH_SIZE x2 + WRITE_SIZE, per
    launch x launches per step) from the committed summary, or None."""
    path = os.path.join(REPO, "profiles", "pmc_latest.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    meta = d.get("_workload", {})
    if (meta.get("pods"), meta.get("nodes"), world) != (P, N, 1):
        return None
    steps = d.get("k2_block_n32", {}).get("calls")
    if not steps:
        return None
    tot = 0.0
    for k, v in d.items():
        if isinstance(v, dict) and "hbm_bytes_per_launch" in v and v.get("calls"):
            tot += v["hbm_bytes_per_launch"] * v["calls"] / steps
    return tot


def committed_pmc(kernel: str, P: int, N: int, world: int) -> dict:
    """PMC-derived per-launch figures of `kernel` from the committed rocprofv3 summary of
    this same workload (profiles/pmc_latest.json, written by tools/profile.sh +
    tools/pmc_summary.py: FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, in bytes).  Only
    used when it was taken on the same P x N at one GPU; {} otherwise."""
    path = os.path.join(REPO, "profiles", "pmc_latest.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return {}
    meta = d.get("_workload", {})
    if (meta.get("pods"), meta.get("nodes"), world) != (P, N, 1):
        return {}
    out = dict(d.get(kernel, {}))
    out["_source"] = "profiles/pmc_latest.json (" + meta.get("profile", "?") + ")"
    return out


def cpu_baselines(nodes, pods, mode, target_s: float, threads: int, gpu_res):
    """The C oracle at T=1 and T=`threads` (the box's CPU share and k8s' 16-goroutine
    parallelizer); T=nproc is reported, not run (nproc counts the whole machine, beyond this
    box's share).  The headline entry is the T=`threads` one."""
    one = cpu_baseline(nodes, pods, mode, target_s / 2, 1, gpu_res)
    many = cpu_baseline(nodes, pods, mode, target_s / 2, threads, gpu_res)
    many["by_threads"] = {"1": {k: one[k] for k in ("value", "sample", "sample_picks_match_gpu")},
                          str(threads): {k: many[k] for k in ("value", "sample")}}
    many["cpu_model"] = cpu_model()
    many["nproc"] = os.cpu_count()
    many["nproc_note"] = (f"T=nproc ({os.cpu_count()}) not run: the GPU box's CPU share is "
                          f"{threads} threads (OMP_NUM_THREADS), nproc counts the whole machine")
    return many


def cpu_baseline(nodes, pods, mode, target_s: float, threads: int, gpu_res):
    """Time the C oracle (scalar, reference-shaped) on a bounded pod sample; also checks the
    sample's picks against the GPU's (the oracle is the checker here)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # noqa: E402  (cpu_baseline leg only)
    oracle.lib()
    probe = min(pods.n_pods, 4 * threads)
    t0 = time.perf_counter()
    oracle.schedule(nodes, pods.slice(0, probe), mode, threads=threads)
    rate = probe * nodes.n_nodes / (time.perf_counter() - t0)
    sample = int(max(probe, min(pods.n_pods, rate * target_s / nodes.n_nodes)))
    sub = pods.slice(0, sample)
    t0 = time.perf_counter()
    want = oracle.schedule(nodes, sub, mode, threads=threads)
    dt = time.perf_counter() - t0
    parity = bool(np.array_equal(want.pick, gpu_res.pick[:sample]) and
                  np.array_equal(want.status, gpu_res.status[:sample]))
    return {"value": sample * nodes.n_nodes / dt, "unit": "pairs/s", "cores": threads,
            "kind": "port",
            "sample": f"first {sample} pods x all {nodes.n_nodes} nodes of the same workload, "
                      f"C oracle (yoda_oracle.c, reference-shaped: per pod filter, "
                      f"CollectMaxValues, score, normalize, select), OpenMP {threads} threads, "
                      f"{dt:.1f} s",
            "sample_picks_match_gpu": parity}


def bench_greedy(args):
    """Config 5: greedy batched assignment (sequential assume in sort.Less order).
    value = pods scheduled per second, reference-faithful mode (flags 0: allocated memory
    feeds Allocate, algorithm.go:299-303); `capacity` = the same batch with the CardNumber
    decrement (YODA_GREEDY_CARD_CAPACITY, the build-defined extension BASELINE config 5 names).
    N=1: one handle (yoda_greedy); N>1: nodes sharded across ranks, windows merged over RCCL
    by libyoda's own driver (yoda_comm_greedy; --greedy-driver python: yoda_amd/dist.py
    sharded_greedy over torch.distributed).  Rank 0 checks a queue-order prefix against the
    sequential oracle (N=1), for both modes."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_index = 0 if os.environ.get("YODA_BENCH_SAME_DEVICE") == "1" else local_rank
    device = torch.device("cuda", dev_index)
    torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("YODA_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    cfg = 5
    nodes, pods = synth.make_config(cfg, pods=args.pods, nodes=args.nodes)
    y = Yoda(dev_index)
    runs = {}
    if world == 1:
        y.upload_nodes(nodes)
        runs = greedy_runs(y, pods, device)
    else:
        import torch.distributed as dist
        from yoda_amd.dist import HandleShard, Reducer, agree_on_path, shard_bounds, sharded_greedy
        b = shard_bounds(nodes.n_nodes, world)
        lo, hi = int(b[rank]), int(b[rank + 1])
        shard = nodes.slice(lo, hi)
        y.upload_nodes(shard, node_offset=lo)
        red = Reducer()
        agree_on_path(red, [y], [shard], [lo], device)
        hs = [HandleShard(y, device)]
        native = args.greedy_driver == "libyoda"
        if native:  # libyoda's own RCCL communicator (yoda_comm_init), id broadcast by torch
            from yoda_amd.dist import LibExchange
            LibExchange(y, device)

        def run_greedy(pd, flags, st=None):
            if not native:
                return sharded_greedy(hs, red, nodes, pd, flags, stats=st)
            pk = y.comm_greedy(nodes, pd, MODE_SCV, flags)
            if st is not None:
                st.update(y.comm_greedy_stats())
            return pk

        for flags in (0, 1):
            run_greedy(pods.slice(0, min(pods.n_pods, 4096)), flags)  # warm-up
            dist.barrier()
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            st = {}
            picks = run_greedy(pods, flags, st)
            torch.cuda.synchronize(device)
            dt = time.perf_counter() - t0
            t = torch.tensor([dt], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            runs[flags] = {"seconds": float(t.item()), "picks": picks, "windows": st["windows"],
                           "driver": "yoda_comm_greedy" if native else "dist.sharded_greedy",
                           ("exact_fallback_pods" if flags == 0 else "window_restarts"):
                           st["exact_pods"] if flags == 0 else st["restarts"],
                           "refreshes": st.get("refreshes", 0)}
            if native:
                runs[flags]["collectives"] = st["collectives"]
            if args.check and rank == 0:
                full = Yoda(dev_index)
                full.upload_nodes(nodes)
                if not np.array_equal(full.greedy(pods, MODE_SCV, flags), picks):
                    raise SystemExit(f"--check: sharded greedy picks (flags {flags}) differ "
                                     "from the single handle")
                full.close()
                runs[flags]["check"] = "sharded greedy picks == single-handle yoda_greedy"
    r0, r1 = runs[0], runs[1]
    out = {"metric": "greedy batch: pods assigned/s (config 5, exact vs the sequential oracle)",
           "value": pods.n_pods / r0["seconds"], "unit": "pods/s", "n_gpus": world,
           "seconds": r0["seconds"], "higher_is_better": True,
           "data": "synthetic (yoda_amd/synth.py config 5)",
           "config": {"workload": f"config5: {pods.n_pods} pods x {nodes.n_nodes} nodes greedy",
                      "pods": pods.n_pods, "nodes": nodes.n_nodes, "path": y.path,
                      "parallelism": f"node-shard x{world}" + (" (RCCL window merges)"
                                                               if world > 1 else "")},
           "pairs_per_s_equiv": pods.n_pods * nodes.n_nodes / r0["seconds"],
           "assigned": int((r0["picks"] >= 0).sum())}
    out.update({k: v for k, v in r0.items() if k not in ("seconds", "picks")})
    out["capacity"] = {"flags": "YODA_GREEDY_CARD_CAPACITY", "value": pods.n_pods / r1["seconds"],
                       "unit": "pods/s", "seconds": r1["seconds"],
                       "assigned": int((r1["picks"] >= 0).sum())}
    out["capacity"].update({k: v for k, v in r1.items() if k not in ("seconds", "picks")})
    if world > 1:
        if rank == 0:
            print(json.dumps(out), flush=True)
        y.close()
        import torch.distributed as dist
        dist.destroy_process_group()
        return
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # noqa: E402  (cpu_baseline leg only)
        # the sequential oracle on a prefix of the queue (greedy is order-dependent, so a
        # prefix in queue order is an exact sub-problem)
        order = oracle.queue_order(pods)
        for flags, dst in ((0, out), (1, out["capacity"])):
            probe = min(pods.n_pods, 16)
            t0 = time.perf_counter()
            oracle.greedy(nodes, pods.take(order[:probe]), MODE_SCV, flags)
            per_pod = max((time.perf_counter() - t0) / probe, 1e-9)
            n = int(max(probe, min(pods.n_pods, args.cpu_seconds / 2 / per_pod)))
            prefix = pods.take(order[:n])
            t0 = time.perf_counter()
            want, _ = oracle.greedy(nodes, prefix, MODE_SCV, flags)
            cdt = time.perf_counter() - t0
            got = y.greedy(prefix, MODE_SCV, flags)
            dst["cpu_baseline"] = {"value": n / cdt, "unit": "pods/s", "cores": 1, "kind": "port",
                                   "sample": f"first {n} pods in queue order, sequential oracle "
                                             f"(yoda_oracle.c oracle_greedy, flags {flags}), "
                                             f"{cdt:.1f} s",
                                   "sample_picks_match_gpu": bool(np.array_equal(got, want))}
    print(json.dumps(out), flush=True)
    y.close()


def greedy_runs(y, pods, device) -> dict:
    """Config 5 on one handle (nodes uploaded): flags 0 (reference-faithful assume) and 1 (the
    card-capacity decrement), each after a 4096-pod warm-up batch; seconds host to host."""
    runs = {}
    for flags in (0, 1):
        y.greedy(pods.slice(0, min(pods.n_pods, 4096)), MODE_SCV, flags)  # warm-up
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        picks = y.greedy(pods, MODE_SCV, flags)
        dt = time.perf_counter() - t0
        windows, fallbacks, times = y.greedy_stats(times=True)
        runs[flags] = {"seconds": dt, "picks": picks, "windows": windows,
                       "exact_fallback_pods": fallbacks, "host_times_ms": times}
        if flags:
            runs[flags]["window_restarts"] = y.greedy_restarts()
    return runs


def greedy_leg(dev_index: int) -> dict:
    """extra.greedy: config 5 at full size (1M pods x 100k nodes, sort.Less queue order,
    sequential assume) on this GPU, both flags -- the driver-observed config-5 seconds.  Every
    pick of both runs is checked against the oracle's per-window digests in the GPU suite
    (tests/test_gpu_greedy_config5.py); here the picks are summarised by a SHA-256 digest."""
    import hashlib
    device = torch.device("cuda", dev_index)
    nodes, pods = synth.make_config(5)
    z = Yoda(dev_index)
    z.upload_nodes(nodes)
    runs = greedy_runs(z, pods, device)
    z.close()
    out = {"workload": f"config5: {pods.n_pods} pods x {nodes.n_nodes} nodes greedy"}
    for flags, key in ((0, "flags0"), (1, "capacity")):
        r = runs[flags]
        out[key] = {k: v for k, v in r.items() if k != "picks"}
        out[key]["assigned"] = int((r["picks"] >= 0).sum())
        out[key]["picks_sha256"] = hashlib.sha256(r["picks"].astype(np.int32).tobytes()).hexdigest()
    out["seconds"] = out["flags0"]["seconds"]
    return out


def _timed_steps(step, barrier, n: int) -> float:
    step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    barrier()
    return (time.perf_counter() - t0) / n * 1e3


def row_latency(dev_index: int, node_counts=(5000, 100000), cycles: int = 60) -> dict:
    """Plugin row mode: one scheduling cycle's PreFilter through the
    Python plugin mirror (yoda_amd/plugin.py) = pack the pod (Go label semantics), upload it,
    yoda_score_rows (Filter bits + raw Score of every node) and copy the row back; and the
    bare C-ABI part of it (upload_pods + score_rows).  P = 1, config-3 nodes."""
    from yoda_amd.pack import pods_to_dicts
    from yoda_amd.plugin import CycleState, YodaPlugin
    out = {}
    for n in node_counts:
        nodes, pods = synth.make_config(3, pods=cycles, nodes=n)
        z = Yoda(dev_index)
        z.upload_nodes(nodes)
        plugin = YodaPlugin(z, [f"node-{i}" for i in range(n)], nodes)
        dicts = pods_to_dicts(pods)
        for d in dicts[:3]:
            plugin.pre_filter(CycleState(), d)
        t_plugin, t_abi, t_b = [], [], []
        for p, d in enumerate(dicts):
            t0 = time.perf_counter()
            plugin.pre_filter(CycleState(), d)
            t_plugin.append((time.perf_counter() - t0) * 1e3)
            one = pods.slice(p, p + 1)
            t0 = time.perf_counter()
            z.upload_pods(one)
            z.score_rows(MODE_SCV)
            t_abi.append((time.perf_counter() - t0) * 1e3)
            # Mode B (BalancedCpuDiskIOPriority, what the shipped binary scores per cycle)
            t0 = time.perf_counter()
            z.upload_pods(one)
            z.score_rows(MODE_DISKIO)
            t_b.append((time.perf_counter() - t0) * 1e3)
        z.close()
        q = lambda v, x: float(np.percentile(v, x))  # noqa: E731
        out[str(n)] = {"prefilter_ms_p50": q(t_plugin, 50), "prefilter_ms_p99": q(t_plugin, 99),
                       "capi_ms_p50": q(t_abi, 50), "capi_ms_p99": q(t_abi, 99),
                       "capi_diskio_ms_p50": q(t_b, 50), "capi_diskio_ms_p99": q(t_b, 99),
                       "cycles": cycles}
    return out


def diskio_classes(pods) -> int:
    """Distinct Mode-B pod classes of a batch: (alpha, beta) bit pairs (algorithm.go:105-106,
    the grouping libyoda's Mode-B batch path evaluates once per class)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        beta = 1.0 / (1.0 + pods.rcpu.astype(np.float64) / pods.rio)
    alpha = 1 - beta
    key = np.stack([alpha.view(np.uint64), beta.view(np.uint64)], axis=1)
    return int(np.unique(key, axis=0).shape[0])


def disclosure(y, nodes, pods, step, barrier, args) -> dict:
    """What the headline depends on, measured after the
    timed region on the same GPU: the block kernels' work classes for this batch (device
    counters), the per-pair kernels on the same workload, and the workloads the headline does
    not cover (synth.VARIANTS): mixed-model nodes, memory in bytes, the U64 record path,
    config 4 at its declared size and at 100k x 100k, and Mode B with the pods as generated
    and with a distinct request per pod -- each with its K1/K2 HIP-event times and class
    fractions."""
    out = {}
    y.class_stats(True)
    step()
    barrier()
    y.class_stats(False)
    out["classes"] = y.class_stats()
    dev_index = torch.cuda.current_device()
    variants = {}

    def timed(name, nd, pd, mode, kw, steps):
        z = Yoda(dev_index)
        z.upload_nodes(nd, **kw)
        z.upload_pods(pd)
        z.set_stream(torch.cuda.current_stream().cuda_stream)
        z.run(mode)
        barrier()
        z.profile(True)
        ms = _timed_steps(lambda: z.run(mode), barrier, steps)
        z.profile(False)
        k1, k2, nl = z.profile_read()
        v = {"desc": synth.VARIANTS.get(name, name), "pods": pd.n_pods, "nodes": nd.n_nodes,
             "mode": "diskio" if mode == MODE_DISKIO else "scv", "path": z.path,
             "ms_per_step": ms, "pairs_per_s": pd.n_pods * nd.n_nodes / (ms / 1e3),
             "k1_ms": k1 / max(nl, 1), "k2_ms": k2 / max(nl, 1)}
        if mode == MODE_SCV and z.path == "n32":
            z.class_stats(True)
            z.run(mode)
            barrier()
            z.class_stats(False)
            v["classes"] = z.class_stats()
        if mode == MODE_DISKIO:
            D = diskio_classes(pd)
            v["pod_classes"] = D
            # K2B roofline (Mode B): D x N class-node pairs, each 3 f64 VALU ops
            # (a = alpha V, b = beta U, d = a - b) + 2 compares + a carry-add = 6 VALU
            # instructions per 64 pairs on one SIMD (4 cycles each, full rate) -- issue-bound;
            # bytes: 16 B per node record and 24 B out per pod
            cn_pairs = D * nd.n_nodes
            simd_rate = 1024 * 2.4e9 / 4  # wave instructions / s: 256 CUs x 4 SIMDs, 2.4 GHz
            ideal_ms = cn_pairs * 6 / 64 / simd_rate * 1e3
            k2 = v["k2_ms"]
            v["k2b_roofline"] = {
                "bound": "valu_issue", "class_node_pairs": cn_pairs, "valu_per_pair": 6,
                "ideal_ms": ideal_ms, "frac": ideal_ms / k2 if k2 > 0 else None,
                "unique_bytes": nd.n_nodes * 16 + pd.n_pods * 24,
                "hbm_frac": ((nd.n_nodes * 16 + pd.n_pods * 24) / (k2 / 1e3) / 1e9 / HBM_PEAK_GBS
                             if k2 > 0 else None)}
        variants[name] = v
        z.close()

    timed("per_pair_kernels", nodes, pods, MODE_SCV, dict(per_node_k1=True, per_node_k2=True), 3)
    variants["per_pair_kernels"]["desc"] = "config 3 on the per-pair kernels (no block classes)"
    for name, nd, pd, mode, kw in synth.variant_workloads(
            ["mixed50", "bytes", "bw1000", "f64", "u64", "c4", "het100k", "diskio",
             "diskio_distinct"]):
        timed(name, nd, pd, mode, kw, 3 if name in ("u64", "f64") else 5)
    out["variants"] = variants
    out["plugin_row_latency"] = row_latency(dev_index)
    if not args.no_greedy:
        out["greedy"] = greedy_leg(dev_index)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--greedy-driver", choices=("libyoda", "python"), default="libyoda",
                    help="--workload greedy at N>1: libyoda's yoda_comm_greedy (RCCL inside "
                         "libyoda) or the Python dist.sharded_greedy (torch.distributed)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--pods", type=int, default=None)
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--mode", choices=["scv", "diskio"], default="scv")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the disclosure runs (work classes, per-pair path, mixed-model "
                         "and F64 variants) after the timed region")
    ap.add_argument("--no-greedy", action="store_true",
                    help="skip the config-5 greedy leg of the disclosure runs (extra.greedy)")
    ap.add_argument("--check", action="store_true",
                    help="N>1: rank 0 re-evaluates the batch on one unsharded handle and "
                         "asserts identical picks / statuses / ties (rehearsal)")
    ap.add_argument("--shard", choices=["nodes", "pods"], default="pods",
                    help="--gpus N > 1: pods (default) = each rank evaluates a pod slice "
                         "against the whole node snapshot, no collective (dist.pod_partition); "
                         "nodes = node blocks merged by RCCL all-reduces, the north_star's "
                         "packed-key merge (yoda_amd/dist.py).  Default from the one-GPU rank "
                         "probes of tools/rank_probe.py (DESIGN.md §7, profiles/r06/rank8/): "
                         "at 8 ranks the slowest pod rank takes 0.36 ms, a node rank 0.35 ms "
                         "before its three collectives")
    ap.add_argument("--exchange", choices=["torch", "libyoda"], default="libyoda",
                    help="--shard nodes: libyoda (default) = libyoda's own RCCL exchanges "
                         "(yoda_comm_run: maxima MAX + counts SUM in one group, the packed "
                         "(score, node) key MAX, the winners' ties SUM; fused pack/unpack "
                         "kernels); torch = the same merge through torch.distributed "
                         "(yoda_amd/dist.py ShardExchange, elementwise torch ops around it: "
                         "0.43 vs 0.35 ms per 8-way rank on the probe)")
    ap.add_argument("--no-balance", action="store_true",
                    help="--shard nodes: keep equal node blocks (default: re-cut them once "
                         "after warm-up so every rank's measured K1 + K2 time is equal)")
    ap.add_argument("--workload", choices=["eval", "greedy", "row"], default="eval",
                    help="eval: the headline batch (config 3); greedy: config 5 sequential "
                         "assume; row: the plugin's per-cycle row latency (P = 1)")
    args = ap.parse_args()
    if args.workload == "greedy":
        return bench_greedy(args)
    if args.workload == "row":
        torch.cuda.set_device(0)
        print(json.dumps({"metric": "plugin PreFilter latency (one pod vs every node)",
                          "unit": "ms", "higher_is_better": False,
                          "row_latency": row_latency(0)}), flush=True)
        return
    mode = MODE_SCV if args.mode == "scv" else MODE_DISKIO

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # Rehearsal knobs (one-GPU boxes): YODA_BENCH_SAME_DEVICE=1 puts every rank on cuda:0,
    # YODA_DIST_BACKEND=gloo exchanges over gloo.  The driver's runs use neither (RCCL).
    dev_index = 0 if os.environ.get("YODA_BENCH_SAME_DEVICE") == "1" else local_rank
    device = torch.device("cuda", dev_index)
    torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("YODA_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    nodes, pods = synth.make_config(args.config, pods=args.pods, nodes=args.nodes)
    P, N = pods.n_pods, nodes.n_nodes
    from yoda_amd.dist import ShardExchange, pod_partition, shard_bounds
    pod_shard = world > 1 and args.shard == "pods"
    y = Yoda(dev_index)
    if pod_shard:
        # rank r: pods part[r] x ALL nodes; nothing to exchange (dist.pod_partition)
        my_pods_idx = pod_partition(pods, world)[rank]
        my_pods = pods.take(my_pods_idx)
        lo, hi = 0, N
        shard = nodes
        y.upload_nodes(nodes)
        y.upload_pods(my_pods)
    else:
        my_pods = pods
        b = shard_bounds(N, world)
        lo, hi = int(b[rank]), int(b[rank + 1])
        shard = nodes.slice(lo, hi)
        y.upload_nodes(shard, node_offset=lo)
        y.upload_pods(pods)
    y.set_stream(torch.cuda.current_stream(device).cuda_stream)
    k_slots = int(nodes.card_count.max()) if N else 1
    k_slots = 1 << max(0, (k_slots - 1).bit_length())

    def make_exchange():
        if args.exchange == "libyoda":
            from yoda_amd.dist import LibExchange
            return LibExchange(y, device, shard=shard, offset=lo)
        return ShardExchange.distributed(y, device, shard=shard, offset=lo)

    if world > 1 and not pod_shard:
        ex = make_exchange()
        step = lambda: ex.step(mode)  # noqa: E731
    else:
        step = lambda: y.run(mode)  # noqa: E731

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize(device)

    for _ in range(args.warmup):
        step()
    barrier()
    if world > 1 and not pod_shard and not args.no_balance:
        # Setup, before the timed region: re-cut the node blocks so every rank's K1 + K2
        # time is equal (the cost per node is data-dependent), then re-upload.
        import torch.distributed as dist
        from yoda_amd.dist import balanced_bounds
        for _ in range(2):
            y.profile(True)
            for _ in range(3):
                step()
            barrier()
            y.profile(False)
            k1, k2, nl = y.profile_read()
            cost = torch.tensor([(k1 + k2) / max(nl, 1)], dtype=torch.float64, device=device)
            costs = [torch.zeros_like(cost) for _ in range(world)]
            dist.all_gather(costs, cost)
            nb = balanced_bounds(b, [float(t.item()) for t in costs])
            if np.array_equal(nb, b) or np.abs(nb - b).max() < 64:
                break
            b = nb
            lo, hi = int(b[rank]), int(b[rank + 1])
            shard = nodes.slice(lo, hi)
            y.upload_nodes(shard, node_offset=lo)
            ex = make_exchange()
            step = lambda: ex.step(mode)  # noqa: E731
            for _ in range(max(args.warmup, 1)):
                step()
            barrier()
    y.profile(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    y.profile(False)
    k1_ms, k2_ms, launches = y.profile_read()
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # End-to-end (pod H2D + kernels + picks D2H), single GPU only: reported, never `value`.
    e2e_ms = None
    if world == 1:
        # median of 9 after 2 untimed batches (the first upload of the loop wakes the host
        # pool and touches the staging pages): the host pod SoA -> yoda_upload_pods (pack +
        # one pinned H2D) -> yoda_run -> picks and statuses back to host memory
        ts = []
        for it in range(11):
            t0 = time.perf_counter()
            y.upload_pods(pods)
            y.run(mode)
            y.download_picks()
            if it >= 2:
                ts.append((time.perf_counter() - t0) * 1e3)
        e2e_ms = float(np.median(ts))
    res = y.download()

    ms_per_step = elapsed / args.steps * 1e3
    value = P * N / (elapsed / args.steps)
    n_local = hi - lo
    p_local = my_pods.n_pods
    # Per kernel (K1 = Filter + maxima, K2 = score + argmax): its algorithmic bytes per launch
    # over its HIP-event launch time (events on the launch stream), the PMC counter bytes and
    # issue figures of the committed rocprofv3 summary; the line's roofline is the DOMINANT
    # kernel's (the longer average launch), whichever it is.
    k1_avg = k1_ms / max(launches, 1)
    k2_avg = k2_ms / max(launches, 1)
    names = kernel_names(y.path, mode)
    per_kernel = {}
    for tag, name, avg, algo in (
            ("k1", names[0], k1_avg, k1_unique_bytes(p_local, n_local, k_slots, y.path, mode)),
            ("k2", names[1], k2_avg, k2_unique_bytes(p_local, n_local, k_slots, y.path, mode))):
        pmc = committed_pmc(name, P, N, world)
        ach = algo / (avg / 1e3) / 1e9 if avg > 0 else 0.0
        tr = pmc.get("hbm_bytes_per_launch")
        per_kernel[tag] = {
            "kernel": name, "avg_launch_ms": avg, "algo_bytes_per_launch": algo,
            "achieved": ach, "frac": ach / HBM_PEAK_GBS,
            "traffic": tr,
            # counter bytes over the committed profile's own launch time, against peak
            "traffic_frac": (tr / (pmc["avg_ns"] / 1e9) / 1e9 / HBM_PEAK_GBS
                             if tr and pmc.get("avg_ns") else None),
            "traffic_over_algo": tr / algo if tr and algo else None,
            "write_bytes": pmc.get("hbm_write_bytes"),
            "pmc_avg_ms": pmc["avg_ns"] / 1e6 if pmc.get("avg_ns") else None,
            # the issue roofline (what binds these kernels): VALU and SALU issue
            # cycles / available cycles, and the share of wave-cycles waiting on memory
            "issue": {k: pmc[k] for k in ("valu_issue_util", "salu_issue_util",
                                          "wave_frac_waitcnt", "wave_frac_issue_stall",
                                          "wave_frac_issuing") if k in pmc}}
    dom_tag = "k2" if k2_avg >= k1_avg else "k1"
    dom = per_kernel[dom_tag]
    pmc_src = committed_pmc(dom["kernel"], P, N, world).get("_source")
    step_traffic = committed_step_traffic(P, N, world)
    step_bytes = step_unique_bytes(p_local, n_local, k_slots, y.path, mode)

    out = {
        "metric": "pod-node pair evals/sec (filter+score+select) at 100k×100k; bit-exact picks",
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        # arithmetic of the dominant kernel: N32 = u32 compares/sums + f32/f64 quotients
        "dtype": {"n32": "u32+f32+f64", "f64": "f64", "u64": "u64"}[y.path]
        if mode == MODE_SCV else "f64",
        "data": "synthetic (seeded SCV node records and pod requests, yoda_amd/synth.py)",
        "config": {"workload": f"config{args.config}: {P} pods x {N} nodes, "
                               f"{'Mode A SCV GPU score' if mode == MODE_SCV else 'Mode B diskIO'}"
                               f", K={k_slots} card slots",
                   "pods": P, "nodes": N, "mode": args.mode,
                   "path": y.path,
                   "parallelism": (f"pod-shard x{world} (whole node snapshot per GPU, "
                                   "no collective)" if pod_shard else
                                   f"node-shard x{world}" + (
                                       (" (RCCL inside libyoda: all-reduce + all-gather)"
                                        if args.exchange == "libyoda" else
                                        " (RCCL all-reduce merge)") if world > 1 else "")),
                   "node_bounds": [int(v) for v in b] if world > 1 and not pod_shard
                   else None},
        # the dominant kernel's algorithmic (unique) bytes per launch / its HIP-event launch
        # time, against HBM peak; `traffic` = its measured HBM bytes per launch (PMC).  What
        # binds it is instruction issue / memory latency at its occupancy, not HBM bandwidth
        # (DESIGN.md §4): `bound` says so, `frac` stays the HBM fraction, and `issue` carries
        # the PMC issue utilisation and wait fractions beside it; `per_kernel` holds both.
        "roofline": {"bound": "issue/latency", "frac_of": "hbm", "kernel": dom["kernel"],
                     "dominant_by_time": dom["kernel"],
                     "achieved": dom["achieved"],
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": dom["frac"],
                     "traffic": dom["traffic"],
                     "algo_bytes_per_launch": dom["algo_bytes_per_launch"],
                     "avg_launch_ms": dom["avg_launch_ms"], "k1_avg_ms": k1_avg,
                     "k2_avg_ms": k2_avg,
                     "issue": dom["issue"],
                     "per_kernel": per_kernel,
                     "fractions": {
                         # the whole step's algorithmic bytes / step time / peak
                         "unique_bytes_step": step_bytes / (ms_per_step / 1e3) / 1e9
                         / HBM_PEAK_GBS},
                     "step_traffic_bytes": step_traffic,
                     "step_unique_bytes": step_bytes,
                     "per_pair_model_bytes": bytes_per_pair(k_slots, mode),
                     "pmc_source": pmc_src},
        "e2e_ms": e2e_ms,
        "status_counts": {str(s): int((res.status == s).sum()) for s in np.unique(res.status)},
    }
    if world > 1 and args.check and rank == 0:
        full = Yoda(dev_index)
        full.upload_nodes(nodes)
        ref = full.eval(pods, mode)
        full.close()
        sel = my_pods_idx if pod_shard else slice(None)
        for f in ("pick", "status", "n_ties", "n_feasible"):
            if not np.array_equal(getattr(res, f), getattr(ref, f)[sel]):
                raise SystemExit(f"--check: sharded {f} differs from the unsharded handle")
        out["check"] = ("rank 0's pod shard" if pod_shard else "merged") + \
            " picks/statuses/ties/feasible == unsharded"
    if rank == 0 and world == 1 and not args.no_extras and mode == MODE_SCV:
        out["extra"] = disclosure(y, nodes, pods, step, barrier, args)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baselines(nodes, pods, mode, args.cpu_seconds,
                                            args.cpu_threads, res)
    if rank == 0:
        print(json.dumps(out), flush=True)
    y.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
