#!/usr/bin/env python3
"""bench.py — pod-node pair evals/s of the Yoda Filter/Score/select hot path on MI355X.

Metric (BASELINE.json): pod-node pair evals/sec (filter+score+select) at 100k x 100k,
bit-exact picks.  One step = feasibility + PreScore maxima + score + NormalizeScore/select of
ALL P pods over ALL N nodes (percentageOfNodesToScore 100), node snapshot and pods already
resident in HBM, picks left in device memory.  Workload: BASELINE config 3 (100k pods x 100k
nodes, K=8, seed 7; synthetic data).  --gpus N (strong scaling: total work fixed): by
default the nodes are sharded across ranks and the per-pod results merged with RCCL
all-reduces (yoda_amd/dist.py); --shard pods gives each rank a pod slice and the whole node
snapshot instead, with no collective (dist.pod_partition).

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
    """SURVEY.md §8d / BASELINE.md: one consult of the compact node record,
    B_node = 32*K + 40 B (Mode B: 16 B)."""
    return 16 if mode == MODE_DISKIO else 32 * k + 40


def kernel_names(path: str, mode: int):
    """(K1, K2) kernel names of a record path, as rocprofv3 / tools/pmc_summary.py name them."""
    if mode == MODE_DISKIO:
        return "k_fill_diskio_state", "k2_diskio"
    return {"n32": ("k1_block_n32", "k2_block_n32"),
            "f64": ("k1_filter_maxima", "k2_score"),
            "u64": ("k1_filter_maxima", "k2_score_generic")}[path]


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
    value = pods scheduled per second.  N=1: one handle (yoda_greedy); N>1: nodes sharded
    across ranks, windows merged over RCCL (yoda_amd/dist.py sharded_greedy).  Rank 0 checks
    a queue-order prefix against the sequential oracle (N=1)."""
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
    flags = 0
    y = Yoda(dev_index)
    if world == 1:
        y.upload_nodes(nodes)
        y.greedy(pods.slice(0, min(pods.n_pods, 4096)), MODE_SCV, flags)  # warm-up
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        picks = y.greedy(pods, MODE_SCV, flags)
        dt = time.perf_counter() - t0
        windows, fallbacks, times = y.greedy_stats(times=True)
        extra = {"windows": windows, "exact_fallback_pods": fallbacks, "host_times_ms": times}
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
        sharded_greedy(hs, red, nodes, pods.slice(0, min(pods.n_pods, 4096)), flags)  # warm-up
        dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        st = {}
        picks = sharded_greedy(hs, red, nodes, pods, flags, stats=st)
        torch.cuda.synchronize(device)
        dt = time.perf_counter() - t0
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        extra = {"windows": st["windows"], "exact_fallback_pods": st["exact_pods"]}
        if args.check and rank == 0:
            full = Yoda(dev_index)
            full.upload_nodes(nodes)
            if not np.array_equal(full.greedy(pods, MODE_SCV, flags), picks):
                raise SystemExit("--check: sharded greedy picks differ from the single handle")
            full.close()
            extra["check"] = "sharded greedy picks == single-handle yoda_greedy"
    out = {"metric": "greedy batch: pods assigned/s (config 5, exact vs the sequential oracle)",
           "value": pods.n_pods / dt, "unit": "pods/s", "n_gpus": world, "seconds": dt,
           "higher_is_better": True, "data": "synthetic (yoda_amd/synth.py config 5)",
           "config": {"workload": f"config5: {pods.n_pods} pods x {nodes.n_nodes} nodes greedy",
                      "pods": pods.n_pods, "nodes": nodes.n_nodes, "path": y.path,
                      "parallelism": f"node-shard x{world}" + (" (RCCL window merges)"
                                                               if world > 1 else "")},
           "pairs_per_s_equiv": pods.n_pods * nodes.n_nodes / dt,
           "assigned": int((picks >= 0).sum())}
    out.update(extra)
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
        probe = min(pods.n_pods, 16)
        t0 = time.perf_counter()
        oracle.greedy(nodes, pods.take(order[:probe]), MODE_SCV, flags)
        per_pod = max((time.perf_counter() - t0) / probe, 1e-9)
        n = int(max(probe, min(pods.n_pods, args.cpu_seconds / per_pod)))
        prefix = pods.take(order[:n])
        t0 = time.perf_counter()
        want, _ = oracle.greedy(nodes, prefix, MODE_SCV, flags)
        cdt = time.perf_counter() - t0
        got = y.greedy(prefix, MODE_SCV, flags)
        out["cpu_baseline"] = {"value": n / cdt, "unit": "pods/s", "cores": 1, "kind": "port",
                               "sample": f"first {n} pods in queue order, sequential oracle "
                                         f"(yoda_oracle.c oracle_greedy), {cdt:.1f} s",
                               "sample_picks_match_gpu": bool(np.array_equal(got, want))}
    print(json.dumps(out), flush=True)
    y.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--pods", type=int, default=None)
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--mode", choices=["scv", "diskio"], default="scv")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", action="store_true",
                    help="N>1: rank 0 re-evaluates the batch on one unsharded handle and "
                         "asserts identical picks / statuses / ties (rehearsal)")
    ap.add_argument("--shard", choices=["nodes", "pods"], default="nodes",
                    help="--gpus N > 1: nodes = node blocks merged by RCCL all-reduces "
                         "(yoda_amd/dist.py); pods = each rank evaluates a pod slice against "
                         "the whole node snapshot, no collective (dist.pod_partition; slower "
                         "per rank on one MI355X, profiles/r01/current/shard_timing.txt)")
    ap.add_argument("--no-balance", action="store_true",
                    help="--shard nodes: keep equal node blocks (default: re-cut them once "
                         "after warm-up so every rank's measured K1 + K2 time is equal)")
    ap.add_argument("--workload", choices=["eval", "greedy"], default="eval",
                    help="eval: the headline batch (config 3); greedy: config 5 sequential assume")
    args = ap.parse_args()
    if args.workload == "greedy":
        return bench_greedy(args)
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

    if world > 1 and not pod_shard:
        ex = ShardExchange.distributed(y, device, shard=shard, offset=lo)
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
            ex = ShardExchange.distributed(y, device, shard=shard, offset=lo)
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
        t0 = time.perf_counter()
        res = y.eval(pods, mode)
        e2e_ms = (time.perf_counter() - t0) * 1e3
    else:
        res = y.download()

    ms_per_step = elapsed / args.steps * 1e3
    value = P * N / (elapsed / args.steps)
    n_local = hi - lo
    # dominant kernel of this rank: K2 (score) unless K1 takes longer
    k1_avg = k1_ms / max(launches, 1)
    k2_avg = k2_ms / max(launches, 1)
    names = kernel_names(y.path, mode)
    dom, dom_ms = (names[1], k2_avg) if k2_avg >= k1_avg else (names[0], k1_avg)
    p_local = my_pods.n_pods
    algo_bytes = p_local * n_local * bytes_per_pair(k_slots, mode)
    achieved = algo_bytes / (dom_ms / 1e3) / 1e9 if dom_ms > 0 else 0.0
    pmc = committed_pmc(dom, P, N, world)

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
                                   f"node-shard x{world}" + (" (RCCL all-reduce merge)"
                                                            if world > 1 else "")),
                   "node_bounds": [int(v) for v in b] if world > 1 and not pod_shard
                   else None},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": pmc.get("hbm_bytes_per_launch"),
                     "avg_launch_ms": dom_ms, "k1_avg_ms": k1_avg, "k2_avg_ms": k2_avg,
                     "bytes_per_pair": bytes_per_pair(k_slots, mode),
                     "pairs_per_launch": p_local * n_local,
                     # achieved > peak: a node record is consulted once per 64-pod wave,
                     # not once per pair; the binding limits are these:
                     "traffic_gbs": (pmc["hbm_bytes_per_launch"] / (dom_ms / 1e3) / 1e9
                                     if pmc.get("hbm_bytes_per_launch") and dom_ms > 0
                                     else None),
                     "issue": {k: pmc[k] for k in ("valu_issue_util", "salu_issue_util",
                                                   "wave_frac_waitcnt",
                                                   "wave_frac_issue_stall",
                                                   "wave_frac_issuing") if k in pmc},
                     "pmc_source": pmc.get("_source")},
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
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(nodes, pods, mode, args.cpu_seconds,
                                           args.cpu_threads, res)
    if rank == 0:
        print(json.dumps(out), flush=True)
    y.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
