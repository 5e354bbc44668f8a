#!/usr/bin/env python3
"""Full-size parity fixtures: per-block digests of the C oracle's outputs on BASELINE configs
3 and 5 at their declared sizes, and on every variant workload bench.py reports
(tests/golden/fullsize.json).

    python tests/golden/make_fullsize.py [config3] [variant_<name> ...] [config5_0] [config5_1]
                                         [--threads T]

* config 3 (100k pods x 100k nodes, seed 7): every pod is an independent cycle
  (scheduler.go:158-183 then selectHost) -> oracle_schedule over all 100k pods; one digest
  per 1,024 pods (input order) over (pick, status, n_feasible, n_ties, top_score, maxima) --
  n_ties and top_score where the status is 0, the six CollectMaxValues maxima
  (collection.go:30-76) of every pod.
* variant_<name> (synth.VARIANTS: mixed50, bytes, bw1000, het100k, diskio, diskio_distinct):
  the same per-1,024-pod digests of the oracle over every pod of the variant workload, built
  by synth.variant_workloads exactly as bench.py's `extra.variants` builds it.  Mode B
  (BalancedCpuDiskIOPriority, algorithm.go:99-119) has no maxima, so its digests omit them.
* config 5 (1M pods x 100k nodes, seed 13, both greedy flags): the sequential greedy in
  sort.go:8-10 queue order with the algorithm.go:299-303 assume (and the CardNumber
  decrement under YODA_GREEDY_CARD_CAPACITY) -> oracle_greedy_mt (node-parallel cycles,
  the same decisions as oracle_greedy); one digest per 6,144-pod queue window over the picks.
  Runs in segments of queue positions with the node state carried between them, and keeps a
  resumable checkpoint under tests/golden/_full/ (not committed; ~1 h per flag on 8 cores).

A digest is the first 16 hex digits of SHA-256 over the block's arrays, each little-endian
in a fixed dtype, concatenated in the order listed.  The fixture also records a digest of
the generated inputs, so a GPU-side mismatch caused by generator drift (another numpy) is told
apart from a kernel mismatch.

The expected outputs are the oracle's (a restatement of the Go text): the reference itself
holds no vectors and cannot run here ("parity unpinned").
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "kubernetes-scheduler_amd"), os.path.join(REPO, "oracle")]

from yoda_amd import synth  # noqa: E402

OUT = os.path.join(HERE, "fullsize.json")
CACHE = os.path.join(HERE, "_full")
C3_BLOCK = 1024
C5_WINDOW = 6144
C5_SEGMENT = 8 * C5_WINDOW


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes())
    return h.hexdigest()[:16]


def input_digest(nodes, pods, mode_b: bool = False) -> str:
    """Digest of the generated snapshot and batch (every SoA field the path reads; with
    mode_b also the Mode-B node metrics and pod requests)."""
    nodes, pods = nodes.normalized(), pods.normalized()
    nf = [nodes.card_number, nodes.card_count, nodes.free_memory_sum, nodes.total_memory_sum,
          nodes.alloc_memory, nodes.card_free_memory, nodes.card_total_memory, nodes.card_clock,
          nodes.card_bandwidth, nodes.card_core, nodes.card_power, nodes.card_healthy]
    pf = [pods.has_number, pods.number, pods.has_memory, pods.memory, pods.has_clock,
          pods.clock, pods.priority]
    if mode_b:
        nf += [nodes.cpu, nodes.disk_io]
        pf += [pods.rio, pods.rcpu]
    return digest(*[np.asarray(a) for a in nf + pf])


def eval_digests(res, block=C3_BLOCK, mode: int = 0):
    """One digest per `block` pods (input order) of an evaluation batch's outputs: pick,
    status, n_feasible, n_ties and top_score (zero where the status is not 0: no pick, so no
    score), and in Mode A the six maxima."""
    P = len(res.pick)
    ok = np.asarray(res.status) == 0
    ties = np.where(ok, res.n_ties, 0).astype(np.uint32)
    top = np.where(ok, res.top_score, 0).astype(np.int64)
    out = []
    for b in range(0, P, block):
        s = slice(b, min(P, b + block))
        arrays = [res.pick[s].astype(np.int32), res.status[s].astype(np.int32),
                  res.n_feasible[s].astype(np.uint32), ties[s], top[s]]
        if mode == 0:
            arrays.append(np.asarray(res.maxima[s], np.uint64))
        out.append(digest(*arrays))
    return out


config3_digests = eval_digests
FIELDS_A = ("pick i32, status i32, n_feasible u32, n_ties u32 and top_score i64 (0 unless "
            "status 0), maxima u64[6] (input order)")
FIELDS_B = "pick i32, status i32, n_feasible u32, n_ties u32 and top_score i64 (0 unless status 0)"
# the variant workloads bench.py reports (synth.VARIANTS) whose outputs differ from config 3's
# (f64 / u64 / per-pair kernels compute config 3 itself and are checked against "config3")
VARIANTS = ("mixed50", "bytes", "bw1000", "het100k", "diskio", "diskio_distinct")


def greedy_window_digests(pick, order, window=C5_WINDOW):
    pq = np.asarray(pick, np.int32)[order]
    return [digest(pq[w:w + window]) for w in range(0, len(pq), window)]


def apply_assumes(alloc, cardn, pods, idx_pods, picks, flags):
    """The assume of each placed pod (algorithm.go:299-303; CardNumber -= number, saturating,
    under the capacity flag), in queue order."""
    ok = picks >= 0
    p, n = idx_pods[ok], picks[ok].astype(np.int64)
    mem = np.where(pods.has_memory[p] == 1, pods.memory[p], 0).astype(np.uint64)
    np.add.at(alloc, n, mem)  # uint64 wrap, like Go
    if flags & 1:
        num = np.where(pods.has_number[p] == 1, pods.number[p], 1).astype(np.uint64)
        for node, k in zip(n, num):  # sequential: saturation depends on order
            cardn[node] = cardn[node] - k if cardn[node] >= k else np.uint64(0)


def run_config3(threads):
    import oracle
    nodes, pods = synth.make_config(3)
    t = time.time()
    res = oracle.schedule(nodes, pods, 0, threads=threads)
    print(f"config3: oracle {time.time() - t:.0f} s", flush=True)
    os.makedirs(CACHE, exist_ok=True)
    np.savez(os.path.join(CACHE, "config3.npz"), pick=res.pick, status=res.status,
             n_feasible=res.n_feasible, n_ties=res.n_ties, top_score=res.top_score,
             maxima=res.maxima)
    return {"inputs": input_digest(nodes, pods), "pods": pods.n_pods, "nodes": nodes.n_nodes,
            "mode": 0, "block": C3_BLOCK, "fields": FIELDS_A, "digests": eval_digests(res)}


def variant_inputs(name):
    """(nodes, pods, mode) of a bench variant, exactly as bench.py builds it."""
    ((_, nodes, pods, mode, _kw),) = synth.variant_workloads([name])
    return nodes, pods, mode


def run_variant(name, threads):
    import oracle
    nodes, pods, mode = variant_inputs(name)
    t = time.time()
    res = oracle.schedule(nodes, pods, mode, threads=threads)
    print(f"variant {name}: oracle {time.time() - t:.0f} s", flush=True)
    return {"inputs": input_digest(nodes, pods, mode_b=mode == 1), "pods": pods.n_pods,
            "nodes": nodes.n_nodes, "mode": mode, "block": C3_BLOCK,
            "desc": synth.VARIANTS[name], "fields": FIELDS_A if mode == 0 else FIELDS_B,
            "feasible_pairs": int(res.n_feasible.astype(np.int64).sum()),
            "digests": eval_digests(res, C3_BLOCK, mode)}


def run_config5(flags, threads):
    import oracle
    nodes, pods = synth.make_config(5)
    P = pods.n_pods
    order = oracle.queue_order(pods)
    os.makedirs(CACHE, exist_ok=True)
    ck = os.path.join(CACHE, f"config5_{flags}.npz")
    pick = np.full(P, -3, np.int32)
    top = np.zeros(P, np.int64)
    ties = np.zeros(P, np.uint32)
    alloc = np.array(nodes.alloc_memory, np.uint64)
    cardn = np.array(nodes.card_number, np.uint64)
    q = 0
    if os.path.exists(ck):
        z = np.load(ck)
        pick, top, ties, alloc, cardn, q = (z["pick"], z["top"], z["ties"], z["alloc"],
                                             z["cardn"], int(z["q"]))
        print(f"config5 flags {flags}: resuming at queue position {q}", flush=True)
    t0 = time.time()
    while q < P:
        q1 = min(P, q + C5_SEGMENT)
        snap = nodes.slice(0, nodes.n_nodes)
        snap.alloc_memory = alloc.copy()
        snap.card_number = cardn.copy()
        pk, _, tp, ti = oracle.greedy_mt(snap, pods, flags, q, q1, threads=threads)
        seg = order[q:q1]
        pick[seg], top[seg], ties[seg] = pk[seg], tp[seg], ti[seg]
        apply_assumes(alloc, cardn, pods, seg, pk[seg], flags)
        q = q1
        np.savez(ck + ".tmp.npz", pick=pick, top=top, ties=ties, alloc=alloc, cardn=cardn, q=q)
        os.replace(ck + ".tmp.npz", ck)
        el = time.time() - t0
        print(f"config5 flags {flags}: {q}/{P} queue positions, {el:.0f} s", flush=True)
    return {"inputs": input_digest(nodes, pods), "pods": P, "nodes": nodes.n_nodes,
            "flags": flags, "window": C5_WINDOW,
            "fields": "pick i32 over 6144 queue positions (sort.go:8-10 order)",
            "placed": int((pick >= 0).sum()),
            "digests": greedy_window_digests(pick, order)}


def main(argv):
    threads = 8
    if "--threads" in argv:
        threads = int(argv[argv.index("--threads") + 1])
    which = [a for a in argv if not a.startswith("--") and not a.isdigit()] or \
        ["config3"] + [f"variant_{v}" for v in VARIANTS] + ["config5_0", "config5_1"]
    fx = json.load(open(OUT)) if os.path.exists(OUT) else {}
    fx["_about"] = ("C-oracle digests at BASELINE configs 3 and 5 and the bench's variant "
                    "workloads, full size (tests/golden/make_fullsize.py). Parity unpinned by "
                    "reference vectors.")
    for w in which:
        if w == "config3":
            fx["config3"] = run_config3(threads)
        elif w.startswith("variant_"):
            fx[w] = run_variant(w[len("variant_"):], threads)
        elif w.startswith("config5_"):
            fx[w] = run_config5(int(w[-1]), threads)
        else:
            raise SystemExit(f"unknown fixture {w}")
        with open(OUT, "w") as f:
            json.dump(fx, f, indent=1, sort_keys=True)
            f.write("\n")
        print("wrote", OUT, w, flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
