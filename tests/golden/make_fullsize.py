#!/usr/bin/env python3
"""Full-size parity fixtures: per-block digests of the C oracle's outputs on BASELINE configs
3 and 5 at their declared sizes (tests/golden/fullsize.json).

    python tests/golden/make_fullsize.py [config3] [config5_0] [config5_1] [--threads T]

* config 3 (100k pods x 100k nodes, seed 7): every pod is an independent cycle
  (scheduler.go:158-183 then selectHost) -> oracle_schedule over all 100k pods; one digest
  per 1,024 pods (input order) over (pick, status, n_feasible, n_ties, top_score).
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


def input_digest(nodes, pods) -> str:
    """Digest of the generated snapshot and batch (every SoA field the path reads)."""
    nodes, pods = nodes.normalized(), pods.normalized()
    nf = [nodes.card_number, nodes.card_count, nodes.free_memory_sum, nodes.total_memory_sum,
          nodes.alloc_memory, nodes.card_free_memory, nodes.card_total_memory, nodes.card_clock,
          nodes.card_bandwidth, nodes.card_core, nodes.card_power, nodes.card_healthy]
    pf = [pods.has_number, pods.number, pods.has_memory, pods.memory, pods.has_clock,
          pods.clock, pods.priority]
    return digest(*[np.asarray(a) for a in nf + pf])


def config3_digests(res, block=C3_BLOCK):
    P = len(res.pick)
    out = []
    for b in range(0, P, block):
        s = slice(b, min(P, b + block))
        out.append(digest(res.pick[s].astype(np.int32), res.status[s].astype(np.int32),
                          res.n_feasible[s].astype(np.uint32), res.n_ties[s].astype(np.uint32),
                          res.top_score[s].astype(np.int64)))
    return out


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
             n_feasible=res.n_feasible, n_ties=res.n_ties, top_score=res.top_score)
    return {"inputs": input_digest(nodes, pods), "pods": pods.n_pods, "nodes": nodes.n_nodes,
            "block": C3_BLOCK, "fields": "pick i32, status i32, n_feasible u32, n_ties u32, "
            "top_score i64 (input order)", "digests": config3_digests(res)}


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
        ["config3", "config5_0", "config5_1"]
    fx = json.load(open(OUT)) if os.path.exists(OUT) else {}
    fx["_about"] = ("C-oracle digests at BASELINE configs 3 and 5, full size "
                    "(tests/golden/make_fullsize.py). Parity unpinned by reference vectors.")
    for w in which:
        if w == "config3":
            fx["config3"] = run_config3(threads)
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
