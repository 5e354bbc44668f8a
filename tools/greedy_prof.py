#!/usr/bin/env python3
"""One config-5 greedy batch per flag (after a warm-up), for rocprofv3 kernel traces:
    rocprofv3 --kernel-trace --stats -d out -- python3 tools/greedy_prof.py --flags 1"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler_amd"))

from yoda_amd import synth  # noqa: E402
from yoda_amd.capi import Yoda  # noqa: E402
from yoda_amd.soa import MODE_SCV  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--flags", type=int, nargs="+", default=[1])
args = ap.parse_args()
nodes, pods = synth.make_config(5)
y = Yoda(0)
y.upload_nodes(nodes)
for flags in args.flags:
    y.greedy(pods.slice(0, 4096), MODE_SCV, flags)
    t0 = time.perf_counter()
    y.greedy(pods, MODE_SCV, flags)
    w, f, t = y.greedy_stats(times=True)
    print(f"flags {flags}: {time.perf_counter() - t0:.3f} s, windows {w}, fallbacks {f}, {t}",
          flush=True)
y.close()
