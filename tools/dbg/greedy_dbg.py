import sys, os
sys.path[:0] = ["kubernetes-scheduler_amd", "oracle", "tests"]
import numpy as np
import oracle
from yoda_amd import synth
from yoda_amd.capi import Yoda
from yoda_amd.soa import MODE_SCV
nodes, pods = synth.make_config(5, pods=400, nodes=300)
pods.priority[:] = 0
pods.memory[:] = 1
pods.has_memory[:] = 1
y = Yoda(0)
want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
for k1, k2 in ((False, False), (True, False), (False, True), (True, True)):
    for order in (True, False):
        y.set_pod_order(order)
        y.upload_nodes(nodes, per_node_k1=k1, per_node_k2=k2)
        got = y.eval(pods, MODE_SCV)
        bad = {f: int((getattr(got, f) != getattr(want, f)).sum()) for f in ("pick", "status", "n_feasible", "top_score", "n_ties")}
        badm = int((got.maxima != want.maxima).any(axis=1).sum())
        print("k1pn", k1, "k2pn", k2, "order", order, bad, "maxima", badm, flush=True)
        if bad["pick"]:
            i = np.nonzero(got.pick != want.pick)[0][:5]
            print("  pods", i, "got", got.pick[i], got.top_score[i], "want", want.pick[i], want.top_score[i])
y.set_pod_order(True)
y.upload_nodes(nodes)
g = y.greedy(pods, MODE_SCV)
w = oracle.greedy(nodes, pods)[0]
i = np.nonzero(g != w)[0]
print("greedy mismatches", len(i), i[:10], g[i[:10]], w[i[:10]], y.greedy_stats(times=True))
print("--- as in the test: Mode B greedy first")
nodes, pods = synth.make_config(5, pods=400, nodes=300)
pods.priority[:] = 0
y.upload_nodes(nodes)
from yoda_amd.soa import MODE_DISKIO
gb = y.greedy(pods, MODE_DISKIO)
print("modeB mismatches", int((gb != oracle.greedy(nodes, pods, MODE_DISKIO)[0]).sum()))
pods.memory[:] = 1
pods.has_memory[:] = 1
g = y.greedy(pods, MODE_SCV)
w = oracle.greedy(nodes, pods)[0]
i = np.nonzero(g != w)[0]
print("greedy mismatches", len(i), i[:10], g[i[:10]], w[i[:10]], y.greedy_stats(times=True))
y.upload_pods(pods)
y.run(MODE_SCV)
got = y.download()
want = oracle.schedule(nodes, pods, MODE_SCV, threads=8)
print({f: int((getattr(got, f) != getattr(want, f)).sum()) for f in ("pick", "status", "n_feasible", "top_score", "n_ties")})
