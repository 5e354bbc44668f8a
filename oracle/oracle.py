"""ctypes wrapper of the C oracle (oracle/build/libyoda_oracle.so) + SoA <-> pyoracle glue.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker / CPU baseline.  Never by the product package.
Parity unpinned by reference fixtures (none exist); see yoda_oracle.c.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
sys.path.insert(0, os.path.join(_REPO, "kubernetes-scheduler_amd"))
sys.path.insert(0, _HERE)

from yoda_amd.soa import CEvalOut, CNodeSoA, CPodSoA, EvalResult, NodeSoA, PodSoA  # noqa: E402
import pyoracle  # noqa: E402

LIB_PATH = os.path.join(_HERE, "build", "libyoda_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_schedule.argtypes = [C.POINTER(CNodeSoA), C.POINTER(CPodSoA), C.c_int, C.c_int,
                                      C.POINTER(CEvalOut)]
        L.oracle_schedule_range.argtypes = [C.POINTER(CNodeSoA), C.POINTER(CPodSoA), C.c_int,
                                            C.c_uint32, C.c_uint32, C.c_int, C.POINTER(CEvalOut)]
        L.oracle_schedule_memo.argtypes = [C.POINTER(CNodeSoA), C.POINTER(CPodSoA), C.c_uint32,
                                           C.c_int, C.POINTER(CEvalOut)]
        L.oracle_pod_detail.argtypes = [C.POINTER(CNodeSoA), C.POINTER(CPodSoA), C.c_uint32,
                                        C.c_int, C.POINTER(C.c_uint8), C.POINTER(C.c_int64),
                                        C.POINTER(C.c_int64)]
        L.oracle_greedy.argtypes = [C.POINTER(CNodeSoA), C.POINTER(CPodSoA), C.c_int, C.c_uint32,
                                    C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.oracle_queue_order.argtypes = [C.POINTER(CPodSoA), C.POINTER(C.c_uint32)]
        L.oracle_greedy_mt.argtypes = [C.POINTER(CNodeSoA), C.POINTER(CPodSoA), C.c_uint32,
                                       C.c_uint32, C.c_uint32, C.c_int, C.POINTER(C.c_int32),
                                       C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                       C.POINTER(C.c_uint32)]
        _lib = L
    return _lib


def schedule(nodes: NodeSoA, pods: PodSoA, mode: int = 0, threads: int = 1,
             p0: int = 0, p1: int | None = None) -> EvalResult:
    """Independent per-pod cycles for pods [p0, p1) (results for other pods left empty)."""
    nodes, pods = nodes.normalized(), pods.normalized()
    p1 = pods.n_pods if p1 is None else p1
    res = EvalResult.empty(pods.n_pods)
    cn, cp, co = nodes.c(), pods.c(), res.c()
    rc = lib().oracle_schedule_range(C.byref(cn), C.byref(cp), mode, p0, p1, threads, C.byref(co))
    if rc != 0:
        raise RuntimeError(f"oracle_schedule rc={rc}")
    return res


def schedule_memo(nodes: NodeSoA, pods: PodSoA, first: int, threads: int = 1) -> EvalResult:
    """Mode B with the B3 Redis memo quirk, node `first` scored first in every cycle
    (documentation mode: SURVEY §8a B3; the product path computes the uncached B1)."""
    nodes, pods = nodes.normalized(), pods.normalized()
    res = EvalResult.empty(pods.n_pods)
    cn, cp, co = nodes.c(), pods.c(), res.c()
    rc = lib().oracle_schedule_memo(C.byref(cn), C.byref(cp), first, threads, C.byref(co))
    if rc != 0:
        raise RuntimeError(f"oracle_schedule_memo rc={rc}")
    return res


def pod_detail(nodes: NodeSoA, pods: PodSoA, p: int, mode: int = 0):
    nodes, pods = nodes.normalized(), pods.normalized()
    n = nodes.n_nodes
    feas = np.zeros(n, np.uint8)
    raw = np.zeros(n, np.int64)
    norm = np.zeros(n, np.int64)
    cn, cp = nodes.c(), pods.c()
    rc = lib().oracle_pod_detail(C.byref(cn), C.byref(cp), p, mode,
                                 feas.ctypes.data_as(C.POINTER(C.c_uint8)),
                                 raw.ctypes.data_as(C.POINTER(C.c_int64)),
                                 norm.ctypes.data_as(C.POINTER(C.c_int64)))
    return rc, feas.astype(bool), raw, norm


def greedy(nodes: NodeSoA, pods: PodSoA, mode: int = 0, flags: int = 0):
    nodes, pods = nodes.normalized(), pods.normalized()
    pick = np.full(pods.n_pods, -3, np.int32)
    status = np.full(pods.n_pods, -1, np.int32)
    cn, cp = nodes.c(), pods.c()
    rc = lib().oracle_greedy(C.byref(cn), C.byref(cp), mode, flags,
                             pick.ctypes.data_as(C.POINTER(C.c_int32)),
                             status.ctypes.data_as(C.POINTER(C.c_int32)))
    if rc != 0:
        raise RuntimeError(f"oracle_greedy rc={rc}")
    return pick, status


def greedy_mt(nodes: NodeSoA, pods: PodSoA, flags: int = 0, q0: int = 0, q1: int | None = None,
              threads: int = 8):
    """Mode-A greedy with node-parallel cycles (oracle_greedy_mt): queue positions [q0, q1)
    from the node state given.  Returns (pick, status, top_score, n_ties) over all pods
    (pods outside the range keep pick -3)."""
    nodes, pods = nodes.normalized(), pods.normalized()
    P = pods.n_pods
    q1 = P if q1 is None else q1
    pick = np.full(P, -3, np.int32)
    status = np.full(P, -1, np.int32)
    top = np.zeros(P, np.int64)
    ties = np.zeros(P, np.uint32)
    cn, cp = nodes.c(), pods.c()
    rc = lib().oracle_greedy_mt(C.byref(cn), C.byref(cp), flags, q0, q1, threads,
                                pick.ctypes.data_as(C.POINTER(C.c_int32)),
                                status.ctypes.data_as(C.POINTER(C.c_int32)),
                                top.ctypes.data_as(C.POINTER(C.c_int64)),
                                ties.ctypes.data_as(C.POINTER(C.c_uint32)))
    if rc != 0:
        raise RuntimeError(f"oracle_greedy_mt rc={rc}")
    return pick, status, top, ties


def queue_order(pods: PodSoA) -> np.ndarray:
    pods = pods.normalized()
    order = np.zeros(pods.n_pods, np.uint32)
    cp = pods.c()
    lib().oracle_queue_order(C.byref(cp), order.ctypes.data_as(C.POINTER(C.c_uint32)))
    return order


# ---- SoA <-> pyoracle objects -------------------------------------------------------------
def to_py(nodes: NodeSoA, pods: PodSoA):
    nodes, pods = nodes.normalized(), pods.normalized()
    scvs = []
    for i in range(nodes.n_nodes):
        cards = []
        for j in range(int(nodes.card_count[i])):
            cards.append(pyoracle.Card(
                free_memory=int(nodes.card_free_memory[i, j]),
                total_memory=int(nodes.card_total_memory[i, j]),
                clock=int(nodes.card_clock[i, j]), bandwidth=int(nodes.card_bandwidth[i, j]),
                core=int(nodes.card_core[i, j]), power=int(nodes.card_power[i, j]),
                health="Healthy" if nodes.card_healthy[i, j] else "Unhealthy"))
        scvs.append(pyoracle.Scv(card_number=int(nodes.card_number[i]), card_list=cards,
                                 free_memory_sum=int(nodes.free_memory_sum[i]),
                                 total_memory_sum=int(nodes.total_memory_sum[i]),
                                 alloc_memory=int(nodes.alloc_memory[i]),
                                 cpu=float(nodes.cpu[i]), disk_io=float(nodes.disk_io[i])))
    plist = []
    for p in range(pods.n_pods):
        plist.append(pyoracle.Pod(
            number=int(pods.number[p]) if pods.has_number[p] else None,
            memory=int(pods.memory[p]) if pods.has_memory[p] else None,
            clock=int(pods.clock[p]) if pods.has_clock[p] else None,
            priority=int(pods.priority[p]), rio=float(pods.rio[p]), rcpu=int(pods.rcpu[p])))
    return scvs, plist


def from_py(scvs, plist, max_cards: int | None = None):
    """pyoracle objects -> (NodeSoA, PodSoA)."""
    n = len(scvs)
    k = max_cards or max([len(s.card_list) for s in scvs] + [1])
    z = lambda dt: np.zeros((n, k), dt)  # noqa: E731
    f, t, ck, bw, co, pw, h = (z(np.uint64), z(np.uint64), z(np.uint64), z(np.uint64),
                               z(np.uint64), z(np.uint64), z(np.uint8))
    for i, s in enumerate(scvs):
        for j, c in enumerate(s.card_list):
            f[i, j], t[i, j], ck[i, j] = c.free_memory, c.total_memory, c.clock
            bw[i, j], co[i, j], pw[i, j] = c.bandwidth, c.core, c.power
            h[i, j] = c.health == "Healthy"
    nodes = NodeSoA(
        card_number=np.array([s.card_number for s in scvs], np.uint64),
        card_count=np.array([len(s.card_list) for s in scvs], np.uint32),
        free_memory_sum=np.array([s.free_memory_sum for s in scvs], np.uint64),
        total_memory_sum=np.array([s.total_memory_sum for s in scvs], np.uint64),
        alloc_memory=np.array([s.alloc_memory for s in scvs], np.uint64),
        card_free_memory=f, card_total_memory=t, card_clock=ck, card_bandwidth=bw,
        card_core=co, card_power=pw, card_healthy=h,
        cpu=np.array([s.cpu for s in scvs], np.float64),
        disk_io=np.array([s.disk_io for s in scvs], np.float64)).normalized()
    pods = PodSoA(
        has_number=np.array([p.number is not None for p in plist], np.uint8),
        number=np.array([p.number or 0 for p in plist], np.uint64),
        has_memory=np.array([p.memory is not None for p in plist], np.uint8),
        memory=np.array([p.memory or 0 for p in plist], np.uint64),
        has_clock=np.array([p.clock is not None for p in plist], np.uint8),
        clock=np.array([p.clock or 0 for p in plist], np.uint64),
        priority=np.array([p.priority for p in plist], np.int64),
        rio=np.array([p.rio for p in plist], np.float64),
        rcpu=np.array([p.rcpu for p in plist], np.int64)).normalized()
    return nodes, pods
