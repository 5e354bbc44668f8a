"""The reference's scheduler-framework plugin surface, backed by libyoda.

Mirrors pkg/yoda/scheduler.go (and sort.go) method for method — same names, argument
meaning and Status codes — so a caller of the reference plugin finds the same contract:

  PreFilter  scheduler.go:91-94    packs the pod, ONE libyoda call for the whole row
                                   (yoda_score_rows: Filter bits + raw Score of every node),
                                   kept in CycleState
  Filter     scheduler.go:96-99    lookup (the SCV predicates, filter.go:11-58)
  PreScore   scheduler.go:101-114  no-op: the inputs are the uploaded snapshot (the reference
                                   flushes Redis and queries Prometheus here — out of scope)
  Score      scheduler.go:116-156  lookup of the row (Uint64ToInt64 already applied)
  NormalizeScore scheduler.go:158-183  the reference algorithm, int64 wrap-around included
  PreBind    scheduler.go:189-196  node must exist in the snapshot
  Less       sort.go:8-10          scv/priority descending

`schedule_one` runs one kube-scheduler v1.22.3 cycle over these methods (Filter all nodes,
the single-feasible-node shortcut, PreScore, Score, NormalizeScore, range check, selectHost).
The Go drop-in has the same structure over cgo.
"""
from __future__ import annotations

import random
from dataclasses import dataclass
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np

from .pack import pack_pods
from .soa import MODE_SCV, NodeSoA

NAME = "yoda"
MAX_NODE_SCORE = 100
MIN_NODE_SCORE = 0

# k8s framework Code values
SUCCESS, ERROR, UNSCHEDULABLE = 0, 1, 2


@dataclass
class Status:
    code: int = SUCCESS
    message: str = ""

    def is_success(self) -> bool:
        return self.code == SUCCESS


class CycleState(dict):
    """framework.CycleState: per-pod scheduling-cycle storage."""

    def write(self, key, value):
        self[key] = value

    def read(self, key):
        if key not in self:
            raise KeyError(f"{key!r} not found in CycleState")
        return self[key]


@dataclass
class NodeScore:
    name: str
    score: int


@dataclass
class _Row:
    feasible: np.ndarray  # bool [N]
    scores: np.ndarray    # int64 [N], -1 where infeasible


def _wrap_i64(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >> 63 else x


def _go_div(a: int, b: int) -> int:
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


class YodaPlugin:
    """PreFilter/Filter/PreScore/Score/NormalizeScore/PreBind + Less, over a libyoda handle
    (or any backend with upload_pods(PodSoA) and score_rows(mode))."""

    def __init__(self, backend, node_names: Sequence[str], nodes: Optional[NodeSoA] = None,
                 mode: int = MODE_SCV):
        self.backend = backend
        self.node_names = list(node_names)
        self.index = {n: i for i, n in enumerate(self.node_names)}
        self.mode = mode
        # Mode A Score divides by TotalMemorySum (algorithm.go:294,309): Go panics on 0
        self.zero_total = (np.asarray(nodes.total_memory_sum) == 0) if nodes is not None \
            else np.zeros(len(self.node_names), bool)

    def name(self) -> str:
        return NAME

    # ---- extension points ---------------------------------------------------------------
    def pre_filter(self, state: CycleState, pod: Mapping) -> Status:
        self.backend.upload_pods(pack_pods([pod]))
        feas, scores = self.backend.score_rows(self.mode)
        state.write(NAME + "/row", _Row(feas[0], scores[0]))
        return Status()

    def filter(self, state: CycleState, pod: Mapping, node_name: str) -> Status:
        row: _Row = state.read(NAME + "/row")
        if row.feasible[self.index[node_name]]:
            return Status()
        return Status(UNSCHEDULABLE, "node(s) didn't match the scv card requirements")

    def pre_score(self, state: CycleState, pod: Mapping, nodes: Sequence[str]) -> Status:
        return Status()

    def score(self, state: CycleState, pod: Mapping, node_name: str) -> Tuple[int, Status]:
        try:
            row: _Row = state.read(NAME + "/row")
        except KeyError as e:
            return 0, Status(ERROR, str(e))
        i = self.index[node_name]
        if self.mode == MODE_SCV and self.zero_total[i]:
            return 0, Status(ERROR, "runtime error: integer divide by zero")
        return int(row.scores[i]), Status()

    def score_extensions(self):
        return self

    def normalize_score(self, state: CycleState, pod: Mapping,
                        scores: List[NodeScore]) -> Status:
        """scheduler.go:158-183 verbatim (int64 arithmetic with Go wrap-around)."""
        highest, lowest = 0, scores[0].score
        for ns in scores:
            lowest = min(lowest, ns.score)
            highest = max(highest, ns.score)
        if highest == lowest:
            lowest -= 1
        for ns in scores:
            ns.score = _go_div(_wrap_i64((ns.score - lowest) * MAX_NODE_SCORE), highest - lowest)
        return Status()

    def pre_bind(self, state: CycleState, pod: Mapping, node_name: str) -> Status:
        if node_name not in self.index:
            return Status(ERROR, f"prebind get node info error: {node_name}")
        return Status()

    @staticmethod
    def less(pod_info1: Mapping, pod_info2: Mapping) -> bool:
        """sort.Less (sort.go:8-10)."""
        from .gostrconv import pod_priority

        def prio(p):
            labels = (p.get("metadata", {}) or {}).get("labels", {}) or {}
            return pod_priority(str(labels["scv/priority"])) if "scv/priority" in labels else 0
        return prio(pod_info1) > prio(pod_info2)


def select_host(scores: Sequence[NodeScore], rng: Optional[random.Random] = None) -> str:
    """k8s v1.22.3 selectHost: reservoir-sampled tie-break with rng; with rng=None the
    lowest-index member of the tie set (the build's deterministic rule)."""
    best = scores[0].score
    selected = scores[0].name
    cnt = 1
    for ns in scores[1:]:
        if ns.score > best:
            best, selected, cnt = ns.score, ns.name, 1
        elif ns.score == best:
            cnt += 1
            if rng is not None and rng.randrange(cnt) == 0:
                selected = ns.name
    return selected


def schedule_one(plugin: YodaPlugin, pod: Mapping, rng: Optional[random.Random] = None,
                 weight: int = 1) -> Tuple[Optional[str], Status]:
    """One scheduling cycle with yoda as the only Filter/Score plugin
    (percentageOfNodesToScore 100).  Returns (node name or None, status)."""
    state = CycleState()
    st = plugin.pre_filter(state, pod)
    if not st.is_success():
        return None, st
    feasible = [n for n in plugin.node_names if plugin.filter(state, pod, n).is_success()]
    if not feasible:
        return None, Status(UNSCHEDULABLE, "0 nodes are available")
    if len(feasible) == 1:
        return feasible[0], Status()
    st = plugin.pre_score(state, pod, feasible)
    if not st.is_success():
        return None, st
    scores = []
    for n in feasible:
        s, st = plugin.score(state, pod, n)
        if not st.is_success():
            return None, st
        scores.append(NodeScore(n, s))
    plugin.score_extensions().normalize_score(state, pod, scores)
    for ns in scores:
        if ns.score > MAX_NODE_SCORE or ns.score < MIN_NODE_SCORE:
            return None, Status(ERROR, f"plugin yoda returns an invalid score {ns.score}")
        ns.score *= weight
    return select_host(scores, rng), Status()
