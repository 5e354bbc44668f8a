"""Independent pure-Python restatement of the reference Yoda scheduling semantics.

TEST INFRASTRUCTURE ONLY (see oracle/yoda_oracle.c header): used by tests/ to cross-check
the C oracle on small clusters and to generate golden fixtures.  Never imported by the
product package.

PARITY STATUS: parity unpinned by reference fixtures (the reference has none and cannot be
built here: no Go toolchain).  Pinned by the hand-derived known-answer tests of SURVEY.md
§8c (tests/test_oracle.py).

Written from the Go text independently of yoda_oracle.c: objects instead of arrays,
Python ints masked to 64 bits instead of C unsigned arithmetic.
"""
from __future__ import annotations

import math
import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

U64 = (1 << 64) - 1
I64_MAX = (1 << 63) - 1

# pkg/yoda/score/algorithm.go:24-35
BANDWIDTH_WEIGHT = 1
CLOCK_WEIGHT = 1
CORE_WEIGHT = 2
POWER_WEIGHT = 1
FREE_MEMORY_WEIGHT = 3
TOTAL_MEMORY_WEIGHT = 1
ACTUAL_WEIGHT = 2
ALLOCATE_WEIGHT = 3

MAX_NODE_SCORE = 100  # k8s framework.MaxNodeScore

PICK_NONE = -1
PICK_ERROR = -2
STATUS_OK, STATUS_UNSCHEDULABLE, STATUS_DIV_ZERO, STATUS_SCORE_RANGE = 0, 1, 2, 3


@dataclass
class Card:
    """SCV api/v1 Card as used by the reference (filter.go:53,57; collection.go:58-75)."""
    free_memory: int
    total_memory: int
    clock: int
    bandwidth: int
    core: int
    power: int
    health: str = "Healthy"


@dataclass
class Scv:
    """SCV Status fields used by the reference (filter.go:13,22; algorithm.go:294,305-309)."""
    card_number: int
    card_list: List[Card]
    free_memory_sum: int
    total_memory_sum: int
    alloc_memory: int = 0          # Σ scv/memory of pods on the node (algorithm.go:299-303)
    cpu: float = 0.0               # advisor.NodeInfo.Cpu  (Mode B)
    disk_io: float = 0.0           # advisor.NodeInfo.DiskIO (Mode B)


@dataclass
class Pod:
    """Parsed pod labels (already converted with Go strconv semantics)."""
    number: Optional[int] = None   # scv/number  -> strToUint (None = label absent)
    memory: Optional[int] = None   # scv/memory  -> StrToUint64
    clock: Optional[int] = None    # scv/clock   -> strToUint
    priority: int = 0              # scv/priority -> Atoi
    rio: float = 0.0               # ParseFloat(annotations["diskIO"], 32)
    rcpu: int = 0                  # CalculatePodResourceRequest(cpu)


@dataclass
class MaxValue:  # collection.go:14-21
    bandwidth: int = 1
    clock: int = 1
    core: int = 1
    free_memory: int = 1
    power: int = 1
    total_memory: int = 1

    def as_list(self):
        return [self.bandwidth, self.clock, self.core, self.free_memory, self.power,
                self.total_memory]


def pod_fits_number(pod: Pod, s: Scv):  # filter.go:11-16
    if pod.number is not None:
        return pod.number <= s.card_number, pod.number
    return s.card_number > 0, 1


def pod_fits_memory(number: int, pod: Pod, s: Scv):  # filter.go:18-33
    if pod.memory is not None:
        fits = sum(1 for c in s.card_list if c.health == "Healthy" and c.free_memory >= pod.memory)
        return fits >= number, pod.memory
    return True, 0


def pod_fits_clock(number: int, pod: Pod, s: Scv):  # filter.go:35-50
    if pod.clock is not None:
        fits = sum(1 for c in s.card_list if c.health == "Healthy" and c.clock == pod.clock)
        return fits >= number, pod.clock
    return True, 0


def fits(pod: Pod, s: Scv):
    """collection.go:41-44 gating; returns (ok, memory, clock)."""
    ok, number = pod_fits_number(pod, s)
    if not ok:
        return False, 0, 0
    fm, memory = pod_fits_memory(number, pod, s)
    fc, clock = pod_fits_clock(number, pod, s)
    return (fm and fc), memory, clock


def collect_max_values(pod: Pod, scvs: Sequence[Scv]) -> MaxValue:  # collection.go:30-55
    mv = MaxValue()
    for s in scvs:
        ok, memory, clock = fits(pod, s)
        if not ok:
            continue
        for c in s.card_list:
            if c.free_memory >= memory and c.clock >= clock:  # :46 — no health check
                mv.free_memory = max(mv.free_memory, c.free_memory)
                mv.clock = max(mv.clock, c.clock)
                mv.total_memory = max(mv.total_memory, c.total_memory)
                mv.bandwidth = max(mv.bandwidth, c.bandwidth)
                mv.core = max(mv.core, c.core)
                mv.power = max(mv.power, c.power)
    return mv


def card_score(mv: MaxValue, c: Card) -> int:  # algorithm.go:280-291
    bw = ((c.bandwidth * 100) & U64) // mv.bandwidth
    clk = ((c.clock * 100) & U64) // mv.bandwidth  # quirk: divided by MaxBandwidth (:283)
    core = ((c.core * 100) & U64) // mv.core
    pw = ((c.power * 100) & U64) // mv.power
    fm = ((c.free_memory * 100) & U64) // mv.free_memory
    tm = ((c.total_memory * 100) & U64) // mv.total_memory
    first = (bw * BANDWIDTH_WEIGHT + clk * CLOCK_WEIGHT + core * CORE_WEIGHT
             + pw * POWER_WEIGHT) & U64
    return (first + fm * FREE_MEMORY_WEIGHT + tm * TOTAL_MEMORY_WEIGHT) & U64


def basic_score(mv: MaxValue, pod: Pod, s: Scv) -> int:  # algorithm.go:264-278
    ok, memory, clock = fits(pod, s)
    total = 0
    if ok:
        for c in s.card_list:
            if c.free_memory >= memory and c.clock >= clock:
                total = (total + card_score(mv, c)) & U64
    return total


class DivideByZero(Exception):
    """Go integer division by zero: the reference panics."""


def actual_score(s: Scv) -> int:  # algorithm.go:293-295
    if s.total_memory_sum == 0:
        raise DivideByZero()
    return (((s.free_memory_sum * 100) & U64) // s.total_memory_sum * ACTUAL_WEIGHT) & U64


def allocate_score(s: Scv) -> int:  # algorithm.go:297-310
    if s.total_memory_sum < s.alloc_memory:
        return 0
    if s.total_memory_sum == 0:
        raise DivideByZero()
    t = (((s.total_memory_sum - s.alloc_memory) * 100) & U64) // s.total_memory_sum
    return (t * ALLOCATE_WEIGHT) & U64


def uint64_to_int64(u: int) -> int:  # filter.go:84-86
    return 0 if u > I64_MAX else u


def _to_i64(x: int) -> int:
    x &= U64
    return x - (1 << 64) if x >> 63 else x


def _go_div(a: int, b: int) -> int:
    """Go int64 division truncates toward zero."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def _cvttsd2sq(x: float) -> int:
    if math.isnan(x) or x >= 2.0 ** 63 or x < -(2.0 ** 63):
        return -(1 << 63)
    return int(x)  # int() truncates toward zero


def go_float64_to_uint64(x: float) -> int:  # amd64 lowering of uint64(float64)
    if x < 2.0 ** 63:
        return _cvttsd2sq(x) & U64
    return (_cvttsd2sq(x - 2.0 ** 63) & U64) | (1 << 63)


def diskio_score(pod: Pod, s: Scv) -> int:  # algorithm.go:99-119
    rio = pod.rio
    rcpu = float(pod.rcpu)
    with _fpe_ignored():
        q = _fdiv(rcpu, rio)
        beta = _fdiv(1.0, 1.0 + q)
    alpha = 1 - beta
    v = s.cpu / 100.0
    u = s.disk_io / 50.0
    li = abs(_fmul(alpha, v) - _fmul(beta, u))
    si = 10.0 - _fmul(10.0, li)
    return uint64_to_int64(go_float64_to_uint64(si))


def diskio_score_memo(pod: Pod, s: Scv, computed: bool) -> int:
    """B3 memo quirk (algorithm.go:57-63,116): the cycle's first Score call computes and
    returns uint64(S); later calls read FormatFloat(S, 'f', -1, 64) back through
    StrToUint64 (filter.go:67-73), so only a finite, integral S >= 0 survives."""
    if computed:
        return diskio_score(pod, s)
    with _fpe_ignored():
        q = _fdiv(float(pod.rcpu), pod.rio)
        beta = _fdiv(1.0, 1.0 + q)
    alpha = 1 - beta
    li = abs(_fmul(alpha, s.cpu / 100.0) - _fmul(beta, s.disk_io / 50.0))
    si = 10.0 - _fmul(10.0, li)
    if math.isnan(si) or math.isinf(si) or si != math.trunc(si) or si < 0 or si >= 2.0 ** 63:
        return 0
    return int(si)


class _fpe_ignored:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _fdiv(a: float, b: float) -> float:
    """IEEE-754 division (Python raises on /0; Go does not)."""
    if b == 0.0:
        if a == 0.0 or math.isnan(a):
            return math.nan
        neg = (math.copysign(1.0, a) < 0) != (math.copysign(1.0, b) < 0)
        return -math.inf if neg else math.inf
    return a / b


def _fmul(a: float, b: float) -> float:
    if (math.isinf(a) and b == 0.0) or (math.isinf(b) and a == 0.0):
        return math.nan
    return a * b


@dataclass
class CycleResult:
    pick: int
    status: int
    n_feasible: int
    n_ties: int = 0
    top_score: int = 0
    maxima: List[int] = field(default_factory=lambda: [1] * 6)
    tie_set: List[int] = field(default_factory=list)


def schedule_one(pod: Pod, scvs: Sequence[Scv], mode: int = 0,
                 memo_first: int | None = None) -> CycleResult:
    """One kube-scheduler v1.22.3 cycle with yoda as the only scorer (see yoda_oracle.c).
    memo_first (Mode B only): the B3 memo quirk with that node's Score call first."""
    if mode == 1:
        feasible = list(range(len(scvs)))  # Filter pass-through (scheduler.go:96-99)
        mv = MaxValue()
    else:
        feasible = [i for i, s in enumerate(scvs) if fits(pod, s)[0]]
        mv = collect_max_values(pod, scvs)
    r = CycleResult(pick=PICK_NONE, status=STATUS_UNSCHEDULABLE, n_feasible=len(feasible),
                    maxima=mv.as_list())
    if not feasible:
        return r
    if len(feasible) == 1:  # k8s returns the only feasible node without scoring
        r.pick, r.status, r.n_ties, r.tie_set = feasible[0], STATUS_OK, 1, [feasible[0]]
        try:
            r.top_score = _score(pod, scvs[feasible[0]], mv, mode, memo_first, feasible[0])
        except DivideByZero:
            r.top_score = 0
        return r
    scores = []
    try:
        for i in feasible:
            scores.append(_score(pod, scvs[i], mv, mode, memo_first, i))
    except DivideByZero:
        r.pick, r.status = PICK_ERROR, STATUS_DIV_ZERO
        return r
    # NormalizeScore — scheduler.go:158-183
    highest, lowest = 0, scores[0]
    for sc in scores:
        lowest = min(lowest, sc)
        highest = max(highest, sc)
    if highest == lowest:
        lowest -= 1
    norm = [_go_div(_to_i64((sc - lowest) * MAX_NODE_SCORE), highest - lowest) for sc in scores]
    if any(v < 0 or v > MAX_NODE_SCORE for v in norm):
        r.pick, r.status = PICK_ERROR, STATUS_SCORE_RANGE
        return r
    best = max(norm)
    ties = [feasible[k] for k, v in enumerate(norm) if v == best]
    r.pick, r.status, r.n_ties, r.tie_set = ties[0], STATUS_OK, len(ties), ties
    r.top_score = scores[feasible.index(ties[0])]
    return r


def _score(pod: Pod, s: Scv, mv: MaxValue, mode: int, memo_first=None, n: int = -1) -> int:
    if mode == 1:
        if memo_first is not None:
            return diskio_score_memo(pod, s, n == memo_first)
        return diskio_score(pod, s)
    raw = basic_score(mv, pod, s)
    raw = (raw + allocate_score(s)) & U64
    raw = (raw + actual_score(s)) & U64
    return uint64_to_int64(raw)


def greedy(pods: Sequence[Pod], scvs: Sequence[Scv], mode: int = 0, card_capacity: bool = False):
    """Sequential batch in sort.Less order (sort.go:8-10), ties by index; SURVEY §3.4."""
    import copy
    scvs = [copy.deepcopy(s) for s in scvs]
    order = sorted(range(len(pods)), key=lambda i: (-pods[i].priority, i))
    picks = [PICK_NONE] * len(pods)
    for i in order:
        r = schedule_one(pods[i], scvs, mode)
        picks[i] = r.pick
        if r.pick >= 0:
            if pods[i].memory is not None:
                scvs[r.pick].alloc_memory = (scvs[r.pick].alloc_memory + pods[i].memory) & U64
            if card_capacity:
                num = pods[i].number if pods[i].number is not None else 1
                cn = scvs[r.pick].card_number
                scvs[r.pick].card_number = cn - num if cn >= num else 0
    return picks


def f32_round(x: float) -> float:
    """Round a float64 to the nearest float32 (as ParseFloat(s, 32) returns)."""
    return struct.unpack("<f", struct.pack("<f", x))[0]
