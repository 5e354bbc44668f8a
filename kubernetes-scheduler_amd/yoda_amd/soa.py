"""Struct-of-arrays containers for node snapshots and pod batches, and their C-ABI views.

The ctypes structures mirror include/yoda.h field for field.  NodeSoA / PodSoA own numpy
arrays; `.c()` returns the C struct pointing into them (the container must outlive it).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

MAX_CARDS = 16

# include/yoda.h constants
MODE_SCV = 0
MODE_DISKIO = 1
PICK_NONE = -1
PICK_ERROR = -2
STATUS_OK = 0
STATUS_UNSCHEDULABLE = 1
STATUS_DIV_ZERO = 2
STATUS_SCORE_RANGE = 3
UPLOAD_FORCE_GENERIC = 1
RUN_BITMASK = 1
GREEDY_CARD_CAPACITY = 1

_u8p = C.POINTER(C.c_uint8)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_f64p = C.POINTER(C.c_double)


class CNodeSoA(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint32),
        ("max_cards", C.c_uint32),
        ("card_number", _u64p),
        ("card_count", _u32p),
        ("free_memory_sum", _u64p),
        ("total_memory_sum", _u64p),
        ("alloc_memory", _u64p),
        ("card_free_memory", _u64p),
        ("card_total_memory", _u64p),
        ("card_clock", _u64p),
        ("card_bandwidth", _u64p),
        ("card_core", _u64p),
        ("card_power", _u64p),
        ("card_healthy", _u8p),
        ("cpu", _f64p),
        ("disk_io", _f64p),
    ]


class CPodSoA(C.Structure):
    _fields_ = [
        ("n_pods", C.c_uint32),
        ("has_number", _u8p),
        ("number", _u64p),
        ("has_memory", _u8p),
        ("memory", _u64p),
        ("has_clock", _u8p),
        ("clock", _u64p),
        ("priority", _i64p),
        ("rio", _f64p),
        ("rcpu", _i64p),
    ]


class CEvalOut(C.Structure):
    _fields_ = [
        ("pick", _i32p),
        ("status", _i32p),
        ("n_feasible", _u32p),
        ("n_ties", _u32p),
        ("top_score", _i64p),
        ("maxima", _u64p),
    ]


def _ptr(a: Optional[np.ndarray], ctype):
    if a is None:
        return C.cast(None, C.POINTER(ctype))
    assert a.flags["C_CONTIGUOUS"], "SoA arrays must be C-contiguous"
    return a.ctypes.data_as(C.POINTER(ctype))


@dataclass
class NodeSoA:
    """A node snapshot (or shard).  Card arrays are [N, K]."""
    card_number: np.ndarray        # u64 [N]
    card_count: np.ndarray         # u32 [N]
    free_memory_sum: np.ndarray    # u64 [N]
    total_memory_sum: np.ndarray   # u64 [N]
    alloc_memory: np.ndarray       # u64 [N]
    card_free_memory: np.ndarray   # u64 [N, K]
    card_total_memory: np.ndarray  # u64 [N, K]
    card_clock: np.ndarray         # u64 [N, K]
    card_bandwidth: np.ndarray     # u64 [N, K]
    card_core: np.ndarray          # u64 [N, K]
    card_power: np.ndarray         # u64 [N, K]
    card_healthy: np.ndarray       # u8  [N, K]
    cpu: np.ndarray                # f64 [N]
    disk_io: np.ndarray            # f64 [N]

    @property
    def n_nodes(self) -> int:
        return int(self.card_number.shape[0])

    @property
    def max_cards(self) -> int:
        return int(self.card_free_memory.shape[1])

    def normalized(self) -> "NodeSoA":
        """Copy with canonical dtypes, contiguity and zeroed unused card slots."""
        n, k = self.card_free_memory.shape
        if not 1 <= k <= MAX_CARDS:
            raise ValueError(f"max_cards must be in 1..{MAX_CARDS}, got {k}")
        cnt = np.ascontiguousarray(self.card_count, dtype=np.uint32)
        if cnt.size and int(cnt.max()) > k:
            raise ValueError("card_count exceeds max_cards")
        used = np.arange(k)[None, :] < cnt[:, None]

        def cards(a, dt):
            a = np.array(a, dtype=dt, copy=True).reshape(n, k)
            a[~used] = 0
            return np.ascontiguousarray(a)

        return NodeSoA(
            card_number=np.ascontiguousarray(self.card_number, dtype=np.uint64),
            card_count=cnt,
            free_memory_sum=np.ascontiguousarray(self.free_memory_sum, dtype=np.uint64),
            total_memory_sum=np.ascontiguousarray(self.total_memory_sum, dtype=np.uint64),
            alloc_memory=np.ascontiguousarray(self.alloc_memory, dtype=np.uint64),
            card_free_memory=cards(self.card_free_memory, np.uint64),
            card_total_memory=cards(self.card_total_memory, np.uint64),
            card_clock=cards(self.card_clock, np.uint64),
            card_bandwidth=cards(self.card_bandwidth, np.uint64),
            card_core=cards(self.card_core, np.uint64),
            card_power=cards(self.card_power, np.uint64),
            card_healthy=cards(self.card_healthy, np.uint8),
            cpu=np.ascontiguousarray(self.cpu, dtype=np.float64),
            disk_io=np.ascontiguousarray(self.disk_io, dtype=np.float64),
        )

    def slice(self, lo: int, hi: int) -> "NodeSoA":
        """Nodes [lo, hi) — a contiguous shard."""
        return NodeSoA(**{f: np.ascontiguousarray(getattr(self, f)[lo:hi])
                          for f in self.__dataclass_fields__})

    def c(self) -> CNodeSoA:
        return CNodeSoA(
            n_nodes=self.n_nodes,
            max_cards=self.max_cards,
            card_number=_ptr(self.card_number, C.c_uint64),
            card_count=_ptr(self.card_count, C.c_uint32),
            free_memory_sum=_ptr(self.free_memory_sum, C.c_uint64),
            total_memory_sum=_ptr(self.total_memory_sum, C.c_uint64),
            alloc_memory=_ptr(self.alloc_memory, C.c_uint64),
            card_free_memory=_ptr(self.card_free_memory, C.c_uint64),
            card_total_memory=_ptr(self.card_total_memory, C.c_uint64),
            card_clock=_ptr(self.card_clock, C.c_uint64),
            card_bandwidth=_ptr(self.card_bandwidth, C.c_uint64),
            card_core=_ptr(self.card_core, C.c_uint64),
            card_power=_ptr(self.card_power, C.c_uint64),
            card_healthy=_ptr(self.card_healthy, C.c_uint8),
            cpu=_ptr(self.cpu, C.c_double),
            disk_io=_ptr(self.disk_io, C.c_double),
        )


@dataclass
class PodSoA:
    has_number: np.ndarray  # u8 [P]
    number: np.ndarray      # u64 [P]
    has_memory: np.ndarray  # u8 [P]
    memory: np.ndarray      # u64 [P]
    has_clock: np.ndarray   # u8 [P]
    clock: np.ndarray       # u64 [P]
    priority: np.ndarray    # i64 [P]
    rio: np.ndarray         # f64 [P]
    rcpu: np.ndarray        # i64 [P]

    @property
    def n_pods(self) -> int:
        return int(self.number.shape[0])

    def normalized(self) -> "PodSoA":
        f = {"has_number": np.uint8, "number": np.uint64, "has_memory": np.uint8,
             "memory": np.uint64, "has_clock": np.uint8, "clock": np.uint64,
             "priority": np.int64, "rio": np.float64, "rcpu": np.int64}
        return PodSoA(**{k: np.ascontiguousarray(getattr(self, k), dtype=t) for k, t in f.items()})

    def slice(self, lo: int, hi: int) -> "PodSoA":
        return PodSoA(**{f: np.ascontiguousarray(getattr(self, f)[lo:hi])
                         for f in self.__dataclass_fields__})

    def take(self, idx) -> "PodSoA":
        return PodSoA(**{f: np.ascontiguousarray(getattr(self, f)[idx])
                         for f in self.__dataclass_fields__})

    def c(self) -> CPodSoA:
        return CPodSoA(
            n_pods=self.n_pods,
            has_number=_ptr(self.has_number, C.c_uint8),
            number=_ptr(self.number, C.c_uint64),
            has_memory=_ptr(self.has_memory, C.c_uint8),
            memory=_ptr(self.memory, C.c_uint64),
            has_clock=_ptr(self.has_clock, C.c_uint8),
            clock=_ptr(self.clock, C.c_uint64),
            priority=_ptr(self.priority, C.c_int64),
            rio=_ptr(self.rio, C.c_double),
            rcpu=_ptr(self.rcpu, C.c_int64),
        )


@dataclass
class EvalResult:
    pick: np.ndarray        # i32 [P]
    status: np.ndarray      # i32 [P]
    n_feasible: np.ndarray  # u32 [P]
    n_ties: np.ndarray      # u32 [P]
    top_score: np.ndarray   # i64 [P]
    maxima: np.ndarray      # u64 [P, 6]

    @staticmethod
    def empty(p: int) -> "EvalResult":
        return EvalResult(pick=np.full(p, -3, np.int32), status=np.full(p, -1, np.int32),
                          n_feasible=np.zeros(p, np.uint32), n_ties=np.zeros(p, np.uint32),
                          top_score=np.zeros(p, np.int64), maxima=np.zeros((p, 6), np.uint64))

    def c(self) -> CEvalOut:
        return CEvalOut(pick=_ptr(self.pick, C.c_int32), status=_ptr(self.status, C.c_int32),
                        n_feasible=_ptr(self.n_feasible, C.c_uint32),
                        n_ties=_ptr(self.n_ties, C.c_uint32),
                        top_score=_ptr(self.top_score, C.c_int64),
                        maxima=_ptr(self.maxima, C.c_uint64))
