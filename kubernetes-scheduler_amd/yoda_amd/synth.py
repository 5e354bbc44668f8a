"""Seeded synthetic clusters and pod batches for BASELINE.json configs 1-5.

There is no network and no real cluster: node SCV records and pods are generated with
numpy from a fixed seed, vectorised so that 100k nodes / 1M pods take well under a second.
"""
from __future__ import annotations

import numpy as np

from .soa import NodeSoA, PodSoA

# GPU models: (total MiB per card, clock MHz, bandwidth, cores, power W) — SURVEY §8d
TOTALS = np.array([16384, 32768, 81920], dtype=np.uint64)
CLOCKS = np.array([1410, 1500, 1755], dtype=np.uint64)
BANDWIDTHS = np.array([900, 1200, 2000], dtype=np.uint64)
CORES = np.array([80, 108, 132], dtype=np.uint64)
POWERS = np.array([300, 400, 700], dtype=np.uint64)

# test-pod.yaml: cpu 100m, annotation diskIO "10"  -> Rcpu 100, Rio 10
TEST_POD_RCPU, TEST_POD_RIO = 100, 10.0
# test-pod-multi.yaml: 2 x 250m, diskIO "10m" (not a float: ParseFloat error -> 0)
TEST_POD_MULTI_RCPU, TEST_POD_MULTI_RIO = 500, 0.0


def make_nodes(n: int, seed: int, cards: int = 8, unhealthy: float = 0.05,
               heterogeneous: bool = False) -> NodeSoA:
    """Homogeneous fleet: 8 cards/node, one GPU model per node, ~5% unhealthy cards.

    heterogeneous=True (config 4): CardNumber in {0,1,2,4,8,16} with len(CardList) equal to
    it except for 1% of nodes where they differ; card slots = 16."""
    rng = np.random.default_rng(seed)
    if heterogeneous:
        k = 16
        counts = rng.choice(np.array([0, 1, 2, 4, 8, 16], dtype=np.uint32), size=n)
        card_number = counts.astype(np.uint64)
        mismatch = rng.random(n) < 0.01
        alt = rng.integers(0, 17, size=n).astype(np.uint32)
        counts = np.where(mismatch, alt, counts).astype(np.uint32)
    else:
        k = cards
        counts = np.full(n, cards, dtype=np.uint32)
        card_number = counts.astype(np.uint64)
    model = rng.integers(0, 3, size=n)
    if heterogeneous:  # mixed memory: per-card model for memory, per-node for the rest
        mem_model = rng.integers(0, 3, size=(n, k))
        total = TOTALS[mem_model]
    else:
        total = np.repeat(TOTALS[model][:, None], k, axis=1)
    free = (rng.random((n, k)) * (total.astype(np.float64) + 1)).astype(np.uint64)
    free = np.minimum(free, total)
    clock = np.repeat(CLOCKS[model][:, None], k, axis=1)
    bw = np.repeat(BANDWIDTHS[model][:, None], k, axis=1)
    core = np.repeat(CORES[model][:, None], k, axis=1)
    power = np.repeat(POWERS[model][:, None], k, axis=1)
    healthy = (rng.random((n, k)) >= unhealthy).astype(np.uint8)
    used = np.arange(k)[None, :] < counts[:, None]
    for a in (free, total, clock, bw, core, power, healthy):
        a[~used] = 0
    free_sum = free.sum(axis=1, dtype=np.uint64)
    total_sum = total.sum(axis=1, dtype=np.uint64)
    alloc = (rng.random(n) * (total_sum.astype(np.float64) / 2)).astype(np.uint64)
    cpu = rng.random(n) * 100.0
    disk = rng.random(n) * 100.0
    return NodeSoA(card_number=card_number, card_count=counts, free_memory_sum=free_sum,
                   total_memory_sum=total_sum, alloc_memory=alloc, card_free_memory=free,
                   card_total_memory=total, card_clock=clock, card_bandwidth=bw,
                   card_core=core, card_power=power, card_healthy=healthy, cpu=cpu,
                   disk_io=disk).normalized()


def make_pods(p: int, seed: int, heterogeneous: bool = False, priorities: bool = False) -> PodSoA:
    """Config 2/3/5 pods: scv/number in {absent 20%, 1, 2, 4, 8}; scv/memory present 80%,
    U[0, 81920]; scv/clock present 50% from the node clock set.  Mode-B fields follow
    test-pod.yaml (Rcpu 100, Rio 10).

    heterogeneous=True (config 4): number in {2,4,8,16}, high memory U[40000, 81920], so
    most pairs are infeasible; half the pods are test-pod-multi.yaml-shaped for Mode B."""
    rng = np.random.default_rng(seed)
    if heterogeneous:
        has_number = np.ones(p, np.uint8)
        number = rng.choice(np.array([2, 4, 8, 16], dtype=np.uint64), size=p)
        has_memory = np.ones(p, np.uint8)
        memory = rng.integers(40000, 81921, size=p).astype(np.uint64)
        multi = rng.random(p) < 0.5
        rcpu = np.where(multi, TEST_POD_MULTI_RCPU, TEST_POD_RCPU).astype(np.int64)
        rio = np.where(multi, TEST_POD_MULTI_RIO, TEST_POD_RIO).astype(np.float64)
    else:
        choice = rng.integers(0, 5, size=p)
        has_number = (choice > 0).astype(np.uint8)
        number = np.array([0, 1, 2, 4, 8], dtype=np.uint64)[choice]
        has_memory = (rng.random(p) < 0.8).astype(np.uint8)
        memory = np.where(has_memory == 1, rng.integers(0, 81921, size=p), 0).astype(np.uint64)
        rcpu = np.full(p, TEST_POD_RCPU, np.int64)
        rio = np.full(p, TEST_POD_RIO, np.float64)
    has_clock = (rng.random(p) < 0.5).astype(np.uint8)
    clock = np.where(has_clock == 1, CLOCKS[rng.integers(0, 3, size=p)], 0).astype(np.uint64)
    priority = (rng.integers(0, 10, size=p) if priorities else np.zeros(p)).astype(np.int64)
    return PodSoA(has_number=has_number, number=number, has_memory=has_memory, memory=memory,
                  has_clock=has_clock, clock=clock, priority=priority, rio=rio,
                  rcpu=rcpu).normalized()


def test_pod(p: int = 1) -> PodSoA:
    """example/test-pod.yaml: no scv/* labels, cpu 100m, diskIO "10" (config 1)."""
    z = np.zeros(p)
    return PodSoA(has_number=z, number=z, has_memory=z, memory=z, has_clock=z, clock=z,
                  priority=z, rio=np.full(p, TEST_POD_RIO), rcpu=np.full(p, TEST_POD_RCPU)
                  ).normalized()


def _copy(soa):
    return type(soa)(**{f: np.array(getattr(soa, f)) for f in soa.__dataclass_fields__})


def mixed_models(nodes: NodeSoA, frac: float = 0.5, seed: int = 12) -> NodeSoA:
    """The same fleet with a fraction `frac` of its nodes holding a mix of GPU models: each
    real card of such a node draws its own (clock, bandwidth, cores, power) model, so the
    one-model shortcuts of the block kernels do not apply to it."""
    out = _copy(nodes)
    rng = np.random.default_rng(seed)
    pick = rng.random(out.n_nodes) < frac
    k = out.card_clock.shape[1]
    models = rng.integers(0, 3, size=(int(pick.sum()), k))
    real = np.arange(k)[None, :] < out.card_count[pick][:, None]
    for arr, table in ((out.card_clock, CLOCKS), (out.card_bandwidth, BANDWIDTHS),
                       (out.card_core, CORES), (out.card_power, POWERS)):
        arr[pick] = np.where(real, table[models], 0)
    return out.normalized()


def memory_in_bytes(nodes: NodeSoA, pods: PodSoA):
    """The same workload with every memory quantity in bytes instead of MiB (card free/total,
    the sums, the allocated memory, scv/memory): fields above 2^32, the F64 record path."""
    mib = np.uint64(1 << 20)
    n = _copy(nodes)
    for f in ("card_free_memory", "card_total_memory", "free_memory_sum", "total_memory_sum",
              "alloc_memory"):
        setattr(n, f, getattr(n, f) * mib)
    p = _copy(pods)
    p.memory = p.memory * mib
    return n.normalized(), p.normalized()


def wide_fields(nodes: NodeSoA, fields=("bandwidth",), factor: int = 1000) -> NodeSoA:
    """The same fleet with small card fields scaled (e.g. bandwidth in MB/s instead of GB/s):
    beyond 16 bits, the N32 kernels with unpacked K1 partials and f64 quotients.
    Scale the pods' scv/clock labels with the clock, or the Filter changes."""
    n = _copy(nodes)
    for f in fields:
        setattr(n, "card_" + f, getattr(n, "card_" + f) * np.uint64(factor))
    return n.normalized()


def distinct_diskio(pods: PodSoA, seed: int = 11) -> PodSoA:
    """The same pods with a distinct Mode-B request each: diskIO annotation U(0.5, 100) and a
    CPU request U{50..4000} millicores, so no two pods share (alpha, beta) and the Mode-B batch
    path evaluates every (pod, node) pair (algorithm.go:105-106)."""
    p = _copy(pods)
    rng = np.random.default_rng(seed)
    p.rio = 0.5 + rng.random(p.n_pods) * 99.5
    p.rcpu = rng.integers(50, 4001, p.n_pods).astype(np.int64)
    return p.normalized()


CONFIGS = {
    1: dict(pods=1, nodes=100, seed=1, desc="example/test-pod.yaml x 100 synthetic nodes"),
    2: dict(pods=1000, nodes=5000, seed=42, desc="1k pods x 5k nodes"),
    3: dict(pods=100_000, nodes=100_000, seed=7, desc="100k pods x 100k nodes"),
    4: dict(pods=10_000, nodes=20_000, seed=11, desc="heterogeneous fleet, high infeasibility"),
    5: dict(pods=1_000_000, nodes=100_000, seed=13, desc="1M pods x 100k nodes greedy"),
}


def make_config(cfg: int, pods: int | None = None, nodes: int | None = None):
    """(NodeSoA, PodSoA) for a BASELINE config; pods/nodes override the sizes (for tests)."""
    c = CONFIGS[cfg]
    p = c["pods"] if pods is None else pods
    n = c["nodes"] if nodes is None else nodes
    seed = c["seed"]
    if cfg == 1:
        return make_nodes(n, seed), test_pod(p)
    het = cfg == 4
    return (make_nodes(n, seed, heterogeneous=het),
            make_pods(p, seed + 1000, heterogeneous=het, priorities=(cfg == 5)))


# Workloads the headline does not cover (bench.py `extra.variants`, tools/variants.py):
# name -> description.  Mode 0 = SCV (Mode A), 1 = diskIO (Mode B), as yoda_amd.soa.
VARIANTS = {
    "c3": "config 3 as generated (the headline workload)",
    "mixed50": "config 3 with 50% of the nodes holding mixed GPU models",
    "mixed100": "config 3 with every node holding mixed GPU models",
    "bytes": "config 3 with memory in bytes instead of MiB (fields above 2^32: memory ranks)",
    "u64": "config 3 forced onto the U64 record path (the reference's uint64 arithmetic)",
    "f64": "config 3 forced onto the F64 record path (per-pair kernels, fields <= 2^44)",
    "bw1000": "config 3 with bandwidth x 1000 (small fields beyond 16 bits: N32, f64 quotients)",
    "c4": "config 4 at its declared size (10k pods x 20k nodes, heterogeneous fleet)",
    "het100k": "config-4 generator at 100k pods x 100k nodes",
    "diskio": "config 3, Mode B (BalancedCpuDiskIOPriority), pods as generated (one spec)",
    "diskio_distinct": "config 3, Mode B, a distinct diskIO/CPU request per pod",
    "c4diskio": "config 4, Mode B",
}


def variant_workloads(names):
    """Yield (name, nodes, pods, mode, upload kwargs) for the VARIANTS names (config 3 built
    once and shared)."""
    c3 = None

    def get_c3():
        nonlocal c3
        if c3 is None:
            c3 = make_config(3)
        return c3

    for name in names:
        if name not in VARIANTS:
            raise ValueError(f"unknown variant {name}")
        mode, kw = 0, {}
        if name in ("c4", "c4diskio"):
            n, p = make_config(4)
        elif name == "het100k":
            n, p = make_config(4, pods=100_000, nodes=100_000)
        else:
            n, p = get_c3()
        if name == "mixed50":
            n = mixed_models(n, 0.5)
        elif name == "mixed100":
            n = mixed_models(n, 1.0)
        elif name == "bytes":
            n, p = memory_in_bytes(n, p)
        elif name == "u64":
            kw = {"force_generic": True}
        elif name == "f64":
            kw = {"force_f64": True}
        elif name == "bw1000":
            n = wide_fields(n, ("bandwidth",), 1000)
        elif name == "diskio_distinct":
            p = distinct_diskio(p)
        if name.startswith("diskio") or name == "c4diskio":
            mode = 1
        yield name, n, p, mode, kw
