"""Host packers: k8s / SCV / advisor objects -> the SoA buffers of include/yoda.h.

Inputs are plain dicts shaped like the API objects (JSON/YAML-decoded), so snapshots can be
files instead of live Prometheus / API-server reads:

  pod          k8s core/v1 Pod: metadata.labels scv/number|memory|clock|priority,
               metadata.annotations diskIO, spec.containers/initContainers/overhead cpu
  scv          NJUPT-ISL/SCV api/v1 Scv (go.mod:6, not vendored).  The Go field names are
               pinned by the reference's use (Status.CardNumber, CardList[].{Health,
               FreeMemory, TotalMemory, Clock, Bandwidth, Core, Power}, FreeMemorySum,
               TotalMemorySum: filter.go:13-57, collection.go:45-75, algorithm.go:294-309);
               their JSON tags are not in the container, so keys are matched as Go's
               encoding/json matches them: exact first, then case-insensitively -- the
               kubebuilder lowerCamelCase tags (cardList, freeMemory, ...) and the field names
               both decode
  advisor      advisor.Result.Info (advisor.go:22-32): {node name: {Cpu, Memory, DiskIO, ...}},
               built from the five Prometheus query responses by pack_advisor
               (advisor.go:149-265)
"""
from __future__ import annotations

import json
import math
import re
from fractions import Fraction
from typing import Dict, Iterable, List, Mapping, Optional, Sequence

import numpy as np

from .gostrconv import parse_float, pod_priority, str_to_uint
from .soa import MAX_CARDS, NodeSoA, PodSoA

# ---- k8s resource.Quantity (apimachinery) -------------------------------------------------
_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": 1,
        "k": 10 ** 3, "M": 10 ** 6, "G": 10 ** 9, "T": 10 ** 12, "P": 10 ** 15, "E": 10 ** 18}
_QTY = re.compile(r"^([+-]?)([0-9]*)(?:\.([0-9]*))?(.*)$")


def parse_quantity(s: str) -> Fraction:
    """resource.ParseQuantity value as an exact rational (raises ValueError if invalid)."""
    s = str(s).strip()
    m = _QTY.match(s)
    if not m or not (m.group(2) or m.group(3)):
        raise ValueError(f"invalid quantity {s!r}")
    sign, ip, fp, suf = m.group(1), m.group(2) or "", m.group(3) or "", m.group(4)
    v = Fraction(int(ip + fp) if (ip + fp) else 0, 10 ** len(fp))
    if suf in _BIN:
        v *= _BIN[suf]
    elif suf in _DEC:
        v *= _DEC[suf]
    elif re.fullmatch(r"[eE][+-]?[0-9]+", suf):
        v *= Fraction(10) ** int(suf[1:])
    else:
        raise ValueError(f"invalid quantity suffix {s!r}")
    return -v if sign == "-" else v


def milli_value(s: str) -> int:
    """Quantity.MilliValue(): ceil(q * 1000)."""
    return math.ceil(parse_quantity(s) * 1000)


def value(s: str) -> int:
    """Quantity.Value(): ceil(q)."""
    return math.ceil(parse_quantity(s))


DEFAULT_MILLI_CPU_REQUEST = 100  # k8s v1.22.3 pkg/scheduler/util/non_zero.go


def nonzero_cpu_request(requests: Optional[Mapping[str, str]]) -> int:
    """schedutil.GetNonzeroRequestForResource(cpu): 100m when unset (not when zero)."""
    if not requests or "cpu" not in requests:
        return DEFAULT_MILLI_CPU_REQUEST
    return milli_value(requests["cpu"])


def pod_cpu_request(pod: Mapping) -> int:
    """score.CalculatePodResourceRequest(pod, cpu, true) (algorithm.go:238-262): sum of
    containers, max'd with each init container, + overhead (Quantity.Value(), as the
    reference writes it — cores, not millicores)."""
    spec = pod.get("spec", {}) or {}
    req = 0
    for c in spec.get("containers", []) or []:
        req += nonzero_cpu_request(((c.get("resources") or {}).get("requests")))
    for c in spec.get("initContainers", []) or []:
        v = nonzero_cpu_request(((c.get("resources") or {}).get("requests")))
        req = max(req, v)
    over = spec.get("overhead")
    if over and "cpu" in over:
        req += value(over["cpu"])
    return req


# ---- pods ----------------------------------------------------------------------------------
def pack_pods(pods: Sequence[Mapping]) -> PodSoA:
    P = len(pods)
    out = {k: np.zeros(P, dt) for k, dt in (
        ("has_number", np.uint8), ("number", np.uint64), ("has_memory", np.uint8),
        ("memory", np.uint64), ("has_clock", np.uint8), ("clock", np.uint64),
        ("priority", np.int64), ("rio", np.float64), ("rcpu", np.int64))}
    for i, pod in enumerate(pods):
        meta = pod.get("metadata", {}) or {}
        labels = meta.get("labels", {}) or {}
        ann = meta.get("annotations", {}) or {}
        for key, has, val in (("scv/number", "has_number", "number"),
                              ("scv/memory", "has_memory", "memory"),
                              ("scv/clock", "has_clock", "clock")):
            if key in labels:                       # filter.go:12,19,36
                out[has][i] = 1
                out[val][i] = str_to_uint(str(labels[key]))
        if "scv/priority" in labels:                # sort.go:13
            out["priority"][i] = pod_priority(str(labels["scv/priority"]))
        # algorithm.go:103: Rio, _ := strconv.ParseFloat(pod.Annotations["diskIO"], 32)
        out["rio"][i] = parse_float(str(ann.get("diskIO", "")), 32)[0]
        out["rcpu"][i] = pod_cpu_request(pod)
    return PodSoA(**out).normalized()


# ---- advisor: Prometheus query responses -> advisor.Result.Info ---------------------------
def _ci_get(obj, key):
    """encoding/json field matching: the exact key first, then a case-insensitive one."""
    if not isinstance(obj, dict):
        return None
    if key in obj:
        return obj[key]
    low = key.lower()
    for k, v in obj.items():
        if isinstance(k, str) and k.lower() == low:
            return v
    return None


def prometheus_results(body) -> list:
    """getCpu / getMemory / ... (advisor.go:63-147): `_ = json.Unmarshal(body, &res)` then
    res.Data.Result.  The unmarshal error is ignored: an invalid body gives no results; a
    body (str/bytes) or an already-decoded dict is accepted."""
    if isinstance(body, (bytes, bytearray)):
        body = body.decode("utf-8", "replace")
    if isinstance(body, str):
        try:
            body = json.loads(body)
        except ValueError:
            return []
    res = _ci_get(_ci_get(body, "Data"), "Result")
    return res if isinstance(res, list) else []


def _metric(r, field: str) -> str:
    v = _ci_get(_ci_get(r, "Metric"), field)
    return v if isinstance(v, str) else ""


def _value(r) -> float:
    """strconv.ParseFloat(Value[1].(string), 64); the type assertion panics in Go when the
    sample is not a string (TypeError here), ParseFloat errors are returned (ValueError)."""
    val = _ci_get(r, "Value")
    if not isinstance(val, list) or len(val) < 2:
        raise IndexError("Value[1]: index out of range")      # a Go panic
    if not isinstance(val[1], str):
        raise TypeError("interface conversion: Value[1] is not string")  # a Go panic
    v, ok = parse_float(val[1], 64)
    if not ok:
        raise ValueError(f'strconv.ParseFloat: parsing "{val[1]}"')
    return v


def pack_advisor(cpu, memory, disk_io, net_up=None, net_down=None):
    """advisor.Result.Init (advisor.go:149-265) restated over the bodies of its five
    Prometheus queries (cpuQueryL, memoryQueryL, diskIOQueryL, networkIOUpQueryL,
    networkIODownQueryL, advisor.go:16-20), so a snapshot can be a set of files.  A body of
    None stands for a failed HTTP query.  Returns (info, err): info maps node name ->
    {"Cpu", "Memory", "DiskIO", "NetworkIOUp", "NetworkIODown"}, err is the error Init would
    return (info is then what it had built so far), or None.  The rules Init applies:
      - names are strings.Trim(kubernetes_io_hostname, " ") (:157);
      - the CPU query creates the entries; a duplicate CPU name keeps the first (:159-161);
      - memory rows only update existing names, with no instance fallback (:186-191);
      - disk and network rows fall back to the instance label when the hostname is empty
        (:200-202, :225-227, :248-250) and only update existing names (later rows win);
      - a ParseFloat error in the CPU/memory/disk rows returns it (:163-165, :183, :205);
        the network queries end Init silently, with no error, on a failed query or a bad
        value (:217-219, :230-232, :239-241, :253-255)."""
    info = {}
    if cpu is None:
        return info, "cpu query failed"
    for r in prometheus_results(cpu):
        name = _metric(r, "kubernetes_io_hostname").strip(" ")
        if name in info:
            continue  # "Error! cpu info no exist!": the first entry stays
        try:
            v = _value(r)
        except ValueError as e:
            return info, str(e)
        info[name] = {"Cpu": v, "Memory": 0.0, "DiskIO": 0.0, "NetworkIOUp": 0.0,
                      "NetworkIODown": 0.0}
    if memory is None:
        return info, "memory query failed"
    for r in prometheus_results(memory):
        name = _metric(r, "kubernetes_io_hostname").strip(" ")
        if name in info:
            try:
                info[name]["Memory"] = _value(r)
            except ValueError as e:
                return info, str(e)
    if disk_io is None:
        return info, "diskIO query failed"
    for r in prometheus_results(disk_io):
        name = _metric(r, "kubernetes_io_hostname").strip(" ") or _metric(r, "instance").strip(" ")
        if name in info:
            try:
                info[name]["DiskIO"] = _value(r)
            except ValueError as e:
                return info, str(e)
    for body, key in ((net_up, "NetworkIOUp"), (net_down, "NetworkIODown")):
        if body is None:
            return info, None
        for r in prometheus_results(body):
            name = (_metric(r, "kubernetes_io_hostname").strip(" ")
                    or _metric(r, "instance").strip(" "))
            if name in info:
                try:
                    info[name][key] = _value(r)
                except ValueError:
                    return info, None
    return info, None


# ---- nodes ---------------------------------------------------------------------------------
def node_alloc_memory(node_names: Sequence[str], bound_pods: Iterable[Mapping]) -> np.ndarray:
    """Σ scv/memory of the pods already on each node (algorithm.go:299-303), uint64 wrap."""
    idx = {n: i for i, n in enumerate(node_names)}
    alloc = [0] * len(node_names)
    for pod in bound_pods:
        node = (pod.get("spec", {}) or {}).get("nodeName")
        labels = (pod.get("metadata", {}) or {}).get("labels", {}) or {}
        if node in idx and "scv/memory" in labels:
            alloc[idx[node]] = (alloc[idx[node]] + str_to_uint(str(labels["scv/memory"]))) \
                & ((1 << 64) - 1)
    return np.array(alloc, dtype=np.uint64)


def pack_scvs(scvs: Sequence[Mapping], bound_pods: Iterable[Mapping] = (),
              advisor: Optional[Mapping[str, Mapping]] = None,
              max_cards: Optional[int] = None) -> NodeSoA:
    """SCV CRD objects (one per node, in node order) -> NodeSoA.  `advisor` (Mode B) maps
    node name -> advisor.NodeInfo fields {"Cpu", "DiskIO", ...}; a node missing from it
    makes the reference panic (algorithm.go:70,73), so it is an error here."""
    names = [(s.get("metadata", {}) or {}).get("name", str(i)) for i, s in enumerate(scvs)]
    status = [(_ci_get(s, "status") or {}) for s in scvs]
    cards = [(_ci_get(st, "cardList") or []) for st in status]
    k = max_cards or max([len(c) for c in cards] + [1])
    if k > MAX_CARDS or any(len(c) > k for c in cards):
        raise ValueError(f"more than {min(k, MAX_CARDS)} cards on a node")
    N = len(scvs)
    z = lambda dt: np.zeros((N, k), dt)  # noqa: E731
    f, t, ck, bw, co, pw, h = (z(np.uint64), z(np.uint64), z(np.uint64), z(np.uint64),
                               z(np.uint64), z(np.uint64), z(np.uint8))
    num = lambda obj, key: int(_ci_get(obj, key) or 0)  # noqa: E731
    for i, cl in enumerate(cards):
        for j, c in enumerate(cl):
            f[i, j] = num(c, "freeMemory")
            t[i, j] = num(c, "totalMemory")
            ck[i, j] = num(c, "clock")
            bw[i, j] = num(c, "bandwidth")
            co[i, j] = num(c, "core")
            pw[i, j] = num(c, "power")
            h[i, j] = _ci_get(c, "health") == "Healthy"   # filter.go:53,57
    st = status
    cpu = np.zeros(N)
    disk = np.zeros(N)
    if advisor is not None:
        for i, n in enumerate(names):
            if n not in advisor:
                raise KeyError(f"node {n!r} missing from the advisor snapshot")
            cpu[i] = float(advisor[n].get("Cpu", 0.0))
            disk[i] = float(advisor[n].get("DiskIO", 0.0))
    return NodeSoA(
        card_number=np.array([num(x, "cardNumber") for x in st], np.uint64),
        card_count=np.array([len(c) for c in cards], np.uint32),
        free_memory_sum=np.array([num(x, "freeMemorySum") for x in st], np.uint64),
        total_memory_sum=np.array([num(x, "totalMemorySum") for x in st], np.uint64),
        alloc_memory=node_alloc_memory(names, bound_pods),
        card_free_memory=f, card_total_memory=t, card_clock=ck, card_bandwidth=bw,
        card_core=co, card_power=pw, card_healthy=h, cpu=cpu, disk_io=disk).normalized()


def scvs_from_soa(nodes: NodeSoA, prefix: str = "node-") -> List[Dict]:
    """Inverse of pack_scvs (for fixtures and examples)."""
    out = []
    for i in range(nodes.n_nodes):
        cl = [{"health": "Healthy" if nodes.card_healthy[i, j] else "Unhealthy",
               "freeMemory": int(nodes.card_free_memory[i, j]),
               "totalMemory": int(nodes.card_total_memory[i, j]),
               "clock": int(nodes.card_clock[i, j]),
               "bandwidth": int(nodes.card_bandwidth[i, j]),
               "core": int(nodes.card_core[i, j]), "power": int(nodes.card_power[i, j])}
              for j in range(int(nodes.card_count[i]))]
        out.append({"apiVersion": "core.run-linux.com/v1", "kind": "Scv",
                    "metadata": {"name": f"{prefix}{i}"},
                    "status": {"cardNumber": int(nodes.card_number[i]), "cardList": cl,
                               "freeMemorySum": int(nodes.free_memory_sum[i]),
                               "totalMemorySum": int(nodes.total_memory_sum[i])}})
    return out


def pods_to_dicts(pods: PodSoA, prefix: str = "pod-") -> List[Dict]:
    """PodSoA -> k8s-style pod dicts that pack_pods maps back to the same SoA (labels as
    decimal strings; rio written with repr so ParseFloat(., 32) returns it; rcpu as a
    millicore request)."""
    out = []
    for i in range(pods.n_pods):
        labels = {}
        if pods.has_number[i]:
            labels["scv/number"] = str(int(pods.number[i]))
        if pods.has_memory[i]:
            labels["scv/memory"] = str(int(pods.memory[i]))
        if pods.has_clock[i]:
            labels["scv/clock"] = str(int(pods.clock[i]))
        if pods.priority[i]:
            labels["scv/priority"] = str(int(pods.priority[i]))
        rio = float(pods.rio[i])
        ann = {"diskIO": repr(rio) if np.isfinite(rio) else ("+Inf" if rio > 0 else "-Inf")} \
            if rio != 0 else {}
        out.append({"metadata": {"name": f"{prefix}{i}", "labels": labels, "annotations": ann},
                    "spec": {"containers": [{"name": "c", "resources": {"requests": {
                        "cpu": f"{int(pods.rcpu[i])}m"}}}]}})
    return out
