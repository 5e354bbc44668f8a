"""Host side (CPU): Go strconv semantics, k8s quantities, the SCV / pod / advisor packers
and the plugin mirror (yoda_amd/plugin.py) driven by an oracle-backed row backend."""
import math
import os
import random

import numpy as np
import pytest

import oracle
from yoda_amd import gostrconv as g
from yoda_amd import synth
from yoda_amd.pack import (milli_value, pack_pods, pack_scvs, pod_cpu_request, pods_to_dicts,
                           scvs_from_soa, value)
from yoda_amd.plugin import (CycleState, NodeScore, Status, YodaPlugin, schedule_one,
                             select_host)
from yoda_amd.soa import MODE_DISKIO, MODE_SCV

U64 = (1 << 64) - 1

# example/test-pod.yaml and example/test-pod-multi.yaml of the reference, as data
TEST_POD = {"metadata": {"name": "test", "labels": {"app": "test"},
                         "annotations": {"diskIO": "10"}},
            "spec": {"containers": [{"name": "iotest-v1", "resources": {
                "requests": {"cpu": "100m", "memory": "400Mi"}}}]}}
TEST_POD_MULTI = {"metadata": {"name": "test", "labels": {"app": "test"},
                               "annotations": {"diskIO": "10m"}},
                  "spec": {"containers": [
                      {"name": "nginx", "resources": {"requests": {"memory": "512Mi",
                                                                   "cpu": "250m"}}},
                      {"name": "nginx2", "resources": {"requests": {"memory": "512Mi",
                                                                    "cpu": "250m"}}}]}}


@pytest.mark.parametrize("s,want", [
    ("10", 10), ("+5", 5), ("0", 0), ("-1", U64), ("-0", 0), ("abc", 0), ("", 0), (" 5", 0),
    ("10m", 0), ("1_000", 0), ("9223372036854775807", (1 << 63) - 1),
    ("9223372036854775808", 0), ("-9223372036854775808", 1 << 63), ("18446744073709551615", 0),
    ("000000000000000000042", 42)])
def test_str_to_uint(s, want):
    """filter.strToUint / StrToUint64 (filter.go:60-74)."""
    assert g.str_to_uint(s) == want


@pytest.mark.parametrize("s,want", [
    ("7", 7), ("-3", -3), ("x", 0), ("99999999999999999999", (1 << 63) - 1),
    ("-99999999999999999999", -(1 << 63))])
def test_pod_priority(s, want):
    """sort.GetPodPriority keeps Atoi's value on a range error (sort.go:14-15)."""
    assert g.pod_priority(s) == want


@pytest.mark.parametrize("s,want,ok", [
    ("10", 10.0, True), ("10m", 0.0, False), ("", 0.0, False), ("0.1", float(np.float32(0.1)), True),
    ("1e39", math.inf, False), ("-1e39", -math.inf, False), ("inf", math.inf, True),
    ("-Infinity", -math.inf, True), ("0x1p-2", 0.25, True), ("1e-50", 0.0, True),
    ("3.4028235e38", float(np.finfo(np.float32).max), True), (".5", 0.5, True), ("5.", 5.0, True),
    ("1e", 0.0, False), ("+", 0.0, False), ("1_0", 10.0, True), ("_1", 0.0, False)])
def test_parse_float32(s, want, ok):
    """strconv.ParseFloat(s, 32) as algorithm.go:103 uses it."""
    v, got_ok = g.parse_float(s, 32)
    assert got_ok == ok and v == want


@pytest.mark.parametrize("s,want,ok", [
    ("1e999999999", math.inf, False), ("-1e999999999", -math.inf, False),
    ("1e-999999999", 0.0, True), ("0e999999999", 0.0, True), ("0x1p999999999", math.inf, False),
    ("1" * 5000, math.inf, False), ("1" * 5000 + "e-4990", 1111111111.1111112, True),
    ("0." + "0" * 5000 + "25e5001", 2.5, True), ("1e" + "9" * 5000, math.inf, False)])
def test_parse_float_bounded(s, want, ok):
    """Huge exponents and long mantissas are decided from the digit counts (Go returns
    ±Inf / range error or 0 at once); the packer must neither stall nor raise on them."""
    import time
    t0 = time.perf_counter()
    v, got_ok = g.parse_float(s, 64)
    assert (v, got_ok) == (want, ok)
    assert g.parse_float(s, 32)[1] == ok
    assert time.perf_counter() - t0 < 1.0


@pytest.mark.parametrize("digits", [20, 5000])
def test_long_integer_labels_clamp(digits):
    """A 20- or 5000-digit scv/* label is a range error in Go's Atoi: StrToUint64 gives 0,
    GetPodPriority the clamped MaxInt64 / MinInt64 (no CPython int-string limit error)."""
    assert g.str_to_uint("9" * digits) == 0
    assert g.pod_priority("9" * digits) == (1 << 63) - 1
    assert g.pod_priority("-" + "9" * digits) == -(1 << 63)
    assert g.atoi("0" * digits + "42") == (42, True)
    pod = {"metadata": {"labels": {"scv/memory": "7" * digits, "scv/priority": "8" * digits},
                        "annotations": {"diskIO": "1e" + "9" * digits}}}
    p = pack_pods([pod])
    assert (p.has_memory[0], p.memory[0], p.priority[0]) == (1, 0, (1 << 63) - 1)
    assert p.rio[0] == math.inf


def test_parse_float_matches_correct_rounding():
    rng = np.random.default_rng(3)
    for _ in range(3000):
        s = f"{int(rng.integers(1, 10 ** 17))}e{int(rng.integers(-340, 312))}"
        assert g.parse_float(s, 64)[0] == float(s), s


def test_parse_float32_rounds_once():
    # correctly rounded to float32 directly from the decimal (no double rounding)
    rng = np.random.default_rng(0)
    for x in rng.random(500) * 1000:
        s = f"{x:.12f}"
        assert g.parse_float(s, 32)[0] == float(np.float32(float(s))) or \
            abs(g.parse_float(s, 32)[0] - float(s)) <= abs(float(np.float32(float(s))) - float(s))
    assert math.isnan(g.parse_float("NaN", 32)[0])


@pytest.mark.parametrize("q,milli,val", [
    ("100m", 100, 1), ("250m", 250, 1), ("1", 1000, 1), ("0.5", 500, 1), ("1.0005", 1001, 2),
    ("2k", 2_000_000, 2000), ("1Ki", 1_024_000, 1024), ("1e3", 1_000_000, 1000), ("0", 0, 0),
    ("1n", 1, 1)])
def test_quantities(q, milli, val):
    assert milli_value(q) == milli and value(q) == val


def test_pod_cpu_request():
    """CalculatePodResourceRequest (algorithm.go:238-262) + GetNonzeroRequestForResource."""
    assert pod_cpu_request(TEST_POD) == 100
    assert pod_cpu_request(TEST_POD_MULTI) == 500
    no_req = {"spec": {"containers": [{"name": "a"}, {"name": "b", "resources": {}}]}}
    assert pod_cpu_request(no_req) == 200                      # default 100m each
    zero = {"spec": {"containers": [{"resources": {"requests": {"cpu": "0"}}}]}}
    assert pod_cpu_request(zero) == 0                         # explicit zero is kept
    init = {"spec": {"containers": [{"resources": {"requests": {"cpu": "100m"}}}],
                     "initContainers": [{"resources": {"requests": {"cpu": "2"}}}],
                     "overhead": {"cpu": "250m"}}}
    assert pod_cpu_request(init) == 2000 + 1                  # Value() of the overhead


def test_pack_example_pods():
    pods = pack_pods([TEST_POD, TEST_POD_MULTI])
    assert list(pods.rcpu) == [100, 500]
    assert list(pods.rio) == [10.0, 0.0]                      # "10m" is not a float
    assert not pods.has_number.any() and not pods.has_memory.any()


def test_pack_labels():
    pod = {"metadata": {"labels": {"scv/number": "-1", "scv/memory": "8000", "scv/clock": "x",
                                   "scv/priority": "3"}}}
    p = pack_pods([pod])
    assert (p.has_number[0], p.number[0]) == (1, U64)
    assert (p.has_memory[0], p.memory[0]) == (1, 8000)
    assert (p.has_clock[0], p.clock[0]) == (1, 0)
    assert p.priority[0] == 3 and p.rcpu[0] == 0


def test_scv_roundtrip_and_alloc():
    nodes = synth.make_nodes(20, seed=9, cards=4)
    scvs = scvs_from_soa(nodes)
    bound = [{"metadata": {"labels": {"scv/memory": "1000"}}, "spec": {"nodeName": "node-3"}},
             {"metadata": {"labels": {"scv/memory": "-1"}}, "spec": {"nodeName": "node-3"}},
             {"metadata": {"labels": {"app": "x"}}, "spec": {"nodeName": "node-4"}}]
    advisor = {f"node-{i}": {"Cpu": float(nodes.cpu[i]), "DiskIO": float(nodes.disk_io[i])}
               for i in range(20)}
    back = pack_scvs(scvs, bound, advisor)
    for f in ("card_number", "card_count", "card_free_memory", "card_total_memory",
              "card_clock", "card_bandwidth", "card_core", "card_power", "card_healthy",
              "free_memory_sum", "total_memory_sum", "cpu", "disk_io"):
        np.testing.assert_array_equal(getattr(back, f), getattr(nodes, f), err_msg=f)
    assert back.alloc_memory[3] == (1000 + U64) & U64 and back.alloc_memory[4] == 0
    with pytest.raises(KeyError):
        pack_scvs(scvs, advisor={"node-0": {"Cpu": 1.0}})


def test_pods_to_dicts_roundtrip():
    pods = synth.make_pods(50, seed=4)
    back = pack_pods(pods_to_dicts(pods))
    for f in pods.__dataclass_fields__:
        np.testing.assert_array_equal(getattr(back, f), getattr(pods, f), err_msg=f)


# ---- plugin mirror -------------------------------------------------------------------------
class OracleRows:
    """Row backend over the C oracle (test stand-in for libyoda's yoda_score_rows)."""

    def __init__(self, nodes):
        self.nodes = nodes

    def upload_pods(self, pods):
        self.pods = pods

    def score_rows(self, mode):
        feas, rows = [], []
        for p in range(self.pods.n_pods):
            _, f, raw, _ = oracle.pod_detail(self.nodes, self.pods, p, mode)
            feas.append(f)
            rows.append(np.where(f, raw, -1))
        return np.array(feas), np.array(rows)


@pytest.mark.parametrize("mode", [MODE_SCV, MODE_DISKIO])
def test_plugin_cycle_matches_oracle(mode):
    nodes, pods = synth.make_config(2, pods=40, nodes=300)
    nodes.total_memory_sum[7] = 0
    names = [f"node-{i}" for i in range(nodes.n_nodes)]
    plugin = YodaPlugin(OracleRows(nodes), names, nodes, mode)
    want = oracle.schedule(nodes, pods, mode)
    for p, pod in enumerate(pods_to_dicts(pods)):
        node, st = schedule_one(plugin, pod)
        if want.status[p] == 0:
            assert st.is_success() and node == names[want.pick[p]], p
        else:
            assert node is None and not st.is_success(), p


def test_plugin_random_tiebreak_stays_in_tie_set():
    nodes, pods = synth.make_config(2, pods=10, nodes=200)
    names = [f"n{i}" for i in range(nodes.n_nodes)]
    plugin = YodaPlugin(OracleRows(nodes), names, nodes)
    rng = random.Random(7)
    for p, pod in enumerate(pods_to_dicts(pods)):
        _, feas, raw, norm = oracle.pod_detail(nodes, pods, p)
        node, st = schedule_one(plugin, pod, rng)
        if st.is_success() and feas.sum() > 1:
            top = norm[feas].max()
            assert norm[names.index(node)] == top


def test_normalize_score_reference_algorithm():
    pl = YodaPlugin(None, ["a", "b", "c"])
    s = [NodeScore("a", 5), NodeScore("b", 5), NodeScore("c", 5)]
    pl.normalize_score(CycleState(), {}, s)
    assert [x.score for x in s] == [100, 100, 100]       # highest == lowest -> lowest--
    s = [NodeScore("a", 1718), NodeScore("b", 4061)]
    pl.normalize_score(CycleState(), {}, s)
    assert [x.score for x in s] == [0, 100]
    assert select_host([NodeScore("a", 3), NodeScore("b", 9), NodeScore("c", 9)]) == "b"


def test_less_and_status():
    hi = {"metadata": {"labels": {"scv/priority": "5"}}}
    lo = {"metadata": {"labels": {}}}
    assert YodaPlugin.less(hi, lo) and not YodaPlugin.less(lo, hi)
    assert Status().is_success()


# ---- advisor ingestion (advisor.go:149-265) ---------------------------------------------
ADV = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "advisor")


def _adv(name):
    return open(os.path.join(ADV, name + ".json")).read()


def test_pack_advisor_fixtures():
    """The five query responses -> Result.Info, against the hand-derived expectation:
    trimmed hostnames, first CPU entry wins, instance fallback for disk/network only, orphan
    rows dropped, later disk rows win, a bad network value ends Init without an error."""
    import json
    from yoda_amd.pack import pack_advisor
    info, err = pack_advisor(_adv("cpu"), _adv("memory"), _adv("diskio"), _adv("net_up"),
                             _adv("net_down"))
    want = json.load(open(os.path.join(ADV, "expected.json")))
    assert err is None and info == want["info"]


def test_pack_advisor_errors():
    from yoda_amd.pack import pack_advisor
    body = lambda rows: {"data": {"result": [{"metric": {"kubernetes_io_hostname": n},  # noqa: E731
                                              "value": [0, v]} for n, v in rows]}}
    info, err = pack_advisor(None, "{}", "{}")
    assert info == {} and err                                   # failed CPU query
    info, err = pack_advisor(body([("a", "1"), ("b", "x")]), "{}", "{}")
    assert list(info) == ["a"] and "ParseFloat" in err          # partial result + the error
    info, err = pack_advisor(body([("a", "1")]), body([("a", "1e999")]), "{}")
    assert err and info["a"]["Memory"] == 0.0                   # range error is an error too
    info, err = pack_advisor("not json", "{}", "{}")
    assert info == {} and err is None                           # Unmarshal error ignored
    info, err = pack_advisor(body([("a", "2")]), "{}", "{}", None)
    assert err is None and info["a"]["Cpu"] == 2.0              # failed network query: no error
    with pytest.raises(TypeError):                              # Value[1].(string) panics
        pack_advisor({"data": {"result": [{"metric": {"kubernetes_io_hostname": "a"},
                                           "value": [0, 1.5]}]}}, "{}", "{}")
    # encoding/json matches keys case-insensitively
    info, _ = pack_advisor({"Data": {"Result": [{"Metric": {"KUBERNETES_IO_HOSTNAME": "a"},
                                                 "Value": [0, "3"]}]}}, "{}", "{}")
    assert info["a"]["Cpu"] == 3.0


def test_advisor_feeds_mode_b():
    """Advisor metrics -> pack_scvs -> Mode B (BalancedCpuDiskIOPriority, algorithm.go:99-119)
    for example/test-pod.yaml (Rcpu 100, Rio 10): scores 5, 9, 0, 2 (SURVEY §8c KAT 2 form)."""
    from yoda_amd.pack import pack_advisor
    info, err = pack_advisor(_adv("cpu"), _adv("memory"), _adv("diskio"), _adv("net_up"),
                             _adv("net_down"))
    nodes = synth.make_nodes(4, seed=3)
    scvs = scvs_from_soa(nodes)
    for s, name in zip(scvs, ["node-a", "node-b", "node-c", "node-d"]):
        s["metadata"]["name"] = name
    soa = pack_scvs(scvs, advisor=info)
    np.testing.assert_array_equal(soa.cpu, [50.0, 5.25, 120.0, 0.0])
    np.testing.assert_array_equal(soa.disk_io, [12.5, 0.5, 0.0, 400.0])
    pods = pack_pods([TEST_POD])
    for n, want in enumerate([5, 9, 0, 2]):
        _, _, raw, _ = oracle.pod_detail(soa, pods, 0, MODE_DISKIO)
        assert raw[n] == want, (n, raw)
    assert oracle.schedule(soa, pods, MODE_DISKIO).pick[0] == 1


def test_pack_scvs_go_json_key_matching():
    """SCV keys decode as encoding/json would: lowerCamelCase tags and Go field names alike."""
    camel = {"metadata": {"name": "n0"}, "status": {"cardNumber": 2, "freeMemorySum": 7,
             "totalMemorySum": 9, "cardList": [{"health": "Healthy", "freeMemory": 3,
                                                "totalMemory": 4, "clock": 1500, "bandwidth": 900,
                                                "core": 80, "power": 300}]}}
    pascal = {"metadata": {"name": "n1"}, "Status": {"CardNumber": 2, "FreeMemorySum": 7,
              "TotalMemorySum": 9, "CardList": [{"Health": "Healthy", "FreeMemory": 3,
                                                 "TotalMemory": 4, "Clock": 1500,
                                                 "Bandwidth": 900, "Core": 80, "Power": 300}]}}
    a, b = pack_scvs([camel]), pack_scvs([pascal])
    for f in a.__dataclass_fields__:
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    assert a.card_healthy[0, 0] == 1 and a.card_clock[0, 0] == 1500 and a.card_number[0] == 2
