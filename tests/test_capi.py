"""CPU checks of the C-ABI boundary: libyoda loads and exports every entry point that
include/yoda.h declares (no compute: there is no GPU here)."""
import ctypes as C
import re

from yoda_amd import capi


def test_header_declares_entry_points():
    syms = capi.header_symbols()
    for s in ("yoda_create", "yoda_destroy", "yoda_upload_nodes", "yoda_eval", "yoda_greedy",
              "yoda_last_error", "yoda_shard_phase1", "yoda_shard_finalize"):
        assert s in syms


def test_library_exports_every_header_symbol():
    lib = C.CDLL(capi.LIB_PATH)
    missing = [s for s in capi.header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    assert set(capi.header_symbols()) == set(capi._SIGS), \
        set(capi.header_symbols()) ^ set(capi._SIGS)


def test_abi_version_and_null_handles():
    L = capi.lib()
    assert L.yoda_abi_version() == 1
    # NULL handle / pointers are rejected without touching a GPU
    assert L.yoda_destroy(None) == -1
    assert L.yoda_run(None, 0, 0) == -1
    assert L.yoda_download(None, None) == -1
    assert L.yoda_create(0, None) == -1
    assert L.yoda_last_error(None) == b"null handle"


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        return
    h = C.c_void_p()
    rc = capi.lib().yoda_create(0, C.byref(h))
    assert rc == -6 and not h.value  # YODA_ERR_NO_DEVICE


def test_struct_layouts_match_header():
    text = open(capi.HEADER_PATH).read()
    for cname, pystruct in (("yoda_node_soa", capi.CNodeSoA), ("yoda_pod_soa", capi.CPodSoA),
                            ("yoda_eval_out", capi.CEvalOut)):
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), text, re.S).group(1)
        fields = re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\*?\s*\*?\s*([a-z_0-9]+);", body, re.M)
        assert fields == [f for f, _ in pystruct._fields_], cname


# Policy knobs of the A/B harness: read from the environment only by libyoda_ab.so
# (`make -C kubernetes-scheduler_amd/csrc ab`, -DYODA_AB_KNOBS).  The release library must
# ignore them -- a scheduler inherits its environment -- so their names are not even in it.
AB_KNOBS = ("YODA_NODE_PERM", "YODA_ORDER_PAD", "YODA_NO_GTAB", "YODA_CHUNK_ROUNDS",
            "YODA_MIN_CHUNK_NODES", "YODA_K1_MAX_CHUNKS", "YODA_BLOCK_WITNESS",
            "YODA_TOPK_PER_PAIR", "YODA_TOPK_ROUNDS", "YODA_UPLOAD_THREADS",
            "YODA_GREEDY_WINDOW", "YODA_GREEDY_TOPK", "YODA_GREEDY_REFRESH",
            "YODA_GREEDY_GROW_PCT", "YODA_GREEDY_CAP_TOPK", "YODA_GREEDY_CAP_SCAN",
            "YODA_GREEDY_FAIL_DIV")


def test_release_library_ignores_ab_knobs():
    data = open(capi.LIB_PATH if "libyoda_ab" not in capi.LIB_PATH else
                capi.LIB_PATH.replace("libyoda_ab", "libyoda"), "rb").read()
    found = [k for k in AB_KNOBS if k.encode() in data]
    assert not found, f"release libyoda.so reads tuning knobs from the environment: {found}"
    # the diagnostics may (traces and counters, never results or policy)
    assert b"YODA_K2_TRACE" in data


def test_comm_check_devices_names_shared_gpu():
    """yoda_comm_check_devices (host only): two ranks on one GPU are named before RCCL's init
    would fail on them with a bare "invalid usage" (the round-4 n2_libyoda failure)."""
    import pytest
    capi.comm_check_devices(["0000:05:00.0", "0000:15:00.0", "0000:65:00.0"])
    capi.comm_check_devices(["0000:05:00.0"])
    with pytest.raises(capi.YodaError, match=r"SAME_DEVICE: ranks 1 and 3 .*0000:15:00.0"):
        capi.comm_check_devices(["0000:05:00.0", "0000:15:00.0", "0000:25:00.0",
                                 "0000:15:00.0"])
    L = capi.lib()
    assert L.yoda_comm_check_devices(None, 2, 32, None, None) == -1
    assert L.yoda_comm_check_devices(b"\0" * 64, 2, 32, None, None) == -1  # empty id
    assert L.yoda_device_bus_id(None, None, 0) == -1
    assert L.yoda_device_key(None, None, 0) == -1


def test_comm_check_devices_multi_host_keys():
    """PCI bus ids repeat across identical servers, so the check compares device
    keys (yoda_device_key: host hash / bus id) -- the same bus id on two hosts passes, the same
    (host, bus id) pair is still refused."""
    import pytest
    a, b = "0123456789abcdef/0000:c1:00.0", "fedcba9876543210/0000:c1:00.0"
    capi.comm_check_devices([a, b])
    with pytest.raises(capi.YodaError, match=r"SAME_DEVICE: ranks 0 and 2"):
        capi.comm_check_devices([a, b, a])
