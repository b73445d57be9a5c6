"""C-ABI library: loads, exports every gpc.h symbol, and its compiler realizes the reference's
golden flow tables (CPU only -- no classify calls here)."""
import copy
import re
import subprocess

import numpy as np
import pytest

from antrea_amd import gpc
from oracle import compiler as oc
from tests.util import assign_tables, load_golden, normalize_flows

GOLD = load_golden("np_batch_install.json")


@pytest.fixture(scope="module", autouse=True)
def _built():
    from antrea_amd.build import build
    build()


def test_exports_every_header_symbol():
    hdr = open(gpc.os.path.join(gpc.os.path.dirname(gpc.HERE), "include", "gpc.h")).read()
    declared = set(re.findall(r"^(?:int|void|const char\*)\s+(gpc_\w+)\(", hdr, re.M))
    assert declared == set(gpc.EXPORTS)
    syms = subprocess.run(["nm", "-D", "--defined-only", gpc.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (gpc_\w+)", syms))
    assert declared <= exported, declared - exported
    lib = gpc.load()
    assert lib.gpc_abi_version() == 6  # 6: pool collections stat; 5: point-extension stats (4: multi-device contexts; 3: ct_mark column, DNS trio, flow keys; 2: IPv6)


@pytest.mark.parametrize("case", GOLD["cases"], ids=[c["name"] for c in GOLD["cases"]])
def test_batch_install_golden(case):
    c = gpc.Classifier()
    c.batch_install_policy_rule_flows(assign_tables(copy.deepcopy(case["rules"])))
    got = normalize_flows(c.dump_flows())
    want = normalize_flows(case["expected_flows"])
    assert got == want, "\nmissing: %s\nextra: %s" % (sorted(want - got), sorted(got - want))


@pytest.mark.parametrize("case", GOLD["cases"], ids=[c["name"] for c in GOLD["cases"]])
def test_incremental_install_golden(case):
    c = gpc.Classifier()
    for r in assign_tables(copy.deepcopy(case["rules"])):
        c.install_policy_rule_flows(r)
    assert normalize_flows(c.dump_flows()) == normalize_flows(case["expected_flows"])


def test_errors_mirror_reference():
    c = gpc.Classifier()
    with pytest.raises(gpc.GpcError) as e:
        c.add_policy_rule_address(99, "src", ["10.0.0.1"])
    assert e.value.code == gpc.GPC_ENOTFOUND  # ConjunctionNotFound
    r = {"direction": "Out", "from": ["10.0.0.1"], "service": [{"protocol": "TCP", "port": 80}], "flow_id": 7,
         "table": "EgressRule"}
    c.install_policy_rule_flows(r)
    with pytest.raises(gpc.GpcError) as e:
        c.add_policy_rule_address(7, "dst", ["10.0.0.2"])
    assert e.value.code == gpc.GPC_ENOCLAUSE  # "no clause is using addrType"
    one = {k: np.zeros(1, dt) for k, dt in (("src", np.uint32), ("dst", np.uint32), ("sport", np.uint16),
                                            ("dport", np.uint16), ("proto", np.uint8), ("out_port", np.uint32))}
    with pytest.raises(gpc.GpcError):
        c.classify_host(one)  # nothing committed (and no device on this host): fails loudly


def test_batch_limit_checked_before_any_device_work():
    """n > GPC_MAX_BATCH (2^32 - 256, the launch grid limit) is -GPC_EINVAL on both classify entry
    points before the library touches the device (so also here, without one); the header constant
    equals that limit."""
    import ctypes as C
    hdr = open(gpc.os.path.join(gpc.os.path.dirname(gpc.HERE), "include", "gpc.h")).read()
    assert re.search(r"#define GPC_MAX_BATCH \(4294967296ull - 256ull\)", hdr)
    c = gpc.Classifier(ipv4=True, ipv6=True)
    soa = gpc.gpc_pkt_soa()
    dummy = (C.c_uint8 * 64)()
    for name in ("src", "dst", "sport", "dport", "proto", "out_port", "src6", "dst6"):
        setattr(soa, name, C.addressof(dummy))
    for n in ((1 << 32) - 255, 1 << 40):
        assert c.lib.gpc_classify(c.h, C.byref(soa), C.c_size_t(n), C.addressof(dummy), 0, None) == -gpc.GPC_EINVAL
        assert c.lib.gpc_classify6(c.h, C.byref(soa), C.c_size_t(n), C.addressof(dummy), 0, None) == -gpc.GPC_EINVAL


def test_create_multi_arguments():
    """gpc_create_multi: 1..GPC_MAX_DEVICES slots of non-negative ordinals (no device is touched
    before the first commit, so this runs here); out-of-range slots are -GPC_EINVAL before any
    device work."""
    import ctypes as C
    hdr = open(gpc.os.path.join(gpc.os.path.dirname(gpc.HERE), "include", "gpc.h")).read()
    assert re.search(r"#define GPC_MAX_DEVICES 16\b", hdr)
    lib = gpc.load()
    cfg = gpc.gpc_config(ipv4_enabled=1, enable_antrea_policy=1, compact_after=-1)
    h = C.c_void_p()
    for devs in ([], [0] * 17, [0, -1]):
        arr = (C.c_int32 * max(1, len(devs)))(*devs)
        assert lib.gpc_create_multi(C.byref(cfg), arr, len(devs), C.byref(h)) == -gpc.GPC_EINVAL, devs
    c = gpc.Classifier(devices=[0, 1, 0])
    assert c.n_devices == 3
    soa = gpc.gpc_pkt_soa()
    dummy = (C.c_uint8 * 64)()
    assert lib.gpc_classify_on(c.h, 3, C.byref(soa), 1, C.addressof(dummy), None, 0, None) == -gpc.GPC_EINVAL
    assert lib.gpc_classify6_on(c.h, 7, C.byref(soa), 1, C.addressof(dummy), 0, None) == -gpc.GPC_EINVAL
    p = C.POINTER(C.c_uint64)()
    s = C.POINTER(C.c_uint32)()
    n = C.c_size_t()
    assert lib.gpc_counters_on(c.h, 3, C.byref(p), C.byref(s), C.byref(n)) == -gpc.GPC_EINVAL
    assert gpc.Classifier().n_devices == 1
