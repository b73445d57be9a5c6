"""Caller-side logic vs the reference's unit-test goldens: pkg/util/ip/ip_test.go:32-113 and
pkg/agent/controller/networkpolicy/priority_test.go:42-351."""
import ipaddress

import pytest

from antrea_amd import caller as cl

N = ipaddress.ip_network


def test_diff_cidrs():
    got = cl.diff_from_cidrs(N("10.20.0.0/16"), [N("10.20.1.0/24")])
    want = ["10.20.128.0/17", "10.20.64.0/18", "10.20.32.0/19", "10.20.16.0/20", "10.20.8.0/21", "10.20.4.0/22",
            "10.20.2.0/23", "10.20.0.0/24"]
    assert sorted(map(str, got)) == sorted(want)
    got = cl.diff_from_cidrs(N("10.20.0.0/16"), [N("10.20.1.0/24"), N("10.20.2.0/28")])
    want = ["10.20.128.0/17", "10.20.64.0/18", "10.20.32.0/19", "10.20.16.0/20", "10.20.8.0/21", "10.20.4.0/22",
            "10.20.0.0/24", "10.20.3.0/24", "10.20.2.128/25", "10.20.2.64/26", "10.20.2.32/27", "10.20.2.16/28"]
    assert sorted(map(str, got)) == sorted(want)


def test_merge_cidrs():
    a, b, c, d = N("10.10.0.0/16"), N("10.20.0.0/16"), N("10.20.1.2/32"), N("10.20.1.3/32")
    assert set(cl.merge_cidrs([a, b, c, d])) == {a, b}
    assert cl.merge_cidrs([a]) == [a]
    assert set(cl.merge_cidrs([c, d])) == {c, d}
    assert set(cl.merge_cidrs([a, d])) == {a, d}
    assert cl.merge_cidrs([]) == []


@pytest.mark.parametrize("seed", range(10))
def test_diff_cidrs_exact_cover(seed):
    import random
    rng = random.Random(seed)
    for _ in range(20):
        plen = rng.randint(8, 28)
        base = rng.getrandbits(32) & ~((1 << (32 - plen)) - 1)
        allow = N((base, plen))
        exc = []
        for _ in range(rng.randint(1, 3)):
            el = rng.randint(plen, 32)
            eb = (base | (rng.getrandbits(32) & ((1 << (32 - plen)) - 1))) & ~((1 << (32 - el)) - 1)
            exc.append(N((eb, el)))
        pieces = cl.diff_from_cidrs(allow, exc)
        # sample points: in allow minus excepts <=> in exactly one piece
        for _ in range(200):
            ip = base | (rng.getrandbits(32) & ((1 << (32 - plen)) - 1))
            ipa = ipaddress.ip_address(ip)
            inside = not any(ipa in e for e in exc)
            hits = sum(ipa in p for p in pieces)
            assert hits == (1 if inside else 0)


p110 = (1, 1.0, 0)
p1120, p1121 = (1, 1.2, 0), (1, 1.2, 1)
p1130, p1131, p1132, p1133 = (1, 1.3, 0), (1, 1.3, 1), (1, 1.3, 2), (1, 1.3, 3)
p1140, p1141, p1142 = (1, 1.4, 0), (1, 1.4, 1), (1, 1.4, 2)
p190, p191, p192, p193 = (1, 9.0, 0), (1, 9.0, 1), (1, 9.0, 2), (1, 9.0, 3)


@pytest.mark.parametrize("prios,ofs", [([p110, p1120, p1121], [10000, 9999, 9998]),
                                       ([p1121, p1120, p110], [9998, 9999, 10000])])
def test_update_priority_assignment(prios, ofs):
    pa = cl.PriorityAssigner(False)
    for p, o in zip(prios, ofs):
        pa.update_priority_assignment(o, p)
    assert pa.priority_map == {p110: 10000, p1120: 9999, p1121: 9998}
    assert pa.sorted == [p1121, p1120, p110]


REASSIGN = [
    ("push-down-single", 10000, 10001, [p1140, p1121, p1120], [10000, 10001, 10002],
     {p1140: 9996, p1133: 9997, p1132: 9998, p1131: 9999, p1130: 10000, p1121: 10001, p1120: 10002},
     {p1140: [10000, 9996]}),
    ("push-down-multiple", 10000, 10001, [p190, p1140, p1121, p1120], [9998, 10000, 10001, 10002],
     {p190: 9995, p1140: 9996, p1133: 9997, p1132: 9998, p1131: 9999, p1130: 10000, p1121: 10001, p1120: 10002},
     {p1140: [10000, 9996], p190: [9998, 9995]}),
    ("push-up-single", 10000, 10002, [p1142, p1141, p1140, p1121], [9998, 9999, 10000, 10002],
     {p1142: 9998, p1141: 9999, p1140: 10000, p1133: 10001, p1132: 10002, p1131: 10003, p1130: 10004, p1121: 10005},
     {p1121: [10002, 10005]}),
    ("push-up-multiple", 10000, 10002, [p1142, p1141, p1140, p1121, p1120], [9998, 9999, 10000, 10002, 10003],
     {p1142: 9998, p1141: 9999, p1140: 10000, p1133: 10001, p1132: 10002, p1131: 10003, p1130: 10004,
      p1121: 10005, p1120: 10006},
     {p1121: [10002, 10005], p1120: [10003, 10006]}),
    ("reassign-minimum-possible", 10000, 10002, [p193, p192, p191, p190, p1140, p1121, p1120],
     [9994, 9995, 9996, 9997, 10000, 10002, 10003],
     {p193: 9994, p192: 9995, p191: 9996, p190: 9997, p1140: 10000, p1133: 10001, p1132: 10002, p1131: 10003,
      p1130: 10004, p1121: 10005, p1120: 10006},
     {p1121: [10002, 10005], p1120: [10003, 10006]}),
]


@pytest.mark.parametrize("name,lower,upper,orig,ofs,want_map,want_upd", REASSIGN, ids=[r[0] for r in REASSIGN])
def test_reassign_boundary_priorities(name, lower, upper, orig, ofs, want_map, want_upd):
    pa = cl.PriorityAssigner(False)
    for p, o in zip(orig, ofs):
        pa.update_priority_assignment(o, p)
    upd = {}
    pa.reassign_boundary_priorities(lower, upper, [p1133, p1132, p1131, p1130], upd)
    assert pa.priority_map == want_map
    assert upd == want_upd


def _ins(pa):
    return pa.initial_of_priority(p1133), pa.initial_of_priority(p1130)


def test_insert_consecutive_priorities():
    reg = [p1133, p1132, p1131, p1130]
    lo, hi = _ins(cl.PriorityAssigner(False))
    z = cl.ZONE_OFFSET
    cases = [
        ([], [], {lo: p1133, lo + 1: p1132, lo + 2: p1131, hi: p1130}),
        ([p110], [lo + 100], {lo: p1133, lo + 1: p1132, lo + 2: p1131, hi: p1130, lo + 100: p110}),
        ([p1140], [lo - 100], {lo - 100: p1140, lo: p1133, lo + 1: p1132, lo + 2: p1131, hi: p1130}),
        ([p1141, p1140, p1121, p1120], [lo - 100, lo - 99, lo + 99, lo + 100],
         {lo - 100: p1141, lo - 99: p1140, lo: p1133, lo + 1: p1132, lo + 2: p1131, hi: p1130, lo + 99: p1121,
          lo + 100: p1120}),
        ([p1141, p1140], [lo + 1, lo + 2],
         {lo + 1: p1141, lo + 2: p1140, lo + 3 + z: p1133, lo + 4 + z: p1132, lo + 5 + z: p1131, lo + 6 + z: p1130}),
        ([p1121, p1120], [lo + 1, lo + 2],
         {lo - z - 3: p1133, lo - z - 2: p1132, lo - z - 1: p1131, lo - z: p1130, lo + 1: p1121, lo + 2: p1120}),
        ([p1141, p1140, p1121, p1120], [lo + 1, lo + 2, lo + 9, lo + 10],
         {lo + 1: p1141, lo + 2: p1140, lo + 4: p1133, lo + 5: p1132, lo + 6: p1131, lo + 7: p1130, lo + 9: p1121,
          lo + 10: p1120}),
        ([p1141, p1140, p1121, p1120], [lo - 1, lo, lo + 5, lo + 6],
         {lo - 1: p1141, lo: p1140, lo + 1: p1133, lo + 2: p1132, lo + 3: p1131, lo + 4: p1130, lo + 5: p1121,
          lo + 6: p1120}),
    ]
    for orig, ofs, want in cases:
        pa = cl.PriorityAssigner(False)
        for p, o in zip(orig, ofs):
            pa.update_priority_assignment(o, p)
        pa.insert_consecutive_priorities(reg, {})
        assert pa.of_priority_map == want


def test_register_priorities():
    pa = cl.PriorityAssigner(False)
    i1132 = pa.initial_of_priority(p1132)
    i191 = pa.initial_of_priority(p191)
    pa.update_priority_assignment(i1132 - 1, p1140)
    pa.update_priority_assignment(i1132 + 2, p1121)
    pa.update_priority_assignment(i1132 + 3, p1120)
    pa.register_priorities([p1132, p1131, p1130, p190, p191])
    assert pa.of_priority_map == {i1132 - 2: p1140, i1132 - 1: p1132, i1132: p1131, i1132 + 1: p1130,
                                  i1132 + 2: p1121, i1132 + 3: p1120, i191: p191, i191 + 1: p190}


def test_register_duplicate_and_all():
    pa1, pa2 = cl.PriorityAssigner(False), cl.PriorityAssigner(False)
    pa1.register_priorities([p1131, p1130])
    pa2.register_priorities([p1130, p1131, p1130, p1130, p1130, p1131, p1130])
    assert pa1.get_of_priority(p1130) == pa2.get_of_priority(p1130)
    assert pa1.get_of_priority(p1131) == pa2.get_of_priority(p1131)
    pa = cl.PriorityAssigner(True)
    pa.register_priorities([(253, 5.0, i) for i in range(0, 171)])
    with pytest.raises(RuntimeError):
        pa.register_priorities([(253, 5.0, 171)])
    pa = cl.PriorityAssigner(False)
    pa.register_priorities([(5, 5.0, i) for i in range(0, 10000 - 100 + 1)])
    pa.register_priorities([(10, 5.0, i) for i in range(0, 65000 - 10001 + 1)])
    with pytest.raises(RuntimeError):
        pa.register_priorities([(253, 5.0, 171)])


def test_initial_of_priority_appendix_a3():
    pa = cl.PriorityAssigner(False)
    assert pa.initial_of_priority((250, 5.0, 0)) == 14500
    assert pa.initial_of_priority((250, 5.0, 1)) == 14499
    assert pa.initial_of_priority((250, 4.0, 0)) == 14600
