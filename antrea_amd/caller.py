"""Caller-side host logic of the path (what pod_reconciler does before calling openflow.Client).

The drop-in boundary is the openflow.Client NP surface (include/gpc.h); in an Antrea deployment the
Go reconciler keeps doing this part. It is restated here because the synthetic workloads of
bench.py and the tests need PolicyRules exactly as the reconciler would build them:

* ipBlock -> OF addresses: `DiffFromCIDRs`, `diffFromCIDR`, `MergeCIDRs`, `IPNetToNetIPNet`
  (pkg/util/ip/ip.go:47-143, 149) as used by `ipBlocksToOFAddresses` (pod_reconciler.go:1198-1233).
* rule table selection `getOFRuleTable` (pod_reconciler.go:353-388).
* `priorityAssigner` (pkg/agent/controller/networkpolicy/priority.go:27-398), uint16 arithmetic
  wrapping exactly as Go's does.
Pinned by pkg/util/ip/ip_test.go:32-113 and priority_test.go:42-351 (tests/test_caller.py).
"""
from __future__ import annotations

import ipaddress
import math
from typing import Dict, List, Optional, Tuple

# ------------------------------------------------------------------------------ ip.go


def ipnet_to_netipnet(cidr: str):
    """IPNetToNetIPNet: normalise non-standard CIDRs (ip.go:149-160)."""
    return ipaddress.ip_network(cidr, strict=False)


def _contains(net, ip_int, version):
    return net.version == version and int(net.network_address) == (ip_int & int(net.netmask))


def merge_cidrs(blocks: List) -> List:
    """MergeCIDRs (ip.go:122-143): drop CIDRs covered by another (stable by prefix length)."""
    blocks = sorted(blocks, key=lambda n: int(n.netmask))
    i = 0
    while i < len(blocks):
        j = i + 1
        while j < len(blocks):
            if _contains(blocks[i], int(blocks[j].network_address), blocks[j].version):
                del blocks[j]
            else:
                j += 1
        i += 1
    return blocks


def _diff_from_cidr(allow, except_):
    """diffFromCIDR (ip.go:79-109)."""
    bits = allow.max_prefixlen
    a_start = int(allow.network_address)
    e_start = int(except_.network_address)
    out = []
    for i in range(allow.prefixlen + 1, except_.prefixlen + 1):
        ip = (e_start ^ (1 << (bits - i))) | a_start
        mask = ((1 << bits) - 1) ^ ((1 << (bits - i)) - 1)
        out.append(ipaddress.ip_network((ip & mask, i)))
    return out


def diff_from_cidrs(allow, excepts: List) -> List:
    """DiffFromCIDRs (ip.go:47-75)."""
    excepts = merge_cidrs(list(excepts))
    new = [allow]
    for ex in excepts:
        changed = True
        while changed:
            changed = False
            for i, ind in enumerate(new):
                ex_ip = int(ex.network_address)
                if _contains(ind, ex_ip, ex.version):
                    res = _diff_from_cidr(ind, ex)
                    del new[i]
                    new.extend(res)
                    changed = True
                    break
                if _contains(ex, int(ind.network_address), ind.version):
                    del new[i]
                    changed = True
                    break
    return new


def ip_blocks_to_of_addresses(blocks: List[dict], ipv4=True, ipv6=False, ct_match=False) -> List[dict]:
    """ipBlocksToOFAddresses (pod_reconciler.go:1198-1233). block = {"cidr": str, "except": [str]}."""
    out = []
    for b in blocks:
        net = ipnet_to_netipnet(b["cidr"])
        if not ((net.version == 4 and ipv4) or (net.version == 6 and ipv6)):
            continue
        for d in diff_from_cidrs(net, [ipnet_to_netipnet(e) for e in b.get("except", [])]):
            out.append({"ctipnet" if ct_match else "ipnet": str(d)})
    return out


# ------------------------------------------------------------------------------ table choice
BASELINE_TIER, BANP_TIER = 253, 254


def of_rule_table(direction: str, antrea_policy: bool, tier_priority: Optional[int]) -> str:
    """getOFRuleTable (pod_reconciler.go:353-388), unicast rules."""
    if not antrea_policy:
        return "IngressRule" if direction == "In" else "EgressRule"
    if tier_priority not in (BASELINE_TIER, BANP_TIER):
        return "AntreaPolicyIngressRule" if direction == "In" else "AntreaPolicyEgressRule"
    return "IngressDefaultRule" if direction == "In" else "EgressDefaultRule"


# ------------------------------------------------------------------------------ priority.go
ZONE_OFFSET = 5
DEFAULT_TIER_PRIORITY = 250
BASELINE_BOTTOM, BASELINE_TOP = 10, 180
POLICY_BOTTOM, POLICY_TOP = 100, 65000


def u16(x: int) -> int:
    return x & 0xFFFF


Priority = Tuple[int, float, int]  # (TierPriority, PolicyPriority, RulePriority)


def p_less(p: Priority, q: Priority) -> bool:
    """types.Priority.Less (pkg/agent/types/networkpolicy.go:122-130)."""
    if p[0] == q[0]:
        if p[1] == q[1]:
            return p[2] > q[2]
        return p[1] > q[1]
    return p[0] > q[0]


def _search(n, f):
    lo, hi = 0, n
    while lo < hi:
        mid = (lo + hi) // 2
        if not f(mid):
            lo = mid + 1
        else:
            hi = mid
    return lo


class PriorityAssigner:
    def __init__(self, is_baseline: bool = False):
        self.priority_map: Dict[Priority, int] = {}
        self.of_priority_map: Dict[int, Priority] = {}
        self.sorted: List[Priority] = []
        self.is_baseline = is_baseline
        self.bottom = BASELINE_BOTTOM if is_baseline else POLICY_BOTTOM
        self.top = BASELINE_TOP if is_baseline else POLICY_TOP

    def initial_of_priority(self, p: Priority) -> int:
        tier_base, prio_base = 200, 20.0
        if p[0] == DEFAULT_TIER_PRIORITY:
            prio_base = 100.0
        if self.is_baseline:
            tier_base, prio_base = 0, 10.0
        tier_off = u16(tier_base * u16(p[0]))
        prio_off = u16(int(math.trunc(p[1] * prio_base)))
        off = u16(tier_off + prio_off + u16(p[2]))
        if u16(self.top - self.bottom) < off:
            return self.bottom
        return u16(self.top - off)

    def update_priority_assignment(self, of: int, p: Priority):
        if p not in self.priority_map:
            idx = _search(len(self.sorted), lambda i: p_less(p, self.sorted[i]))
            self.sorted.insert(idx, p)
        self.of_priority_map[of] = p
        self.priority_map[p] = of

    def find_reassign_boundaries(self, lower: int, upper: int, num_new: int, gap: int):
        target = num_new - gap
        cost_map = {}
        low, high = lower, upper
        sift_down = sift_up = empt_low = empt_high = 0
        while low >= self.bottom and empt_low < target:
            if low in self.of_priority_map:
                sift_down += 1
            else:
                empt_low += 1
                cost_map[empt_low] = [low, u16(upper - 1), sift_down]
            low = u16(low - 1)
        while high <= self.top and empt_high < target:
            if high in self.of_priority_map:
                sift_up += 1
            else:
                empt_high += 1
                idx = target - empt_high
                c = cost_map.get(idx)
                if c is not None:
                    c[2] = sift_down + sift_up
                    c[1] = high
                elif idx == 0:
                    cost_map[idx] = [u16(lower + 1), high, sift_up]
            high = u16(high + 1)
        min_cost, min_idx = 2 ** 31 - 1, 0
        for i in range(target, -1, -1):
            c = cost_map.get(i)
            if c is not None and c[2] < min_cost and u16(c[1] - c[0]) + 1 == num_new + c[2]:
                min_cost, min_idx = c[2], i
        if min_cost == 2 ** 31 - 1:
            raise RuntimeError("failed to push boundary priorities to reach numNewPriorities")
        return cost_map[min_idx][0], cost_map[min_idx][1]

    def reassign_boundary_priorities(self, lower, upper, to_register, updates):
        num_new, gap = len(to_register), u16(upper - lower - 1)
        low, high = self.find_reassign_boundaries(lower, upper, num_new, gap)
        sl = [self.of_priority_map[i] for i in range(low, lower + 1) if i in self.of_priority_map]
        sh = [self.of_priority_map[i] for i in range(upper, high + 1) if i in self.of_priority_map]
        all_p = sl + list(to_register) + sh
        reassigned = sl + sh
        for p in reassigned:
            if p not in updates:
                updates[p] = [self.priority_map[p], None]
        for i, p in enumerate(all_p):
            self.update_priority_assignment(u16(low + i), p)
        for p in reassigned:
            updates[p][1] = self.priority_map[p]

    def get_of_priority(self, p: Priority):
        return self.priority_map.get(p), p in self.priority_map

    def register_priorities(self, priorities: List[Priority]):
        seen = set()
        to_reg = []
        for p in priorities:
            if p not in seen:
                seen.add(p)
                if p not in self.priority_map:
                    to_reg.append(p)
        n = len(to_reg)
        if n == 0:
            return {}, None
        if u16(n + len(self.sorted)) > u16(self.top - self.bottom + 1):
            raise RuntimeError("number of priorities to be registered is greater than available openflow priorities")
        import functools
        to_reg.sort(key=functools.cmp_to_key(lambda a, b: -1 if p_less(a, b) else (1 if p_less(b, a) else 0)))
        groups, i = [], 0
        for j in range(1, n + 1):
            if j == n or not _consecutive(to_reg[j], to_reg[j - 1]):
                groups.append(to_reg[i:j])
                i = j
        updates = {}
        for g in groups:
            self.insert_consecutive_priorities(g, updates)
        return {v[0]: v[1] for v in updates.values()}, None

    def insert_consecutive_priorities(self, priorities: List[Priority], updates):
        n = len(priorities)
        p_low, p_high = priorities[0], priorities[-1]
        ins_low = self.initial_of_priority(p_low)
        ins_high = self.initial_of_priority(p_high)
        idx = _search(len(self.sorted), lambda i: p_less(p_low, self.sorted[i]))
        upper, lower = self.top, self.bottom
        if idx > 0:
            lower = self.priority_map[self.sorted[idx - 1]]
        if idx < len(self.sorted):
            upper = self.priority_map[self.sorted[idx]]
        if u16(upper - lower - 1) < n:
            return self.reassign_boundary_priorities(lower, upper, priorities, updates)
        if ins_low > lower and ins_high < upper:
            pass
        elif u16(upper - lower - 1) >= n + 2 * ZONE_OFFSET:
            if ins_low <= lower:
                ins_low = u16(lower + ZONE_OFFSET + 1)
            else:
                ins_low = u16(upper - ZONE_OFFSET - n)
        else:
            ins_low = u16(lower + u16(upper - lower - n) // 2 + 1)
        for i, p in enumerate(priorities):
            self.update_priority_assignment(u16(ins_low + i), p)

    def release(self, of: int):
        p = self.of_priority_map.pop(of, None)
        if p is None:
            return
        self.priority_map.pop(p, None)
        idx = _search(len(self.sorted), lambda i: p_less(p, self.sorted[i])) - 1
        if idx >= 0 and self.sorted[idx] == p:
            del self.sorted[idx]


def _consecutive(p: Priority, q: Priority) -> bool:
    """Priority.IsConsecutive (types/networkpolicy.go:142-147)."""
    return p[0] == q[0] and p[1] == q[1] and abs(p[2] - q[2]) == 1
