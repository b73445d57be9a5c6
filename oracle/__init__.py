"""CPU oracle for the Antrea NetworkPolicy flow-matching path.

TEST INFRASTRUCTURE ONLY. Nothing in the product (`antrea_amd/`, `include/`) imports,
links or executes anything under `oracle/`. Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` use it, and only as the checker.

Contents
--------
* `compiler.py`   -- restatement of the conjunctive-match compiler of
                     `pkg/agent/openflow/network_policy.go` + the NetworkPolicy flow builders of
                     `pkg/agent/openflow/pipeline.go` + `third_party/networkpolicy/port_range.go`,
                     emitting flows in the ovs-ofctl text format of `pkg/ovs/openflow/utils.go`.
                     Pinned by the golden flow strings of
                     `pkg/agent/openflow/network_policy_test.go:349-364, 447-475`.
* `flowtext.py`   -- parser for that text format (the oracle classifier consumes flow text, so it
                     can evaluate any Antrea flow dump, not only what `compiler.py` emits).
* `ovs_cls.py`    -- restatement of the OVS 2.17.7 userspace classifier semantics
                     (`lib/classifier.c` `classifier_lookup__` with conjunctive matches; third-party,
                     not vendored in the reference) and of the Antrea policy-table walk
                     (`docs/design/ovs-pipeline.md:1159-1330, 1633-1812`). Pure Python; small cases.
* `ovs_cls.c`     -- the same classifier semantics in plain C (larger cases, and the timed
                     `cpu_baseline` of bench.py: OVS-style tuple-space search over priority-sorted
                     subtables with early exit).

Parity status: the compiler side is pinned by the reference's golden flow strings and change
counts. The packet->verdict side is restated from OVS semantics (no OVS source or binary in this
container): it is pinned only by the hand-derived known answers of SURVEY.md Appendix A, which are
committed under tests/golden/. Conj-ID ties between equal-priority conjunctions are implementation
defined in OVS (`docs/antrea-network-policy.md:1966-1980`): both oracle and product report them with
the TIE flag and resolve them to the lowest conjunction id.
"""
