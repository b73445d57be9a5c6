// Conjunctive-match compiler: the NetworkPolicy half of openflow.Client, MI355X build.
//
// Restates pkg/agent/openflow/network_policy.go (contexts, clauses, conjunctions, install /
// uninstall / address churn / priority reassignment) and the NP flow builders of pipeline.go.
// `installed_` plays the role of ovs-vswitchd's flow table: every change is applied to it as one
// all-or-nothing bundle, and the device image is built from it (image.cpp).
#pragma once

#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "gpc.h"
#include "model.hpp"

namespace gpc {

// types.MatchKey values (network_policy.go:38-81)
enum MatchKeyId : uint8_t {
  MK_DST_IP, MK_SRC_IP, MK_DST_IPNET, MK_SRC_IPNET,
  MK_CT_DST_IP, MK_CT_SRC_IP, MK_CT_DST_IPNET, MK_CT_SRC_IPNET,
  MK_DST_IPV6, MK_SRC_IPV6, MK_DST_IPNETV6, MK_SRC_IPNETV6,
  MK_CT_DST_IPV6, MK_CT_SRC_IPV6, MK_CT_DST_IPNETV6, MK_CT_SRC_IPNETV6,
  MK_DST_OFPORT, MK_SRC_OFPORT,
  MK_TCP_DST, MK_TCPV6_DST, MK_UDP_DST, MK_UDPV6_DST, MK_SCTP_DST, MK_SCTPV6_DST,
  MK_TCP_SRC, MK_TCPV6_SRC, MK_UDP_SRC, MK_UDPV6_SRC, MK_SCTP_SRC, MK_SCTPV6_SRC,
  MK_ICMP_TYPE, MK_ICMP_CODE, MK_ICMPV6_TYPE, MK_ICMPV6_CODE,
  MK_SVC_GROUP, MK_IGMP, MK_LABEL_ID, MK_CT_STATE
};

enum ValTag : uint8_t { V_IP, V_IPNET, V_INT, V_BITRANGE, V_ICMP, V_CTSTATE };

struct MatchValue {
  ValTag tag = V_INT;
  IPAddr ip;
  int plen = 0;
  uint32_t u = 0;      // INT / ICMP value / BITRANGE value / CTSTATE data
  int32_t mask = -1;   // BITRANGE mask (-1 nil) / CTSTATE mask
  bool nil = false;    // ICMP nil pointer
};

struct MatchPair {
  MatchKeyId key;
  MatchValue val;
};

struct ConjAction {
  uint32_t conj_id = 0;
  uint8_t clause_id = 0, n_clause = 0;
};

struct ConjMatch {
  uint8_t table = 0;
  bool has_prio = false;
  uint16_t prio = 0;
  std::vector<MatchPair> pairs;
  std::string key() const;  // generateGlobalMapKey equivalence classes
};

struct Context {  // conjMatchFlowContext (network_policy.go:442-461)
  ConjMatch match;
  std::map<uint32_t, ConjAction> actions;
  std::map<uint32_t, bool> deny_all;
  std::unique_ptr<Flow> flow, drop_flow;
  bool drop_logging = false;
};
using CtxPtr = std::shared_ptr<Context>;

struct Clause {  // clause (network_policy.go:685-695)
  ConjAction action;
  std::map<std::string, CtxPtr> matches;
  uint8_t rule_table = 0;
  uint8_t drop_table = 0;  // 0 = none
};

struct Conjunction {  // policyRuleConjunction (network_policy.go:664-677)
  uint32_t id = 0;
  std::unique_ptr<Clause> from, to, svc;
  std::vector<Flow> action_flows, metric_flows;
  bool has_ref = false;
  uint8_t policy_type = 0;
  std::string ns, pname, uid, rule_name, log_label;
  uint8_t rule_table = 0;
  int32_t tier = 0;
  std::vector<Clause*> clauses() const;
};
using ConjPtr = std::shared_ptr<Conjunction>;

struct FlowChange {
  enum Type { INSERT, MODIFY, DELETE } type = MODIFY;
  std::unique_ptr<Flow> flow;  // null: DENY-ALL bookkeeping only
};

struct CtxChange {  // conjMatchFlowContextChange (network_policy.go:551-575)
  CtxPtr ctx;
  FlowChange::Type ctx_type = FlowChange::MODIFY;
  Clause* clause = nullptr;
  FlowChange::Type act_type = FlowChange::INSERT;
  bool has_act = false;
  ConjAction act;
  bool has_match_flow = false;
  FlowChange match_flow;
  bool has_drop = false;
  FlowChange drop_flow;
};

class FeatureNP {
 public:
  explicit FeatureNP(const gpc_config& cfg);

  int initialize();
  int install_rule(const gpc_rule& r);
  int batch_install(const gpc_rule* rules, size_t n);
  int uninstall_rule(uint32_t id, std::vector<uint16_t>* stale);
  int add_rule_addrs(uint32_t id, int addr_type, const gpc_addr* a, size_t n, const uint16_t* prio, bool logging, bool mcnp);
  int del_rule_addrs(uint32_t id, int addr_type, const gpc_addr* a, size_t n, const uint16_t* prio);
  int reassign_priorities(const uint16_t* from, const uint16_t* to, size_t n, uint8_t table);
  int policy_info(uint32_t id, gpc_policy_info* out) const;
  int new_dns_conjunction(uint32_t id);
  std::vector<std::string> flow_keys(const std::string& name, const std::string& ns, uint8_t type) const;

  const std::map<std::string, Flow>& installed() const { return installed_; }
  // Flow-text ingest: applies parsed flows as one bundle. replace = drop the
  // realized NP tables and the compiler's rule caches first (the context then serves the loaded
  // flows only). Loaded flows are not known to the compiler, so commits rebuild the whole image.
  int load_flows(const std::vector<Flow>& flows, bool replace);
  bool foreign() const { return foreign_; }
  // Non-conjunctive, non-conj_id flows of the rule tables (drop / skip flows): the hard
  // pseudo-rules of the image (image.cpp); mirrored here so a delta commit can rebuild them.
  const std::map<std::string, Flow>& hard_flows() const { return hard_; }

  // Change tracking for delta commits: the rules whose realized flows changed since the last
  // take_dirty(). A soft flow whose conjunction actions changed dirties exactly the conj ids
  // added or removed (a shared context gaining rule B does not dirty rule A).
  struct Dirty {
    std::set<uint32_t> conj;
    uint8_t hard_tables = 0;  // bit t-1 for rule table t; kDirtyClassifier: IngressSecurityClassifier
  };
  static constexpr uint8_t kDirtyClassifier = 0x80;
  Dirty take_dirty() {
    Dirty d = std::move(dirty_);
    dirty_ = Dirty();
    return d;
  }
  const std::map<uint32_t, ConjPtr>& policies() const { return policy_cache_; }
  std::string dump() const;
  uint64_t generation() const { return generation_; }

 private:
  // flow builders (pipeline.go)
  Flow conjunctive_match_flow(const ConjMatch& m, const std::map<uint32_t, ConjAction>& acts) const;
  Flow default_drop_flow(uint8_t table, const std::vector<MatchPair>& pairs, bool logging) const;
  Flow mcnp_drop_flow(uint8_t table, const std::vector<MatchPair>& pairs) const;
  std::vector<Flow> conjunction_action_flows(uint32_t id, uint8_t table, uint8_t next, const uint16_t* prio, bool logging) const;
  Flow conjunction_deny_flow(uint32_t id, uint8_t table, uint16_t prio, int disposition, bool logging) const;
  Flow conjunction_pass_flow(uint32_t id, uint8_t table, uint16_t prio, bool logging) const;
  std::vector<Flow> allow_metric_flows(uint32_t id, bool ingress) const;
  Flow deny_metric_flow(uint32_t id, bool ingress) const;
  Flow dns_packet_in_flow(uint32_t id) const;
  void add_flow_match(Match& m, const MatchPair& p) const;

  // clause logic
  ConjPtr calculate_action_flows(const gpc_rule& r, int* err);
  void calculate_clauses(Conjunction& c, const gpc_rule& r);
  std::vector<std::pair<Clause*, ConjMatch>> rule_matches(const Conjunction& c, const gpc_rule& r, int* err) const;
  bool add_conj_match_flow(Clause* cl, const ConjMatch& m, bool logging, bool mcnp, CtxChange* out);
  bool del_conj_match_flow(Clause* cl, const std::string& key, CtxChange* out);
  void update_context_status(CtxChange& ch);
  void apply_changes(std::vector<CtxChange>& chs);
  void apply_bundle(std::vector<const Flow*> add, std::vector<const Flow*> del);
  std::vector<uint16_t> stale_priorities(const Conjunction& c) const;

  gpc_config cfg_;
  std::vector<uint8_t> ip_protocols_;  // 4 and/or 6
  std::map<std::string, CtxPtr> global_cache_;
  std::map<uint32_t, ConjPtr> policy_cache_;
  std::map<std::string, Flow> installed_;
  std::map<std::string, Flow> hard_;
  Dirty dirty_;
  bool foreign_ = false;
  uint64_t generation_ = 0;
  void note_flow(const Flow& f);
  void note_change(const Flow& old, const Flow& nw);
};

// ovs-ofctl flow text -> Flow (flowtext.cpp). 1 = parsed, 0 = skipped line (blank, header, table
// outside the NP path), -GPC_EINVAL with *err set.
int parse_flow_text(const std::string& line, Flow* f, std::string* err);

// helpers shared with tests / image builder
std::vector<std::pair<uint16_t, uint16_t>> bitwise_match(uint16_t start, uint16_t end);  // port_range.go:45

}  // namespace gpc
