// Control-plane operation log (api.cpp): every call that changes the realized NetworkPolicy flows
// is recorded with owned copies of its arguments, so the background compactor's shadow compiler
// can replay the same sequence and reach the same flow table without touching the live compiler.
// Compiler calls are deterministic in their arguments, so replay is exact (failed calls fail the
// same way and change nothing).
#pragma once

#include <string>
#include <vector>

#include "compiler.hpp"
#include "gpc.h"

namespace gpc {

struct OwnedRule {
  gpc_rule r{};
  std::vector<gpc_addr> from, to;
  std::vector<gpc_service> svc;
  std::string str[5];
  bool has_str[5] = {false, false, false, false, false};

  explicit OwnedRule(const gpc_rule& in) : r(in) {
    if (in.n_from > 0 && in.from) from.assign(in.from, in.from + in.n_from);
    if (in.n_to > 0 && in.to) to.assign(in.to, in.to + in.n_to);
    if (in.n_service > 0 && in.service) svc.assign(in.service, in.service + in.n_service);
    const char* s[5] = {in.name, in.log_label, in.policy_namespace, in.policy_name, in.policy_uid};
    for (int i = 0; i < 5; i++)
      if (s[i]) {
        has_str[i] = true;
        str[i] = s[i];
      }
  }
  gpc_rule get() const {  // the rule with pointers into this object's storage
    gpc_rule o = r;
    o.from = from.empty() ? nullptr : from.data();
    o.to = to.empty() ? nullptr : to.data();
    o.service = svc.empty() ? nullptr : svc.data();
    const char** s[5] = {&o.name, &o.log_label, &o.policy_namespace, &o.policy_name, &o.policy_uid};
    for (int i = 0; i < 5; i++) *s[i] = has_str[i] ? str[i].c_str() : nullptr;
    return o;
  }
};

struct Op {
  enum Kind { INIT, INSTALL, BATCH, UNINSTALL, ADD, DEL, REASSIGN, LOAD, DNS_NEW, COMMIT } kind = COMMIT;
  std::vector<OwnedRule> rules;
  uint32_t id = 0;
  int32_t addr_type = 0;
  std::vector<gpc_addr> addrs;
  bool has_prio = false, logging = false, mcnp = false, replace = false;
  uint16_t prio = 0;
  std::vector<uint16_t> from, to;
  uint8_t table = 0;
  std::vector<Flow> flows;
  uint64_t commit_no = 0;  // COMMIT marker: the state after this op is commit `commit_no`

  int apply(FeatureNP& np) const {
    switch (kind) {
      case INIT: return np.initialize();
      case INSTALL: {
        gpc_rule g = rules[0].get();
        return np.install_rule(g);
      }
      case BATCH: {
        std::vector<gpc_rule> rs;
        rs.reserve(rules.size());
        for (auto& o : rules) rs.push_back(o.get());
        return np.batch_install(rs.data(), rs.size());
      }
      case UNINSTALL: {
        std::vector<uint16_t> st;
        return np.uninstall_rule(id, &st);
      }
      case ADD: return np.add_rule_addrs(id, addr_type, addrs.data(), addrs.size(), has_prio ? &prio : nullptr, logging, mcnp);
      case DEL: return np.del_rule_addrs(id, addr_type, addrs.data(), addrs.size(), has_prio ? &prio : nullptr);
      case REASSIGN: return np.reassign_priorities(from.data(), to.data(), from.size(), table);
      case LOAD: return np.load_flows(flows, replace);
      case DNS_NEW: return np.new_dns_conjunction(id);
      case COMMIT: return GPC_OK;
    }
    return GPC_OK;
  }
};

}  // namespace gpc
