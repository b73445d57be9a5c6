// TEST-ONLY: the host half of the library (conjunctive-match compiler, image builders, journal,
// flow-text parser, Service feature) under AddressSanitizer + UndefinedBehaviorSanitizer -- the
// build's counterpart of the reference's `go test -race` unit tier (Makefile:284). Compiled and run
// by tests/test_sanitize.py with g++ -fsanitize=address,undefined -fno-sanitize-recover=all; any
// report aborts the process. Exercises seeded random rule sets (every address kind, both families,
// port ranges, ICMP, IGMP, all actions and tables), batch / single install, address churn,
// uninstall / reinstall, priority reassignment, the DNS conjunction, full and IPv6 image builds,
// delta journals, a dump -> parse -> load round trip and a Service image.
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "compiler.hpp"
#include "image.hpp"
#include "service.hpp"

using namespace gpc;

namespace {

struct RuleStore {  // owns the arrays a gpc_rule points into
  std::vector<gpc_addr> from, to;
  std::vector<gpc_service> svc;
  std::string name, ns, pname, uid, label;
  gpc_rule r{};
};

gpc_addr rand_addr(std::mt19937& g, bool src) {
  gpc_addr a{};
  const int kind = int(g() % 7);
  const bool v6 = g() % 4 == 0;
  a.family = v6 ? 6 : 4;
  switch (kind) {
    case 0: a.kind = GPC_ADDR_IP; break;
    case 1: a.kind = GPC_ADDR_IPNET; a.prefix_len = uint8_t(v6 ? 96 + g() % 33 : 8 + g() % 25); break;
    case 2: a.kind = GPC_ADDR_OFPORT; a.value = 3 + g() % 50; break;
    case 3: a.kind = src ? GPC_ADDR_IP : GPC_ADDR_SVC_GROUP; a.value = 1 + g() % 20; break;
    case 4: a.kind = GPC_ADDR_CT_IP; break;
    case 5: a.kind = GPC_ADDR_CT_IPNET; a.prefix_len = uint8_t(v6 ? 100 : 16 + g() % 17); break;
    default: a.kind = src ? GPC_ADDR_LABEL_ID : GPC_ADDR_IP; a.value = g() % 4; break;
  }
  if (v6) {
    a.ip[0] = 0xfd;
    for (int i = 10; i < 16; i++) a.ip[i] = uint8_t(g());
  } else {
    a.ip[0] = 10;
    for (int i = 1; i < 4; i++) a.ip[i] = uint8_t(g());
  }
  return a;
}

gpc_service rand_service(std::mt19937& g) {
  gpc_service s{};
  const int k = int(g() % 6);
  s.protocol = uint8_t(k == 0 ? GPC_PROTO_NONE : k == 1 ? GPC_PROTO_TCP : k == 2 ? GPC_PROTO_UDP
                       : k == 3 ? GPC_PROTO_SCTP : k == 4 ? GPC_PROTO_ICMP : GPC_PROTO_IGMP);
  if (s.protocol == GPC_PROTO_ICMP) {
    s.has_icmp_type = g() % 2;
    s.icmp_type = int32_t(g() % 16);
    s.has_icmp_code = s.has_icmp_type && g() % 2;
    s.icmp_code = 0;
  } else if (s.protocol == GPC_PROTO_IGMP) {
    s.has_igmp_type = 1;
    s.igmp_type = 0x11;
  } else if (g() % 5) {
    s.has_port = 1;
    s.port = uint16_t(1 + g() % 60000);
    if (g() % 2) {
      s.has_end_port = 1;
      s.end_port = uint16_t(std::min<uint32_t>(65535, s.port + g() % 3000));
    }
    if (g() % 6 == 0) {
      s.has_src_port = 1;
      s.src_port = uint16_t(1024 + g() % 1000);
      s.has_src_end_port = g() % 2;
      s.src_end_port = uint16_t(s.src_port + g() % 64);
    }
  }
  return s;
}

RuleStore make_rule(std::mt19937& g, uint32_t id) {
  RuleStore st;
  const bool in = g() % 2;
  const bool anp = g() % 3 != 0;
  gpc_rule& r = st.r;
  r.direction = uint8_t(in ? GPC_DIR_IN : GPC_DIR_OUT);
  r.table = uint8_t(anp ? (in ? GPC_TABLE_ANTREA_POLICY_INGRESS_RULE : GPC_TABLE_ANTREA_POLICY_EGRESS_RULE)
                        : (in ? GPC_TABLE_INGRESS_RULE : GPC_TABLE_EGRESS_RULE));
  if (anp && g() % 8 == 0) r.table = uint8_t(in ? GPC_TABLE_INGRESS_DEFAULT_RULE : GPC_TABLE_EGRESS_DEFAULT_RULE);
  r.policy_type = uint8_t(anp ? GPC_POLICY_ACNP : GPC_POLICY_K8S);
  r.action = uint8_t(g() % 4);
  if (r.action == GPC_RULE_PASS && (r.table == GPC_TABLE_INGRESS_DEFAULT_RULE || r.table == GPC_TABLE_EGRESS_DEFAULT_RULE))
    r.action = GPC_RULE_DROP;
  r.has_priority = anp ? 1 : uint8_t(g() % 2);
  r.priority = uint16_t(anp ? 100 + g() % 30000 : 190 + g() % 20);
  r.enable_logging = g() % 5 == 0;
  r.flow_id = id;
  r.tier_priority = int32_t(g() % 256);
  const int nf = int(g() % 5) - 1, nt = int(g() % 5) - 1, ns = int(g() % 4) - 1;
  for (int i = 0; i < nf; i++) st.from.push_back(rand_addr(g, true));
  for (int i = 0; i < nt; i++) st.to.push_back(rand_addr(g, false));
  for (int i = 0; i < ns; i++) st.svc.push_back(rand_service(g));
  r.n_from = nf;
  r.n_to = nt;
  r.n_service = ns;
  st.name = "rule-" + std::to_string(id);
  st.ns = "ns";
  st.pname = "p" + std::to_string(id % 17);
  st.uid = "uid";
  st.label = "label";
  return st;
}

void bind(RuleStore& st) {
  st.r.from = st.from.empty() ? nullptr : st.from.data();
  st.r.to = st.to.empty() ? nullptr : st.to.data();
  st.r.service = st.svc.empty() ? nullptr : st.svc.data();
  st.r.name = st.name.c_str();
  st.r.policy_namespace = st.ns.c_str();
  st.r.policy_name = st.pname.c_str();
  st.r.policy_uid = st.uid.c_str();
  st.r.log_label = st.label.c_str();
}

int check(int rc, const char* what) {
  if (rc < 0 && rc != -GPC_EINVAL && rc != -GPC_ENOTFOUND && rc != -GPC_ENOCLAUSE) {
    std::fprintf(stderr, "%s failed: %d\n", what, rc);
    std::exit(2);
  }
  return rc;
}

}  // namespace

int main(int argc, char** argv) {
  const uint32_t seed = argc > 1 ? uint32_t(std::atoi(argv[1])) : 1;
  const int n_rules = argc > 2 ? std::atoi(argv[2]) : 400;
  std::mt19937 g(seed);
  gpc_config cfg{};
  cfg.ipv4_enabled = 1;
  cfg.ipv6_enabled = 1;
  cfg.enable_antrea_policy = 1;
  cfg.enable_deny_tracking = int32_t(seed & 1);
  cfg.ovs_meters = int32_t((seed >> 1) & 1);
  cfg.cookie = 0x1020000000000ull;
  FeatureNP np(cfg);
  check(np.initialize(), "initialize");
  std::vector<RuleStore> rules;
  rules.reserve(size_t(n_rules));
  for (int i = 0; i < n_rules; i++) rules.push_back(make_rule(g, uint32_t(i + 1)));
  for (auto& st : rules) bind(st);
  std::vector<gpc_rule> batch;
  for (int i = 0; i < n_rules / 2; i++) batch.push_back(rules[size_t(i)].r);
  check(np.batch_install(batch.data(), batch.size()), "batch_install");
  for (int i = n_rules / 2; i < n_rules; i++) check(np.install_rule(rules[size_t(i)].r), "install_rule");
  check(np.new_dns_conjunction(100000), "new_dns_conjunction");

  SlotMap slots;
  HostImage img, img6;
  int rc = build_image(np, slots, &img);
  std::printf("image: rc %d, %zu words, %u flows%s%s\n", rc, img.blob.size(), img.n_flows, img.error.empty() ? "" : ", ",
              img.error.c_str());
  rc = build_image6(np, slots, &img6);
  std::printf("image6: rc %d, %zu words\n", rc, img6.blob.size());
  (void)np.take_dirty();
  Journal jn;
  jn.reset(&img);
  std::vector<uint16_t> stale;
  for (int step = 0; step < 200; step++) {
    RuleStore& st = rules[g() % rules.size()];
    const uint32_t id = st.r.flow_id;
    switch (g() % 6) {
      case 0:
      case 1: {
        gpc_addr a[3] = {rand_addr(g, true), rand_addr(g, true), rand_addr(g, true)};
        check(np.add_rule_addrs(id, GPC_SRC_ADDRESS, a, 3, st.r.has_priority ? &st.r.priority : nullptr, false, false),
              "add_rule_addrs");
        check(np.del_rule_addrs(id, GPC_SRC_ADDRESS, a, 1, st.r.has_priority ? &st.r.priority : nullptr), "del_rule_addrs");
        break;
      }
      case 2:
        check(np.uninstall_rule(id, &stale), "uninstall_rule");
        for (uint16_t p : stale) (void)p;
        break;
      case 3:
        check(np.install_rule(st.r), "reinstall");
        break;
      case 4: {
        const uint16_t from = st.r.priority, to = uint16_t(st.r.priority + 1);
        check(np.reassign_priorities(&from, &to, 1, st.r.table), "reassign");
        break;
      }
      default: {
        gpc_addr a = rand_addr(g, false);
        check(np.add_rule_addrs(100000, GPC_DST_ADDRESS, &a, 1, nullptr, false, false), "dns add");
        break;
      }
    }
    FeatureNP::Dirty d = np.take_dirty();
    std::string err;
    const int jrc = step % 50 == 49 ? 1 : jn.apply(np, slots, d.conj, uint8_t(d.hard_tables & 0x3f), &err);
    if (jrc) {
      if (jrc < 0 && step < 5) std::printf("journal apply: %s\n", err.c_str());
      HostImage full;
      (void)build_image(np, slots, &full, step % 2 == 0);
      img = std::move(full);
      jn.reset(&img);
    }
  }
  std::printf("journal: %zu pool words, %u live\n", jn.pool.size(), jn.n_live);

  // dump -> parse -> load round trip into a second compiler, and its image
  const std::string dump = np.dump();
  std::vector<Flow> flows;
  size_t pos = 0, n_lines = 0;
  while (pos < dump.size()) {
    size_t e = dump.find('\n', pos);
    if (e == std::string::npos) e = dump.size();
    Flow f;
    std::string err;
    if (parse_flow_text(dump.substr(pos, e - pos), &f, &err) == 1) flows.push_back(f);
    n_lines++;
    pos = e + 1;
  }
  FeatureNP np2(cfg);
  check(np2.load_flows(flows, true), "load_flows");
  HostImage img2;
  (void)build_image(np2, slots, &img2);
  std::printf("round trip: %zu lines, %zu flows parsed, image %zu words %s\n", n_lines, flows.size(), img2.blob.size(),
              img2.error.c_str());

  // Service feature
  FeatureService svc(cfg);
  for (uint32_t i = 0; i < 50; i++) {
    gpc_endpoint eps[4]{};
    const size_t ne = g() % 5;
    for (size_t k = 0; k < ne; k++) {
      eps[k].family = 4;
      eps[k].port = uint16_t(1024 + g() % 60000);
      eps[k].is_local = g() % 2;
      eps[k].has_node_name = 1;
      eps[k].ip[0] = 10;
      eps[k].ip[1] = uint8_t(g());
      eps[k].ip[2] = uint8_t(g());
      eps[k].ip[3] = uint8_t(g());
      if (eps[k].is_local) check(svc.install_pod(eps[k].ip, 4, 3 + g() % 50), "install_pod");
    }
    check(svc.install_service_group(2 * i + 1, false, eps, ne), "install_service_group");
    check(svc.install_endpoint_flows(uint8_t(1 + g() % 3), 4, eps, ne), "install_endpoint_flows");
    gpc_service_config c{};
    c.family = 4;
    c.protocol = uint8_t(1 + g() % 3);
    c.port = uint16_t(1 + g() % 65535);
    c.cluster_group_id = 2 * i + 1;
    c.local_group_id = 2 * i + 2;
    c.ip[0] = 10;
    c.ip[1] = 96;
    c.ip[2] = uint8_t(i >> 8);
    c.ip[3] = uint8_t(i);
    check(svc.install_service_flows(c), "install_service_flows");
    if (g() % 5 == 0) check(svc.uninstall_service_flows(c.ip, 4, c.port, c.protocol), "uninstall_service_flows");
  }
  std::vector<uint32_t> sblob;
  std::string serr;
  rc = svc.build_image(&sblob, &serr);
  std::printf("service image: rc %d, %zu words; %zu flow bytes, %zu group bytes\n", rc, sblob.size(), svc.dump_flows().size(),
              svc.dump_groups().size());
  std::printf("sanitize ok (seed %u)\n", seed);
  return 0;
}
