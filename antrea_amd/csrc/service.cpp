// AntreaProxy flows / groups (service.hpp). Flow text is golden-exact against
// pkg/agent/openflow/client_test.go:1024-1330 (Test_client_InstallServiceGroup,
// Test_client_InstallEndpointFlows, Test_client_InstallServiceFlows).
#include "service.hpp"

#include <cstdio>
#include <cstring>

#include "core.hpp"

namespace gpc {

namespace {

// fields.go register marks used by the Service path
constexpr uint32_t kRewriteMac = 1u << 9;          // reg0[9]   RewriteMACRegMark
constexpr uint32_t kSvcNoEp = 1u << 14;            // reg0[14]  SvcNoEpRegMark
constexpr uint32_t kEpStateMask = 0x7u << 16;      // reg4[16..18] ServiceEPStateField
constexpr uint32_t kEpToSelect = 0x1u << 16;
constexpr uint32_t kEpSelected = 0x2u << 16;
constexpr uint32_t kToNodePort = 1u << 19;         // reg4[19]  ToNodePortAddressRegMark
constexpr uint32_t kToExternal = 1u << 21;         // reg4[21]  ToExternalAddressRegMark
constexpr uint32_t kVirtualNodePortDNAT = 0xa9fe00fcu;  // config.VirtualNodePortDNATIPv4 169.254.0.252
constexpr uint32_t kRemoteEndpoint = 1u << 26;     // reg4[26]  RemoteEndpointRegMark
constexpr uint32_t kEpUnionMask = 0x7ffffu;        // reg4[0..18] EpUnionField

uint8_t ip_proto(uint8_t p) {  // gpc_protocol -> IP protocol number
  switch (p) {
    case GPC_PROTO_TCP: return 6;
    case GPC_PROTO_UDP: return 17;
    case GPC_PROTO_SCTP: return 132;
  }
  return 0;
}

const char* proto_name(uint8_t p, uint8_t family) {  // binding.Protocol string (cache keys)
  switch (p) {
    case GPC_PROTO_TCP: return family == 6 ? "tcp6" : "tcp";
    case GPC_PROTO_UDP: return family == 6 ? "udp6" : "udp";
    case GPC_PROTO_SCTP: return family == 6 ? "sctp6" : "sctp";
  }
  return "?";
}

IPAddr to_ip(const uint8_t* b, uint8_t family) {
  IPAddr a;
  a.fam = family == 6 ? 6 : 4;
  std::memcpy(a.b, b, a.fam == 4 ? 4 : 16);
  return a;
}

Action set_reg(uint32_t r, uint32_t v, uint32_t m = 0xffffffffu) {
  Action a{ACT_SET_REG};
  a.a = r;
  a.b = v;
  a.c = m;
  a.has_mask = m != 0xffffffffu;
  return a;
}

void match_reg(Match& m, int r, uint32_t v, uint32_t mask) {  // several marks of one register merge
  if (m.reg_present & (1u << r)) {
    m.reg_v[r] |= v;
    m.reg_m[r] |= mask;
  } else {
    m.set_reg(r, v, mask);
  }
}

void set_proto(Match& m, uint8_t proto, uint8_t family) {
  m.has_dl = true;
  m.dl_type = family == 6 ? kEthIPv6 : kEthIP;
  m.has_proto = proto != 0;
  m.nw_proto = proto;
}

}  // namespace

FeatureService::FeatureService(const gpc_config& cfg) : cfg_(cfg) {}

uint64_t FeatureService::cookie() const {  // cookie.Service category of the same round
  return cfg_.cookie ? ((cfg_.cookie & ~(0xffull << 40)) | (3ull << 40)) : 0;
}

// serviceEndpointGroup (pipeline.go:2553-2592)
int FeatureService::install_service_group(uint32_t gid, bool affinity, const gpc_endpoint* eps, size_t n) {
  Group g;
  g.id = gid;
  const uint8_t resubmit = affinity ? TB_SERVICE_LB : TB_ENDPOINT_DNAT;
  if (n == 0) {
    Bucket b;
    b.acts = {set_reg(0, kSvcNoEp, kSvcNoEp)};
    Action r{ACT_RESUBMIT};
    r.a = TB_ENDPOINT_DNAT;
    b.acts.push_back(r);
    g.buckets.push_back(b);
  }
  for (size_t i = 0; i < n; i++) {
    const gpc_endpoint& e = eps[i];
    if (e.family != 4 && e.family != 6) return -GPC_EINVAL;
    if (e.family == 6) return -GPC_EINVAL;  // IPv6 Endpoints: xxreg3 loads are not modelled
    Bucket b;
    b.id = uint32_t(i);
    if (!e.is_local && e.has_node_name && !e.is_node_ip) b.acts.push_back(set_reg(4, kRemoteEndpoint, kRemoteEndpoint));
    b.acts.push_back(set_reg(3, to_ip(e.ip, 4).v4()));
    b.acts.push_back(set_reg(4, e.port, 0xffff));
    Action r{ACT_RESUBMIT};
    r.a = resubmit;
    b.acts.push_back(r);
    g.buckets.push_back(b);
  }
  groups_[gid] = g;
  generation_++;
  return GPC_OK;
}

int FeatureService::uninstall_service_group(uint32_t gid) {
  groups_.erase(gid);
  generation_++;
  return GPC_OK;
}

static std::string endpoint_key(const gpc_endpoint& e, uint8_t proto) {  // generateEndpointFlowCacheKey
  char buf[96];
  std::snprintf(buf, sizeof buf, "E%s%s%x", to_ip(e.ip, e.family).str().c_str(), proto_name(proto, e.family), e.port);
  return buf;
}

// InstallEndpointFlows (client.go:750-770): endpointDNATFlow (pipeline.go:2502-2528) per Endpoint,
// plus podHairpinSNATFlow (pipeline.go:3052-3064) for local Endpoints.
int FeatureService::install_endpoint_flows(uint8_t proto, uint8_t family, const gpc_endpoint* eps, size_t n) {
  if (!ip_proto(proto) || family != 4) return -GPC_EINVAL;
  std::map<std::string, std::vector<Flow>> add;
  for (size_t i = 0; i < n; i++) {
    const gpc_endpoint& e = eps[i];
    if (e.family != 4) return -GPC_EINVAL;
    const uint32_t ip = to_ip(e.ip, 4).v4();
    std::vector<Flow> fl;
    Flow f;
    f.table = TB_ENDPOINT_DNAT;
    f.priority = kPriorityNormal;
    f.cookie = cookie();
    set_proto(f.m, ip_proto(proto), 4);
    f.m.set_reg(3, ip);
    f.m.set_reg(4, kEpSelected | e.port, kEpUnionMask);
    Action ct{ACT_CT_DNAT};
    ct.a = dnat_next_table();
    ct.b = kCtZone;
    ct.c = ip;
    ct.lv = e.port;
    f.acts = {ct};
    fl.push_back(f);
    if (e.is_local) {
      Flow h;
      h.table = TB_SNAT_MARK;
      h.priority = kPriorityLow;
      h.cookie = cookie();
      h.m.has_ct_state = true;
      h.m.ct_data = 0x21;  // +new+trk
      h.m.ct_mask = 0x21;
      set_proto(h.m, 0, 4);
      h.m.nw_src.set = h.m.nw_dst.set = true;
      h.m.nw_src.addr = h.m.nw_dst.addr = to_ip(e.ip, 4);
      Action hp{ACT_CT_HAIRPIN};
      hp.a = TB_SNAT;
      hp.b = kCtZone;
      h.acts = {hp};
      fl.push_back(h);
    }
    add[endpoint_key(e, proto)] = fl;
  }
  for (auto& kv : add) cached_[kv.first] = kv.second;
  generation_++;
  return GPC_OK;
}

int FeatureService::uninstall_endpoint_flows(uint8_t proto, uint8_t family, const gpc_endpoint* eps, size_t n) {
  if (!ip_proto(proto) || family != 4) return -GPC_EINVAL;
  for (size_t i = 0; i < n; i++) cached_.erase(endpoint_key(eps[i], proto));
  generation_++;
  return GPC_OK;
}

static std::string service_key(const IPAddr& ip, uint16_t port, uint8_t proto) {  // generateServicePortFlowCacheKey
  char buf[96];
  std::snprintf(buf, sizeof buf, "S%s%s%x", ip.str().c_str(), proto_name(proto, ip.fam), port);
  return buf;
}

// InstallServiceFlows (client.go:790-807) -> serviceLBFlows (pipeline.go:2373-2431).
int FeatureService::install_service_flows(const gpc_service_config& c) {
  if (!ip_proto(c.protocol) || c.family != 4) return -GPC_EINVAL;
  if (c.affinity_timeout || c.is_dsr || c.is_nested || (c.is_external && c.traffic_policy_local))
    return -GPC_EINVAL;  // learn / DSR / multi-cluster / short-circuit flows: not modelled
  const IPAddr ip = to_ip(c.ip, 4);
  const uint32_t gid = c.traffic_policy_local ? c.local_group_id : c.cluster_group_id;  // TrafficPolicyGroupID
  Flow f;
  f.table = TB_SERVICE_LB;
  f.priority = kPriorityNormal;
  f.cookie = cookie();
  set_proto(f.m, ip_proto(c.protocol), 4);
  f.m.has_tp_dst = true;
  f.m.tp_dst = c.port;
  f.m.tp_dst_m = 0xffff;
  match_reg(f.m, 4, kEpToSelect, kEpStateMask);
  if (c.is_nodeport) {  // ToNodePortAddressRegMark instead of the Service IP (pipeline.go:2381-2387)
    match_reg(f.m, 4, kToNodePort, kToNodePort);
  } else {
    f.m.nw_dst.set = true;
    f.m.nw_dst.addr = ip;
  }
  f.acts.push_back(set_reg(0, kRewriteMac, kRewriteMac));
  f.acts.push_back(set_reg(4, kEpSelected, kEpStateMask));
  if (c.is_external) f.acts.push_back(set_reg(4, kToExternal, kToExternal));
  if (cfg_.enable_antrea_policy) f.acts.push_back(set_reg(7, gid));
  Action g{ACT_GROUP};
  g.a = gid;
  f.acts.push_back(g);
  cached_[service_key(ip, c.port, c.protocol)] = {f};
  generation_++;
  return GPC_OK;
}

int FeatureService::uninstall_service_flows(const uint8_t* ip, uint8_t family, uint16_t port, uint8_t proto) {
  if (!ip_proto(proto) || family != 4) return -GPC_EINVAL;
  cached_.erase(service_key(to_ip(ip, family), port, proto));
  generation_++;
  return GPC_OK;
}

int FeatureService::install_pod(const uint8_t* ip, uint8_t family, uint32_t ofport) {
  if (family != 4) return -GPC_EINVAL;
  pods_[to_ip(ip, 4).v4()] = ofport;
  generation_++;
  return GPC_OK;
}

int FeatureService::set_node_port_addresses(const uint32_t* v4, size_t n) {
  for (auto it = cached_.begin(); it != cached_.end();)
    it = it->first.compare(0, 2, "NP") == 0 ? cached_.erase(it) : std::next(it);
  std::vector<uint32_t> addrs;
  for (size_t i = 0; i < n; i++)
    if ((v4[i] >> 24) != 127u) addrs.push_back(v4[i]);  // loopback: not NodePort traffic from a Pod
  if (n) addrs.push_back(kVirtualNodePortDNAT);  // the gateway's DNATed NodePort connections
  for (uint32_t a : addrs) {
    Flow f;
    f.table = TB_NODEPORT_MARK;
    f.priority = kPriorityNormal;
    f.cookie = cookie();
    set_proto(f.m, 0, 4);
    f.m.nw_dst.set = true;
    f.m.nw_dst.addr.fam = 4;
    for (int k = 0; k < 4; k++) f.m.nw_dst.addr.b[k] = uint8_t(a >> (24 - 8 * k));
    f.acts.push_back(set_reg(4, kToNodePort, kToNodePort));
    char key[24];
    std::snprintf(key, sizeof key, "NP%08x", a);
    cached_[key] = {f};
  }
  generation_++;
  return GPC_OK;
}

int FeatureService::uninstall_pod(const uint8_t* ip, uint8_t family) {
  if (family != 4) return -GPC_EINVAL;
  pods_.erase(to_ip(ip, 4).v4());
  generation_++;
  return GPC_OK;
}

std::string FeatureService::dump_flows() const {
  std::string s;
  for (auto& kv : cached_)
    for (auto& f : kv.second) s += f.str() + "\n";
  return s;
}

std::string FeatureService::dump_groups() const {
  std::string s;
  for (auto& kv : groups_) s += kv.second.str() + "\n";
  return s;
}

// --------------------------------------------------------------------------- device image
namespace {

struct SvcHash {  // 2-choice cuckoo table of (key, value), kSvcSlots slots per bucket
  uint32_t log2 = 0;
  std::vector<uint64_t> keys;
  std::vector<uint32_t> vals;
  bool build(const std::vector<std::pair<uint64_t, uint32_t>>& kv) {
    constexpr uint32_t S = kSvcSlots;
    for (log2 = 1; double(S << log2) * 0.6 < double(kv.size() + 1); log2++) {
    }
    for (int attempt = 0; attempt < 8; attempt++, log2++) {
      const uint32_t nb = 1u << log2, mask = nb - 1;
      keys.assign(size_t(nb) * S, 0);
      vals.assign(size_t(nb) * S, 0);
      bool ok = true;
      for (auto& e : kv) {
        uint64_t k = e.first;
        uint32_t v = e.second;
        int kicks = 0;
        while (true) {
          bool placed = false;
          for (uint32_t b : {hash_b1(k, mask), hash_b2(k, mask)}) {
            for (uint32_t i = 0; i < S && !placed; i++)
              if (!keys[size_t(b) * S + i]) {
                keys[size_t(b) * S + i] = k;
                vals[size_t(b) * S + i] = v;
                placed = true;
              }
            if (placed) break;
          }
          if (placed) break;
          if (++kicks > 500) {
            ok = false;
            break;
          }
          const uint32_t b = (kicks & 1) ? hash_b2(k, mask) : hash_b1(k, mask);
          const uint32_t i = uint32_t(kicks) % S;
          std::swap(k, keys[size_t(b) * S + i]);
          std::swap(v, vals[size_t(b) * S + i]);
        }
        if (!ok) break;
      }
      if (ok) return true;
    }
    return false;
  }
};

}  // namespace

int FeatureService::build_image(std::vector<uint32_t>* blob, std::string* err) const {
  blob->clear();
  // EndpointDNAT flows: (proto, endpoint ip, port) -> DNAT exists
  std::map<std::tuple<uint8_t, uint32_t, uint16_t>, bool> dnat;
  struct Svc {
    uint64_t key;
    uint32_t gid;
    bool reg7;
  };
  std::vector<Svc> svcs;
  std::vector<uint32_t> node_port_addrs;
  bool any_node_port = false;
  for (auto& kv : cached_)
    for (auto& f : kv.second) {
      if (f.table == TB_NODEPORT_MARK) {
        if (!f.m.nw_dst.set || f.m.nw_dst.plen >= 0) {
          *err = "unsupported NodePortMark flow: " + f.str();
          return -GPC_EINVAL;
        }
        node_port_addrs.push_back(f.m.nw_dst.addr.v4());
      } else if (f.table == TB_ENDPOINT_DNAT) {
        if (!(f.m.reg_present & (1u << 3)) || !(f.m.reg_present & (1u << 4)) || f.acts.empty() ||
            f.acts[0].kind != ACT_CT_DNAT) {
          *err = "unsupported EndpointDNAT flow: " + f.str();
          return -GPC_EINVAL;
        }
        dnat[{f.m.nw_proto, f.m.reg_v[3], uint16_t(f.m.reg_v[4] & 0xffffu)}] = true;
      } else if (f.table == TB_SERVICE_LB) {
        // a NodePort Service (ToNodePortAddressRegMark, no Service IP) is keyed by address 0
        const bool node_port = (f.m.reg_present & (1u << 4)) && (f.m.reg_m[4] & kToNodePort) && (f.m.reg_v[4] & kToNodePort);
        any_node_port |= node_port;
        Svc s{svc_key(f.m.nw_proto, node_port ? 0u : f.m.nw_dst.addr.v4(), f.m.tp_dst), 0, false};
        bool grp = false;
        for (auto& a : f.acts) {
          if (a.kind == ACT_GROUP) s.gid = a.a, grp = true;
          if (a.kind == ACT_SET_REG && a.a == 7) s.reg7 = true;
        }
        if (!grp || node_port == f.m.nw_dst.set || (f.m.nw_dst.set && f.m.nw_dst.plen >= 0) || !f.m.has_tp_dst ||
            f.m.tp_dst_m != 0xffff) {
          *err = "unsupported ServiceLB flow: " + f.str();
          return -GPC_EINVAL;
        }
        svcs.push_back(s);
      }
    }
  std::vector<uint32_t> svc_words, ep_words;
  std::vector<std::pair<uint64_t, uint32_t>> kv;
  for (auto& s : svcs) {
    uint32_t first = uint32_t(ep_words.size() / 4), n = 0;
    auto git = groups_.find(s.gid);
    if (git != groups_.end()) {
      for (auto& b : git->second.buckets) {
        uint32_t ip = 0, port = 0, flags = 0;
        bool noep = false, to_dnat = false;
        for (auto& a : b.acts) {
          if (a.kind == ACT_SET_REG && a.a == 3) ip = a.b;
          if (a.kind == ACT_SET_REG && a.a == 4 && a.c == 0xffffu) port = a.b;
          if (a.kind == ACT_SET_REG && a.a == 4 && (a.b & kRemoteEndpoint)) flags |= GPC_LB_REMOTE;
          if (a.kind == ACT_SET_REG && a.a == 0 && (a.b & kSvcNoEp)) noep = true;
          if (a.kind == ACT_RESUBMIT) to_dnat = a.a == TB_ENDPOINT_DNAT;
        }
        if (!to_dnat) {
          *err = "unsupported group bucket (session affinity): " + git->second.str();
          return -GPC_EINVAL;
        }
        if (noep) continue;
        auto d = dnat.find({uint8_t((s.key >> 48) & 0xff), ip, uint16_t(port)});
        if (d != dnat.end()) flags |= GPC_LB_DNAT;
        uint32_t out_port = 0, dest = GPC_DEST_GATEWAY;
        auto pit = pods_.find(ip);
        if (pit != pods_.end()) {
          out_port = pit->second;
          dest = GPC_DEST_POD;
        } else if (flags & GPC_LB_REMOTE) {
          dest = GPC_DEST_TUNNEL;
        }
        ep_words.insert(ep_words.end(), {ip, port | (flags << 16), out_port, dest});
        n++;
      }
    }
    uint32_t lg = 6;
    while ((1u << lg) < n) lg++;
    if (n >= (1u << 24)) {
      *err = "too many Endpoints in one group";
      return -GPC_EINVAL;
    }
    kv.push_back({s.key, uint32_t(svc_words.size() / 4)});
    svc_words.insert(svc_words.end(), {first, n | (lg << 24), s.gid, s.reg7 ? kSvcLoadReg7 : 0u});
  }
  SvcHash h;
  if (!h.build(kv)) {
    *err = "Service hash construction failed";
    return -GPC_ENOMEM;
  }
  const uint32_t nb = 1u << h.log2;
  SvcHdr hdr{};
  hdr.map_log2 = 12;  // about 16 map bits per Service: most non-Service packets stop at the map
  while (hdr.map_log2 < 22 && (1ull << hdr.map_log2) < 16ull * kv.size()) hdr.map_log2++;
  hdr.map_off = 32;
  hdr.hash_off = hdr.map_off + (1u << (hdr.map_log2 - 5));  // 128-B aligned
  hdr.hash_log2 = h.log2;
  hdr.svc_off = hdr.hash_off + nb * kSvcBucketWords;
  hdr.n_svc = uint32_t(svc_words.size() / 4);
  hdr.ep_off = hdr.svc_off + uint32_t(svc_words.size());
  hdr.n_ep = uint32_t(ep_words.size() / 4);
  // NodePort addresses: probed only when some ServiceLB flow is a NodePort one
  if (!any_node_port) node_port_addrs.clear();
  if (node_port_addrs.size() > kSvcMaxNodePortAddrs) {
    *err = "too many NodePort addresses";
    return -GPC_EINVAL;
  }
  hdr.np_off = hdr.ep_off + uint32_t(ep_words.size());
  hdr.n_np = uint32_t(node_port_addrs.size());
  blob->assign(hdr.np_off + node_port_addrs.size(), 0u);
  std::copy(node_port_addrs.begin(), node_port_addrs.end(), blob->begin() + hdr.np_off);
  std::memcpy(blob->data(), &hdr, sizeof hdr);
  for (auto& e : kv) {
    const uint32_t mb = svc_map_bit(e.first, hdr.map_log2);
    (*blob)[hdr.map_off + (mb >> 5)] |= 1u << (mb & 31u);
  }
  for (uint32_t b = 0; b < nb; b++) {
    uint32_t* w = blob->data() + hdr.hash_off + size_t(b) * kSvcBucketWords;
    for (uint32_t i = 0; i < kSvcSlots; i++) {
      const uint64_t k = h.keys[size_t(b) * kSvcSlots + i];
      w[kSvcSlotWords * i] = uint32_t(k);
      w[kSvcSlotWords * i + 1] = uint32_t(k >> 32);
      w[kSvcSlotWords * i + 2] = h.vals[size_t(b) * kSvcSlots + i];
    }
  }
  std::copy(svc_words.begin(), svc_words.end(), blob->begin() + hdr.svc_off);
  std::copy(ep_words.begin(), ep_words.end(), blob->begin() + hdr.ep_off);
  return GPC_OK;
}

}  // namespace gpc
