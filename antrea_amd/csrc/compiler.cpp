// Host-side conjunctive-match compiler (see compiler.hpp). Reference anchors are cited per
// function; the structure follows network_policy.go so that change sets and the realized flow
// table are the ones Antrea would send to OVS.
#include "compiler.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <tuple>

namespace gpc {

// ============================================================================ model / text
static const char* kTableNames[TB_COUNT] = {"",
                                            "AntreaPolicyEgressRule",
                                            "EgressRule",
                                            "EgressDefaultRule",
                                            "AntreaPolicyIngressRule",
                                            "IngressRule",
                                            "IngressDefaultRule",
                                            "EgressMetric",
                                            "IngressMetric",
                                            "L3Forwarding",
                                            "ConntrackCommit",
                                            "Output",
                                            "ServiceLB",
                                            "EndpointDNAT",
                                            "SNATMark",
                                            "SNAT",
                                            "IngressSecurityClassifier",
                                            "NodePortMark"};

const char* table_name(uint8_t t) { return t < TB_COUNT ? kTableNames[t] : "?"; }

uint8_t next_table(uint8_t t) {  // pipeline order, pipeline.go:150-176
  switch (t) {
    case TB_AP_EGRESS: return TB_EGRESS;
    case TB_EGRESS: return TB_EGRESS_DEFAULT;
    case TB_EGRESS_DEFAULT: return TB_EGRESS_METRIC;
    case TB_EGRESS_METRIC: return TB_L3_FORWARDING;
    case TB_AP_INGRESS: return TB_INGRESS;
    case TB_INGRESS: return TB_INGRESS_DEFAULT;
    case TB_INGRESS_DEFAULT: return TB_INGRESS_METRIC;
    case TB_INGRESS_METRIC: return TB_CONNTRACK_COMMIT;
    default: return TB_NONE;
  }
}

bool IPAddr::operator<(const IPAddr& o) const {
  if (fam != o.fam) return fam < o.fam;
  return std::memcmp(b, o.b, 16) < 0;
}
bool IPAddr::operator==(const IPAddr& o) const { return fam == o.fam && std::memcmp(b, o.b, 16) == 0; }

IPAddr IPAddr::masked(int plen) const {
  IPAddr r = *this;
  int nbytes = fam == 4 ? 4 : 16;
  for (int i = 0; i < nbytes; i++) {
    int keep = plen - 8 * i;
    uint8_t m = keep >= 8 ? 0xff : keep <= 0 ? 0 : uint8_t(0xff << (8 - keep));
    r.b[i] = b[i] & m;
  }
  for (int i = nbytes; i < 16; i++) r.b[i] = 0;
  return r;
}

std::string IPAddr::str() const {  // net.IP.String()
  char buf[64];
  if (fam == 4) {
    std::snprintf(buf, sizeof buf, "%u.%u.%u.%u", b[0], b[1], b[2], b[3]);
    return buf;
  }
  uint16_t g[8];
  for (int i = 0; i < 8; i++) g[i] = uint16_t(b[2 * i] << 8 | b[2 * i + 1]);
  int best = -1, bestlen = 0;
  for (int i = 0; i < 8;) {
    if (g[i] != 0) { i++; continue; }
    int j = i;
    while (j < 8 && g[j] == 0) j++;
    if (j - i > bestlen) { best = i; bestlen = j - i; }
    i = j;
  }
  if (bestlen < 2) best = -1;
  std::string s;
  for (int i = 0; i < 8; i++) {
    if (i == best) {
      s += "::";
      i += bestlen - 1;
      continue;
    }
    if (!s.empty() && s.back() != ':') s += ":";
    std::snprintf(buf, sizeof buf, "%x", g[i]);
    s += buf;
  }
  return s;
}

static std::string ipmatch_str(const IPMatch& m) {  // utils.go getFieldDataString Ipv4SrcField..
  std::string s = m.addr.str();
  if (m.plen >= 0 && m.plen < m.addr.bits()) s += "/" + std::to_string(m.plen);
  return s;
}

static std::string proto_str(uint16_t eth, uint8_t proto) {  // utils.go:298-354
  if (eth == kEthIP) {
    switch (proto) {
      case 0: return "ip";
      case 6: return "tcp";
      case 17: return "udp";
      case 132: return "sctp";
      case 1: return "icmp";
      case 2: return "igmp";
    }
  } else if (eth == kEthIPv6) {
    switch (proto) {
      case 0: return "ipv6";
      case 6: return "tcp6";
      case 17: return "udp6";
      case 132: return "sctp6";
      case 58: return "icmp6";
    }
  } else if (eth == 0x0806 && proto == 0) {
    return "arp";
  }
  return "";
}

std::string Match::str(uint16_t priority) const {  // getFlowModMatch, utils.go:905-1098
  static const char* cts[8] = {"new", "est", "rel", "rpl", "inv", "trk", "snat", "dnat"};
  char buf[128];
  std::string s = "priority=" + std::to_string(priority);
  if (has_conj) s += ",conj_id=" + std::to_string(conj_id);
  if (has_ct_state) {
    s += ",ct_state=";
    for (int i = 0; i < 8; i++)
      if (ct_mask & (1u << i)) s += std::string((ct_data & (1u << i)) ? "+" : "-") + cts[i];
  }
  if (has_ct_mark) {  // matchCtMarkToString (utils.go:287), Uint32Message data / mask
    if (ct_mark_m == 0xffffffffu) std::snprintf(buf, sizeof buf, ",ct_mark=0x%x", ct_mark_v);
    else std::snprintf(buf, sizeof buf, ",ct_mark=0x%x/0x%x", ct_mark_v, ct_mark_m);
    s += buf;
  }
  if (has_ct_label) {
    std::snprintf(buf, sizeof buf, ",ct_label=0x%llx/0x%llx", (unsigned long long)label_v, (unsigned long long)label_m);
    s += buf;
  }
  if (ct_nw_src.set) s += std::string(ct_nw_src.addr.fam == 4 ? ",ct_nw_src=" : ",ct_ipv6_src=") + ipmatch_str(ct_nw_src);
  if (ct_nw_dst.set) s += std::string(ct_nw_dst.addr.fam == 4 ? ",ct_nw_dst=" : ",ct_ipv6_dst=") + ipmatch_str(ct_nw_dst);
  if (has_dl) s += "," + proto_str(dl_type, has_proto ? nw_proto : 0);
  for (int i = 0; i < 16; i++) {
    if (!(reg_present & (1u << i))) continue;
    if (reg_m[i] == 0xffffffffu)
      std::snprintf(buf, sizeof buf, ",reg%d=0x%x", i, reg_v[i]);
    else
      std::snprintf(buf, sizeof buf, ",reg%d=0x%x/0x%x", i, reg_v[i], reg_m[i]);
    s += buf;
  }
  if (has_tun) s += ",tun_id=" + std::to_string(tun_id);
  if (has_in_port) s += ",in_port=" + std::to_string(in_port);
  if (nw_src.set) s += std::string(nw_src.addr.fam == 4 ? ",nw_src=" : ",ipv6_src=") + ipmatch_str(nw_src);
  if (nw_dst.set) s += std::string(nw_dst.addr.fam == 4 ? ",nw_dst=" : ",ipv6_dst=") + ipmatch_str(nw_dst);
  if (has_icmp_type) s += ",icmp_type=" + std::to_string(icmp_type);
  if (has_icmp_code) s += ",icmp_code=" + std::to_string(icmp_code);
  if (has_tp_src) {
    if (tp_src_m == 0xffff) s += ",tp_src=" + std::to_string(tp_src);
    else { std::snprintf(buf, sizeof buf, ",tp_src=0x%x/0x%x", tp_src, tp_src_m); s += buf; }
  }
  if (has_tp_dst) {
    if (tp_dst_m == 0xffff) s += ",tp_dst=" + std::to_string(tp_dst);
    else { std::snprintf(buf, sizeof buf, ",tp_dst=0x%x/0x%x", tp_dst, tp_dst_m); s += buf; }
  }
  return s;
}

std::string Action::str() const {  // utils.go:600-760 (the subset NP flows use)
  char buf[256];
  switch (kind) {
    case ACT_CONJ:
      std::snprintf(buf, sizeof buf, "conjunction(%u,%u/%u)", a, b, c);
      return buf;
    case ACT_SET_REG:
      if (has_mask) std::snprintf(buf, sizeof buf, "set_field:0x%x/0x%x->reg%u", b, c, a);
      else std::snprintf(buf, sizeof buf, "set_field:0x%x->reg%u", b, a);
      return buf;
    case ACT_CT_COMMIT:
      std::snprintf(buf, sizeof buf, "ct(commit,table=%s,zone=%u,exec(set_field:0x%llx/0x%llx->ct_label))", table_name(uint8_t(a)), b,
                    (unsigned long long)lv, (unsigned long long)lm);
      return buf;
    case ACT_GOTO: return std::string("goto_table:") + table_name(uint8_t(a));
    case ACT_GROUP: return "group:" + std::to_string(a);
    case ACT_DROP: return "drop";
    case ACT_CT_DNAT:  // endpointDNATFlow, pipeline.go:2511-2528
      std::snprintf(buf, sizeof buf,
                    "ct(commit,table=%s,zone=%u,nat(dst=%u.%u.%u.%u:%u),exec(set_field:0x10/0x10->ct_mark,"
                    "move:NXM_NX_REG0[0..3]->NXM_NX_CT_MARK[0..3]))",
                    table_name(uint8_t(a)), b, c >> 24, (c >> 16) & 255u, (c >> 8) & 255u, c & 255u, unsigned(lv));
      return buf;
    case ACT_CT_HAIRPIN:  // podHairpinSNATFlow, pipeline.go:3052-3064
      std::snprintf(buf, sizeof buf, "ct(commit,table=%s,zone=%u,exec(set_field:0x20/0x20->ct_mark,set_field:0x40/0x40->ct_mark))",
                    table_name(uint8_t(a)), b);
      return buf;
    case ACT_RESUBMIT: return std::string("resubmit:") + table_name(uint8_t(a));
    case ACT_METER: return "meter:" + std::to_string(a);
    case ACT_CONTROLLER: {  // nxActionController2ToString (utils.go:800-838)
      std::string ud;
      for (uint32_t i = 0; i < a && i < 4; i++) {
        std::snprintf(buf, sizeof buf, "%s%02x", i ? "." : "", (b >> (8 * i)) & 0xffu);
        ud += buf;
      }
      return "controller(id=" + std::to_string(kControllerId) + ",reason=no_match,userdata=" + ud + ",max_len=65535)";
    }
  }
  return "";
}

std::string Group::str() const {  // ofctrl group text as the reference tests print it (client_test.go:1024-1090)
  std::string s = "group_id=" + std::to_string(id) + ",type=select";
  for (auto& b : buckets) {
    s += ",bucket=bucket_id:" + std::to_string(b.id) + ",weight:" + std::to_string(b.weight) + ",actions=";
    for (size_t i = 0; i < b.acts.size(); i++) s += (i ? "," : "") + b.acts[i].str();
  }
  return s;
}

std::string Flow::str() const {  // FlowModToString, utils.go:1222-1224
  char buf[64];
  std::string s;
  if (cookie) {
    std::snprintf(buf, sizeof buf, "cookie=0x%llx, ", (unsigned long long)cookie);
    s += buf;
  }
  s += std::string("table=") + table_name(table) + ", " + m.str(priority) + " actions=";
  std::string a;
  for (auto& x : acts) {
    if (x.kind == ACT_DROP) continue;
    if (!a.empty()) a += ",";
    a += x.str();
  }
  return s + (a.empty() ? "drop" : a);
}

std::string Flow::identity() const { return std::string(table_name(table)) + "|" + m.str(priority); }

// ============================================================================ port ranges
// PortRange.BitwiseMatch (third_party/networkpolicy/port_range.go:45-132): largest aligned block
// ending inside the range, then recurse left and right. Exact cover, ordered by value.
std::vector<std::pair<uint16_t, uint16_t>> bitwise_match(uint16_t start, uint16_t end) {
  std::vector<std::pair<uint16_t, uint16_t>> out;
  if (start == 0 || end == 0 || start > end) return out;
  if (start == end) {
    out.push_back({start, 0xffff});
    return out;
  }
  uint32_t window = uint32_t(end - start) + 1;
  int bl = int(std::floor(std::log2(double(window))));
  auto get_range = [](uint16_t e, int b, uint32_t* rs, uint32_t* re) {
    uint32_t len = (1u << b) - 1;
    *rs = e & ~len & 0xffff;
    *re = *rs + len;
  };
  uint32_t rs, re;
  get_range(end, bl, &rs, &re);
  while (re > end) get_range(end, --bl, &rs, &re);
  if (start != rs) {
    auto l = bitwise_match(start, uint16_t(rs - 1));
    out.insert(out.end(), l.begin(), l.end());
  }
  out.push_back({uint16_t(rs), uint16_t(0xffff ^ ((1u << bl) - 1))});
  if (end != re) {
    auto r = bitwise_match(uint16_t(re + 1), end);
    out.insert(out.end(), r.begin(), r.end());
  }
  return out;
}

// ============================================================================ match keys
static bool mk_is_ipv6(MatchKeyId k) {
  return (k >= MK_DST_IPV6 && k <= MK_CT_SRC_IPNETV6) || k == MK_TCPV6_DST || k == MK_UDPV6_DST || k == MK_SCTPV6_DST ||
         k == MK_TCPV6_SRC || k == MK_UDPV6_SRC || k == MK_SCTPV6_SRC || k == MK_ICMPV6_TYPE || k == MK_ICMPV6_CODE;
}

static IPAddr addr_ip(const gpc_addr& a) {
  IPAddr ip;
  ip.fam = a.family == 6 ? 6 : 4;
  std::memcpy(ip.b, a.ip, ip.fam == 4 ? 4 : 16);
  return ip;
}

// Address.GetMatchKey + GetValue (network_policy.go:97-307)
static bool address_pair(const gpc_addr& a, bool src, MatchPair* out) {
  bool v6 = a.family == 6;
  MatchValue v;
  switch (a.kind) {
    case GPC_ADDR_IP:
      out->key = src ? (v6 ? MK_SRC_IPV6 : MK_SRC_IP) : (v6 ? MK_DST_IPV6 : MK_DST_IP);
      v.tag = V_IP;
      v.ip = addr_ip(a);
      break;
    case GPC_ADDR_IPNET:
      out->key = src ? (v6 ? MK_SRC_IPNETV6 : MK_SRC_IPNET) : (v6 ? MK_DST_IPNETV6 : MK_DST_IPNET);
      v.tag = V_IPNET;
      v.plen = a.prefix_len;
      if (v.plen > (v6 ? 128 : 32)) return false;
      v.ip = addr_ip(a).masked(v.plen);  // IPNetToNetIPNet normalisation (pkg/util/ip/ip.go:149)
      break;
    case GPC_ADDR_OFPORT:
      out->key = src ? MK_SRC_OFPORT : MK_DST_OFPORT;
      v.tag = V_INT;
      v.u = a.value;
      break;
    case GPC_ADDR_SVC_GROUP:
      out->key = MK_SVC_GROUP;
      v.tag = V_INT;
      v.u = a.value;
      break;
    case GPC_ADDR_CT_IP:
      out->key = src ? (v6 ? MK_CT_SRC_IPV6 : MK_CT_SRC_IP) : (v6 ? MK_CT_DST_IPV6 : MK_CT_DST_IP);
      v.tag = V_IP;
      v.ip = addr_ip(a);
      break;
    case GPC_ADDR_CT_IPNET:
      out->key = src ? (v6 ? MK_CT_SRC_IPNETV6 : MK_CT_SRC_IPNET) : (v6 ? MK_CT_DST_IPNETV6 : MK_CT_DST_IPNET);
      v.tag = V_IPNET;
      v.plen = a.prefix_len;
      if (v.plen > (v6 ? 128 : 32)) return false;
      v.ip = addr_ip(a).masked(v.plen);
      break;
    case GPC_ADDR_LABEL_ID:
      out->key = MK_LABEL_ID;
      v.tag = V_INT;
      v.u = a.value;
      break;
    default:
      return false;
  }
  out->val = v;
  return true;
}

// matchPair.KeyString / generateGlobalMapKey (network_policy.go:336-400). Only the equivalence
// classes matter: an IP and the same IP with a full mask share one key.
std::string ConjMatch::key() const {
  std::string s = "t" + std::to_string(table) + ",p" + std::to_string(has_prio ? prio : kPriorityNormal);
  for (auto& p : pairs) {
    MatchKeyId k = p.key;
    const MatchValue& v = p.val;
    std::string vs;
    switch (v.tag) {
      case V_IP:
        vs = v.ip.str() + "/" + std::to_string(v.ip.bits());
        if (k == MK_DST_IP) k = MK_DST_IPNET;
        else if (k == MK_SRC_IP) k = MK_SRC_IPNET;
        else if (k == MK_DST_IPV6) k = MK_DST_IPNETV6;
        else if (k == MK_SRC_IPV6) k = MK_SRC_IPNETV6;
        break;
      case V_IPNET: vs = v.ip.str() + "/" + std::to_string(v.plen); break;
      case V_BITRANGE: vs = std::to_string(v.u) + "/" + std::to_string(v.mask < 0 ? 65535 : v.mask); break;
      case V_ICMP: vs = v.nil ? "<nil>" : std::to_string(v.u); break;
      case V_CTSTATE: vs = std::to_string(v.u) + "/" + std::to_string(v.mask); break;
      default: vs = std::to_string(v.u); break;
    }
    s += ",k" + std::to_string(int(k)) + "=" + vs;
  }
  return s;
}

std::vector<Clause*> Conjunction::clauses() const {
  std::vector<Clause*> v;
  if (from) v.push_back(from.get());
  if (to) v.push_back(to.get());
  if (svc) v.push_back(svc.get());
  return v;
}

// ============================================================================ FeatureNP
FeatureNP::FeatureNP(const gpc_config& cfg) : cfg_(cfg) {
  if (cfg.ipv4_enabled) ip_protocols_.push_back(4);
  if (cfg.ipv6_enabled) ip_protocols_.push_back(6);
}

static bool egress_table(uint8_t t) { return t == TB_AP_EGRESS || t == TB_EGRESS || t == TB_EGRESS_DEFAULT; }

static void set_proto(Match& m, uint16_t eth, int proto) {  // ofFlowBuilder.MatchProtocol (ofctrl_builder.go:408-446)
  m.has_dl = true;
  m.dl_type = eth;
  if (proto >= 0) {
    m.has_proto = true;
    m.nw_proto = uint8_t(proto);
  }
}

static void ct_new(Match& m, bool set) {
  m.has_ct_state = true;
  m.ct_mask |= 1;
  if (set) m.ct_data |= 1;
  else m.ct_data &= uint8_t(~1u);
}

static void l4_of(MatchKeyId k, uint16_t* eth, int* proto) {
  switch (k) {
    case MK_TCP_DST: case MK_TCP_SRC: *eth = kEthIP; *proto = 6; return;
    case MK_TCPV6_DST: case MK_TCPV6_SRC: *eth = kEthIPv6; *proto = 6; return;
    case MK_UDP_DST: case MK_UDP_SRC: *eth = kEthIP; *proto = 17; return;
    case MK_UDPV6_DST: case MK_UDPV6_SRC: *eth = kEthIPv6; *proto = 17; return;
    case MK_SCTP_DST: case MK_SCTP_SRC: *eth = kEthIP; *proto = 132; return;
    case MK_SCTPV6_DST: case MK_SCTPV6_SRC: *eth = kEthIPv6; *proto = 132; return;
    default: *eth = kEthIP; *proto = -1; return;
  }
}

// featureNetworkPolicy.addFlowMatch (pipeline.go:1896-2000)
void FeatureNP::add_flow_match(Match& m, const MatchPair& p) const {
  const MatchValue& v = p.val;
  auto ipm = [&](IPMatch& f) {
    f.set = true;
    f.addr = v.ip;
    f.plen = v.tag == V_IPNET ? v.plen : -1;
  };
  switch (p.key) {
    case MK_DST_OFPORT: m.set_reg(1, v.u); break;
    case MK_SRC_OFPORT: m.has_in_port = true; m.in_port = v.u; break;
    case MK_DST_IP: case MK_DST_IPNET: set_proto(m, kEthIP, -1); ipm(m.nw_dst); break;
    case MK_DST_IPV6: case MK_DST_IPNETV6: set_proto(m, kEthIPv6, -1); ipm(m.nw_dst); break;
    case MK_SRC_IP: case MK_SRC_IPNET: set_proto(m, kEthIP, -1); ipm(m.nw_src); break;
    case MK_SRC_IPV6: case MK_SRC_IPNETV6: set_proto(m, kEthIPv6, -1); ipm(m.nw_src); break;
    case MK_CT_DST_IP: case MK_CT_DST_IPNET: ct_new(m, true); set_proto(m, kEthIP, -1); ipm(m.ct_nw_dst); break;
    case MK_CT_DST_IPV6: case MK_CT_DST_IPNETV6: ct_new(m, true); set_proto(m, kEthIPv6, -1); ipm(m.ct_nw_dst); break;
    case MK_CT_SRC_IP: case MK_CT_SRC_IPNET: ct_new(m, true); set_proto(m, kEthIP, -1); ipm(m.ct_nw_src); break;
    case MK_CT_SRC_IPV6: case MK_CT_SRC_IPNETV6: ct_new(m, true); set_proto(m, kEthIPv6, -1); ipm(m.ct_nw_src); break;
    case MK_TCP_DST: case MK_TCPV6_DST: case MK_UDP_DST: case MK_UDPV6_DST: case MK_SCTP_DST: case MK_SCTPV6_DST: {
      uint16_t eth; int proto;
      l4_of(p.key, &eth, &proto);
      set_proto(m, eth, proto);
      if (v.u > 0) {
        m.has_tp_dst = true;
        m.tp_dst = uint16_t(v.u);
        m.tp_dst_m = v.mask < 0 ? 0xffff : uint16_t(v.mask);
      }
      break;
    }
    case MK_TCP_SRC: case MK_TCPV6_SRC: case MK_UDP_SRC: case MK_UDPV6_SRC: case MK_SCTP_SRC: case MK_SCTPV6_SRC: {
      uint16_t eth; int proto;
      l4_of(p.key, &eth, &proto);
      set_proto(m, eth, proto);
      if (v.u > 0) {
        m.has_tp_src = true;
        m.tp_src = uint16_t(v.u);
        m.tp_src_m = v.mask < 0 ? 0xffff : uint16_t(v.mask);
      }
      break;
    }
    case MK_ICMP_TYPE: case MK_ICMPV6_TYPE:
      set_proto(m, p.key == MK_ICMP_TYPE ? kEthIP : kEthIPv6, p.key == MK_ICMP_TYPE ? 1 : 58);
      if (!v.nil) { m.has_icmp_type = true; m.icmp_type = uint8_t(v.u); }
      break;
    case MK_ICMP_CODE: case MK_ICMPV6_CODE:
      set_proto(m, p.key == MK_ICMP_CODE ? kEthIP : kEthIPv6, p.key == MK_ICMP_CODE ? 1 : 58);
      if (!v.nil) { m.has_icmp_code = true; m.icmp_code = uint8_t(v.u); }
      break;
    case MK_SVC_GROUP: m.set_reg(7, v.u); break;
    case MK_IGMP: set_proto(m, kEthIP, 2); break;
    case MK_LABEL_ID: m.has_tun = true; m.tun_id = v.u; break;
    case MK_CT_STATE:
      m.has_ct_state = true;
      m.ct_data = uint8_t((m.ct_data & ~uint32_t(v.mask)) | v.u);
      m.ct_mask = uint8_t(m.ct_mask | v.mask);
      break;
  }
}

// conjunctiveMatchFlow (pipeline.go:2019-2037); actions in conj-id order ("deterministic" mode).
Flow FeatureNP::conjunctive_match_flow(const ConjMatch& cm, const std::map<uint32_t, ConjAction>& acts) const {
  Flow f;
  f.table = cm.table;
  f.priority = cm.has_prio ? cm.prio : kPriorityNormal;
  f.cookie = cfg_.cookie;
  for (auto& p : cm.pairs) add_flow_match(f.m, p);
  for (auto& kv : acts) {
    Action a{ACT_CONJ};
    a.a = kv.second.conj_id;
    a.b = kv.second.clause_id;
    a.c = kv.second.n_clause;
    f.acts.push_back(a);
  }
  return f;
}

static Action set_reg(uint32_t reg, uint32_t v, int64_t mask = -1) {
  Action a{ACT_SET_REG};
  a.a = reg;
  a.b = v;
  if (mask >= 0) { a.has_mask = true; a.c = uint32_t(mask); }
  return a;
}
static Action go(uint8_t t) {
  Action a{ACT_GOTO};
  a.a = t;
  return a;
}

// defaultDropFlow (pipeline.go:2040-2065)
Flow FeatureNP::default_drop_flow(uint8_t table, const std::vector<MatchPair>& pairs, bool logging) const {
  Flow f;
  f.table = table;
  f.priority = kPriorityNormal;
  f.cookie = cfg_.cookie;
  for (auto& p : pairs) add_flow_match(f.m, p);
  if (logging || cfg_.enable_deny_tracking) {
    uint32_t ops = (logging ? 1u : 0u) + (cfg_.enable_deny_tracking ? 2u : 0u);
    f.acts = {set_reg(0, 1u << 11, 0x1800), set_reg(0, ops << 25, 0xfe000000u), set_reg(0, 2u << 21, 0x600000),
              set_reg(2, table, 0xff), go(TB_OUTPUT)};
  } else {
    f.acts = {Action{ACT_DROP}};
  }
  return f;
}

// multiClusterNetworkPolicySecurityDropFlow (pipeline.go:2068-2076)
Flow FeatureNP::mcnp_drop_flow(uint8_t table, const std::vector<MatchPair>& pairs) const {
  Flow f;
  f.table = table;
  f.priority = kPriorityNormal;
  f.cookie = cfg_.cookie;
  f.m.has_tun = true;
  f.m.tun_id = kUnknownLabelIdentity;
  for (auto& p : pairs) add_flow_match(f.m, p);
  f.acts = {Action{ACT_DROP}};
  return f;
}

// conjunctionActionFlow (pipeline.go:1718-1808), unicast tables, no L7 redirect.
std::vector<Flow> FeatureNP::conjunction_action_flows(uint32_t id, uint8_t table, uint8_t next, const uint16_t* prio,
                                                      bool logging) const {
  std::vector<Flow> out;
  bool eg = egress_table(table);
  for (uint8_t fam : ip_protocols_) {
    Flow f;
    f.table = table;
    f.priority = prio ? *prio : kPriorityLow;
    f.cookie = cfg_.cookie;
    f.m.has_conj = true;
    f.m.conj_id = id;
    set_proto(f.m, fam == 4 ? kEthIP : kEthIPv6, -1);
    f.acts.push_back(set_reg(eg ? 5 : 6, id));
    Action ct{ACT_CT_COMMIT};
    ct.a = next;
    ct.b = fam == 4 ? kCtZone : kCtZoneV6;
    ct.lv = eg ? (uint64_t(id) << 32) : uint64_t(id);
    ct.lm = eg ? 0xffffffff00000000ull : 0xffffffffull;
    f.acts.push_back(ct);
    if (logging) {
      f.acts.push_back(set_reg(0, 0, 0x1800));
      f.acts.push_back(set_reg(0, 2u << 21, 0x600000));
      f.acts.push_back(set_reg(0, 1u << 25, 0xfe000000u));
      f.acts.push_back(set_reg(2, table, 0xff));
      f.acts.push_back(go(TB_OUTPUT));
    }
    out.push_back(f);
  }
  return out;
}

// conjunctionActionDenyFlow (pipeline.go:1812-1859)
Flow FeatureNP::conjunction_deny_flow(uint32_t id, uint8_t table, uint16_t prio, int disposition, bool logging) const {
  Flow f;
  f.table = table;
  f.priority = prio;
  f.cookie = cfg_.cookie;
  f.m.has_conj = true;
  f.m.conj_id = id;
  uint8_t metric = egress_table(table) ? TB_EGRESS_METRIC : TB_INGRESS_METRIC;
  f.acts = {set_reg(3, id), set_reg(0, 0x400, 0x400)};
  uint32_t ops = 0;
  if (cfg_.enable_deny_tracking) {
    ops += 2;
    f.acts.push_back(set_reg(0, uint32_t(disposition) << 11, 0x1800));
  }
  if (logging) {
    ops += 1;
    f.acts.push_back(set_reg(0, uint32_t(disposition) << 11, 0x1800));
  }
  if (disposition == 2) ops += 4;
  if (logging || cfg_.enable_deny_tracking || disposition == 2) {
    f.acts.push_back(set_reg(0, ops << 25, 0xfe000000u));
    f.acts.push_back(set_reg(2, table, 0xff));
    Action g{ACT_GROUP};
    g.a = metric == TB_EGRESS_METRIC ? kLogGroupEgressMetric : kLogGroupIngressMetric;  // resubmits to the metric table
    f.acts.push_back(g);
  } else {
    f.acts.push_back(go(metric));
  }
  return f;
}

// conjunctionActionPassFlow (pipeline.go:1861-1886)
Flow FeatureNP::conjunction_pass_flow(uint32_t id, uint8_t table, uint16_t prio, bool logging) const {
  Flow f;
  f.table = table;
  f.priority = prio;
  f.cookie = cfg_.cookie;
  f.m.has_conj = true;
  f.m.conj_id = id;
  bool eg = egress_table(table);
  uint8_t next = eg ? TB_EGRESS : TB_INGRESS;
  f.acts = {set_reg(eg ? 5 : 6, id)};
  if (logging) {
    f.acts.push_back(set_reg(0, 3u << 11, 0x1800));
    f.acts.push_back(set_reg(0, 1u << 25, 0xfe000000u));
    f.acts.push_back(set_reg(2, table, 0xff));
    Action g{ACT_GROUP};
    g.a = next == TB_EGRESS ? kLogGroupEgressRule : kLogGroupIngressRule;  // resubmits to the K8s rule table
    f.acts.push_back(g);
  } else {
    f.acts.push_back(go(next));
  }
  return f;
}

// allowRulesMetricFlows (pipeline.go:1604-1651)
std::vector<Flow> FeatureNP::allow_metric_flows(uint32_t id, bool ingress) const {
  std::vector<Flow> out;
  uint8_t metric = ingress ? TB_INGRESS_METRIC : TB_EGRESS_METRIC;
  for (uint8_t fam : ip_protocols_) {
    for (int isnew = 1; isnew >= 0; isnew--) {
      Flow f;
      f.table = metric;
      f.priority = kPriorityNormal;
      f.cookie = cfg_.cookie;
      set_proto(f.m, fam == 4 ? kEthIP : kEthIPv6, -1);
      ct_new(f.m, isnew);
      f.m.has_ct_label = true;
      f.m.label_v = ingress ? uint64_t(id) : (uint64_t(id) << 32);
      f.m.label_m = ingress ? 0xffffffffull : 0xffffffff00000000ull;
      f.acts = {go(next_table(metric))};
      out.push_back(f);
    }
  }
  return out;
}

// denyRuleMetricFlow (pipeline.go:1653-1670)
Flow FeatureNP::deny_metric_flow(uint32_t id, bool ingress) const {
  Flow f;
  f.table = ingress ? TB_INGRESS_METRIC : TB_EGRESS_METRIC;
  f.priority = kPriorityNormal;
  f.cookie = cfg_.cookie;
  f.m.set_reg(0, 0x400, 0x400);
  f.m.set_reg(3, id);
  f.acts = {Action{ACT_DROP}};
  return f;
}

// ---------------------------------------------------------------------------- OVS stand-in
static bool is_rule_table(uint8_t t) { return t >= TB_AP_EGRESS && t <= TB_INGRESS_DEFAULT; }
static bool is_hard_flow(const Flow& f) { return is_rule_table(f.table) && !f.m.has_conj && !f.is_soft(); }

// Which image rule a flow belongs to (image.cpp gathers exactly these kinds).
void FeatureNP::note_flow(const Flow& f) {
  if (is_rule_table(f.table)) {
    if (f.m.has_conj) {
      dirty_.conj.insert(f.m.conj_id);
    } else if (f.is_soft()) {
      for (auto& a : f.acts) dirty_.conj.insert(a.a);
    } else {
      dirty_.hard_tables |= uint8_t(1u << (f.table - 1));
    }
  } else if (f.table == TB_INGRESS_CLASSIFIER) {
    dirty_.hard_tables |= kDirtyClassifier;  // ImageHdr.isc changes: the next commit rebuilds
  } else if (f.table == TB_EGRESS_METRIC || f.table == TB_INGRESS_METRIC) {
    const Match& m = f.m;
    if (m.has_ct_label) dirty_.conj.insert(f.table == TB_INGRESS_METRIC ? uint32_t(m.label_v & 0xffffffffu) : uint32_t(m.label_v >> 32));
    if (m.reg_present & (1u << 3)) dirty_.conj.insert(m.reg_v[3]);
  }
}

void FeatureNP::note_change(const Flow& old, const Flow& nw) {
  if (is_rule_table(nw.table) && old.is_soft() && nw.is_soft()) {  // context flow: actions added / removed
    auto key = [](const Action& a) { return std::make_tuple(a.a, a.b, a.c); };
    std::set<std::tuple<uint32_t, uint32_t, uint32_t>> o, n;
    for (auto& a : old.acts) o.insert(key(a));
    for (auto& a : nw.acts) n.insert(key(a));
    for (auto& k : o)
      if (!n.count(k)) dirty_.conj.insert(std::get<0>(k));
    for (auto& k : n)
      if (!o.count(k)) dirty_.conj.insert(std::get<0>(k));
    return;
  }
  note_flow(old);
  note_flow(nw);
}

void FeatureNP::apply_bundle(std::vector<const Flow*> add, std::vector<const Flow*> del) {
  for (auto* f : del) {
    auto it = installed_.find(f->identity());
    if (it == installed_.end()) continue;
    note_flow(it->second);
    if (is_hard_flow(it->second)) hard_.erase(it->first);
    installed_.erase(it);
  }
  for (auto* f : add) {
    std::string id = f->identity();
    auto it = installed_.find(id);
    if (it != installed_.end()) {
      note_change(it->second, *f);
      if (is_hard_flow(it->second)) hard_.erase(id);
      it->second = *f;
    } else {
      note_flow(*f);
      it = installed_.emplace(std::move(id), *f).first;
    }
    if (is_hard_flow(*f)) hard_[it->first] = *f;
  }
  generation_++;
}

int FeatureNP::load_flows(const std::vector<Flow>& flows, bool replace) {
  std::vector<const Flow*> add, del;
  std::vector<Flow> old;
  if (replace) {
    old.reserve(installed_.size());
    for (auto& kv : installed_) old.push_back(kv.second);
    for (auto& f : old) del.push_back(&f);
    global_cache_.clear();
    policy_cache_.clear();
  }
  for (auto& f : flows) add.push_back(&f);
  apply_bundle(add, del);
  foreign_ = true;
  return GPC_OK;
}

// featureNetworkPolicy.initFlows (network_policy.go:2126-2142): ingressClassifierFlows on a K8s
// Node (pipeline.go:2144-2182), skipPolicyRuleCheckFlows (network_policy.go:2167-2211) and
// initLoggingFlows (:2249-2269).
int FeatureNP::initialize() {
  uint8_t eg = TB_EGRESS, in = TB_INGRESS;
  uint16_t prio = kPriorityHigh;
  if (cfg_.enable_antrea_policy) {
    eg = TB_AP_EGRESS;
    in = TB_AP_INGRESS;
    prio = kPriorityTopAntreaPolicy;
  }
  std::vector<Flow> flows;
  if (!cfg_.external_node) {
    for (uint32_t mark : {kToGatewayMark, kToTunnelMark, kToUplinkMark}) {
      Flow f;
      f.table = TB_INGRESS_CLASSIFIER;
      f.priority = kPriorityNormal;
      f.cookie = cfg_.cookie;
      f.m.set_reg(0, mark, 0xf0);
      f.acts = {go(TB_INGRESS_METRIC)};
      flows.push_back(f);
    }
    Flow h;  // hairpin Service connections skip to stageConntrack
    h.table = TB_INGRESS_CLASSIFIER;
    h.priority = kPriorityNormal;
    h.cookie = cfg_.cookie;
    h.m.has_ct_mark = true;
    h.m.ct_mark_v = h.m.ct_mark_m = kHairpinCTMark;
    h.acts = {go(TB_CONNTRACK_COMMIT)};
    flows.push_back(h);
  }
  for (uint32_t ops = 1; ops <= 7; ops++) {  // logging | store-deny | reject operations -> packet-in
    Flow f;
    f.table = TB_OUTPUT;
    f.priority = kPriorityNormal;
    f.cookie = cfg_.cookie;
    f.m.set_reg(0, (ops << 25) | (2u << 21), 0xfe600000u);
    if (cfg_.ovs_meters) {
      Action m{ACT_METER};
      m.a = kMeterNP;
      f.acts.push_back(m);
    }
    Action c{ACT_CONTROLLER};
    c.a = 2;
    c.b = kPacketInCategoryNP | (ops << 8);
    f.acts.push_back(c);
    flows.push_back(f);
  }
  for (uint8_t fam : ip_protocols_) {
    for (auto tm : {std::make_pair(eg, uint8_t(TB_EGRESS_METRIC)), std::make_pair(in, uint8_t(TB_INGRESS_METRIC))}) {
      for (int bit : {1, 2}) {  // est, rel
        Flow f;
        f.table = tm.first;
        f.priority = prio;
        f.cookie = cfg_.cookie;
        set_proto(f.m, fam == 4 ? kEthIP : kEthIPv6, -1);
        f.m.has_ct_state = true;
        f.m.ct_data = uint8_t(1u << bit);
        f.m.ct_mask = uint8_t(1u | (1u << bit));
        f.acts = {go(tm.second)};
        flows.push_back(f);
      }
    }
  }
  std::vector<const Flow*> add;
  for (auto& f : flows) add.push_back(&f);
  apply_bundle(add, {});
  return GPC_OK;
}

// ---------------------------------------------------------------------------- clause logic
// clause.addConjunctiveMatchFlow (network_policy.go:791-864)
bool FeatureNP::add_conj_match_flow(Clause* cl, const ConjMatch& m, bool logging, bool mcnp, CtxChange* ch) {
  std::string key = m.key();
  if (cl->matches.count(key)) return false;
  CtxPtr ctx;
  auto it = global_cache_.find(key);
  FlowChange::Type ctx_type = FlowChange::MODIFY;
  bool has_drop = false;
  FlowChange drop;
  if (it == global_cache_.end()) {
    ctx = std::make_shared<Context>();
    ctx->match = m;
    ctx->drop_logging = logging;
    ctx_type = FlowChange::INSERT;
    if (cl->drop_table && !ctx->drop_flow) {
      has_drop = true;
      drop.type = FlowChange::INSERT;
      drop.flow.reset(new Flow(mcnp ? mcnp_drop_flow(cl->drop_table, m.pairs) : default_drop_flow(cl->drop_table, m.pairs, logging)));
    }
  } else {
    ctx = it->second;
    if (ctx->drop_logging != logging) {
      ctx->drop_logging = logging;
      if (cl->drop_table && ctx->drop_flow) {
        has_drop = true;
        drop.type = FlowChange::MODIFY;
        drop.flow.reset(new Flow(default_drop_flow(cl->drop_table, m.pairs, logging)));
      }
    }
  }
  ch->ctx = ctx;
  ch->ctx_type = ctx_type;
  ch->clause = cl;
  ch->act_type = FlowChange::INSERT;
  ch->has_drop = has_drop;
  if (has_drop) ch->drop_flow = std::move(drop);
  if (cl->action.n_clause > 1) {
    if (!ctx->actions.count(cl->action.conj_id)) {  // context.addAction
      auto acts = ctx->actions;
      acts[cl->action.conj_id] = cl->action;
      ch->has_match_flow = true;
      ch->match_flow.type = ctx->flow ? FlowChange::MODIFY : FlowChange::INSERT;
      ch->match_flow.flow.reset(new Flow(conjunctive_match_flow(ctx->match, acts)));
      ch->has_act = true;
      ch->act = cl->action;
    }
  } else {
    ch->has_match_flow = true;
    ch->match_flow.type = FlowChange::INSERT;  // DENY-ALL bookkeeping, no flow
  }
  return true;
}

// clause.deleteConjunctiveMatchFlow (network_policy.go:1049-1098)
bool FeatureNP::del_conj_match_flow(Clause* cl, const std::string& key, CtxChange* ch) {
  auto it = cl->matches.find(key);
  if (it == cl->matches.end()) return false;
  CtxPtr ctx = it->second;
  ch->ctx = ctx;
  ch->clause = cl;
  ch->ctx_type = FlowChange::MODIFY;
  ch->act_type = FlowChange::DELETE;
  uint32_t id = cl->action.conj_id;
  size_t n_actions = ctx->actions.size(), n_deny = ctx->deny_all.size();
  if (cl->action.n_clause > 1) {
    auto ait = ctx->actions.find(id);
    if (ait != ctx->actions.end()) {
      // conjMatchFlowContext.deleteAction (network_policy.go:496-514)
      if (ctx->actions.size() == 1 && ctx->flow) {
        ch->has_match_flow = true;
        ch->match_flow.type = FlowChange::DELETE;
        ch->match_flow.flow.reset(new Flow(*ctx->flow));
      } else {
        auto acts = ctx->actions;
        acts.erase(id);
        if (!(acts.empty() && !ctx->flow)) {
          ch->has_match_flow = true;
          ch->match_flow.type = ctx->flow ? FlowChange::MODIFY : FlowChange::INSERT;
          ch->match_flow.flow.reset(new Flow(conjunctive_match_flow(ctx->match, acts)));
        }
      }
      ch->has_act = true;
      ch->act = ait->second;
      n_actions--;
    }
  } else {
    ch->has_match_flow = true;
    ch->match_flow.type = FlowChange::DELETE;
    n_deny--;
  }
  if (n_actions == 0 && n_deny == 0) {
    if (ctx->drop_flow) {
      ch->has_drop = true;
      ch->drop_flow.type = FlowChange::DELETE;
      ch->drop_flow.flow.reset(new Flow(*ctx->drop_flow));
    }
    ch->ctx_type = FlowChange::DELETE;
  }
  return true;
}

// conjMatchFlowContextChange.updateContextStatus (network_policy.go:583-646)
void FeatureNP::update_context_status(CtxChange& ch) {
  Context& ctx = *ch.ctx;
  std::string key = ctx.match.key();
  if (ch.act_type == FlowChange::INSERT) {
    ch.clause->matches[key] = ch.ctx;
    if (ch.has_act) ctx.actions[ch.act.conj_id] = ch.act;
  } else {
    ch.clause->matches.erase(key);
    if (ch.has_act) ctx.actions.erase(ch.act.conj_id);
  }
  if (ch.has_match_flow) {
    auto& mf = ch.match_flow;
    if (mf.type == FlowChange::INSERT || mf.type == FlowChange::MODIFY) {
      if (mf.flow) ctx.flow.reset(new Flow(*mf.flow));
      else if (ch.act_type == FlowChange::INSERT) ctx.deny_all[ch.clause->action.conj_id] = true;
      else ctx.deny_all.erase(ch.clause->action.conj_id);
    } else {
      if (mf.flow) ctx.flow.reset();
      else ctx.deny_all.erase(ch.clause->action.conj_id);
    }
  }
  if (ch.has_drop) {
    if (ch.drop_flow.type == FlowChange::INSERT) ctx.drop_flow.reset(new Flow(*ch.drop_flow.flow));
    else if (ch.drop_flow.type == FlowChange::DELETE) ctx.drop_flow.reset();
  }
  if (ch.ctx_type == FlowChange::INSERT) global_cache_[key] = ch.ctx;
  else if (ch.ctx_type == FlowChange::DELETE) global_cache_.erase(key);
}

// applyConjunctiveMatchFlows + sendConjunctiveFlows (network_policy.go:1359-1396)
void FeatureNP::apply_changes(std::vector<CtxChange>& chs) {
  std::vector<const Flow*> add, del;
  for (auto& ch : chs) {
    for (FlowChange* fc : {ch.has_match_flow ? &ch.match_flow : nullptr, ch.has_drop ? &ch.drop_flow : nullptr}) {
      if (!fc || !fc->flow) continue;
      if (fc->type == FlowChange::DELETE) del.push_back(fc->flow.get());
      else add.push_back(fc->flow.get());
    }
  }
  apply_bundle(add, del);
  for (auto& ch : chs) update_context_status(ch);
}

static bool contains_label_identity(const gpc_addr* a, int32_t n) {
  for (int32_t i = 0; i < n; i++)
    if (a[i].kind == GPC_ADDR_LABEL_ID) return true;
  return false;
}

static bool is_anp(const gpc_rule& r) { return r.policy_type != GPC_POLICY_K8S; }

// policyRuleConjunction.calculateClauses (network_policy.go:1423-1472)
void FeatureNP::calculate_clauses(Conjunction& c, const gpc_rule& r) {
  bool eg = r.direction == GPC_DIR_OUT;
  uint8_t drop_table = eg ? TB_EGRESS_DEFAULT : TB_INGRESS_DEFAULT;
  uint8_t n = 0, fid = 0, tid = 0, sid = 0;
  if (r.n_from >= 0) fid = ++n;
  if (r.n_to >= 0) tid = ++n;
  if (r.n_service >= 0) sid = ++n;
  auto mk = [&](uint8_t id, uint8_t dt) {
    auto cl = std::make_unique<Clause>();
    cl->action.conj_id = c.id;
    cl->action.clause_id = id;
    cl->action.n_clause = n;
    cl->rule_table = r.table;
    cl->drop_table = dt;
    return cl;
  };
  if (r.n_from >= 0) c.from = mk(fid, (!eg || is_anp(r)) ? 0 : drop_table);
  if (r.n_to >= 0) {
    bool none = eg || (is_anp(r) && !contains_label_identity(r.from, r.n_from));
    c.to = mk(tid, none ? 0 : drop_table);
  }
  if (r.n_service >= 0) c.svc = mk(sid, 0);
}

// calculateActionFlowChangesForRule (network_policy.go:1186-1228)
ConjPtr FeatureNP::calculate_action_flows(const gpc_rule& r, int* err) {
  *err = GPC_OK;
  if (policy_cache_.count(r.flow_id)) return nullptr;
  if (r.table < TB_AP_EGRESS || r.table > TB_INGRESS_DEFAULT) {
    *err = GPC_EINVAL;
    return nullptr;
  }
  auto c = std::make_shared<Conjunction>();
  c->id = r.flow_id;
  c->has_ref = true;
  c->policy_type = r.policy_type;
  c->ns = r.policy_namespace ? r.policy_namespace : "";
  c->pname = r.policy_name ? r.policy_name : "";
  c->uid = r.policy_uid ? r.policy_uid : "";
  c->rule_name = r.name ? r.name : "";
  c->log_label = r.log_label ? r.log_label : "";
  c->tier = r.tier_priority;
  calculate_clauses(*c, r);
  c->rule_table = r.table;
  int n = (r.n_from >= 0) + (r.n_to >= 0) + (r.n_service >= 0);
  bool ingress = !egress_table(r.table);
  uint8_t drop_table = r.direction == GPC_DIR_OUT ? TB_EGRESS_DEFAULT : TB_INGRESS_DEFAULT;
  const uint16_t* prio = r.has_priority ? &r.priority : nullptr;
  if (n > 1) {
    if (is_anp(r) && (r.action == GPC_RULE_DROP || r.action == GPC_RULE_REJECT || r.action == GPC_RULE_PASS) && !prio) {
      *err = GPC_EINVAL;  // Antrea-native deny/pass flows dereference rule.Priority
      return nullptr;
    }
    if (is_anp(r) && r.action == GPC_RULE_DROP) {
      c->metric_flows.push_back(deny_metric_flow(c->id, ingress));
      c->action_flows.push_back(conjunction_deny_flow(c->id, r.table, *prio, 1, r.enable_logging));
    } else if (is_anp(r) && r.action == GPC_RULE_REJECT) {
      c->metric_flows.push_back(deny_metric_flow(c->id, ingress));
      c->action_flows.push_back(conjunction_deny_flow(c->id, r.table, *prio, 2, r.enable_logging));
    } else if (is_anp(r) && r.action == GPC_RULE_PASS) {
      if (r.table == TB_EGRESS_DEFAULT || r.table == TB_INGRESS_DEFAULT) {
        *err = GPC_EINVAL;  // goto_table to a lower table is rejected by OVS (Pass is not allowed in the baseline tier)
        return nullptr;
      }
      c->action_flows.push_back(conjunction_pass_flow(c->id, r.table, *prio, r.enable_logging));
    } else {
      c->metric_flows = allow_metric_flows(c->id, ingress);
      c->action_flows = conjunction_action_flows(c->id, r.table, next_table(drop_table), prio, r.enable_logging);
    }
  }
  return c;
}

static bool service_pairs(const gpc_service& s, const std::vector<uint8_t>& fams, std::vector<std::vector<MatchPair>>* out);

std::vector<std::pair<Clause*, ConjMatch>> FeatureNP::rule_matches(const Conjunction& c, const gpc_rule& r, int* err) const {
  std::vector<std::pair<Clause*, ConjMatch>> out;
  *err = GPC_OK;
  auto mk = [&](uint8_t table) {
    ConjMatch m;
    m.table = table;
    m.has_prio = r.has_priority;
    m.prio = r.priority;
    return m;
  };
  if (c.from) {
    for (int32_t i = 0; i < r.n_from; i++) {
      ConjMatch m = mk(c.from->rule_table);
      MatchPair p;
      if (!address_pair(r.from[i], true, &p)) { *err = GPC_EINVAL; return out; }
      m.pairs.push_back(p);
      out.push_back({c.from.get(), m});
    }
  }
  if (c.to) {
    for (int32_t i = 0; i < r.n_to; i++) {
      ConjMatch m = mk(c.to->rule_table);
      MatchPair p;
      if (!address_pair(r.to[i], false, &p)) { *err = GPC_EINVAL; return out; }
      m.pairs.push_back(p);
      out.push_back({c.to.get(), m});
    }
  }
  if (c.svc) {
    for (int32_t i = 0; i < r.n_service; i++) {
      std::vector<std::vector<MatchPair>> pp;
      if (!service_pairs(r.service[i], ip_protocols_, &pp)) { *err = GPC_EINVAL; return out; }
      for (auto& pairs : pp) {
        ConjMatch m = mk(c.svc->rule_table);
        m.pairs = pairs;
        out.push_back({c.svc.get(), m});
      }
    }
  }
  return out;
}

// portsToBitRanges (network_policy.go:986-1017): BitRange list as MatchValues
static std::vector<MatchValue> ports_to_bit_ranges(bool has_port, uint16_t port, bool has_end, uint16_t end) {
  std::vector<MatchValue> out;
  if (has_end && has_port && end > port) {
    for (auto& br : bitwise_match(port, end)) {
      MatchValue v;
      v.tag = V_BITRANGE;
      v.u = br.first;
      v.mask = br.second;
      out.push_back(v);
    }
  } else {
    MatchValue v;
    v.tag = V_BITRANGE;
    v.u = has_port ? port : 0;
    v.mask = -1;
    out.push_back(v);
  }
  return out;
}

// getServiceMatchPairs (network_policy.go:891-983)
static bool service_pairs(const gpc_service& s, const std::vector<uint8_t>& fams, std::vector<std::vector<MatchPair>>* out) {
  auto dst = ports_to_bit_ranges(s.has_port, s.port, s.has_end_port, s.end_port);
  std::vector<MatchValue> src;
  bool has_src = s.has_src_port;
  if (has_src) src = ports_to_bit_ranges(true, s.src_port, s.has_src_end_port, s.src_end_port);
  auto add_l4 = [&](MatchKeyId dk, MatchKeyId sk) {
    for (auto& d : dst) {
      std::vector<MatchPair> pairs{{dk, d}};
      if (has_src) {
        for (auto& sr : src) {  // Go appends to the same slice per src range (network_policy.go:902-906)
          pairs.push_back({sk, sr});
          out->push_back(pairs);
        }
      } else {
        out->push_back(pairs);
      }
    }
  };
  switch (s.protocol) {
    case GPC_PROTO_UDP:
      for (auto f : fams) f == 4 ? add_l4(MK_UDP_DST, MK_UDP_SRC) : add_l4(MK_UDPV6_DST, MK_UDPV6_SRC);
      break;
    case GPC_PROTO_SCTP:
      for (auto f : fams) f == 4 ? add_l4(MK_SCTP_DST, MK_SCTP_SRC) : add_l4(MK_SCTPV6_DST, MK_SCTPV6_SRC);
      break;
    case GPC_PROTO_ICMP:
      for (auto f : fams) {
        std::vector<MatchPair> pairs;
        MatchKeyId tk = f == 4 ? MK_ICMP_TYPE : MK_ICMPV6_TYPE, ck = f == 4 ? MK_ICMP_CODE : MK_ICMPV6_CODE;
        if (s.has_icmp_type) { MatchValue v; v.tag = V_ICMP; v.u = uint32_t(s.icmp_type); pairs.push_back({tk, v}); }
        if (s.has_icmp_code) { MatchValue v; v.tag = V_ICMP; v.u = uint32_t(s.icmp_code); pairs.push_back({ck, v}); }
        if (pairs.empty()) { MatchValue v; v.tag = V_ICMP; v.nil = true; pairs.push_back({tk, v}); }
        out->push_back(pairs);
      }
      break;
    case GPC_PROTO_IGMP:
      if (s.has_igmp_type && s.igmp_type == 0x11) {  // IGMPQuery
        MatchValue ip;
        ip.tag = V_IP;
        ip.ip.fam = 4;
        if (s.has_group_address) std::memcpy(ip.ip.b, s.group_address, 4);
        else { ip.ip.b[0] = 224; ip.ip.b[1] = 0; ip.ip.b[2] = 0; ip.ip.b[3] = 1; }  // types.McastAllHosts
        MatchValue none;
        out->push_back({{MK_DST_IP, ip}, {MK_IGMP, none}});
      }
      break;
    case GPC_PROTO_TCP:
    case GPC_PROTO_NONE:
    default:
      if (s.protocol == GPC_PROTO_TCP) {
        for (auto f : fams) f == 4 ? add_l4(MK_TCP_DST, MK_TCP_SRC) : add_l4(MK_TCPV6_DST, MK_TCPV6_SRC);
      } else {
        add_l4(MK_TCP_DST, MK_TCP_SRC);
      }
      break;
  }
  return true;
}

// InstallPolicyRuleFlows (network_policy.go:1160-1183)
int FeatureNP::install_rule(const gpc_rule& r) {
  int err;
  ConjPtr c = calculate_action_flows(r, &err);
  if (err) return -err;
  if (!c) return GPC_OK;  // already installed
  bool mcnp = contains_label_identity(r.from, r.n_from);
  auto ms = rule_matches(*c, r, &err);
  if (err) return -err;
  std::vector<CtxChange> chs;
  for (auto& cm : ms) {
    CtxChange ch;
    if (add_conj_match_flow(cm.first, cm.second, r.enable_logging, mcnp, &ch)) chs.push_back(std::move(ch));
  }
  std::vector<const Flow*> add;
  for (auto& f : c->metric_flows) add.push_back(&f);
  for (auto& f : c->action_flows) add.push_back(&f);
  apply_bundle(add, {});
  apply_changes(chs);
  policy_cache_[c->id] = c;
  return GPC_OK;
}

// BatchInstallPolicyRuleFlows (network_policy.go:1310-1356)
int FeatureNP::batch_install(const gpc_rule* rules, size_t n) {
  std::vector<ConjPtr> conjs;
  std::vector<const Flow*> all;
  for (size_t i = 0; i < n; i++) {
    const gpc_rule& r = rules[i];
    int err;
    ConjPtr c = calculate_action_flows(r, &err);
    if (err) return -err;
    if (!c) continue;
    bool mcnp = contains_label_identity(r.from, r.n_from);
    auto ms = rule_matches(*c, r, &err);
    if (err) return -err;
    for (auto& cm : ms) {  // addActionToConjunctiveMatch (network_policy.go:1267-1304)
      Clause* cl = cm.first;
      std::string key = cm.second.key();
      if (cl->matches.count(key)) continue;
      CtxPtr ctx;
      auto it = global_cache_.find(key);
      if (it == global_cache_.end()) {
        ctx = std::make_shared<Context>();
        ctx->match = cm.second;
        ctx->drop_logging = r.enable_logging;
        if (cl->drop_table)
          ctx->drop_flow.reset(new Flow(mcnp ? mcnp_drop_flow(cl->drop_table, cm.second.pairs)
                                             : default_drop_flow(cl->drop_table, cm.second.pairs, r.enable_logging)));
        global_cache_[key] = ctx;
      } else {
        ctx = it->second;
      }
      cl->matches[key] = ctx;
      if (cl->action.n_clause > 1) ctx->actions[cl->action.conj_id] = cl->action;
      else ctx->deny_all[cl->action.conj_id] = true;
    }
    conjs.push_back(c);
  }
  for (auto& c : conjs) {
    for (auto& f : c->action_flows) all.push_back(&f);
    for (auto& f : c->metric_flows) all.push_back(&f);
  }
  for (auto& kv : global_cache_) {
    Context& ctx = *kv.second;
    if (!ctx.actions.empty()) {
      ctx.flow.reset(new Flow(conjunctive_match_flow(ctx.match, ctx.actions)));
      all.push_back(ctx.flow.get());
    }
    if (ctx.drop_flow) all.push_back(ctx.drop_flow.get());
  }
  apply_bundle(all, {});
  for (auto& c : conjs) policy_cache_[c->id] = c;
  return GPC_OK;
}

// getStalePriorities (network_policy.go:1599-1624)
std::vector<uint16_t> FeatureNP::stale_priorities(const Conjunction& c) const {
  std::vector<uint16_t> stale;
  if (c.rule_table == TB_INGRESS || c.rule_table == TB_EGRESS) return stale;
  for (auto& f : c.action_flows) {
    bool is_stale = true;
    for (auto& kv : policy_cache_) {
      const Conjunction& o = *kv.second;
      if (o.id == c.id || o.rule_table != c.rule_table) continue;
      for (auto& of : o.action_flows)
        if (of.priority == f.priority) is_stale = false;
      if (!is_stale) break;
    }
    if (is_stale) stale.push_back(f.priority);
  }
  return stale;
}

// UninstallPolicyRuleFlows (network_policy.go:1570-1595)
int FeatureNP::uninstall_rule(uint32_t id, std::vector<uint16_t>* stale) {
  auto it = policy_cache_.find(id);
  if (it == policy_cache_.end()) return GPC_OK;
  ConjPtr c = it->second;
  if (stale) *stale = stale_priorities(*c);
  std::vector<const Flow*> del;
  for (auto& f : c->action_flows) del.push_back(&f);
  for (auto& f : c->metric_flows) del.push_back(&f);
  apply_bundle({}, del);
  std::vector<CtxChange> chs;
  for (Clause* cl : c->clauses()) {
    std::vector<std::string> keys;
    for (auto& kv : cl->matches) keys.push_back(kv.first);
    for (auto& k : keys) {
      CtxChange ch;
      if (del_conj_match_flow(cl, k, &ch)) chs.push_back(std::move(ch));
    }
  }
  apply_changes(chs);
  policy_cache_.erase(id);
  return GPC_OK;
}

// AddPolicyRuleAddress (network_policy.go:1661-1682)
int FeatureNP::add_rule_addrs(uint32_t id, int addr_type, const gpc_addr* a, size_t n, const uint16_t* prio, bool logging,
                              bool mcnp) {
  auto it = policy_cache_.find(id);
  if (it == policy_cache_.end()) return -GPC_ENOTFOUND;
  Clause* cl = addr_type == GPC_SRC_ADDRESS ? it->second->from.get() : addr_type == GPC_DST_ADDRESS ? it->second->to.get() : nullptr;
  if (!cl) return -GPC_ENOCLAUSE;
  std::vector<CtxChange> chs;
  for (size_t i = 0; i < n; i++) {
    ConjMatch m;
    m.table = cl->rule_table;
    m.has_prio = prio != nullptr;
    m.prio = prio ? *prio : 0;
    MatchPair p;
    if (!address_pair(a[i], addr_type == GPC_SRC_ADDRESS, &p)) return -GPC_EINVAL;
    m.pairs.push_back(p);
    CtxChange ch;
    if (add_conj_match_flow(cl, m, logging, mcnp, &ch)) chs.push_back(std::move(ch));
  }
  apply_changes(chs);
  return GPC_OK;
}

// DeletePolicyRuleAddress (network_policy.go:1686-1710)
int FeatureNP::del_rule_addrs(uint32_t id, int addr_type, const gpc_addr* a, size_t n, const uint16_t* prio) {
  auto it = policy_cache_.find(id);
  if (it == policy_cache_.end()) return -GPC_ENOTFOUND;
  Clause* cl = addr_type == GPC_SRC_ADDRESS ? it->second->from.get() : addr_type == GPC_DST_ADDRESS ? it->second->to.get() : nullptr;
  if (!cl) return -GPC_ENOCLAUSE;
  std::vector<CtxChange> chs;
  for (size_t i = 0; i < n; i++) {
    ConjMatch m;
    m.table = cl->rule_table;
    m.has_prio = prio != nullptr;
    m.prio = prio ? *prio : 0;
    MatchPair p;
    if (!address_pair(a[i], addr_type == GPC_SRC_ADDRESS, &p)) return -GPC_EINVAL;
    m.pairs.push_back(p);
    CtxChange ch;
    if (del_conj_match_flow(cl, m.key(), &ch)) chs.push_back(std::move(ch));
  }
  apply_changes(chs);
  return GPC_OK;
}

// ReassignFlowPriorities (network_policy.go:1746-1889): end state of the bundle.
int FeatureNP::reassign_priorities(const uint16_t* from, const uint16_t* to, size_t n, uint8_t table) {
  struct Move {
    ConjPtr c;
    uint16_t to;
  };
  std::vector<Move> moves;
  std::vector<Flow> adds;
  std::vector<Flow> dels;
  for (size_t i = 0; i < n; i++) {
    for (auto& kv : policy_cache_) {
      ConjPtr c = kv.second;
      if (c->rule_table != table) continue;
      bool hit = false;
      for (auto& f : c->action_flows) {
        if (f.priority == from[i]) {
          Flow nf = f;
          nf.priority = to[i];
          adds.push_back(nf);
          dels.push_back(f);
          hit = true;
        }
      }
      if (!hit) continue;
      for (Clause* cl : c->clauses())
        for (auto& m : cl->matches)
          if (m.second->flow) {
            Flow nf = *m.second->flow;
            nf.priority = to[i];
            adds.push_back(nf);
            dels.push_back(*m.second->flow);
          }
      moves.push_back({c, to[i]});
    }
  }
  // processFlowUpdates: a delete colliding with an add becomes a modification
  std::set<std::string> add_ids;
  for (auto& f : adds) add_ids.insert(f.identity());
  std::vector<const Flow*> a, d;
  for (auto& f : dels)
    if (!add_ids.count(f.identity())) d.push_back(&f);
  for (auto& f : adds) a.push_back(&f);
  apply_bundle(a, d);
  for (auto& mv : moves) {
    Conjunction& c = *mv.c;
    for (auto& f : c.action_flows) f.priority = mv.to;  // every action flow of c had the original priority
    for (Clause* cl : c.clauses()) {
      std::map<std::string, CtxPtr> nm;
      for (auto& kv : cl->matches) {
        global_cache_.erase(kv.second->match.key());
        if (kv.second->flow) kv.second->flow->priority = mv.to;
        kv.second->match.has_prio = true;
        kv.second->match.prio = mv.to;
      }
      for (auto& kv : cl->matches) {
        nm[kv.second->match.key()] = kv.second;
        global_cache_[kv.second->match.key()] = kv.second;
      }
      cl->matches = nm;
    }
  }
  return GPC_OK;
}

// GetPolicyInfoFromConjunction (network_policy.go:1555-1565)
int FeatureNP::policy_info(uint32_t id, gpc_policy_info* out) const {
  std::memset(out, 0, sizeof *out);
  auto it = policy_cache_.find(id);
  if (it == policy_cache_.end() || !it->second->has_ref || it->second->action_flows.empty()) return GPC_OK;
  const Conjunction& c = *it->second;
  out->found = 1;
  out->policy_type = c.policy_type;
  out->of_priority = c.action_flows[0].priority;
  std::snprintf(out->policy_namespace, sizeof out->policy_namespace, "%s", c.ns.c_str());
  std::snprintf(out->policy_name, sizeof out->policy_name, "%s", c.pname.c_str());
  std::snprintf(out->policy_uid, sizeof out->policy_uid, "%s", c.uid.c_str());
  std::snprintf(out->rule_name, sizeof out->rule_name, "%s", c.rule_name.c_str());
  std::snprintf(out->log_label, sizeof out->log_label, "%s", c.log_label.c_str());
  return GPC_OK;
}

// dnsPacketInFlow (pipeline.go:2080-2093)
Flow FeatureNP::dns_packet_in_flow(uint32_t id) const {
  Flow f;
  f.table = TB_AP_INGRESS;
  f.priority = kPriorityDNSIntercept;
  f.cookie = cfg_.cookie;
  f.m.has_conj = true;
  f.m.conj_id = id;
  if (cfg_.ovs_meters) {
    Action m{ACT_METER};
    m.a = kMeterDNS;
    f.acts.push_back(m);
  }
  Action c{ACT_CONTROLLER};
  c.a = 1;
  c.b = kPacketInCategoryDNS;
  f.acts.push_back(c);
  f.acts.push_back(go(TB_INGRESS_METRIC));
  return f;
}

// NewDNSPacketInConjunction (network_policy.go:697-779): a conjunction without NetworkPolicy
// reference whose service clause (1/2) matches solicited DNS responses (ct_state=+rpl+trk, TCP and
// UDP source port 53 per IP family) and whose to clause (2/2) gets the FQDN policy's Pod addresses
// through AddAddressToDNSConjunction.
int FeatureNP::new_dns_conjunction(uint32_t id) {
  if (policy_cache_.count(id)) return GPC_OK;  // "DNS Conjunction has already been added to cache"
  auto c = std::make_shared<Conjunction>();
  c->id = id;
  c->has_ref = false;
  c->rule_table = TB_AP_INGRESS;
  c->action_flows.push_back(dns_packet_in_flow(id));
  auto mk = [&](uint8_t clause) {
    auto cl = std::make_unique<Clause>();
    cl->action.conj_id = id;
    cl->action.clause_id = clause;
    cl->action.n_clause = 2;
    cl->rule_table = TB_AP_INGRESS;
    cl->drop_table = 0;
    return cl;
  };
  c->svc = mk(1);
  c->to = mk(2);
  std::vector<const Flow*> add{&c->action_flows[0]};
  apply_bundle(add, {});
  std::vector<CtxChange> chs;
  for (uint8_t fam : ip_protocols_) {
    for (MatchKeyId k : {fam == 4 ? MK_TCP_SRC : MK_TCPV6_SRC, fam == 4 ? MK_UDP_SRC : MK_UDPV6_SRC}) {
      ConjMatch m;
      m.table = TB_AP_INGRESS;
      m.has_prio = true;
      m.prio = kPriorityDNSIntercept;
      MatchValue ct;
      ct.tag = V_CTSTATE;
      ct.u = 0x28;  // +rpl+trk
      ct.mask = 0x28;
      MatchValue port;
      port.tag = V_BITRANGE;
      port.u = 53;
      port.mask = -1;
      m.pairs = {{MK_CT_STATE, ct}, {k, port}};
      CtxChange ch;
      if (add_conj_match_flow(c->svc.get(), m, false, false, &ch)) chs.push_back(std::move(ch));
    }
  }
  apply_changes(chs);
  policy_cache_[id] = c;
  return GPC_OK;
}

static std::string flow_dump_key(const Flow& f) {  // getFlowDumpKey (pipeline.go:385-387, utils.go:1226-1242)
  std::string m = f.m.str(f.priority), out;
  size_t pos = 0;
  while (pos <= m.size()) {
    size_t e = m.find(',', pos);
    if (e == std::string::npos) e = m.size();
    std::string part = m.substr(pos, e - pos);
    if (part.compare(0, 8, "priority") != 0) out += (out.empty() ? "" : ",") + part;
    pos = e + 1;
  }
  return std::string("table=") + table_name(f.table) + "," + out;
}

// GetNetworkPolicyFlowKeys (network_policy.go:1712-1736) over getAllFlowKeys (:1520-1545): per rule
// of the policy its action flows, conjunctive match flows, then drop flows; duplicates kept.
std::vector<std::string> FeatureNP::flow_keys(const std::string& name, const std::string& ns, uint8_t type) const {
  std::vector<std::string> keys;
  for (auto& kv : policy_cache_) {
    const Conjunction& c = *kv.second;
    if (!c.has_ref || c.pname != name || c.ns != ns || c.policy_type != type) continue;
    std::vector<std::string> drops;
    for (auto& f : c.action_flows) keys.push_back(flow_dump_key(f));
    for (Clause* cl : c.clauses())
      for (auto& m : cl->matches) {
        if (m.second->flow) keys.push_back(flow_dump_key(*m.second->flow));
        if (m.second->drop_flow) drops.push_back(flow_dump_key(*m.second->drop_flow));
      }
    keys.insert(keys.end(), drops.begin(), drops.end());
  }
  return keys;
}

std::string FeatureNP::dump() const {
  std::string s;
  for (auto& kv : installed_) {
    s += kv.second.str();
    s += "\n";
  }
  return s;
}

}  // namespace gpc
