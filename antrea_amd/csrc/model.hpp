// Flow model of the realized OpenFlow table (host side).
//
// A `Flow` is what `openflow.Client` hands to OVS in a bundle (FlowMod). The compiler
// (compiler.cpp) produces them exactly as network_policy.go / pipeline.go do; the image builder
// (image.cpp) turns the realized set into the device classification image. Text rendering follows
// pkg/ovs/openflow/utils.go (FlowModToString, getFlowModMatch field order) so dumps compare
// byte-for-byte with the reference's golden strings.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

namespace gpc {

// Table ids 1..6 are the rule tables (== gpc_table); the rest are pipeline neighbours that appear
// as goto/ct targets (pipeline.go:150-183).
enum TableId : uint8_t {
  TB_NONE = 0,
  TB_AP_EGRESS = 1,
  TB_EGRESS = 2,
  TB_EGRESS_DEFAULT = 3,
  TB_AP_INGRESS = 4,
  TB_INGRESS = 5,
  TB_INGRESS_DEFAULT = 6,
  TB_EGRESS_METRIC = 7,
  TB_INGRESS_METRIC = 8,
  TB_L3_FORWARDING = 9,
  TB_CONNTRACK_COMMIT = 10,
  TB_OUTPUT = 11,
  // AntreaProxy tables (pipeline.go ServiceLB / EndpointDNAT / SNATMark)
  TB_SERVICE_LB = 12,
  TB_ENDPOINT_DNAT = 13,
  TB_SNAT_MARK = 14,
  TB_SNAT = 15,
  TB_INGRESS_CLASSIFIER = 16,  // IngressSecurityClassifier (pipeline.go:2144-2182)
  TB_NODEPORT_MARK = 17,       // NodePortMark (pipeline.go:2280-2314, proxyAll)
  TB_COUNT = 18
};
const char* table_name(uint8_t t);
// Logging-and-resubmit group IDs as initGroups allocates them (network_policy.go:2271-2300, Multicast
// off; client_test.go:2762-2767): keyed by the table the group resubmits to.
constexpr uint32_t kLogGroupEgressRule = 1, kLogGroupEgressMetric = 2, kLogGroupIngressRule = 3,
                   kLogGroupIngressMetric = 4;
inline bool is_egress_table(uint8_t t) { return t == TB_AP_EGRESS || t == TB_EGRESS || t == TB_EGRESS_DEFAULT || t == TB_EGRESS_METRIC; }
uint8_t next_table(uint8_t t);

constexpr uint16_t kPriorityHigh = 210, kPriorityNormal = 200, kPriorityLow = 190;
constexpr uint16_t kPriorityTopAntreaPolicy = 64990, kPriorityDNSIntercept = 64991;
constexpr uint32_t kControllerId = 32776;                      // the agent's OpenFlow controller id
constexpr uint32_t kMeterNP = 256, kMeterDNS = 258;            // client.go:851-858 packet-in meters
constexpr uint32_t kPacketInCategoryNP = 1, kPacketInCategoryDNS = 2;  // packetin.go:44-52
// PktDestinationField reg0[4..7] values (fields.go:54-57) and HairpinCTMark ct_mark[6] (:211-213)
constexpr uint32_t kToTunnelMark = 0x10, kToGatewayMark = 0x20, kToUplinkMark = 0x40, kHairpinCTMark = 0x40;
constexpr uint32_t kCtZone = 0xfff0, kCtZoneV6 = 0xffe6;
constexpr uint32_t kUnknownLabelIdentity = 0xffffff;
constexpr uint16_t kEthIP = 0x0800, kEthIPv6 = 0x86dd;

struct IPAddr {
  uint8_t fam = 4;  // 4 or 6
  uint8_t b[16] = {0};
  bool operator<(const IPAddr& o) const;
  bool operator==(const IPAddr& o) const;
  uint32_t v4() const { return (uint32_t(b[0]) << 24) | (uint32_t(b[1]) << 16) | (uint32_t(b[2]) << 8) | b[3]; }
  std::string str() const;
  int bits() const { return fam == 4 ? 32 : 128; }
  IPAddr masked(int plen) const;
};

struct IPMatch {
  bool set = false;
  IPAddr addr;
  int plen = -1;  // -1: exact (MatchSrcIP) ; else IPNet prefix
};

// One OpenFlow match (only the fields the NetworkPolicy path uses).
struct Match {
  bool has_conj = false;
  uint32_t conj_id = 0;
  bool has_ct_state = false;
  uint8_t ct_data = 0, ct_mask = 0;
  bool has_ct_mark = false;
  uint32_t ct_mark_v = 0, ct_mark_m = 0xffffffffu;
  bool has_ct_label = false;
  uint64_t label_v = 0, label_m = 0;  // ct_label[0..63]
  IPMatch ct_nw_src, ct_nw_dst;
  bool has_dl = false;
  uint16_t dl_type = 0;
  bool has_proto = false;
  uint8_t nw_proto = 0;
  uint16_t reg_present = 0;
  uint32_t reg_v[16] = {0}, reg_m[16] = {0};
  bool has_tun = false;
  uint64_t tun_id = 0;
  bool has_in_port = false;
  uint32_t in_port = 0;
  IPMatch nw_src, nw_dst;
  bool has_icmp_type = false, has_icmp_code = false;
  uint8_t icmp_type = 0, icmp_code = 0;
  bool has_tp_src = false, has_tp_dst = false;
  uint16_t tp_src = 0, tp_src_m = 0xffff, tp_dst = 0, tp_dst_m = 0xffff;

  void set_reg(int r, uint32_t v, uint32_t m = 0xffffffffu) {
    reg_present |= uint16_t(1u << r);
    reg_v[r] = v;
    reg_m[r] = m;
  }
  std::string str(uint16_t priority) const;  // "priority=...,..." (getFlowModMatch)
};

enum ActKind : uint8_t {
  ACT_CONJ, ACT_SET_REG, ACT_CT_COMMIT, ACT_GOTO, ACT_GROUP, ACT_DROP,
  ACT_CT_DNAT,     // ct(commit,table=a,zone=b,nat(dst=c:lv),exec(ServiceCTMark, reg0[0..3]->ct_mark))
  ACT_CT_HAIRPIN,  // ct(commit,table=a,zone=b,exec(ConnSNATCTMark, HairpinCTMark))
  ACT_RESUBMIT,    // resubmit:a (group buckets)
  ACT_METER,       // meter:a
  ACT_CONTROLLER   // controller(id=32776,reason=no_match,userdata=<a bytes of b, low first>,max_len=65535)
};

struct Action {
  ActKind kind;
  uint32_t a = 0, b = 0, c = 0;  // CONJ: id, clause, n ; SET_REG: reg, value, mask ; CT: table, zone ; GOTO: table ; GROUP: id
  bool has_mask = false;
  uint64_t lv = 0, lm = 0;       // CT: ct_label value/mask
  std::string str() const;
};

struct Flow {
  uint8_t table = TB_NONE;
  uint16_t priority = 0;
  Match m;
  std::vector<Action> acts;
  uint64_t cookie = 0;
  std::string str() const;       // FlowModToString
  std::string identity() const;  // table + priority + match (what OVS keys a flow by)
  bool is_soft() const {         // conjunction-only flow
    if (acts.empty()) return false;
    for (auto& a : acts)
      if (a.kind != ACT_CONJ) return false;
    return true;
  }
};

// OpenFlow group (select type): what serviceEndpointGroup builds (pipeline.go:2553-2592).
struct Bucket {
  uint32_t id = 0, weight = 100;
  std::vector<Action> acts;
};
struct Group {
  uint32_t id = 0;
  std::vector<Bucket> buckets;
  std::string str() const;  // "group_id=100,type=select,bucket=bucket_id:0,weight:100,actions=..."
};

}  // namespace gpc
