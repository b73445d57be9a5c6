/*
 * gpc.h -- C-ABI of the MI355X NetworkPolicy packet classifier ("gpuclassify").
 *
 * Drop-in boundary for the NetworkPolicy half of Antrea's `openflow.Client`
 * (reference: pkg/agent/openflow/client.go:56-414; NP methods :128-148, 215-223, 240-251, 310-317;
 * implementation pkg/agent/openflow/network_policy.go). A Go `pkg/agent/gpuclassify` layer binds
 * these symbols over cgo; C++ callers include this header directly; the Python
 * test harness and bench use ctypes.
 *
 * Conventions
 *   - Every call returns 0 on success or a negative GPC_E* code (gpc_strerror()).
 *   - The caller owns every buffer it passes; the library copies what it keeps.
 *   - Control-plane calls (install/uninstall/add/del/reassign/commit) are serialized by an internal
 *     mutex (the role of conjMatchFlowLock + replayMutex, network_policy.go:1161-1167, 2077).
 *   - gpc_classify() may run concurrently with control-plane calls; it always sees exactly one
 *     committed epoch (gpc_commit publishes atomically, as an OpenFlow bundle does:
 *     pkg/ovs/openflow/ofctrl_bridge.go:468-539).
 *   - No torch / HIP types appear in this header; streams are passed as `void*` (hipStream_t).
 */
#ifndef GPC_H
#define GPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPC_ABI_VERSION 6
/* device slots of one context (gpc_create_multi) */
#define GPC_MAX_DEVICES 16

/* ---------------------------------------------------------------------------- error codes */
#define GPC_OK 0
#define GPC_ENOTFOUND 1   /* ConjunctionNotFound (network_policy.go:309-319)                   */
#define GPC_EINVAL 2      /* malformed argument / unsupported flow shape                          */
#define GPC_ENOMEM 3      /* host or device allocation failed                                     */
#define GPC_EDEV 4        /* HIP runtime error / no device                                        */
#define GPC_ENOCLAUSE 5   /* "no clause is using addrType %d" (network_policy.go:1674-1676)       */
#define GPC_EBUNDLE 6     /* flow bundle rejected; caches rolled back (network_policy.go:1344-1349)*/
#define GPC_ERANGE 7      /* output buffer too small (needed size returned)                      */

/* ---------------------------------------------------------------------------- enums */
enum gpc_direction { GPC_DIR_IN = 0, GPC_DIR_OUT = 1 };            /* v1beta2.Direction */

/* Rule tables (pipeline.go:150-176). */
enum gpc_table {
  GPC_TABLE_ANTREA_POLICY_EGRESS_RULE = 1,
  GPC_TABLE_EGRESS_RULE = 2,
  GPC_TABLE_EGRESS_DEFAULT_RULE = 3,
  GPC_TABLE_ANTREA_POLICY_INGRESS_RULE = 4,
  GPC_TABLE_INGRESS_RULE = 5,
  GPC_TABLE_INGRESS_DEFAULT_RULE = 6
};

enum gpc_policy_type {                                             /* v1beta2.NetworkPolicyType */
  GPC_POLICY_K8S = 0,
  GPC_POLICY_ANNP = 1,
  GPC_POLICY_ACNP = 2,
  GPC_POLICY_ANP = 3,
  GPC_POLICY_BANP = 4
};

enum gpc_rule_action {                                             /* crdv1beta1.RuleAction */
  GPC_RULE_ALLOW = 0,
  GPC_RULE_DROP = 1,
  GPC_RULE_REJECT = 2,
  GPC_RULE_PASS = 3
};

enum gpc_addr_kind {                          /* types.Address implementations, network_policy.go */
  GPC_ADDR_IP = 1,        /* IPAddress        :97-131  */
  GPC_ADDR_IPNET = 2,     /* IPNetAddress     :133-167 */
  GPC_ADDR_OFPORT = 3,    /* OFPortAddress    :169-197 */
  GPC_ADDR_SVC_GROUP = 4, /* ServiceGroupIDAddress :199-216 */
  GPC_ADDR_CT_IP = 5,     /* CTIPAddress      :218-252 */
  GPC_ADDR_CT_IPNET = 6,  /* CTIPNetAddress   :254-288 */
  GPC_ADDR_LABEL_ID = 7   /* LabelIDAddress   :290-307 */
};

enum gpc_addr_type { GPC_SRC_ADDRESS = 0, GPC_DST_ADDRESS = 1 };   /* types.AddressType */

enum gpc_protocol {                                                /* v1beta2.Protocol */
  GPC_PROTO_NONE = 0, /* nil protocol: defaults to TCP (network_policy.go:979-981) */
  GPC_PROTO_TCP = 1,
  GPC_PROTO_UDP = 2,
  GPC_PROTO_SCTP = 3,
  GPC_PROTO_ICMP = 4,
  GPC_PROTO_IGMP = 5
};

/* Verdict actions. */
enum gpc_verdict_action {
  GPC_ACT_NONE = 0,           /* stage not reached (packet dropped in the egress stage)        */
  GPC_ACT_NO_MATCH = 1,       /* no policy flow hit: allowed by default (Metric table miss)    */
  GPC_ACT_ALLOW = 2,          /* conj action flow with ct commit (pipeline.go:1718-1808)       */
  GPC_ACT_DROP = 3,           /* conj deny flow, APDeny + reg3 (pipeline.go:1812-1859)          */
  GPC_ACT_REJECT = 4,         /* conj deny flow with reject disposition                        */
  GPC_ACT_ISOLATION_DROP = 5, /* K8s default / MCNP drop flow (pipeline.go:2040-2076)           */
  GPC_ACT_BYPASS = 6          /* ct est/rel skip flow or IngressSecurityClassifier bypass       */
};
#define GPC_VFLAG_PASS 0x1    /* a Pass rule of the AntreaPolicy table was hit on the way      */
#define GPC_VFLAG_TIE 0x2     /* >1 conjunction completed at the winning priority (OVS-defined
                                 order; resolved to the lowest conj id)                        */
#define GPC_VFLAG_PACKETIN 0x4 /* the deciding flow sends the packet to the controller (the DNS
                                  interception flow, pipeline.go:2080-2093: paused, resumed at
                                  IngressMetric)                                               */

/* Packet destination class, as IngressSecurityClassifier sees reg0 (fields.go PktDestinationField). */
enum gpc_dest { GPC_DEST_POD = 0, GPC_DEST_GATEWAY = 1, GPC_DEST_TUNNEL = 2, GPC_DEST_UPLINK = 3 };
#define GPC_CT_NEW 0x01
#define GPC_CT_EST 0x02
#define GPC_CT_REL 0x04
#define GPC_CT_RPL 0x08
#define GPC_CT_TRK 0x20
#define GPC_CT_MARK_HAIRPIN 0x40 /* HairpinCTMark ct_mark[6] (fields.go:211-213)                */

/* ---------------------------------------------------------------------------- records */
typedef struct gpc_ctx gpc_ctx;

typedef struct gpc_config {
  int32_t ipv4_enabled;          /* featureNetworkPolicy.ipProtocols                           */
  int32_t ipv6_enabled;
  int32_t enable_antrea_policy;  /* AntreaPolicy feature gate (egressTables, skip flows)        */
  int32_t enable_deny_tracking;
  uint64_t cookie;               /* cookie printed in flow dumps (round<<48 | category<<40)     */
  int32_t device;                /* HIP device ordinal used by this context                    */
  int32_t compact_after;         /* live journal rules that start a background compaction
                                    (0: max(512, rules / 128); < 0: never in the background)  */
  int32_t ovs_meters;            /* OVS meters supported: packet-in flows carry meter:256/258    */
  int32_t external_node;         /* config.ExternalNode: no IngressSecurityClassifier flows      */
  int32_t group_packets;         /* gpc_classify groups a batch by nw_src before the table walk:
                                    0 = batches of >= 2^18 packets against an image of >= 4 MB
                                    without composite driver indexes (with them grouping
                                    measured slower), > 0 = always, < 0 = never (gpc_classify6:
                                    the same over the code columns; GPC_GROUP_V6=0: never)      */
  int32_t group_key;             /* grouping key of IPv4 batches (gpc_group_key; environment
                                    GPC_GROUP_KEY overrides): 0 = per image, SCAN when waves' scan
                                    lengths are very unequal (long driver lists), else ADDR       */
  int32_t launch_pacing;         /* gpc_classify* host-side wait (see gpc_classify): 0 = a call waits
                                    until the call 8 calls before it on the same stream has
                                    finished; > 0 = that many calls in flight per stream; < 0 = off
                                    (never blocks: a caller that keeps its stream's queue full may
                                    then delay gpc_commit's publish behind its blocking launches) */
  int32_t reserved[1];
} gpc_config;

/* Order a grouped batch is classified in, inside every tile of 16384 packets (results never depend
   on it): ADDR = top bits of nw_src (then nw_dst; GPC_GROUP_SRC_BITS) -- lanes of a wavefront share
   image lines; SCAN = the driver-list length each policy stage will scan -- lanes of a wavefront
   finish their candidate scans together. */
typedef enum gpc_group_key { GPC_GROUP_KEY_AUTO = 0, GPC_GROUP_KEY_ADDR = 1, GPC_GROUP_KEY_SCAN = 2 } gpc_group_key;

typedef struct gpc_addr {        /* 24 bytes */
  uint8_t kind;                  /* gpc_addr_kind */
  uint8_t family;                /* 4 or 6 for IP kinds */
  uint8_t prefix_len;            /* IPNET kinds */
  uint8_t reserved;
  uint32_t value;                /* OFPORT / SVC_GROUP / LABEL_ID */
  uint8_t ip[16];                /* network byte order; IPv4 in ip[0..3] */
} gpc_addr;

typedef struct gpc_service {     /* v1beta2.Service (controlplane/v1beta2/types.go:299-321) */
  uint8_t protocol;              /* gpc_protocol */
  uint8_t has_port, has_end_port, has_src_port, has_src_end_port;
  uint8_t has_icmp_type, has_icmp_code, has_igmp_type;
  uint16_t port, end_port, src_port, src_end_port;
  int32_t icmp_type, icmp_code, igmp_type;
  uint8_t has_group_address;
  uint8_t group_address[4];      /* IGMP query group (IPv4) */
  uint8_t reserved[3];
} gpc_service;

typedef struct gpc_rule {        /* types.PolicyRule (pkg/agent/types/networkpolicy.go:92-108) */
  uint8_t direction;             /* gpc_direction */
  uint8_t table;                 /* gpc_table (PolicyRule.TableID) */
  uint8_t action;                /* gpc_rule_action (PolicyRule.Action; ignored for K8s) */
  uint8_t policy_type;           /* gpc_policy_type (PolicyRef.Type) */
  uint8_t has_priority;          /* PolicyRule.Priority != nil */
  uint8_t enable_logging;
  uint16_t priority;
  uint32_t flow_id;              /* conjunction id */
  int32_t tier_priority;         /* reported in verdicts (not part of PolicyRule) */
  int32_t n_from;                /* < 0 : From == nil (no clause); >= 0 : clause with n addresses */
  int32_t n_to;
  int32_t n_service;
  const gpc_addr* from;
  const gpc_addr* to;
  const gpc_service* service;
  const char* name;              /* may be NULL */
  const char* log_label;
  const char* policy_namespace;
  const char* policy_name;
  const char* policy_uid;
} gpc_rule;

/* Structure-of-arrays packet batch. Required columns: src, dst, sport, dport, proto, out_port.
 * Optional columns may be NULL (default in parentheses). Addresses/ports in host byte order.
 * For ICMP, sport = type and dport = code (OVS keeps them in tp_src/tp_dst). */
typedef struct gpc_pkt_soa {
  const uint32_t* src;           /* nw_src */
  const uint32_t* dst;           /* nw_dst */
  const uint16_t* sport;         /* tp_src */
  const uint16_t* dport;         /* tp_dst */
  const uint8_t* proto;          /* nw_proto */
  const uint32_t* out_port;      /* reg1 TargetOFPortField */
  const uint32_t* in_port;       /* (0) */
  const uint32_t* svc_group;     /* reg7 ServiceGroupIDField (0) */
  const uint32_t* tun_id;        /* label identity (0) */
  const uint32_t* ct_src;        /* ct_nw_src (= src) */
  const uint32_t* ct_dst;        /* ct_nw_dst (= dst) */
  const uint8_t* ct_state;       /* (+new+trk) */
  const uint8_t* dest;           /* gpc_dest (POD) */
  const uint16_t* len;           /* bytes for per-rule counters (0) */
  /* IPv6 batches (gpc_classify6): 16 network-order bytes per packet, 16-byte aligned; src6 and
   * dst6 required (they replace src / dst), ct_src6 / ct_dst6 optional (default src6 / dst6).
   * proto is the upper-layer protocol (ICMPv6 = 58). Ignored by gpc_classify. */
  const uint8_t* src6;           /* ipv6_src */
  const uint8_t* dst6;           /* ipv6_dst */
  const uint8_t* ct_src6;        /* ct_ipv6_src */
  const uint8_t* ct_dst6;        /* ct_ipv6_dst */
  const uint8_t* ct_mark;        /* ct_mark[0..7] (0); GPC_CT_MARK_HAIRPIN steers IngressSecurityClassifier */
} gpc_pkt_soa;

typedef struct gpc_verdict {     /* 8 bytes; gpc_classify writes 2 per packet: [egress, ingress] */
  uint32_t conj_id;              /* reg5/reg6 or reg3 conjunction id (0 if none) */
  uint8_t action;                /* gpc_verdict_action */
  uint8_t table;                 /* 1 = AntreaPolicy*Rule, 2 = *Rule, 3 = *DefaultRule, 0 = none */
  uint8_t tier;                  /* tier priority of the winning rule (0 if none / K8s) */
  uint8_t flags;                 /* GPC_VFLAG_* */
} gpc_verdict;

/* AntreaProxy. proxy.Endpoint (pkg/agent/proxy/types) as serviceEndpointGroup and
 * endpointDNATFlow read it (pipeline.go:2553-2592, 2502-2528). */
typedef struct gpc_endpoint {
  uint8_t family;                /* 4 or 6 */
  uint8_t is_local;              /* Endpoint.GetIsLocal() */
  uint8_t has_node_name;         /* Endpoint.GetNodeName() != "" */
  uint8_t is_node_ip;            /* nodeIPChecker.IsNodeIP(endpoint IP) (hostNetwork Endpoint) */
  uint16_t port;
  uint16_t reserved;
  uint8_t ip[16];
} gpc_endpoint;

typedef struct gpc_service_config { /* types.ServiceConfig (pkg/agent/types/service.go:24-40) */
  uint8_t family;
  uint8_t protocol;              /* gpc_protocol: TCP, UDP or SCTP */
  uint16_t port;                 /* ServicePort */
  uint32_t cluster_group_id, local_group_id;
  uint8_t traffic_policy_local, is_external, is_nodeport, is_nested, is_dsr;
  uint8_t reserved;
  uint16_t affinity_timeout;
  uint8_t ip[16];                /* ServiceIP */
} gpc_service_config;

/* Per-packet load-balancing result (optional output of gpc_classify_lb), 16 bytes. */
typedef struct gpc_lb_result {
  uint32_t endpoint_ip;          /* selected Endpoint (reg3), host byte order; 0 if none      */
  uint16_t endpoint_port;        /* reg4[0..15]                                               */
  uint8_t flags;                 /* GPC_LB_*                                                  */
  uint8_t reserved;
  uint32_t group_id;             /* Service group (reg7 ServiceGroupIDField)                   */
  uint32_t out_port;             /* reg1 after L3Forwarding to the Endpoint (local Pod ofport) */
} gpc_lb_result;
#define GPC_LB_HIT 0x1           /* the packet matched a ServiceLB flow                        */
#define GPC_LB_NO_ENDPOINT 0x2   /* ... of a Service without Endpoints (rejected, pipeline.go
                                    serviceNoEndpointFlow -> SvcReject packet-in)               */
#define GPC_LB_DNAT 0x4          /* an EndpointDNAT flow rewrote the destination               */
#define GPC_LB_REMOTE 0x8        /* RemoteEndpointRegMark: the Endpoint is on another Node      */
/* gpc_verdict.table value of the egress verdict of a packet rejected by EndpointDNAT (no Endpoint). */
#define GPC_VTABLE_ENDPOINT_DNAT 4

typedef struct gpc_policy_info { /* GetPolicyInfoFromConjunction result */
  int32_t found;
  uint8_t policy_type;
  uint16_t of_priority;          /* priority of the first action flow */
  char policy_namespace[64];
  char policy_name[128];
  char policy_uid[64];
  char rule_name[128];
  char log_label[64];
} gpc_policy_info;

typedef struct gpc_trace_step { /* one rule table of a traced packet's walk (gpc_trace) */
  uint32_t table;                /* gpc_table 1..6                                              */
  uint32_t verdict;              /* table decision: 1 miss (-> next table), 2 allow, 3 drop, 4 reject,
                                    5 isolation drop, 6 bypass (to Metric), 7 pass (-> *Rule)   */
  uint32_t flags;                /* GPC_VFLAG_TIE / GPC_VFLAG_PACKETIN of this decision          */
  uint32_t conj_id;              /* deciding conjunction (0: a non-conjunctive flow, or a miss)  */
  uint32_t priority;             /* OpenFlow priority of the deciding flow (0: miss)             */
  uint32_t candidates;           /* driver-index entries the table's lookup had to consider      */
} gpc_trace_step;

typedef struct gpc_rule_metric { /* types.RuleMetric keyed by conjunction id */
  uint32_t conj_id;
  uint32_t reserved;
  uint64_t packets, bytes, sessions;
} gpc_rule_metric;

typedef struct gpc_image_stats { /* shape of the committed device image (for roofline math) */
  uint64_t epoch;
  uint64_t device_bytes;
  uint32_t n_rules[6];           /* per rule table, soft + hard pseudo-rules */
  uint32_t n_hard[6];
  uint32_t n_flows;
  uint32_t n_counter_slots;
  uint64_t bytes_records;        /* rule records (headers + inline clauses)                   */
  uint64_t bytes_ext;            /* out-of-line clause data                                    */
  uint64_t bytes_bucket_offsets; /* driver-index bucket offset arrays                          */
  uint64_t bytes_entries;        /* driver-index entries (16 B each) incl. always lists        */
  uint64_t bytes_hash;           /* image-wide point hash                                      */
  /* delta epochs (gpc_commit): rules changed since the last full build live in an overlay image */
  uint64_t overlay_bytes;        /* journal pool bytes in use (0: base image alone)              */
  uint32_t n_overlay_rules;      /* live rules in the journal                                  */
  uint32_t n_tombstones;         /* superseded or removed rule copies (base + journal)         */
  uint64_t n_full_builds, n_delta_builds;
  uint64_t n_background_builds;  /* full rebuilds done by the background compactor and installed */
  uint32_t group_key;            /* gpc_group_key grouped IPv4 batches of this epoch use (ADDR/SCAN) */
  uint32_t lane_sort;            /* lane-regrouping table per policy stage: egress | ingress << 8   */
  /* IPv6 image (ipv6_enabled): full rebuilds, delta epochs, its journal */
  uint64_t v6_full_builds, v6_delta_builds;
  uint32_t v6_overlay_rules;     /* live rules in the IPv6 journal                               */
  uint32_t v6_prefixes;          /* interned IPv6 prefixes (incl. those added by delta commits)  */
  /* point extensions (ABI 5): rules whose change since the base only added exact values to one
   * clause (AddPolicyRuleAddress of Pod IPs / ofports) keep their base record; the added values
   * are probed per packet instead of walking a journal copy of the rule */
  uint32_t n_ext_rules;          /* rules with point extensions                                  */
  uint32_t n_ext_values;         /* added values they hold                                       */
  /* ABI 6: journal pool collections (the journal's state rewritten into a fresh pool, without
   * superseded extension indexes and dead versions; no image build) */
  uint64_t n_pool_collections;
} gpc_image_stats;

/* ---------------------------------------------------------------------------- lifecycle */
int gpc_create(const gpc_config* cfg, gpc_ctx** out);
/* One control plane over several devices (MI355X: one agent process driving the GPUs of a node).
 * The compiler, host image and journal exist once; every gpc_commit uploads the new epoch to each
 * device in devices[0..n) and publishes it on all of them together (a launch on any slot sees the
 * same epoch number). Slot k is devices[k] (a device may repeat). cfg->device is ignored.
 * gpc_create(cfg) == gpc_create_multi(cfg, &cfg->device, 1). n in [1, GPC_MAX_DEVICES]. */
int gpc_create_multi(const gpc_config* cfg, const int32_t* devices, size_t n, gpc_ctx** out);
/* Device slots of the context. */
int gpc_n_devices(gpc_ctx* ctx);
void gpc_destroy(gpc_ctx* ctx);
/* Client.Initialize NP part: skipPolicyRuleCheckFlows (network_policy.go:2144-2211). */
int gpc_initialize(gpc_ctx* ctx);

/* ---------------------------------------------------------------------------- openflow.Client NP surface */
/* InstallPolicyRuleFlows(*types.PolicyRule) error            network_policy.go:1160 */
int gpc_install_rule(gpc_ctx* ctx, const gpc_rule* rule);
/* BatchInstallPolicyRuleFlows([]*types.PolicyRule) error     network_policy.go:1310 */
int gpc_batch_install(gpc_ctx* ctx, const gpc_rule* rules, size_t n);
/* UninstallPolicyRuleFlows(ruleID) ([]string, error)         network_policy.go:1570
 * Stale OF priorities are returned in stale[0..*n_stale). */
int gpc_uninstall_rule(gpc_ctx* ctx, uint32_t rule_id, uint16_t* stale, size_t stale_cap, size_t* n_stale);
/* AddPolicyRuleAddress(ruleID, addrType, addresses, priority, enableLogging, isMCNPRule) network_policy.go:1661 */
int gpc_add_rule_addrs(gpc_ctx* ctx, uint32_t rule_id, int32_t addr_type, const gpc_addr* addrs, size_t n,
                       const uint16_t* priority_or_null, int32_t enable_logging, int32_t is_mcnp);
/* DeletePolicyRuleAddress(ruleID, addrType, addresses, priority) network_policy.go:1686 */
int gpc_del_rule_addrs(gpc_ctx* ctx, uint32_t rule_id, int32_t addr_type, const gpc_addr* addrs, size_t n,
                       const uint16_t* priority_or_null);
/* ReassignFlowPriorities(map[uint16]uint16, tableID) error   network_policy.go:1873 */
int gpc_reassign_priorities(gpc_ctx* ctx, const uint16_t* from, const uint16_t* to, size_t n, uint8_t table);
/* GetPolicyInfoFromConjunction(ruleID)                        network_policy.go:1555 */
int gpc_get_policy_info(gpc_ctx* ctx, uint32_t rule_id, gpc_policy_info* out);
/* NewDNSPacketInConjunction(id) error                        client.go:311, network_policy.go:697-779
 * A conjunction without NetworkPolicy reference: solicited DNS responses (ct_state=+rpl+trk,
 * TCP/UDP tp_src=53) to the addresses added below are sent to the controller (paused) and resumed
 * at IngressMetric (verdict BYPASS + GPC_VFLAG_PACKETIN). A second call with the same id is a no-op. */
int gpc_new_dns_conjunction(gpc_ctx* ctx, uint32_t id);
/* AddAddressToDNSConjunction(id, addrs) error                 client.go:314, network_policy.go:781-784 */
int gpc_add_dns_conj_addrs(gpc_ctx* ctx, uint32_t id, const gpc_addr* addrs, size_t n);
/* DeleteAddressFromDNSConjunction(id, addrs) error            client.go:317, network_policy.go:786-789 */
int gpc_del_dns_conj_addrs(gpc_ctx* ctx, uint32_t id, const gpc_addr* addrs, size_t n);
/* GetNetworkPolicyFlowKeys(npName, npNamespace, npType) []string   client.go:219, network_policy.go:1712-1736
 * '\n'-separated keys "table=<name>,<match without priority>" (getFlowDumpKey): per rule of the
 * policy its action flows, conjunctive match flows, then drop flows; duplicates kept. */
int gpc_network_policy_flow_keys(gpc_ctx* ctx, const char* name, const char* ns, uint8_t policy_type, char* buf,
                                 size_t cap, size_t* needed, size_t* n_keys);
/* NetworkPolicyMetrics() map[uint32]*types.RuleMetric          network_policy.go:2034
 * Reads the per-rule device counters of this context. */
int gpc_metrics(gpc_ctx* ctx, gpc_rule_metric* out, size_t cap, size_t* n);

/* Flow-text ingest: the realized flows as ovs-ofctl text, one flow per line -- FlowModToString
 * (pkg/ovs/openflow/utils.go:1222-1241) or `ovs-ofctl dump-flows --names` lines -- applied as one
 * bundle, the seam Bridge.AddFlowsInBundle (pkg/ovs/openflow/ofctrl_bridge.go:468) feeds OVS.
 * Flows of tables outside the NetworkPolicy path are skipped. replace != 0 drops the realized NP
 * tables and the compiler's rule caches first. On a parse error nothing is applied and *err_line
 * (1-based) names the line. Publish with gpc_commit (always a full rebuild for loaded flows). */
int gpc_load_flows(gpc_ctx* ctx, const char* text, size_t len, int32_t replace, size_t* n_loaded, size_t* n_skipped,
                   size_t* err_line);

/* ---------------------------------------------------------------------------- AntreaProxy surface */
/* InstallServiceGroup(groupID, withSessionAffinity, endpoints) error       client.go:710 */
int gpc_install_service_group(gpc_ctx* ctx, uint32_t group_id, int32_t with_session_affinity, const gpc_endpoint* eps,
                              size_t n);
/* UninstallServiceGroup(groupID) error                                      client.go:729 */
int gpc_uninstall_service_group(gpc_ctx* ctx, uint32_t group_id);
/* InstallEndpointFlows(protocol, endpoints) error                           client.go:750 */
int gpc_install_endpoint_flows(gpc_ctx* ctx, uint8_t protocol, uint8_t family, const gpc_endpoint* eps, size_t n);
/* UninstallEndpointFlows(protocol, endpoints) error                         client.go:772 */
int gpc_uninstall_endpoint_flows(gpc_ctx* ctx, uint8_t protocol, uint8_t family, const gpc_endpoint* eps, size_t n);
/* InstallServiceFlows(*types.ServiceConfig) error                           client.go:790
 * Supported: ClusterIP / LoadBalancer / ExternalIP / NodePort Services (optionally Local traffic
 * policy) without session affinity, DSR, multi-cluster nesting or the external + Local
 * short-circuit; other configs -GPC_EINVAL. A NodePort Service (is_nodeport; the caller passes the
 * virtual NodePort DNAT IP 169.254.0.252 as its ip, as the proxier does) matches packets to the
 * NodePort addresses (gpc_set_node_port_addresses) by protocol and port (pipeline.go:2381-2387). */
int gpc_install_service_flows(gpc_ctx* ctx, const gpc_service_config* cfg);
/* UninstallServiceFlows(svcIP, svcPort, protocol) error                     client.go:809 */
int gpc_uninstall_service_flows(gpc_ctx* ctx, const uint8_t* ip, uint8_t family, uint16_t port, uint8_t protocol);
/* InstallPodFlows NP-relevant part (client.go:~600): Pod IP -> ofport, the L3Forwarding result
 * (reg1 TargetOFPortField) for traffic DNATed to a local Endpoint. */
int gpc_install_pod(gpc_ctx* ctx, const uint8_t* ip, uint8_t family, uint32_t ofport);
int gpc_uninstall_pod(gpc_ctx* ctx, const uint8_t* ip, uint8_t family);
/* NodePort addresses of the Node (NewClient nodePortAddressesIPv4 with proxyAll; ABI 6): one
 * NodePortMark flow per non-loopback address plus the virtual NodePort DNAT IP 169.254.0.252
 * (pipeline.go:2282-2314), loading ToNodePortAddressRegMark (reg4[19]) for the ServiceLB NodePort
 * flows. `ips`: n IPv4 addresses of 16 bytes each (the address in the first 4); family 4 only;
 * n = 0 removes them (proxyAll off). Replaces the previous set. */
int gpc_set_node_port_addresses(gpc_ctx* ctx, const uint8_t* ips, uint8_t family, size_t n);
/* ovs-ofctl dump-groups style text of the realized groups, '\n' separated. */
int gpc_dump_groups(gpc_ctx* ctx, char* buf, size_t cap, size_t* needed);

/* ---------------------------------------------------------------------------- data path */
/* Publish the realized flow table to the device atomically (the bundle commit,
 * ofctrl_bridge.go:468-539). A rule whose change since the base image only added exact values to
 * one clause (AddPolicyRuleAddress of Pod IPs, ofports, single ports) keeps its base record and the
 * added values become point extensions (gpc_image_stats n_ext_*); the other changed rules are
 * appended to an append-only journal over the base image and their older copies tombstoned (a
 * delta epoch: cost proportional to the changed rules). A background compactor rebuilds the base
 * once compact_after rules are extended or journaled; past max(16384, base rules / 4) live journal
 * rules without one the whole image is rebuilt inline. Launches already queued keep the epoch they
 * were launched with. */
int gpc_commit(gpc_ctx* ctx);
/* Same, but always rebuilds the whole image (compaction: empties the overlay). */
int gpc_compact(gpc_ctx* ctx);
/* ReplayFlows (client.go:1130-1152) for the device: rebuilds every device buffer of the current
 * epoch from the host shadow state (after a device reset); flows, conj ids and counter slots are
 * unchanged, device counters restart from zero. */
int gpc_replay(gpc_ctx* ctx);
/* Largest batch of one gpc_classify* call (the launch grid is limited to 2^32 work-items). */
#define GPC_MAX_BATCH (4294967296ull - 256ull)
/* Classify n packets whose columns are DEVICE pointers; writes 2*n verdicts (device pointer).
 * n > GPC_MAX_BATCH: -GPC_EINVAL, nothing launched.
 * `count` != 0 updates the per-rule counters (Metric-table flows). `stream` is a hipStream_t; the
 * library keeps per-stream scratch (packet grouping) and epoch-lifetime events, keyed by the
 * stream and, for hipStreamPerThread, by the calling thread as well. With group_packets == 0 a
 * batch whose grouping scratch cannot be allocated runs ungrouped; -GPC_ENOMEM only when
 * grouping was forced (group_packets > 0).
 * The launch is asynchronous on `stream`, but the call may BLOCK ON THE HOST (launch pacing): it
 * first waits, outside every lock, until the call gpc_config.launch_pacing (default 8) calls
 * before it on the same stream and slot has finished, so that no launch blocks inside the lock a
 * commit publishes under (a caller that keeps its stream's queue full would otherwise delay every
 * gpc_commit by ~1 s). A caller that must never block sets launch_pacing < 0. */
int gpc_classify(gpc_ctx* ctx, const gpc_pkt_soa* pkts, size_t n, gpc_verdict* out, int32_t count, void* stream);
/* gpc_classify plus the AntreaProxy stage in front of the policy tables: packets to a Service
 * (ServiceLB flow hit) get an Endpoint from the group (select bucket by a symmetric L4 hash of the
 * 5-tuple), are DNATed by the EndpointDNAT flow and continue to the policy stages with nw_dst /
 * tp_dst = the Endpoint, ct_nw_dst = the Service IP, reg7 = the group id and reg1 / destination
 * from the Pod map. lb_out (device, n entries, may be NULL) receives the selection. gpc_classify
 * runs the same stage (it just does not write lb_out). */
int gpc_classify_lb(gpc_ctx* ctx, const gpc_pkt_soa* pkts, size_t n, gpc_verdict* out, gpc_lb_result* lb_out,
                    int32_t count, void* stream);
/* Traceflow-style readback (traceflow/packetin.go:211-270 reads the verdict registers
 * back, ovsctl.go:91-183 wraps ofproto/trace): packet 0 of the HOST columns `pkt` through the
 * current epoch on the device, Service stage included; out[2] = its verdicts (as gpc_classify),
 * steps[0..*n_steps) = each rule table the walk evaluated, in order. Synchronous; debug path. */
int gpc_trace(gpc_ctx* ctx, const gpc_pkt_soa* pkt, gpc_verdict* out, gpc_lb_result* lb_out, gpc_trace_step* steps,
              size_t cap, size_t* n_steps);
/* IPv6 packets (pkts->src6 / dst6 columns) against the IPv6 half of the rule set (the ipv6_* /
 * tcp6 / udp6 / icmp6 flows and the family-less ones), as OVS classifies an IPv6 packet in the
 * same tables. Needs gpc_config.ipv6_enabled. A commit that changes rules publishes an IPv6 delta
 * epoch (the IPv6 base plus a journal of the changed rules; new prefixes are interned into the
 * prefix tree in place and their LPM entries go to the journal's overflow table) and falls back
 * to a full IPv6 rebuild for a new prefix length, a prefix that is not a leaf of the tree, or a
 * journal past its size thresholds (rules, pool words, overflow entries). No AntreaProxy stage for
 * IPv6. Same verdict / counter layout. -GPC_EINVAL if the IPv6 prefixes of the rule set need more
 * than 32 code bits (core.hpp). */
int gpc_classify6(gpc_ctx* ctx, const gpc_pkt_soa* pkts, size_t n, gpc_verdict* out, int32_t count, void* stream);
/* The data path on device slot `slot` of a gpc_create_multi context: pkts / out / lb_out live on
 * that slot's device and `stream` belongs to it (NULL: its null stream). gpc_classify* == slot 0. */
int gpc_classify_on(gpc_ctx* ctx, uint32_t slot, const gpc_pkt_soa* pkts, size_t n, gpc_verdict* out,
                    gpc_lb_result* lb_out, int32_t count, void* stream);
int gpc_classify6_on(gpc_ctx* ctx, uint32_t slot, const gpc_pkt_soa* pkts, size_t n, gpc_verdict* out, int32_t count,
                     void* stream);
int gpc_classify_host_on(gpc_ctx* ctx, uint32_t slot, const gpc_pkt_soa* pkts, size_t n, gpc_verdict* out,
                         gpc_lb_result* lb_out, int32_t count);
int gpc_classify6_host(gpc_ctx* ctx, const gpc_pkt_soa* pkts, size_t n, gpc_verdict* out, int32_t count);
/* Same with HOST pointers (copies in and out; synchronous). */
int gpc_classify_host(gpc_ctx* ctx, const gpc_pkt_soa* pkts, size_t n, gpc_verdict* out, int32_t count);
int gpc_classify_host_lb(gpc_ctx* ctx, const gpc_pkt_soa* pkts, size_t n, gpc_verdict* out, gpc_lb_result* lb_out,
                         int32_t count);
/* Per-rule counters as a device buffer of n_slots x {packets, bytes, sessions} uint64 (for an
 * RCCL all-reduce by the caller), plus the slot -> conj id map (host, valid until the next commit).
 * Sessions as the Metric flows count them: ct_state=+new packets for allow rules, every packet for
 * deny rules (pipeline.go:1604-1670, network_policy.go:1917-1980). Internally the kernels update
 * striped replicas of the array (few rules: many same-address atomics); this call folds them into
 * the returned buffer (synchronizes the device), so call it again to see later classifications. */
int gpc_counters(gpc_ctx* ctx, uint64_t** dev_counters, const uint32_t** slot_conj, size_t* n_slots);
/* The counters of device slot `slot` alone (gpc_counters == slot 0). gpc_metrics sums every slot;
 * gpc_reset_counters zeroes every slot. */
int gpc_counters_on(gpc_ctx* ctx, uint32_t slot, uint64_t** dev_counters, const uint32_t** slot_conj, size_t* n_slots);
int gpc_reset_counters(gpc_ctx* ctx);

/* ---------------------------------------------------------------------------- introspection */
/* ovs-ofctl style dump of the realized flow table (utils.go FlowModToString), '\n' separated. */
int gpc_dump_flows(gpc_ctx* ctx, char* buf, size_t cap, size_t* needed);
int gpc_get_image_stats(gpc_ctx* ctx, gpc_image_stats* out);
/* The last committed image as built on the host (kept as shadow state for re-upload after a
 * device reset). Pointers stay valid until the next gpc_commit. Used by tests to verify the
 * image independently of the device. */
int gpc_debug_image(gpc_ctx* ctx, const uint32_t** blob, size_t* n_words, const void** hdr, size_t* hdr_bytes);
/* The last committed IPv6 image (NULL / 0 when IPv6 is disabled). */
int gpc_debug_image6(gpc_ctx* ctx, const uint32_t** blob, size_t* n_words, const void** hdr, size_t* hdr_bytes);
/* The host copy of the committed Service image (NULL / 0 when no Services). */
int gpc_debug_service_image(gpc_ctx* ctx, const uint32_t** blob, size_t* n_words);
/* Host mirror of the journal pool and the current epoch's journal header offset (NULL / 0 when
 * the epoch is the base image alone). */
int gpc_debug_epoch(gpc_ctx* ctx, const uint32_t** pool, size_t* pool_words, uint32_t* jhdr);
/* The same for the IPv6 image's journal (IPv6 delta epochs). */
int gpc_debug_epoch6(gpc_ctx* ctx, const uint32_t** pool, size_t* pool_words, uint32_t* jhdr);
/* Test hook (fault injection): the next `n` device image uploads of this context's gpc_commit /
 * gpc_compact / gpc_replay fail with GPC_EDEV, as a device error would (the background
 * compactor's uploads and other contexts are unaffected); the host shadow state keeps the new
 * build, and the next successful commit re-uploads every base the device slots do not hold
 * (tests/test_gpu_ipv6_delta.py). */
int gpc_debug_fail_uploads(gpc_ctx* ctx, int n);
/* The epoch (gpc_image_stats.epoch) the last gpc_classify* launch on `stream` was bound to: with
 * classification concurrent to commits, every launch sees exactly this one committed epoch. */
int gpc_stream_epoch(gpc_ctx* ctx, void* stream, uint64_t* epoch);
/* Launch timing (a measurement hook: bench.py's per-kernel roofline). With slots > 0 every
 * gpc_classify* call records HIP events on its own stream before each of its kernels and after
 * the last, into the next of `slots` event sets (reused round-robin: a set not read back by
 * gpc_launch_times before it comes round again is overwritten and counted in `dropped`);
 * slots = 0 (the default) records nothing. */
typedef struct gpc_launch_time {
  char kernel[32];   /* "group_tiles", "classify_egress", "classify_ingress", "classify_both", "unpermute" */
  uint32_t launches; /* launches of that kernel since the previous gpc_launch_times */
  uint32_t dropped;  /* event sets overwritten before they were read (all kinds) */
  double total_ms;   /* summed HIP-event durations */
} gpc_launch_time;
int gpc_set_launch_timing(gpc_ctx* ctx, uint32_t slots);
/* Waits for the recorded events and returns one entry per kernel kind that ran (cap entries at most). */
int gpc_launch_times(gpc_ctx* ctx, gpc_launch_time* out, size_t cap, size_t* n);
const char* gpc_strerror(int err);
int gpc_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GPC_H */
