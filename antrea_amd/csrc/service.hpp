// AntreaProxy feature of the classifier: the ServiceLB / EndpointDNAT flows
// and Endpoint groups of pkg/agent/openflow (client.go:710-815, pipeline.go:2374-2592, 3052), kept
// as the realized flow / group state OVS would hold, and the device Service image built from it.
#pragma once

#include <map>
#include <string>
#include <vector>

#include "gpc.h"
#include "model.hpp"

namespace gpc {

class FeatureService {
 public:
  explicit FeatureService(const gpc_config& cfg);

  int install_service_group(uint32_t gid, bool affinity, const gpc_endpoint* eps, size_t n);
  int uninstall_service_group(uint32_t gid);
  int install_endpoint_flows(uint8_t proto, uint8_t family, const gpc_endpoint* eps, size_t n);
  int uninstall_endpoint_flows(uint8_t proto, uint8_t family, const gpc_endpoint* eps, size_t n);
  int install_service_flows(const gpc_service_config& c);
  int uninstall_service_flows(const uint8_t* ip, uint8_t family, uint16_t port, uint8_t proto);
  int install_pod(const uint8_t* ip, uint8_t family, uint32_t ofport);
  // NodePort addresses (NewClient's nodePortAddressesIPv4 with proxyAll): the NodePortMark flows
  // (pipeline.go:2282-2314) for each non-loopback address and the virtual NodePort DNAT IP
  int set_node_port_addresses(const uint32_t* v4, size_t n);
  int uninstall_pod(const uint8_t* ip, uint8_t family);

  std::string dump_flows() const;   // FlowModToString lines of the realized Service flows
  std::string dump_groups() const;  // Group::str lines
  bool empty() const { return cached_.empty() && groups_.empty(); }
  uint64_t generation() const { return generation_; }

  // Device Service image (core.hpp "Service image"), IPv4. Returns -GPC_EINVAL with *err for a
  // realized flow shape the data path does not implement.
  int build_image(std::vector<uint32_t>* blob, std::string* err) const;

 private:
  uint64_t cookie() const;
  uint8_t dnat_next_table() const { return cfg_.enable_antrea_policy ? TB_AP_EGRESS : TB_EGRESS; }

  gpc_config cfg_;
  std::map<std::string, std::vector<Flow>> cached_;  // featureService.cachedFlows: cache key -> flows
  std::map<uint32_t, Group> groups_;                 // featureService.groupCache
  std::map<uint32_t, uint32_t> pods_;                // IPv4 Pod IP -> ofport
  uint64_t generation_ = 0;
};

}  // namespace gpc
