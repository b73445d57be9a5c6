// Builds the device classification image (core.hpp layout) from the realized flow table.
#pragma once

#include <map>
#include <set>
#include <unordered_map>
#include <string>
#include <vector>

#include "compiler.hpp"
#include "core.hpp"

namespace gpc {

struct HostImage {
  ImageHdr hdr{};
  std::vector<uint32_t> blob;        // hdr offsets index this (uint32 words)
  uint32_t n_rules[6] = {0}, n_hard[6] = {0};
  uint32_t n_flows = 0;
  uint64_t bytes_records = 0, bytes_ext = 0, bytes_bucket_offsets = 0, bytes_entries = 0, bytes_hash = 0;
  std::string error;                 // non-empty: unsupported flow shape
  // rule ids (record word 4 >> 8) for tombstoning this image's rules from a later delta epoch
  uint32_t n_rids = 0;
  std::unordered_map<uint32_t, uint32_t> conj_rid;  // soft rules
  std::vector<uint32_t> hard_rids[6];                // hard pseudo-rules per table
  bool any_noact = false;  // a soft rule without an IPv4 conj_id flow (delta combine needs none)
};

// Stable counter slots per conjunction id (freed on uninstall, reused later; identical on every
// rank that applies the same control-plane calls, so slots line up for the RCCL all-reduce).
class SlotMap {
 public:
  uint32_t get(uint32_t conj);
  void release(uint32_t conj, std::vector<uint32_t>* freed);
  uint32_t size() const { return uint32_t(slot_conj_.size()); }
  const std::vector<uint32_t>& slot_conj() const { return slot_conj_; }

 private:
  std::map<uint32_t, uint32_t> slot_;
  std::vector<uint32_t> slot_conj_;
  std::vector<uint32_t> free_;
};

int build_image(const FeatureNP& np, SlotMap& slots, HostImage* out);
// Delta image of a subset: the rules of `conj` as currently installed (uninstalled ones are
// skipped) plus every hard pseudo-rule of the tables in `hard_tables` (bit t-1 = table t).
int build_overlay(const FeatureNP& np, SlotMap& slots, const std::set<uint32_t>& conj, uint8_t hard_tables, HostImage* out);

}  // namespace gpc
