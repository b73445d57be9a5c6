// Builds the device classification image (core.hpp layout) from the realized flow table.
#pragma once

#include <array>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <unordered_map>
#include <string>
#include <vector>

#include "compiler.hpp"
#include "core.hpp"

namespace gpc {

class V6Codes;  // IPv6 prefix tree and codes (image.cpp)

// A soft rule of a base image as point extensions need it (Journal::apply): where its record is,
// a signature of everything but its match atoms, and per clause the sorted hashes of its atoms.
struct BaseRule {
  uint32_t table = 0, rec_off = 0;
  uint64_t sig = 0;
  // sorted atom hashes per clause, interned per image: rules sharing a peer set (an AddressGroup
  // referenced by many rules, C2g) share one vector (10 M hashes -> 160 k in C2g)
  std::shared_ptr<const std::vector<uint64_t>> atoms[kMaxClauses];
};

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
  uint32_t v6_code_bits = 0, v6_prefixes = 0;  // IPv6 image: deepest code, interned prefixes
  std::shared_ptr<V6Codes> codes6;             // IPv6 image: its prefix tree (delta commits extend it)
  // IPv6 image: LPM entries of the prefixes delta commits interned ({masked address, len} -> code),
  // published through the IPv6 journal's overflow table (extend_image6)
  std::map<std::array<uint32_t, 5>, uint32_t> v6_ovf;
  std::unordered_map<uint32_t, BaseRule> base_rules;  // IPv4 image: soft rules by conj id (point extensions)
};

// Stable counter slots per conjunction id (freed on uninstall, reused later; identical on every
// rank that applies the same control-plane calls, so slots line up for the RCCL all-reduce).
// Slots are allocated only by the control thread (gpc_commit, in conj-id order, before the commit
// is logged for the compactor); the background compactor only looks them up (lookup with
// alloc = false), so numbering never depends on thread timing and a conjunction uninstalled while
// the compactor worked is built uncounted instead of re-acquiring a slot nothing would release.
class SlotMap {
 public:
  uint32_t get(uint32_t conj);
  // The slot of conj; a new one when absent and alloc, else false.
  bool lookup(uint32_t conj, bool alloc, uint32_t* slot);
  void release(uint32_t conj, std::vector<uint32_t>* freed);
  uint32_t size() const {
    std::lock_guard<std::mutex> g(mu_);
    return uint32_t(slot_conj_.size());
  }
  std::vector<uint32_t> slot_conj() const {
    std::lock_guard<std::mutex> g(mu_);
    return slot_conj_;
  }

 private:
  mutable std::mutex mu_;
  std::map<uint32_t, uint32_t> slot_;
  std::vector<uint32_t> slot_conj_;
  std::vector<uint32_t> free_;
};

// alloc = false (background compactor): counter slots are looked up, never allocated.
// Point extensions a compaction keeps as extensions (api.cpp compactor): per conj, the clause and
// the (axis, value) atoms the new base leaves out (the fresh journal re-adds them as extensions).
struct HeldExt {
  uint32_t clause = 0;
  std::vector<std::pair<uint32_t, uint32_t>> values;  // (axis, value), sorted
};
using HeldExts = std::map<uint32_t, HeldExt>;
int build_image(const FeatureNP& np, SlotMap& slots, HostImage* out, bool alloc = true, const HeldExts* hold = nullptr);
// The IPv6 image (core.hpp "IPv6 interning"): full build.
int build_image6(const FeatureNP& np, SlotMap& slots, HostImage* out, bool alloc = true);
class Journal;
// IPv6 delta commits: interns the prefixes of the changed rules `conj` (and of the hard flows of
// `hard_tables`) that the image's tree lacks (V6Codes::add_leaf: no existing code changes) and
// adds their LPM entries and markers to img->v6_ovf; when that grew, the journal gets a new
// overflow table (probed next to the base LPM hash by delta-epoch kernels). Nothing published is
// rewritten. -GPC_EINVAL when a prefix cannot be interned (rebuild the IPv6 image instead).
int extend_image6(const FeatureNP& np, const std::set<uint32_t>& conj, uint8_t hard_tables, HostImage* img, Journal* j6);
// Append-only delta store over one base image (core.hpp "journal"). apply() appends the current
// versions of the changed rules (records, driver-bucket entries, copied-on-write head pages) and a
// new epoch header with the cumulative tombstones; nothing published earlier is rewritten, so the
// device only receives pool[uploaded, size). Cost per commit ~ the changed rules, not the journal.
class Journal {
 public:
  // lg: log2 of the chain-head table; 0 = sized to the base (kJournalLgMin..kJournalLgMax)
  void reset(const HostImage* base, uint32_t lg = 0);
  // IPv6 journal: rules gathered as an IPv6 image over the base's codes (base->codes6)
  void set_family(int fam) { fam_ = fam; }
  // IPv6: the overflow LPM table the next epoch header points at (appended by the next apply)
  void set_v6_overflow(std::vector<uint32_t> table, uint32_t log2) {
    ovf_table_ = std::move(table);
    ovf_log2_ = log2;
    ovf_dirty_ = true;
  }
  void set_base(const HostImage* base) { base_ = base; }  // the base image object moved
  int apply(const FeatureNP& np, SlotMap& slots, const std::set<uint32_t>& conj, uint8_t hard_tables, std::string* err,
            bool alloc = true);
  bool active() const { return hdr_off != 0; }
  // What the current epoch needs of the kernel (core.hpp kModeBase / kModeExt / kModeJournal).
  int mode() const { return journaled_ ? kModeJournal : ext_off_ ? kModeExt : kModeBase; }
  uint32_t n_ext_rules() const { return uint32_t(ext_.size()); }
  HeldExts held_extensions() const;  // the live point extensions, for a compaction that keeps them
  uint32_t n_ext_values() const { return ext_values_; }
  uint32_t n_tombstones() const;
  uint32_t n_dead_versions() const;  // journal versions tombstoned by a later version
  // Pool garbage collection (api.cpp): the same state over the same base in a fresh pool -- the
  // live journaled rules written once more, extensions and base tombstones carried over -- without
  // the dead versions and superseded extension indexes of the old pool (IPv4 journal only).
  int rebuild(const FeatureNP& np, SlotMap& slots, std::string* err);
  std::vector<uint32_t> pool;  // host mirror of the device pool
  size_t uploaded = 0;         // words already on the device
  uint32_t hdr_off = 0;        // JournalHdr of the latest epoch (0: no journal yet)
  uint32_t n_versions = 0, n_live = 0;
  bool any_noact = false;

 private:
  uint32_t append(const uint32_t* w, size_t n, size_t align);
  const HostImage* base_ = nullptr;
  uint32_t lg_ = 16;
  std::vector<uint32_t> heads_, pt_, bdead_, odead_, bpt_, opt_;
  std::set<uint32_t> bdirty_, odirty_;  // tombstone pages changed since the last epoch
  std::unordered_map<uint32_t, uint32_t> live_;  // conj -> journal rule id of its live version
  std::vector<uint32_t> hard_orids_[6], hard_offs_[6];
  JournalTable tables_[6];
  uint32_t bloom_axes_ = 0;  // JournalHdr.bloom_axes
  int fam_ = 4;
  std::vector<uint32_t> ovf_table_;
  uint32_t ovf_off_ = 0, ovf_log2_ = 0;
  bool ovf_dirty_ = false;
  // point extensions (core.hpp ExtHdr): conj -> its base record and the values added to one clause
  struct ExtRule {
    uint32_t table = 0, rec_off = 0, clause = 0, prio = 0;
    std::vector<std::pair<uint32_t, uint32_t>> values;  // (axis, value), sorted
    // composite keys (core.hpp ExtHdr): the exact values of clause 1 - cband when the values extend
    // clause cband of a composite table; empty: plain (table, axis, value) keys
    std::vector<uint32_t> xv;
    // exact composite entries (core.hpp kExtExact): the rule's remaining clause as intervals on iax
    // (iax 15: the rule has no other clause); empty: the record verifies it
    uint32_t conj = 0, iax = 15;
    std::vector<std::pair<uint32_t, uint32_t>> ivs;
    bool operator==(const ExtRule& o) const {
      return table == o.table && rec_off == o.rec_off && clause == o.clause && prio == o.prio && values == o.values &&
             xv == o.xv && conj == o.conj && iax == o.iax && ivs == o.ivs;
    }
  };
  std::map<uint32_t, ExtRule> ext_;
  uint32_t ext_values_ = 0, ext_off_ = 0;
  size_t ext_entries_ = 0;  // index entries: a composite value has one per x
  // two-level index (emit_ext): B's header fields (b_*, presence size, axes), its presence bits, its
  // entries per rule, their tombstones; the rules in D; the rules changed since the last epoch
  ExtHdr extb_{};
  std::vector<uint32_t> extb_pres_, extb_tomb_;
  std::unordered_map<uint32_t, std::vector<uint32_t>> extb_ents_;
  uint32_t extb_dead_ = 0;
  std::set<uint32_t> extd_, ext_dirty_;
  std::set<uint32_t> touched_;  // every rule applied since the reset (rebuild)
  uint8_t touched_hard_ = 0;
  bool ext_force_ = false;  // rebuild: emit the carried-over extension index with the next epoch
  bool journaled_ = false;  // records, tombstones or hard rules since reset (JournalHdr kJUsed)
  uint32_t pt_off_ = 0, bdead_pt_off_ = 0, odead_pt_off_ = 0;  // last published page tables (reused if unchanged)
  uint32_t emit_ext();
};

}  // namespace gpc
