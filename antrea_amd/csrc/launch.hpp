// Internal launch entry of the classification kernel (classify.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "core.hpp"
#include "gpc.h"

namespace gpc {
// Device pointers of one published epoch (core.hpp View): base image, optional journal.
struct EpochArgs {
  const ImageHdr* hdr;
  const uint32_t* blob;
  const uint32_t* pool;   // journal pool (null: base image alone)
  uint32_t jhdr;          // JournalHdr word offset of this epoch
  const uint32_t* svc;    // null: no Services (AntreaProxy stage skipped)
  uint32_t v6_lpm;        // IPv6 image: word offset of its V6Lpm block (host copy of ImageHdr.v6_lpm)
  uint8_t sort_table[2];  // per policy stage launch: table (1-6) whose scan length groups lanes, 0 = none
  uint32_t ctr_stride;    // per-rule counters: words per copy (counter_cap * kCounterWords)
  uint32_t ctr_mask;      // number of striped copies - 1 (a block updates copy blockIdx & mask)
  uint32_t mode;          // with a pool: kModeExt = only point extensions over the base, else the journal
};
// One packet (index 0 of the device columns) through the table walk with a per-table trace.
int launch_trace(const EpochArgs& ep, const gpc_pkt_soa& pk, uint4* out, uint4* lb_out, TraceStep* steps, uint32_t* n_steps,
                 hipStream_t stream);
// Drains the accumulator copies 0..copies-1 ({packets, bytes, non-session packets} per slot, stride
// words per copy) into the published copy `copies` ({packets, bytes, sessions}): core.hpp count_stage.
int launch_fold_counters(unsigned long long* counters, uint64_t stride, uint32_t copies, hipStream_t stream);
// dst[w] += sum over r < copies of src[r * src_stride + w], w < n_words (device-scope atomics: launches
// on other streams may be adding to dst concurrently). Used when the counter array grows.
int launch_merge_counters(unsigned long long* dst, const unsigned long long* src, uint64_t src_stride, uint32_t copies,
                          uint64_t n_words, hipStream_t stream);
// Packet grouping of a batch (classify.hip group_tiles_kernel): the batch is classified in the
// order of an 8-bit key (scan lengths or address bits) within every tile of 16384 packets, from a grouped copy in
// `scratch` (group_scratch_bytes(pk, n, lb) bytes of device memory, live until the launches have run:
// stream-ordered).
struct GroupArgs {
  uint8_t* scratch;
  uint32_t key;        // GPC_GROUP_KEY_ADDR or GPC_GROUP_KEY_SCAN
  uint32_t axes;       // SCAN: bit a = axis a is read by a sub-index of the image (group_axes)
  uint32_t src_bits;   // ADDR: key = top src_bits of nw_src, then the top 8 - src_bits of nw_dst
  uint32_t xcd_order;  // block order (classify.hip logical_block): 1 = the blocks of one tile run on one XCD
  uint32_t unpermute;  // 1: the ingress launch stores in grouped order, unpermute_kernel restores caller order
  uint32_t lb;         // 1: a Service batch with lb_out: its LB results are un-permuted too (scratch for them)
};
uint64_t group_scratch_bytes(const gpc_pkt_soa& pk, uint64_t n, bool lb);
// Launch timing (gpc_set_launch_timing): an event is recorded on the launch stream before every
// kernel of one gpc_classify* call and after the last, named by the kernel that follows it.
struct LaunchMarks {
  static constexpr int kMax = 8;
  hipEvent_t ev[kMax];
  uint8_t kind[kMax];  // LaunchKind of the kernel starting at ev[i] (kLaunchEnd: the closing event)
  int n;
};
enum LaunchKind : uint8_t {
  kLaunchGroup, kLaunchEgress, kLaunchIngress, kLaunchBoth, kLaunchUnpermute, kLaunchCodes, kLaunchKinds, kLaunchEnd
};
inline void launch_mark(LaunchMarks* m, uint8_t kind, hipStream_t s) {
  if (!m || m->n >= LaunchMarks::kMax) return;
  if (hipEventRecord(m->ev[m->n], s) == hipSuccess) m->kind[m->n++] = kind;
}
// park: with Services (ep.svc), 16 B per packet of device scratch for the fields the Service stage
// rewrites, handed from the egress launch to the ingress launch; null: one launch does both stages.
int launch_classify(const EpochArgs& ep, const gpc_pkt_soa& pk, uint64_t n, gpc_verdict* out, uint4* lb_out,
                    unsigned long long* counters, int count, const GroupArgs* group, hipStream_t stream,
                    LaunchMarks* marks = nullptr, uint4* park = nullptr);
// IPv6 batch (pk.src6 / dst6 [/ ct_src6 / ct_dst6]) against the IPv6 image `ep` (base or delta
// epoch): v6_code_kernel maps the addresses to codes in `codes` (v6_code_columns(pk) * n words of
// device memory, live until the launches have run), then launch_classify runs over the code columns
// (`group`: sized by group_scratch_bytes of that IPv4-shaped batch).
uint32_t v6_code_columns(const gpc_pkt_soa& pk);
int launch_classify6(const EpochArgs& ep, const gpc_pkt_soa& pk, uint64_t n, gpc_verdict* out,
                     unsigned long long* counters, int count, const GroupArgs* group, uint32_t* codes, hipStream_t stream,
                     LaunchMarks* marks = nullptr);
}
