// gfx950 classification kernel: one packet per lane, both policy stages.
//
// Memory behaviour: the six packet columns are read once with coalesced loads
// (17 B/packet), the 16-B verdict pair is written with one 128-bit store per lane, and everything
// else is read-only image traffic (driver bucket offsets, candidate ranks, 32-B rule records,
// interval / box / point-hash lines) served from L2 / Infinity Cache when the image fits.
#include <hip/hip_runtime.h>

#include "core.hpp"
#include "gpc.h"
#include "launch.hpp"

// group_tiles_kernel (141 KB) and unpermute_kernel (128 KB) size their LDS for gfx950's 160 KB.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "classify.hip is written for gfx950 (CDNA4: 160 KB LDS per workgroup)"
#endif

namespace gpc {

#if defined(GPC_STAMPS)
__device__ unsigned long long gpc_stamp_acc[32];  // [16 * (kStage == 2) + region], [.. + 15] = waves
#endif

#ifndef GPC_WAVES_PER_EU
#define GPC_WAVES_PER_EU 6
#endif
// Journal-mode kernels run at 5 waves per SIMD: 96 VGPRs hold them without spills (at 6 they
// spill 13-44 VGPRs, 36-52 B of scratch per lane), and C5 measured 6.00 vs 6.10 ms per step
// (profiles/r05rs_occupancy_parking_ab.txt). The base kernels stay at 6 (C3 5.09 ms at 6 waves
// against 5.54 at 5), and since round 6 the extension-mode ones too: the two-level extension probe
// with its bucket ranges loaded up front fits 80 VGPRs without spills (tools/kres.sh).
#ifndef GPC_DELTA_WAVES_PER_EU
#define GPC_DELTA_WAVES_PER_EU 5
#endif
#ifndef GPC_EXT_WAVES_PER_EU
#define GPC_EXT_WAVES_PER_EU 6
#endif
#ifndef GPC_BLOCK
#define GPC_BLOCK 64
#endif
// One wavefront per block for the plain kernels (C3: 14.73 ms at 256 threads, 14.36 at 128, 14.24
// at 64 -- finished waves free their slot without waiting for block siblings); the lane-regrouping
// kernels sort 256 packets across 4 waves, which needs the larger block.
constexpr int kBlock = GPC_BLOCK;
constexpr int kSortBlock = 256;
template <bool kSort>
constexpr int block_threads() { return kSort ? kSortBlock : kBlock; }

// kDelta = false: a base-only epoch (no tombstones, no journal); kSvc = false: no Services. The
// machinery of either folds away at compile time so the common case pays nothing for it.
// kStage: without Services the two policy stages run as two launches over the batch (1 = egress,
// 2 = ingress, which reads the egress verdict back); every lane of a launch then runs the same
// stage, measured 8 % faster on C3 than one launch walking both stages (kStage = 0; lanes leave the
// egress stage at different times). With Services one launch (0) does both stages: a second
// launch would have to repeat the Service lookup, which costs more than the split saves (C4).
// IPv6 batches: a first launch maps every IPv6 address of the batch to its code in
// the IPv6 image (core.hpp v6_codes), one address per lane, into 32-bit code columns; the batch is
// then an IPv4-shaped batch over the codes and takes the IPv4 launches (grouping, both policy
// stages, un-permute) against the IPv6 image unchanged. The length descriptors of the binary search
// are copied to LDS once per block, so a step's only memory access is its two bucket loads.
constexpr int kCodeBlock = 256;
struct V6Cols {
  const uint8_t* c[4];  // src6, dst6, ct_src6, ct_dst6 (16 network-order bytes per packet, 16-B aligned)
};
// kDelta: an IPv6 delta epoch, whose journal header may carry an overflow table (probed in the same
// step). One address per lane: four lanes of a quad cooperating on one address (each loading 16 B of
// a 64-B bucket: whole lines per wave-instruction, a quarter of the independent searches in flight)
// measured slower on C3 in IPv6 (8.92 vs 7.95 ms per 128M addresses).
template <bool kDelta>
__global__ __launch_bounds__(kCodeBlock) void v6_code_kernel(EpochArgs ep, V6Cols cols, uint64_t n,
                                                             uint32_t* __restrict__ codes) {
  __shared__ V6Len desc[kV6MaxLens];
  const V6Lpm* L = reinterpret_cast<const V6Lpm*>(ep.blob + ep.v6_lpm);
  const uint32_t words = L->n_lens * uint32_t(sizeof(V6Len) / 4);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(L->d);
  for (uint32_t j = threadIdx.x; j < words; j += kCodeBlock) reinterpret_cast<uint32_t*>(desc)[j] = src[j];
  __syncthreads();
  const uint64_t i = uint64_t(blockIdx.x) * kCodeBlock + threadIdx.x;
  if (i >= n) return;
  const uint4 v = reinterpret_cast<const uint4*>(cols.c[blockIdx.y])[i];
  const uint32_t a[1][4] = {{__builtin_bswap32(v.x), __builtin_bswap32(v.y), __builtin_bswap32(v.z), __builtin_bswap32(v.w)}};
  const uint32_t* ovf = nullptr;
  uint32_t ovf_log2 = 0;
  if (kDelta) {
    const JournalHdr* jh = reinterpret_cast<const JournalHdr*>(ep.pool + ep.jhdr);
    if (jh->v6_ovf_off) {
      ovf = ep.pool + jh->v6_ovf_off;
      ovf_log2 = jh->v6_ovf_log2;
    }
  }
  uint32_t code;
  if (ovf) {
    v6_codes<1, true>(ep.blob, ep.v6_lpm, a, &code, ovf, ovf_log2, desc);
  } else {
    v6_codes<1>(ep.blob, ep.v6_lpm, a, &code, nullptr, 0, desc);
  }
  codes[uint64_t(blockIdx.y) * n + i] = code;
}

// Lane regrouping for a policy stage launch: the candidate scan of a wavefront runs as long as its
// longest lane (the wave-uniform trip count of eval_part), so when the host saw long driver lists
// in the stage's main table (api.cpp lane_sort_tables) the block's packets are regrouped by their
// scan length in that table before any table work: a counting sort of 256 lanes over 64 length
// bins in LDS, then lane t classifies the packet perm[t] of its block. Verdicts and counters are
// per packet, so the order never shows. Every thread of the block calls this (barriers); returns
// the packet index this lane now owns (>= n: none).
template <int kStage>
__device__ __forceinline__ uint64_t sorted_index(const EpochArgs& ep, const gpc_pkt_soa& pk, uint64_t n,
                                                 const uint4* __restrict__ out, const uint2* __restrict__ mid,
                                                 uint64_t block_base, uint32_t* pkt_lds) {
  constexpr uint32_t kBins = 64;  // one wavefront scans the histogram
  __shared__ uint32_t hist[kBins];
  __shared__ uint16_t perm[kSortBlock];
  const uint64_t i = block_base + threadIdx.x;
  const uint32_t tid = threadIdx.x;
  uint32_t est = 0;
  if (i < n) {
    bool live = true;
    if (kStage == 2) {  // packets the ingress launch settles without table work weigh nothing
      const uint32_t ea = (mid ? mid[i].y : out[i].y) & 0xffu;
      live = ea != RV_DROP && ea != RV_REJECT && ea != RV_ISO_DROP &&
             !ingress_bypass(ep.hdr->isc, pk.dest ? pk.dest[i] : 0u, pk.ct_mark ? pk.ct_mark[i] : 0u);
    }
    if (live) {
      const uint32_t src = pk.src[i], dst = pk.dst[i];
      Pkt p(pkt_lds + tid, kSortBlock);
      make_axes(p, src, dst, pk.sport[i], pk.dport[i], pk.proto[i], pk.out_port[i], pk.in_port ? pk.in_port[i] : 0u,
                pk.svc_group ? pk.svc_group[i] : 0u, pk.tun_id ? pk.tun_id[i] : 0u, pk.ct_src ? pk.ct_src[i] : src,
                pk.ct_dst ? pk.ct_dst[i] : dst, pk.ct_state ? pk.ct_state[i] : uint32_t(GPC_CT_NEW | GPC_CT_TRK));
      const Img im{ep.blob, ep.hdr, nullptr, nullptr};
      est = scan_estimate(im, ep.sort_table[kStage - 1], p);
    }
  }
  const uint32_t bin = est >> 1 < kBins - 1 ? est >> 1 : kBins - 1;
  if (tid < kBins) hist[tid] = 0;
  __syncthreads();
  const uint32_t r = atomicAdd(&hist[bin], 1u);
  __syncthreads();
  if (tid < kBins) {  // exclusive prefix sum over the bins
    const uint32_t v = hist[tid];
    uint32_t x = v;
#pragma unroll
    for (uint32_t d = 1; d < kBins; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, kBins);
      if (tid >= d) x += y;
    }
    hist[tid] = x - v;
  }
  __syncthreads();
  perm[hist[bin] + r] = uint16_t(tid);
  __syncthreads();
  return block_base + perm[tid];
}

// Packet grouping. Lanes of a wavefront that classify packets of one address
// region share driver buckets, candidate lists and rule records, so their loads coalesce and their
// scans run the same length. For a grouped batch a first launch rewrites every tile of kGroupTile
// packets in the order of group_key (top bits of nw_src, then of nw_dst; a counting sort in LDS, then every present
// column staged through LDS: coalesced reads and writes) and records each grouped packet's caller
// index. The egress launch leaves its verdict in mid[] (grouped order); the ingress launch (or the
// single Service launch) stores the verdict pair / LB result at the caller index. The blocks of
// one tile run on one XCD (block_xcd_order), so those scattered stores stay inside one tile's
// window of one L2 and leave it as whole lines. Packets are independent and counters are sums:
// the grouping never shows in the results.
constexpr uint32_t kGroupThreads = 1024, kGroupBins = 256, kGroupTile = 16384;

template <typename T>
__device__ __forceinline__ void group_column(const T* __restrict__ in, T* __restrict__ outc, uint64_t base, uint32_t m,
                                             const uint16_t* from, void* stage) {
  T* buf = reinterpret_cast<T*>(stage);
  __syncthreads();  // the previous column's reads of `stage` are done
  for (uint32_t j = threadIdx.x; j < m; j += kGroupThreads) buf[j] = in[base + j];
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < m; k += kGroupThreads) outc[base + k] = buf[from[k]];
}

// Grouping key of a packet: the top src_bits of nw_src followed by the top 8 - src_bits of nw_dst.
__device__ __forceinline__ uint32_t group_key(uint32_t src, uint32_t dst, uint32_t src_bits) {
  const uint32_t db = 8u - src_bits;
  const uint32_t hi = src_bits ? (src >> (32u - src_bits)) << db : 0u;
  return hi | (db ? dst >> (32u - db) : 0u);
}

// Scan-length key (GroupArgs.key == GPC_GROUP_KEY_SCAN): the candidate scan of a wavefront runs as
// long as its longest lane, so lanes whose walks scan equally long driver lists belong together.
// Per policy stage the packet's driver-list length (core.hpp scan_estimate, summed over the stage's
// tables: the bucket offsets only, no entry is read) binned to 4 bits, floor(1.5 sqrt(len)) capped
// at 15 (finer where most packets are); key = egress bin << 4 | ingress bin. `axes`: the axes the
// image's sub-indexes read (only those columns are loaded); ax: this thread's LDS column of axes.
__device__ __forceinline__ uint32_t scan_bin(uint32_t len) {
  const uint32_t b = uint32_t(1.5f * sqrtf(float(len)));
  return b < 15u ? b : 15u;
}
__device__ __forceinline__ uint32_t scan_key(const EpochArgs& ep, const gpc_pkt_soa& in, uint64_t i, uint32_t axes,
                                             uint32_t* ax) {
  auto has = [&](uint32_t a) { return (axes >> a) & 1u; };
  const uint32_t src = has(AX_SRC) || (has(AX_CTSRC) && !in.ct_src) ? in.src[i] : 0u;
  const uint32_t dst = has(AX_DST) || (has(AX_CTDST) && !in.ct_dst) ? in.dst[i] : 0u;
  const bool l4 = has(AX_L4D) || has(AX_L4S);
  Pkt p(ax, kGroupThreads);
  make_axes(p, src, dst, has(AX_L4S) ? in.sport[i] : 0u, has(AX_L4D) ? in.dport[i] : 0u, l4 ? in.proto[i] : 0u,
            has(AX_REG1) ? in.out_port[i] : 0u, has(AX_INPORT) && in.in_port ? in.in_port[i] : 0u,
            has(AX_REG7) && in.svc_group ? in.svc_group[i] : 0u, has(AX_TUN) && in.tun_id ? in.tun_id[i] : 0u,
            has(AX_CTSRC) && in.ct_src ? in.ct_src[i] : src, has(AX_CTDST) && in.ct_dst ? in.ct_dst[i] : dst,
            has(AX_CTST) && in.ct_state ? in.ct_state[i] : uint32_t(GPC_CT_NEW | GPC_CT_TRK));
  const Img im{ep.blob, ep.hdr, nullptr, nullptr};
  uint32_t e = 0, g = 0;
#pragma unroll
  for (uint32_t t = 1; t <= 3; t++) {
    e += scan_estimate(im, t, p);
    g += scan_estimate(im, t + 3, p);
  }
  return scan_bin(e) << 4 | scan_bin(g);
}

// key_mode GPC_GROUP_KEY_SCAN: scan_key; GPC_GROUP_KEY_ADDR: group_key (IPv6 batches: over the codes).
__global__ __launch_bounds__(kGroupThreads) void group_tiles_kernel(EpochArgs ep, gpc_pkt_soa in, uint64_t n,
                                                                    uint32_t key_mode, uint32_t axes, uint32_t src_bits,
                                                                    gpc_pkt_soa g, uint32_t* __restrict__ orig) {
  __shared__ uint32_t stage[kGroupTile];  // the tile's keys, then one column of the tile
  __shared__ uint16_t from[kGroupTile];   // grouped position -> tile position
  __shared__ uint32_t cur[kGroupBins];
  __shared__ uint32_t axl[AX_N * kGroupThreads];  // scan_key: per-thread packet axes, [axis][thread]
  const uint32_t tid = threadIdx.x;
  const uint64_t base = uint64_t(blockIdx.x) * kGroupTile;
  const uint32_t m = uint32_t(n - base < kGroupTile ? n - base : kGroupTile);
  if (tid < kGroupBins) cur[tid] = 0;
  if (key_mode == GPC_GROUP_KEY_SCAN) {
    for (uint32_t j = tid; j < m; j += kGroupThreads) stage[j] = scan_key(ep, in, base + j, axes, axl + tid);
  } else if (src_bits == 8u) {
    for (uint32_t j = tid; j < m; j += kGroupThreads) stage[j] = in.src[base + j] >> 24;
  } else {
    for (uint32_t j = tid; j < m; j += kGroupThreads) stage[j] = group_key(in.src[base + j], in.dst[base + j], src_bits);
  }
  __syncthreads();
  for (uint32_t j = tid; j < m; j += kGroupThreads) atomicAdd(&cur[stage[j]], 1u);
  __syncthreads();
  if (tid < 64) {  // exclusive prefix over the 256 bins: one wavefront, 4 bins per lane
    const uint32_t c0 = cur[4 * tid], c1 = cur[4 * tid + 1], c2 = cur[4 * tid + 2], c3 = cur[4 * tid + 3];
    const uint32_t v = c0 + c1 + c2 + c3;
    uint32_t x = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (tid >= d) x += y;
    }
    const uint32_t e = x - v;
    cur[4 * tid] = e;
    cur[4 * tid + 1] = e + c0;
    cur[4 * tid + 2] = e + c0 + c1;
    cur[4 * tid + 3] = e + c0 + c1 + c2;
  }
  __syncthreads();
  for (uint32_t j = tid; j < m; j += kGroupThreads) from[atomicAdd(&cur[stage[j]], 1u)] = uint16_t(j);
  __syncthreads();
  for (uint32_t k = tid; k < m; k += kGroupThreads) orig[base + k] = uint32_t(base + from[k]);
#define GPC_GROUP_COL(c, T) \
  if (in.c) group_column<T>(in.c, const_cast<T*>(g.c), base, m, from, stage)
  GPC_GROUP_COL(src, uint32_t);
  GPC_GROUP_COL(dst, uint32_t);
  GPC_GROUP_COL(sport, uint16_t);
  GPC_GROUP_COL(dport, uint16_t);
  GPC_GROUP_COL(proto, uint8_t);
  GPC_GROUP_COL(out_port, uint32_t);
  GPC_GROUP_COL(in_port, uint32_t);
  GPC_GROUP_COL(svc_group, uint32_t);
  GPC_GROUP_COL(tun_id, uint32_t);
  GPC_GROUP_COL(ct_src, uint32_t);
  GPC_GROUP_COL(ct_dst, uint32_t);
  GPC_GROUP_COL(ct_state, uint8_t);
  GPC_GROUP_COL(dest, uint8_t);
  GPC_GROUP_COL(len, uint16_t);
  GPC_GROUP_COL(ct_mark, uint8_t);
#undef GPC_GROUP_COL
}

// Logical block of this workgroup for a grouped batch: workgroups are dispatched round-robin over
// the 8 XCDs, so XCD x (blocks b with b % 8 == x) gets the contiguous logical range
// [x*q + min(x, r), ...) of the G = 8q + r blocks. A bijection whatever the dispatch order.
__device__ __forceinline__ uint64_t block_xcd_order() {
  const uint32_t b = blockIdx.x, G = gridDim.x, q = G >> 3, r = G & 7u, x = b & 7u;
  return uint64_t(x) * q + (x < r ? x : r) + (b >> 3);
}

// Logical block of this workgroup for a grouped batch (GroupArgs.xcd_order):
//   1: XCD-contiguous tiles (block_xcd_order);
//   2: tile-interleaved -- workgroups running at the same time take the same position of many
//      tiles (wave k of tiles t, t+1, ...), so the whole chip works on one key range at a time (the
//      image lines of that address region stay in every L2), as after a global sort by key;
//   3: as 2, with the tiles of XCD x = those with t % 8 == x (its verdict stores stay in its L2).
// kTileBlocks workgroups per full tile; the blocks of a last partial tile keep their order.
template <int kTileBlocks>
__device__ __forceinline__ uint64_t logical_block(uint32_t mode) {
  if (mode == 1) return block_xcd_order();
  const uint32_t b = blockIdx.x, T = gridDim.x / kTileBlocks;
  if (mode < 2 || T == 0 || b >= T * kTileBlocks) return b;
  if (mode == 3 && (T & 7u) == 0) {
    const uint32_t x = b & 7u, j = b >> 3, tx = T >> 3;
    return uint64_t(x + 8u * (j % tx)) * kTileBlocks + j / tx;
  }
  return uint64_t(b % T) * kTileBlocks + b / T;
}

// orig != null: a grouped batch (group_tiles_kernel): pk holds the grouped columns, lane i of the
// logical block order classifies grouped packet i, whose caller index is orig[i]. IPv6 batches come
// here as code columns (v6_code_kernel) against the IPv6 image.
// Packet i of the batch through the Service stage (kSvc) and the policy stage(s) of the launch;
// pkt_lane / pkt_stride: this lane's column of the block's [word][lane] packet table in LDS.
template <int kDelta, bool kSvc, int kStage>
__device__ __forceinline__ void classify_one(const EpochArgs& ep, const gpc_pkt_soa& pk, uint64_t i, uint4* __restrict__ out,
                                             uint4* __restrict__ lb_out, unsigned long long* __restrict__ counters, int count,
                                             const uint32_t* __restrict__ orig, uint2* __restrict__ mid,
                                             uint2* __restrict__ gout, uint4* __restrict__ park, uint32_t* pkt_lane,
                                             uint32_t pkt_stride, uint32_t i_hi) {
  // Ingress launch: only the egress action of the egress half is read here; nothing of it is held
  // over the walk (the result is stored as a half).
  uint32_t ea = 0;
  if (kStage == 2) ea = (mid ? mid[i].y : reinterpret_cast<const uint2*>(out)[2 * i].y) & 0xffu;
  // caller index of this packet (loaded where a result is stored: no register held over the walk)
  auto at = [&](uint64_t k) -> uint64_t { return orig ? uint64_t(orig[k]) : k; };
  // the ingress launch's result: its half of the verdict pair in grouped order into gout
  // (unpermute_kernel joins it with the egress half in mid and stores the pair in caller order with
  // whole-line stores); grouped without the un-permute, or ungrouped with the egress halves in mid
  // (the split store), the pair at the caller index with the egress half re-read from mid; else
  // the ingress half of the pair the egress launch stored
  auto store2 = [&](uint64_t k, uint32_t conj, uint32_t packed) {
    if (gout) {
      gout[k] = make_uint2(conj, packed);
    } else if (mid) {
      const uint2 e = mid[k];
      out[at(k)] = make_uint4(e.x, e.y, conj, packed);
    } else {
      reinterpret_cast<uint2*>(out)[2 * k + 1] = make_uint2(conj, packed);
    }
  };
  uint32_t src = pk.src[i], dst = pk.dst[i];
  const uint32_t ct_src = pk.ct_src ? pk.ct_src[i] : src;
  const uint32_t ct_dst = pk.ct_dst ? pk.ct_dst[i] : dst;  // pre-NAT destination
  uint32_t dport = pk.dport[i];
  const uint32_t sport = pk.sport[i], proto = pk.proto[i];
  uint32_t out_port = pk.out_port[i];
  uint32_t svc_group = pk.svc_group ? pk.svc_group[i] : 0u;
  uint32_t dest = pk.dest ? pk.dest[i] : 0u;
  const uint32_t ct_mark = pk.ct_mark ? pk.ct_mark[i] : 0u;
  // Service stage. kStage 0: one launch does it and both policy stages. kStage 1 / 2 (Service
  // batches split like the others): the egress launch runs it and parks the fields it rewrites
  // (destination, port, reg1 / reg7, destination mark) in park[i]; the ingress launch reads them back
  // instead of repeating the lookup. NO_ENDPOINT: rejected in EndpointDNAT before the policy
  // stages, so the ingress launch sees a REJECT egress action and stores ingress NONE.
  if (kSvc && kStage == 2) {
    // (read after the egress-action check below)
  } else if (kSvc) {
    uint32_t lb[4];
    const uint32_t f = lb_stage(ep.svc, src, dst, sport, dport, proto, svc_group, out_port, dest, lb);
    // grouped with the un-permute (gout): results in grouped order, unpermute_kernel stores them
    if (lb_out) lb_out[gout ? i : at(i)] = make_uint4(lb[0], lb[1], lb[2], lb[3]);
    if (kStage == 1) park[i] = make_uint4(dst, (dport & 0xffffu) | (dest << 16), out_port, svc_group);
    if (f & GPC_LB_NO_ENDPOINT) {  // EndpointDNAT serviceNoEndpointFlow: rejected before the policy stages
      const uint32_t rj = pack_verdict(GPC_ACT_REJECT, GPC_VTABLE_ENDPOINT_DNAT, 0, 0);
      if (kStage == 0 && gout) {
        mid[i] = make_uint2(0u, rj);
        gout[i] = make_uint2(0u, 0u);
      } else if (kStage == 1 && mid) {
        mid[i] = make_uint2(0u, rj);
      } else if (kStage == 1) {
        out[i] = make_uint4(0u, rj, 0u, 0u);
      } else {
        out[at(i)] = make_uint4(0u, rj, 0u, 0u);
      }
      return;
    }
  } else if (kStage != 2 && lb_out) {
    lb_out[at(i)] = make_uint4(0u, 0u, 0u, 0u);
  }
  if (kStage == 2) {  // only packets the egress stage let through reach the ingress tables
    if (ea == RV_DROP || ea == RV_REJECT || ea == RV_ISO_DROP) {
      if (mid) store2(i, 0u, 0u);  // ingress NONE
      return;
    }
    if (kSvc) {  // the fields the egress launch's Service stage rewrote
      const uint4 pv = park[i];
      dst = pv.x;
      dport = pv.y & 0xffffu;
      dest = pv.y >> 16;
      out_port = pv.z;
      svc_group = pv.w;
    }
    if (const uint32_t b = ingress_bypass(ep.hdr->isc, dest, ct_mark)) {  // IngressSecurityClassifier
      store2(i, 0u, pack_verdict(b & 0xffu, 0, 0, (b >> 8) ? 2u : 0u));
      return;
    }
  }
  View im{{ep.blob, ep.hdr, nullptr, ep.pool}, {ep.pool, nullptr, nullptr, ep.pool}, 1u, ep.jhdr, 0u};
  if (kDelta != kModeBase) {
    const JournalHdr* jh = reinterpret_cast<const JournalHdr*>(ep.pool + ep.jhdr);
    im.ext = jh->ext_off;
    if (kDelta == kModeJournal) {
      if (jh->bdead_off) im.base.dead = ep.pool + jh->bdead_off;
      im.n_img = 2u;
    }
  }
  Pkt p(pkt_lane, pkt_stride);
  make_pkt(p, src, dst, sport, dport, proto, out_port, pk.in_port ? pk.in_port[i] : 0u, svc_group,
           pk.tun_id ? pk.tun_id[i] : 0u, ct_src, ct_dst, pk.ct_state ? pk.ct_state[i] : uint32_t(GPC_CT_NEW | GPC_CT_TRK),
           view_bloom_axes(im));
  // The packet index is parked in the lane's LDS column for the walk and read back after it
  // ("memory" clobber: the reload, and that of the packet's ct_state in count_stage, cannot be
  // forwarded from the registers they were stored from), so neither is held in a VGPR over the
  // walk -- they were the base kernels' only spills (20-28 B of scratch per lane).
  pkt_lane[kPktWords * pkt_stride] = uint32_t(i);
  auto late = [&]() -> uint64_t {
    lds_reload();
    return (uint64_t(i_hi) << 32) | pkt_lane[kPktWords * pkt_stride];
  };
  auto count_one = [&](const StageOut& s, uint64_t k) {  // a stage's Metric-table counters
    if (!count || !s.counted) return;
    const uint32_t len = pk.len ? pk.len[k] : 0u;
    unsigned long long* const copy = counters + size_t(blockIdx.x & ep.ctr_mask) * ep.ctr_stride;
    count_stage(s.v, s.slot, len, p.ax[AX_CTST], [&](uint32_t w, unsigned long long v) { atomicAdd(&copy[w], v); });
  };
  if constexpr (kStage == 0) {
    // Both stages in one launch (Services): the egress half is counted and stored before the
    // ingress walk, so nothing of it is held over that walk.
    // (the ingress bypass is parked next to the index: nothing of the Service stage is held in a
    // register over the egress walk)
    pkt_lane[(kPktWords + 1) * pkt_stride] = ingress_bypass(ep.hdr->isc, dest, ct_mark);
    const StageOut s1 = walk_stage<kDelta, false>(im, p, 1u, nullptr, nullptr);
    const uint64_t i1 = late();
    const uint32_t byp = pkt_lane[(kPktWords + 1) * pkt_stride];
    count_one(s1, i1);
    uint2* const o2 = reinterpret_cast<uint2*>(out);
    if (gout) mid[i1] = make_uint2(s1.v.conj, s1.v.packed);  // grouped order (un-permuted afterwards)
    else o2[2 * at(i1)] = make_uint2(s1.v.conj, s1.v.packed);
    const uint32_t a1 = s1.v.packed & 0xffu;
    uint32_t gc = 0u, gp = 0u;  // ingress NONE: dropped in egress
    if (a1 != RV_DROP && a1 != RV_REJECT && a1 != RV_ISO_DROP) {
      if (byp) {  // IngressSecurityClassifier
        gp = pack_verdict(byp & 0xffu, 0, 0, (byp >> 8) ? 2u : 0u);
      } else {
        const StageOut s2 = walk_stage<kDelta, false>(im, p, 4u, nullptr, nullptr);
        count_one(s2, late());
        gc = s2.v.conj;
        gp = s2.v.packed;
      }
    }
    const uint64_t i2 = late();
    if (gout) gout[i2] = make_uint2(gc, gp);
    else o2[2 * at(i2) + 1] = make_uint2(gc, gp);
    return;
  }
  const StageOut s = walk_stage<kDelta, false>(im, p, kStage == 2 ? 4u : 1u, nullptr, nullptr);
  const uint64_t il = late();
  count_one(s, il);
  const VerdictOut e = s.v, g = s.v;
  if (kStage == 2) store2(il, g.conj, g.packed);
  else if (kStage == 1 && mid) mid[il] = make_uint2(e.conj, e.packed);
  else out[il] = make_uint4(e.conj, e.packed, 0u, 0u);  // ingress NONE until the second launch
}

// kDelta: the epoch mode (core.hpp kModeBase / kModeExt / kModeJournal).
template <int kDelta, bool kSvc, int kStage, bool kSort = false>
__global__ __launch_bounds__(block_threads<kSort>()) __attribute__((amdgpu_waves_per_eu(kDelta == kModeJournal ? GPC_DELTA_WAVES_PER_EU : kDelta == kModeExt ? GPC_EXT_WAVES_PER_EU : GPC_WAVES_PER_EU))) void classify_kernel(
    EpochArgs ep, gpc_pkt_soa pk, uint64_t n, uint4* __restrict__ out, uint4* __restrict__ lb_out,
    unsigned long long* __restrict__ counters, int count, const uint32_t* __restrict__ orig, uint2* __restrict__ mid,
    uint32_t xcd_order, uint2* __restrict__ gout, uint4* __restrict__ park) {
  // per-lane packet axes / filter bits: a [word][lane] table in LDS (core.hpp Pkt)
  __shared__ uint32_t pkt_lds[(kPktWords + 2) * block_threads<kSort>()];  // + the parked index and bypass
#if defined(GPC_STAMPS)
  {
    uint32_t* st = gpc_stamp_lds();
    if (threadIdx.x < ST_N + 1) st[threadIdx.x] = threadIdx.x == ST_N ? uint32_t(ST_PRE) : 0u;
    const uint64_t now = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) st[ST_N + 1] = uint32_t(now), st[ST_N + 2] = uint32_t(now >> 32);
    __syncthreads();
  }
  auto body = [&]() {
#else
  {
#endif
  const uint64_t block_base = logical_block<kGroupTile / block_threads<kSort>()>(xcd_order) * block_threads<kSort>();
  uint64_t i = block_base + threadIdx.x;
  if constexpr (kSort) i = sorted_index<kStage>(ep, pk, n, out, mid, block_base, pkt_lds);  // own instantiation: the plain kernel has no barrier
  if (i >= n) return;
  classify_one<kDelta, kSvc, kStage>(ep, pk, i, out, lb_out, counters, count, orig, mid, gout, park,
                                     pkt_lds + threadIdx.x, block_threads<kSort>(), uint32_t(block_base >> 32));
#if defined(GPC_STAMPS)
  };
  body();
  gpc_mark(ST_POST);
  __syncthreads();
  uint32_t* st = gpc_stamp_lds();
  constexpr uint32_t sb = kStage == 2 ? 16u : 0u;
  if (threadIdx.x < ST_N) atomicAdd(&gpc_stamp_acc[sb + threadIdx.x], (unsigned long long)st[threadIdx.x]);
  if (threadIdx.x == 0) atomicAdd(&gpc_stamp_acc[sb + 15], 1ull);
#else
  }
#endif
}

// Verdict pairs of a grouped batch in caller order: the egress half from mid (grouped order, every
// mid_words words) and the ingress half from gout (grouped order, both written with coalesced
// stores by the classification launches) joined and stored at the caller index; with lbg, the
// Service launch's LB results (grouped order) too. One 1024-thread block per grouping tile; each
// half of the tile's caller range is assembled in LDS (128 KB of 16-B records, loads four deep per
// thread) and written with whole-line stores. Replaces 16-B stores scattered over the tile (C3:
// 0.84 ms of 13.5 per 64M packets).
constexpr uint32_t kUnpermHalf = kGroupTile / 2;

// One tile's 16-B records, grouped position k -> caller position orig[k], through buf.
template <typename Load>
__device__ __forceinline__ void permute_tile(uint4* buf, const uint32_t* __restrict__ orig, uint64_t base, uint32_t m,
                                             Load load, uint4* __restrict__ dst) {
  constexpr int kU = 4;  // loads in flight per thread (all issued before any is used)
  // (the staged records are held as word arrays: arrays of uint4 are not promoted to registers)
  for (uint32_t h = 0; h * kUnpermHalf < m; h++) {
    const uint32_t lo = h * kUnpermHalf, cnt = m - lo < kUnpermHalf ? m - lo : kUnpermHalf;
    __syncthreads();  // the previous pass's reads of buf are done
    for (uint32_t k0 = threadIdx.x; k0 < m; k0 += kU * kGroupThreads) {
      uint32_t d[kU], x[kU], y[kU], z[kU], w[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t k = k0 + u * kGroupThreads;
        d[u] = k < m ? orig[base + k] - uint32_t(base) - lo : 0xffffffffu;  // position in this half (wraps if outside)
      }
#pragma unroll
      for (int u = 0; u < kU; u++) {
        x[u] = y[u] = z[u] = w[u] = 0;
        if (d[u] < cnt) {
          const uint4 v = load(base + k0 + u * kGroupThreads);
          x[u] = v.x, y[u] = v.y, z[u] = v.z, w[u] = v.w;
        }
      }
#pragma unroll
      for (int u = 0; u < kU; u++)
        if (d[u] < cnt) buf[d[u]] = make_uint4(x[u], y[u], z[u], w[u]);
    }
    __syncthreads();
    for (uint32_t j0 = threadIdx.x; j0 < cnt; j0 += kU * kGroupThreads) {
      uint32_t x[kU], y[kU], z[kU], w[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) {
        x[u] = y[u] = z[u] = w[u] = 0;
        if (j0 + u * kGroupThreads < cnt) {
          const uint4 v = buf[j0 + u * kGroupThreads];
          x[u] = v.x, y[u] = v.y, z[u] = v.z, w[u] = v.w;
        }
      }
#pragma unroll
      for (int u = 0; u < kU; u++)
        if (j0 + u * kGroupThreads < cnt) dst[base + lo + j0 + u * kGroupThreads] = make_uint4(x[u], y[u], z[u], w[u]);
    }
  }
}

__global__ __launch_bounds__(kGroupThreads) void unpermute_kernel(const uint32_t* __restrict__ mid, uint32_t mid_words,
                                                                  const uint2* __restrict__ gout,
                                                                  const uint32_t* __restrict__ orig, uint64_t n,
                                                                  uint4* __restrict__ out, const uint4* __restrict__ lbg,
                                                                  uint4* __restrict__ lb_out) {
  __shared__ uint4 buf[kUnpermHalf];
  const uint64_t base = uint64_t(blockIdx.x) * kGroupTile;
  const uint32_t m = uint32_t(n - base < kGroupTile ? n - base : kGroupTile);
  permute_tile(
      buf, orig, base, m,
      [&](uint64_t k) {
        const uint2 e = *reinterpret_cast<const uint2*>(mid + k * mid_words), g = gout[k];
        return make_uint4(e.x, e.y, g.x, g.y);
      },
      out);
  if (lbg) permute_tile(buf, orig, base, m, [&](uint64_t k) { return lbg[k]; }, lb_out);
}

static void launch_unpermute(const void* mid, uint32_t mid_words, const uint2* gout, const uint32_t* orig, uint64_t n,
                             uint4* out, const uint4* lbg, uint4* lb_out, hipStream_t stream, LaunchMarks* marks) {
  const uint64_t tiles = (n + kGroupTile - 1) / kGroupTile;
  launch_mark(marks, kLaunchUnpermute, stream);
  hipLaunchKernelGGL(unpermute_kernel, dim3(uint32_t(tiles)), dim3(kGroupThreads), 0, stream,
                     reinterpret_cast<const uint32_t*>(mid), mid_words, gout, orig, n, out, lbg, lb_out);
}

template <int kDelta, bool kSvc>
static void launch(const EpochArgs& ep, const gpc_pkt_soa& pk, uint64_t n, gpc_verdict* out, uint4* lb_out,
                   unsigned long long* counters, int count, const uint32_t* orig, uint2* mid, uint32_t xo, uint2* gout,
                   uint4* park, hipStream_t stream, LaunchMarks* marks) {
  const uint64_t blocks = (n + kBlock - 1) / kBlock;
  uint4* const o = reinterpret_cast<uint4*>(out);
  if (kSvc && park) {  // split like the Service-free batches, the rewritten fields parked in between
    launch_mark(marks, kLaunchEgress, stream);
    hipLaunchKernelGGL((classify_kernel<kDelta, true, 1>), dim3(uint32_t(blocks)), dim3(kBlock), 0, stream, ep, pk, n, o,
                       lb_out, counters, count, orig, mid, xo, gout, park);
    launch_mark(marks, kLaunchIngress, stream);
    hipLaunchKernelGGL((classify_kernel<kDelta, true, 2>), dim3(uint32_t(blocks)), dim3(kBlock), 0, stream, ep, pk, n, o,
                       lb_out, counters, count, orig, mid, xo, gout, park);
    return;
  }
  if (kSvc) {
    launch_mark(marks, kLaunchBoth, stream);
    hipLaunchKernelGGL((classify_kernel<kDelta, true, 0>), dim3(uint32_t(blocks)), dim3(kBlock), 0, stream, ep, pk, n, o,
                       lb_out, counters, count, orig, mid, xo, gout, nullptr);
    return;
  }
  // One launch for both stages unless a stage regroups its lanes by scan length (the sort is per
  // stage). Round 2 measured the split 8 % faster on C3 (lanes leave the egress stage at different
  // times); on the zero-scratch kernels one launch is faster (C3 4.70 -> 4.54 ms per 64 M packets,
  // profiles/r06b_*): no egress verdict round trip through HBM and one read of the packet columns.
  // GPC_FUSED=0 / 1 forces the split / the single launch (A/B experiments).
  static const int fused_env = std::getenv("GPC_FUSED") ? std::atoi(std::getenv("GPC_FUSED")) : -1;
  // (journal epochs keep the split: their fused kernel would spill at 5 waves)
  const bool fused = fused_env == 1 || (fused_env < 0 && kDelta != kModeJournal && !ep.sort_table[0] && !ep.sort_table[1]);
  if (fused) {
    launch_mark(marks, kLaunchBoth, stream);
    hipLaunchKernelGGL((classify_kernel<kDelta, false, 0>), dim3(uint32_t(blocks)), dim3(kBlock), 0, stream, ep, pk, n, o,
                       lb_out, counters, count, orig, mid, xo, gout, nullptr);
    return;
  }
  const uint64_t sblocks = (n + kSortBlock - 1) / kSortBlock;
  launch_mark(marks, kLaunchEgress, stream);
  if (ep.sort_table[0])
    hipLaunchKernelGGL((classify_kernel<kDelta, false, 1, true>), dim3(uint32_t(sblocks)), dim3(kSortBlock), 0, stream,
                       ep, pk, n, o, lb_out, counters, count, orig, mid, xo, nullptr, nullptr);
  else
    hipLaunchKernelGGL((classify_kernel<kDelta, false, 1>), dim3(uint32_t(blocks)), dim3(kBlock), 0, stream, ep, pk, n, o,
                       lb_out, counters, count, orig, mid, xo, nullptr, nullptr);
  launch_mark(marks, kLaunchIngress, stream);
  if (ep.sort_table[1])
    hipLaunchKernelGGL((classify_kernel<kDelta, false, 2, true>), dim3(uint32_t(sblocks)), dim3(kSortBlock), 0, stream,
                       ep, pk, n, o, lb_out, counters, count, orig, mid, xo, gout, nullptr);
  else
    hipLaunchKernelGGL((classify_kernel<kDelta, false, 2>), dim3(uint32_t(blocks)), dim3(kBlock), 0, stream, ep, pk, n, o,
                       lb_out, counters, count, orig, mid, xo, gout, nullptr);
}

// gpc_trace: one packet through the same table walk as classify_kernel (Service stage and journal
// included), recording every rule table it evaluates. One lane; debug path, not the data path.
__global__ void trace_kernel(EpochArgs ep, gpc_pkt_soa pk, uint4* __restrict__ out, uint4* __restrict__ lb_out,
                             TraceStep* __restrict__ steps, uint32_t* __restrict__ n_steps) {
  __shared__ uint32_t pkt_lds[kPktWords];
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t src = pk.src[0], dst = pk.dst[0], dport = pk.dport[0];
  const uint32_t sport = pk.sport[0], proto = pk.proto[0];
  const uint32_t ct_src = pk.ct_src ? pk.ct_src[0] : src;
  const uint32_t ct_dst = pk.ct_dst ? pk.ct_dst[0] : dst;
  uint32_t out_port = pk.out_port[0], svc_group = pk.svc_group ? pk.svc_group[0] : 0u, dest = pk.dest ? pk.dest[0] : 0u;
  const uint32_t ct_mark = pk.ct_mark ? pk.ct_mark[0] : 0u;
  uint32_t lb[4] = {0u, 0u, 0u, 0u};
  *n_steps = 0;
  if (ep.svc) {
    const uint32_t f = lb_stage(ep.svc, src, dst, sport, dport, proto, svc_group, out_port, dest, lb);
    if (f & GPC_LB_NO_ENDPOINT) {
      out[0] = make_uint4(0u, pack_verdict(GPC_ACT_REJECT, GPC_VTABLE_ENDPOINT_DNAT, 0, 0), 0u, 0u);
      lb_out[0] = make_uint4(lb[0], lb[1], lb[2], lb[3]);
      return;
    }
  }
  lb_out[0] = make_uint4(lb[0], lb[1], lb[2], lb[3]);
  View im{{ep.blob, ep.hdr, nullptr, ep.pool}, {ep.pool, nullptr, nullptr, ep.pool}, 1u, ep.jhdr, 0u};
  if (ep.pool) {
    const JournalHdr* jh = reinterpret_cast<const JournalHdr*>(ep.pool + ep.jhdr);
    if (jh->bdead_off) im.base.dead = ep.pool + jh->bdead_off;
    im.n_img = 2u;
    im.ext = jh->ext_off;
  }
  Pkt p(pkt_lds, 1);
  make_pkt(p, src, dst, sport, dport, proto, out_port, pk.in_port ? pk.in_port[0] : 0u, svc_group,
           pk.tun_id ? pk.tun_id[0] : 0u, ct_src, ct_dst, pk.ct_state ? pk.ct_state[0] : uint32_t(GPC_CT_NEW | GPC_CT_TRK),
           view_bloom_axes(im));
  const PacketOut o = classify_packet<kModeJournal, 0, true>(im, p, dest, ct_mark, steps, n_steps);
  out[0] = make_uint4(o.e.conj, o.e.packed, o.g.conj, o.g.packed);
}

int launch_trace(const EpochArgs& ep, const gpc_pkt_soa& pk, uint4* out, uint4* lb_out, TraceStep* steps, uint32_t* n_steps,
                 hipStream_t stream) {
  hipLaunchKernelGGL(trace_kernel, dim3(1), dim3(64), 0, stream, ep, pk, out, lb_out, steps, n_steps);
  return hipGetLastError() == hipSuccess ? 0 : -GPC_EDEV;
}

// One thread per counter slot: the accumulator copies {packets, bytes, non-session packets} are
// drained (atomic exchange: a classification running concurrently on another stream loses no
// update, it lands in the next fold) and added to the published copy as {packets, bytes, sessions}.
__global__ void fold_counters_kernel(unsigned long long* __restrict__ c, uint64_t stride, uint32_t copies) {
  const uint64_t s = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (kCounterWords * s >= stride) return;
  unsigned long long p = 0, b = 0, ns = 0;
  for (uint32_t r = 0; r < copies; r++) {
    unsigned long long* a = c + r * stride + kCounterWords * s;
    p += atomicExch(&a[0], 0ull);
    b += atomicExch(&a[1], 0ull);
    ns += atomicExch(&a[2], 0ull);
  }
  unsigned long long* o = c + uint64_t(copies) * stride + kCounterWords * s;
  if (p) atomicAdd(&o[0], p);
  if (b) atomicAdd(&o[1], b);
  if (p != ns) atomicAdd(&o[2], p - ns);  // (mod 2^64: a fold between a packet's two adds evens out next time)
}

int launch_fold_counters(unsigned long long* counters, uint64_t stride, uint32_t copies, hipStream_t stream) {
  if (!counters || copies == 0 || stride == 0) return 0;
  const uint64_t slots = stride / kCounterWords;
  hipLaunchKernelGGL(fold_counters_kernel, dim3(uint32_t((slots + 255) / 256)), dim3(256), 0, stream, counters, stride, copies);
  return hipGetLastError() == hipSuccess ? 0 : -GPC_EDEV;
}

__global__ void merge_counters_kernel(unsigned long long* __restrict__ dst, const unsigned long long* __restrict__ src,
                                      uint64_t src_stride, uint32_t copies, uint64_t n_words) {
  const uint64_t w = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (w >= n_words) return;
  unsigned long long sum = 0;
  for (uint32_t r = 0; r < copies; r++) sum += src[r * src_stride + w];
  if (sum) atomicAdd(&dst[w], sum);
}

int launch_merge_counters(unsigned long long* dst, const unsigned long long* src, uint64_t src_stride, uint32_t copies,
                          uint64_t n_words, hipStream_t stream) {
  if (!dst || !src || !copies || !n_words) return 0;
  hipLaunchKernelGGL(merge_counters_kernel, dim3(uint32_t((n_words + 255) / 256)), dim3(256), 0, stream, dst, src, src_stride,
                     copies, n_words);
  return hipGetLastError() == hipSuccess ? 0 : -GPC_EDEV;
}

// Launch size: the grid is limited in work-items (gridDim.x * blockDim.x < 2^32 on ROCm), and the
// lane-regrouping kernels use 256-thread blocks.
constexpr uint64_t kMaxPackets = (1ull << 32) - uint64_t(kSortBlock);
static_assert(kMaxPackets == GPC_MAX_BATCH, "gpc.h GPC_MAX_BATCH mirrors the launch limit");

uint64_t group_scratch_bytes(const gpc_pkt_soa& pk, uint64_t n, bool lb) {
  uint64_t per = 4 /*orig*/ + 8 /*mid*/ + 4 + 4 + 2 + 2 + 1 + 4;  // + src dst sport dport proto out_port
  per += (pk.ct_src ? 4 : 0) + (pk.ct_dst ? 4 : 0) + (pk.in_port ? 4 : 0) + (pk.svc_group ? 4 : 0) + (pk.tun_id ? 4 : 0) +
         (pk.ct_state ? 1 : 0) + (pk.dest ? 1 : 0) + (pk.len ? 2 : 0) + (pk.ct_mark ? 1 : 0);
  per += 8;  // gout: the ingress halves of the verdict pairs in grouped order (GroupArgs.unpermute)
  if (lb) per += 16;  // lbg: the Service launch's LB results in grouped order
  return per * n + 22 * 256;  // every region 256-B aligned
}

// Carves the grouped columns, orig and mid out of group->scratch and launches group_tiles_kernel.
static int launch_group(const EpochArgs& ep, const gpc_pkt_soa& pk, uint64_t n, const GroupArgs& group, hipStream_t stream,
                        gpc_pkt_soa* g, uint32_t** orig, uint2** mid, uint2** gout, uint4** lbg, LaunchMarks* marks) {
  if (!group.scratch || group.src_bits > 8 || (group.key != GPC_GROUP_KEY_ADDR && group.key != GPC_GROUP_KEY_SCAN)) return -GPC_EINVAL;
  uint8_t* q = group.scratch;
  auto take = [&](uint64_t bytes) {
    uint8_t* r = q;
    q += (bytes + 255) & ~uint64_t(255);
    return r;
  };
  *g = gpc_pkt_soa{};
  *mid = reinterpret_cast<uint2*>(take(8 * n));
  *orig = reinterpret_cast<uint32_t*>(take(4 * n));
  *gout = reinterpret_cast<uint2*>(take(8 * n));
  if (lbg) *lbg = group.lb ? reinterpret_cast<uint4*>(take(16 * n)) : nullptr;
  g->src = reinterpret_cast<const uint32_t*>(take(4 * n));
  g->dst = reinterpret_cast<const uint32_t*>(take(4 * n));
  g->sport = reinterpret_cast<const uint16_t*>(take(2 * n));
  g->dport = reinterpret_cast<const uint16_t*>(take(2 * n));
  g->proto = take(n);
  g->out_port = reinterpret_cast<const uint32_t*>(take(4 * n));
  if (pk.in_port) g->in_port = reinterpret_cast<const uint32_t*>(take(4 * n));
  if (pk.svc_group) g->svc_group = reinterpret_cast<const uint32_t*>(take(4 * n));
  if (pk.tun_id) g->tun_id = reinterpret_cast<const uint32_t*>(take(4 * n));
  if (pk.ct_src) g->ct_src = reinterpret_cast<const uint32_t*>(take(4 * n));
  if (pk.ct_dst) g->ct_dst = reinterpret_cast<const uint32_t*>(take(4 * n));
  if (pk.ct_state) g->ct_state = take(n);
  if (pk.dest) g->dest = take(n);
  if (pk.len) g->len = reinterpret_cast<const uint16_t*>(take(2 * n));
  if (pk.ct_mark) g->ct_mark = take(n);
  gpc_pkt_soa in = pk;  // the IPv6 address columns are not read (an IPv6 batch comes as code columns)
  in.src6 = in.dst6 = in.ct_src6 = in.ct_dst6 = nullptr;
  if (!group.unpermute) {
    *gout = nullptr;
    if (lbg) *lbg = nullptr;
  }
  const uint64_t tiles = (n + kGroupTile - 1) / kGroupTile;
  launch_mark(marks, kLaunchGroup, stream);
  hipLaunchKernelGGL(group_tiles_kernel, dim3(uint32_t(tiles)), dim3(kGroupThreads), 0, stream, ep, in, n, group.key,
                     group.axes, group.src_bits, *g, *orig);
  return 0;
}

uint32_t v6_code_columns(const gpc_pkt_soa& pk) { return 2u + (pk.ct_src6 ? 1u : 0u) + (pk.ct_dst6 ? 1u : 0u); }

int launch_classify6(const EpochArgs& ep, const gpc_pkt_soa& pk, uint64_t n, gpc_verdict* out,
                     unsigned long long* counters, int count, const GroupArgs* group, uint32_t* codes, hipStream_t stream,
                     LaunchMarks* marks) {
  if (n == 0) return 0;
  if (n > kMaxPackets || !codes) return -GPC_EINVAL;
  V6Cols cols{{pk.src6, pk.dst6, nullptr, nullptr}};
  uint32_t nc = 2;
  gpc_pkt_soa p4 = pk;  // the batch over code columns: src, dst [, ct_src] [, ct_dst]
  p4.src6 = p4.dst6 = p4.ct_src6 = p4.ct_dst6 = nullptr;
  p4.src = codes;
  p4.dst = codes + n;
  p4.ct_src = p4.ct_dst = nullptr;
  if (pk.ct_src6) {
    cols.c[nc] = pk.ct_src6;
    p4.ct_src = codes + uint64_t(nc++) * n;
  }
  if (pk.ct_dst6) {
    cols.c[nc] = pk.ct_dst6;
    p4.ct_dst = codes + uint64_t(nc++) * n;
  }
  launch_mark(marks, kLaunchCodes, stream);
  const dim3 grid(uint32_t((n + kCodeBlock - 1) / kCodeBlock), nc);
  if (ep.pool)  // an IPv6 delta epoch: base + journal (its overflow LPM table)
    hipLaunchKernelGGL(v6_code_kernel<true>, grid, dim3(kCodeBlock), 0, stream, ep, cols, n, codes);
  else
    hipLaunchKernelGGL(v6_code_kernel<false>, grid, dim3(kCodeBlock), 0, stream, ep, cols, n, codes);
  return launch_classify(ep, p4, n, out, nullptr, counters, count, group, stream, marks);
}

int launch_classify(const EpochArgs& ep, const gpc_pkt_soa& pk, uint64_t n, gpc_verdict* out, uint4* lb_out,
                    unsigned long long* counters, int count, const GroupArgs* group, hipStream_t stream,
                    LaunchMarks* marks, uint4* park) {
  if (n == 0) return 0;
  if (n > kMaxPackets) return -GPC_EINVAL;
  gpc_pkt_soa g;
  const gpc_pkt_soa* p = &pk;
  uint32_t* orig = nullptr;
  uint2* mid = nullptr;
  uint32_t xo = 0;
  uint2* gout = nullptr;
  uint4* lbg = nullptr;  // grouped Service batch with the un-permute: LB results in grouped order
  if (group) {
    if (const int rc = launch_group(ep, pk, n, *group, stream, &g, &orig, &mid, &gout, &lbg, marks)) return rc;
    xo = group->xcd_order;
    p = &g;
  }
  EpochArgs e = ep;
  if (group && group->key == GPC_GROUP_KEY_SCAN) e.sort_table[0] = e.sort_table[1] = 0;  // lanes already grouped by scan length
  // epoch mode: a journal (records / tombstones) or only point extensions over the base
  const int mode = !ep.pool ? kModeBase : ep.mode == uint32_t(kModeExt) ? kModeExt : kModeJournal;
  const bool svc = ep.svc != nullptr;
  // with Services one launch does both stages; grouped, it stores both verdict halves (and the LB
  // results) in grouped order for the un-permute, like the two launches without Services
  if (svc && lb_out && gout && !lbg) return -GPC_EINVAL;  // the caller sized the scratch without lb
  uint4* const lbk = lbg ? lbg : lb_out;
  if (mode == kModeJournal && svc) launch<kModeJournal, true>(e, *p, n, out, lbk, counters, count, orig, mid, xo, gout, park, stream, marks);
  else if (mode == kModeJournal) launch<kModeJournal, false>(e, *p, n, out, lb_out, counters, count, orig, mid, xo, gout, nullptr, stream, marks);
  else if (mode == kModeExt && svc) launch<kModeExt, true>(e, *p, n, out, lbk, counters, count, orig, mid, xo, gout, park, stream, marks);
  else if (mode == kModeExt) launch<kModeExt, false>(e, *p, n, out, lb_out, counters, count, orig, mid, xo, gout, nullptr, stream, marks);
  else if (svc) launch<kModeBase, true>(e, *p, n, out, lbk, counters, count, orig, mid, xo, gout, park, stream, marks);
  else launch<kModeBase, false>(e, *p, n, out, lb_out, counters, count, orig, mid, xo, gout, nullptr, stream, marks);
  if (gout) launch_unpermute(mid, 2, gout, orig, n, reinterpret_cast<uint4*>(out), svc ? lbg : nullptr, lb_out, stream, marks);
  launch_mark(marks, kLaunchEnd, stream);
  return hipGetLastError() == hipSuccess ? 0 : -GPC_EDEV;
}

#if defined(GPC_STAMPS)
// Diagnostic builds: copy (and optionally clear) the region-stamp totals (tools/stamps.py).
extern "C" int gpc_stamps_read(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gpc_stamp_acc), sizeof(gpc_stamp_acc)) != hipSuccess) return -GPC_EDEV;
  if (reset) {
    static const unsigned long long zero[32] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(gpc_stamp_acc), zero, sizeof(zero)) != hipSuccess) return -GPC_EDEV;
  }
  return 0;
}
#endif

}  // namespace gpc
