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

namespace gpc {

#ifndef GPC_WAVES_PER_EU
#define GPC_WAVES_PER_EU 6
#endif
#ifndef GPC_BLOCK
#define GPC_BLOCK 256
#endif
constexpr int kBlock = GPC_BLOCK;

// kDelta = false: a base-only epoch (no tombstones, no overlay); the delta-epoch machinery folds
// away at compile time so the common case pays nothing for it.
template <bool kDelta>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GPC_WAVES_PER_EU))) void classify_kernel(EpochArgs ep, gpc_pkt_soa pk, uint64_t n, uint4* __restrict__ out,
                                                          unsigned long long* __restrict__ counters, int count) {
  uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  Pkt p;
  const uint32_t src = pk.src[i], dst = pk.dst[i];
  make_pkt(p, src, dst, pk.sport[i], pk.dport[i], pk.proto[i], pk.out_port[i], pk.in_port ? pk.in_port[i] : 0u,
           pk.svc_group ? pk.svc_group[i] : 0u, pk.tun_id ? pk.tun_id[i] : 0u, pk.ct_src ? pk.ct_src[i] : src,
           pk.ct_dst ? pk.ct_dst[i] : dst, pk.ct_state ? pk.ct_state[i] : uint32_t(GPC_CT_NEW | GPC_CT_TRK));
  const uint32_t dest = pk.dest ? pk.dest[i] : 0u;
  View im{{ep.blob, ep.hdr, kDelta ? ep.dead : nullptr}, {ep.oblob, ep.ohdr, nullptr}, (kDelta && ep.oblob) ? 2u : 1u};
  PacketOut o = classify_packet(im, p, dest);
  if (count && (o.ecounted || o.gcounted)) {
    const uint32_t len = pk.len ? pk.len[i] : 0u;
    count_packet(o, len, p.ax[AX_CTST], [&](uint32_t w, unsigned long long v) { atomicAdd(&counters[w], v); });
  }
  const VerdictOut e = o.e, g = o.g;
  out[i] = make_uint4(e.conj, e.packed, g.conj, g.packed);
}

int launch_classify(const EpochArgs& ep, const gpc_pkt_soa& pk, uint64_t n, gpc_verdict* out,
                    unsigned long long* counters, int count, hipStream_t stream) {
  if (n == 0) return 0;
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (ep.dead || ep.oblob)
    hipLaunchKernelGGL(classify_kernel<true>, dim3(uint32_t(blocks)), dim3(kBlock), 0, stream, ep, pk, n,
                       reinterpret_cast<uint4*>(out), counters, count);
  else
    hipLaunchKernelGGL(classify_kernel<false>, dim3(uint32_t(blocks)), dim3(kBlock), 0, stream, ep, pk, n,
                       reinterpret_cast<uint4*>(out), counters, count);
  return hipGetLastError() == hipSuccess ? 0 : -GPC_EDEV;
}

}  // namespace gpc
