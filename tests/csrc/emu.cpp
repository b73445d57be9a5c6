// TEST-ONLY host emulation of the device kernel body (core.hpp classify_packet) over the image the
// product library built (gpc_debug_image). Lets the CPU test tier verify the image builder and the
// evaluation logic without a GPU. Never linked into libgpc.so; the product has no CPU classify path.
#include <cstddef>
#include <cstdint>

#include <algorithm>
#include <vector>
extern "C" {
unsigned long long gpc_emu_stats[16];
}
#include <map>
static std::vector<uintptr_t> g_lines;
static std::map<uintptr_t, int> g_line_site;
extern "C" {
unsigned long long gpc_emu_site_lines[2048];
// per packet (first 1M): record verifications and entries scanned (SIMT divergence studies)
unsigned gpc_emu_pkt_verif[1 << 20], gpc_emu_pkt_scan[1 << 20];
// per packet: scan passes (while iterations of eval_part), rule_match search iterations, scan_lists iterations
unsigned gpc_emu_pkt_pass[1 << 20], gpc_emu_pkt_search[1 << 20], gpc_emu_pkt_iter[1 << 20];
}
extern "C" void gpc_emu_touch(const void* p, unsigned bytes, int site) {
  uintptr_t a = reinterpret_cast<uintptr_t>(p);
  for (uintptr_t l = a >> 6; l <= (a + bytes - 1) >> 6; l++) {
    g_lines.push_back(l);
    g_line_site.emplace(l, site);
  }
}
#define GPC_EMU_STATS 1
#include "core.hpp"
#include "gpc.h"

using namespace gpc;

extern "C" int emu_classify(const uint32_t* blob, const void* hdr, const uint32_t* pool, uint32_t jhdr,
                            const uint32_t* svc, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, uint32_t* lb_out,
                            unsigned long long* counters) {
  View im{{blob, static_cast<const ImageHdr*>(hdr), nullptr, pool}, {pool, nullptr, nullptr, pool}, 1u, jhdr, 0u};
  int mode = kModeBase;  // as the device launch picks it (api.cpp: JournalHdr jflags)
  if (pool) {
    const JournalHdr* jh = reinterpret_cast<const JournalHdr*>(pool + jhdr);
    im.ext = jh->ext_off;
    mode = (jh->jflags & kJUsed) ? kModeJournal : kModeExt;
    if (mode == kModeJournal) {
      if (jh->bdead_off) im.base.dead = pool + jh->bdead_off;
      im.n_img = 2u;
    }
  }
  for (size_t i = 0; i < n; i++) {
    const uint32_t src = pk->src[i];
    uint32_t dst = pk->dst[i], dport = pk->dport[i];
    const uint32_t sport = pk->sport[i], proto = pk->proto[i];
    uint32_t out_port = pk->out_port[i], svc_group = pk->svc_group ? pk->svc_group[i] : 0u;
    uint32_t dest = pk->dest ? pk->dest[i] : 0u;
    const uint32_t ct_src = pk->ct_src ? pk->ct_src[i] : src, ct_dst = pk->ct_dst ? pk->ct_dst[i] : dst;
    uint32_t lb[4] = {0, 0, 0, 0};
    uint32_t lbf = svc ? lb_stage(svc, src, dst, sport, dport, proto, svc_group, out_port, dest, lb) : 0u;
    if (lb_out)
      for (int k = 0; k < 4; k++) lb_out[4 * i + k] = lb[k];
    if (lbf & GPC_LB_NO_ENDPOINT) {
      uint32_t* w = reinterpret_cast<uint32_t*>(out + 2 * i);
      w[0] = 0;
      w[1] = pack_verdict(GPC_ACT_REJECT, GPC_VTABLE_ENDPOINT_DNAT, 0, 0);
      w[2] = w[3] = 0;
      continue;
    }
    uint32_t pst[kPktWords];
    Pkt p(pst, 1);
    make_pkt(p, src, dst, sport, dport, proto, out_port, pk->in_port ? pk->in_port[i] : 0u, svc_group,
             pk->tun_id ? pk->tun_id[i] : 0u, ct_src, ct_dst, pk->ct_state ? pk->ct_state[i] : uint32_t(GPC_CT_NEW | GPC_CT_TRK),
             view_bloom_axes(im));
    g_lines.clear();
    g_line_site.clear();
    const unsigned long long v0 = ::gpc_emu_stats[3], s0 = ::gpc_emu_stats[4], p0 = ::gpc_emu_stats[8],
                             q0 = ::gpc_emu_stats[9], r0 = ::gpc_emu_stats[10];
    const uint32_t cm = pk->ct_mark ? pk->ct_mark[i] : 0u;
    PacketOut o = mode == kModeJournal ? classify_packet<kModeJournal>(im, p, dest, cm)
                  : mode == kModeExt   ? classify_packet<kModeExt>(im, p, dest, cm)
                                       : classify_packet<kModeBase>(im, p, dest, cm);
    if (counters)
      count_packet(o, pk->len ? pk->len[i] : 0u, p.ax[AX_CTST], [&](uint32_t w, unsigned long long v) { counters[w] += v; });
    std::sort(g_lines.begin(), g_lines.end());
    ::gpc_emu_stats[6] += std::unique(g_lines.begin(), g_lines.end()) - g_lines.begin();  // distinct 64-B lines
    ::gpc_emu_stats[7] += 1;
    if (i < (1u << 20)) {
      gpc_emu_pkt_verif[i] = unsigned(::gpc_emu_stats[3] - v0);
      gpc_emu_pkt_scan[i] = unsigned(::gpc_emu_stats[4] - s0);
      gpc_emu_pkt_pass[i] = unsigned(::gpc_emu_stats[8] - p0);
      gpc_emu_pkt_search[i] = unsigned(::gpc_emu_stats[9] - q0);
      gpc_emu_pkt_iter[i] = unsigned(::gpc_emu_stats[10] - r0);
    }
    for (auto& kv : g_line_site) gpc_emu_site_lines[kv.second & 2047]++;                                                              // packets
    uint32_t* w = reinterpret_cast<uint32_t*>(out + 2 * i);
    w[0] = o.e.conj;
    w[1] = o.e.packed;
    w[2] = o.g.conj;
    w[3] = o.g.packed;
  }
  return 0;
}

// gpc_trace's walk (core.hpp classify_packet<..., kTrace>) for packet 0 of the columns (no Service stage).
extern "C" int emu_trace(const uint32_t* blob, const void* hdr, const uint32_t* pool, uint32_t jhdr, const gpc_pkt_soa* pk,
                         gpc_verdict* out, TraceStep* steps, uint32_t* n_steps) {
  View im{{blob, static_cast<const ImageHdr*>(hdr), nullptr, pool}, {pool, nullptr, nullptr, pool}, 1u, jhdr, 0u};
  if (pool) {
    const JournalHdr* jh = reinterpret_cast<const JournalHdr*>(pool + jhdr);
    if (jh->bdead_off) im.base.dead = pool + jh->bdead_off;
    im.n_img = 2u;
    im.ext = jh->ext_off;
  }
  const uint32_t src = pk->src[0], dst = pk->dst[0];
  uint32_t pst[kPktWords];
  Pkt p(pst, 1);
  make_pkt(p, src, dst, pk->sport[0], pk->dport[0], pk->proto[0], pk->out_port[0], pk->in_port ? pk->in_port[0] : 0u,
           pk->svc_group ? pk->svc_group[0] : 0u, pk->tun_id ? pk->tun_id[0] : 0u, pk->ct_src ? pk->ct_src[0] : src,
           pk->ct_dst ? pk->ct_dst[0] : dst, pk->ct_state ? pk->ct_state[0] : uint32_t(GPC_CT_NEW | GPC_CT_TRK),
           view_bloom_axes(im));
  *n_steps = 0;
  PacketOut o = classify_packet<kModeJournal, 0, true>(im, p, pk->dest ? pk->dest[0] : 0u, pk->ct_mark ? pk->ct_mark[0] : 0u, steps,
                                               n_steps);
  uint32_t* w = reinterpret_cast<uint32_t*>(out);
  w[0] = o.e.conj;
  w[1] = o.e.packed;
  w[2] = o.g.conj;
  w[3] = o.g.packed;
  return 0;
}

// IPv6 batch over the IPv6 image (gpc_debug_image6): addresses mapped to codes as the kernel does.
extern "C" int emu_classify6(const uint32_t* blob, const void* hdr, const uint32_t* pool, uint32_t jhdr,
                             const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, unsigned long long* counters) {
  const ImageHdr* h = static_cast<const ImageHdr*>(hdr);
  View im{{blob, h, nullptr, pool}, {pool, nullptr, nullptr, pool}, 1u, jhdr, 0u};
  const uint32_t* ovf = nullptr;
  uint32_t ovf_log2 = 0;
  if (pool) {  // an IPv6 delta epoch (gpc_debug_epoch6)
    const JournalHdr* jh = reinterpret_cast<const JournalHdr*>(pool + jhdr);
    if (jh->bdead_off) im.base.dead = pool + jh->bdead_off;
    im.n_img = 2u;
    if (jh->v6_ovf_off) {
      ovf = pool + jh->v6_ovf_off;
      ovf_log2 = jh->v6_ovf_log2;
    }
  }
  auto code = [&](const uint8_t* col, size_t i) {
    uint32_t a[4];
    v6_words(col + 16 * i, a);
    return v6_code(blob, h->v6_lpm, a, ovf, ovf_log2);
  };
  auto code2 = [&](const uint8_t* c0, const uint8_t* c1, size_t i, uint32_t* c) {  // the kernel's paired LPM
    uint32_t a[2][4];
    v6_words(c0 + 16 * i, a[0]);
    v6_words(c1 + 16 * i, a[1]);
    if (ovf) v6_codes<2, true>(blob, h->v6_lpm, a, c, ovf, ovf_log2);
    else v6_codes<2>(blob, h->v6_lpm, a, c);
  };
  for (size_t i = 0; i < n; i++) {
    g_lines.clear();
    g_line_site.clear();
    uint32_t sd[2];
    code2(pk->src6, pk->dst6, i, sd);
    const uint32_t src = sd[0], dst = sd[1];
    const uint32_t ct_src = pk->ct_src6 ? code(pk->ct_src6, i) : src, ct_dst = pk->ct_dst6 ? code(pk->ct_dst6, i) : dst;
    const uint32_t dest = pk->dest ? pk->dest[i] : 0u;
    uint32_t pst[kPktWords];
    Pkt p(pst, 1);
    make_pkt(p, src, dst, pk->sport[i], pk->dport[i], pk->proto[i], pk->out_port[i], pk->in_port ? pk->in_port[i] : 0u,
             pk->svc_group ? pk->svc_group[i] : 0u, pk->tun_id ? pk->tun_id[i] : 0u, ct_src, ct_dst,
             pk->ct_state ? pk->ct_state[i] : uint32_t(GPC_CT_NEW | GPC_CT_TRK), view_bloom_axes(im));
    const uint32_t cm = pk->ct_mark ? pk->ct_mark[i] : 0u;
    PacketOut o = pool ? classify_packet<kModeJournal, 0>(im, p, dest, cm) : classify_packet<kModeBase, 0>(im, p, dest, cm);
    std::sort(g_lines.begin(), g_lines.end());
    ::gpc_emu_stats[6] += std::unique(g_lines.begin(), g_lines.end()) - g_lines.begin();  // distinct 64-B lines
    ::gpc_emu_stats[7] += 1;
    for (auto& kv : g_line_site) gpc_emu_site_lines[kv.second & 2047]++;
    if (i < (1u << 20) && !ovf) {  // search rounds of src and dst alone (the code kernel: one address per lane)
      const unsigned long long r0 = ::gpc_emu_stats[11], l0 = ::gpc_emu_stats[12], g0 = ::gpc_emu_stats[13];
      uint32_t a1[1][4], c1;
      v6_words(pk->src6 + 16 * i, a1[0]);
      v6_codes<1>(blob, h->v6_lpm, a1, &c1);
      gpc_emu_pkt_iter[i] = unsigned(::gpc_emu_stats[11] - r0);
      v6_words(pk->dst6 + 16 * i, a1[0]);
      v6_codes<1>(blob, h->v6_lpm, a1, &c1);
      gpc_emu_pkt_search[i] = unsigned(::gpc_emu_stats[11] - r0) - gpc_emu_pkt_iter[i];
      ::gpc_emu_stats[11] = r0;
      ::gpc_emu_stats[12] = l0;
      ::gpc_emu_stats[13] = g0;
    }
    if (counters)
      count_packet(o, pk->len ? pk->len[i] : 0u, p.ax[AX_CTST], [&](uint32_t w, unsigned long long v) { counters[w] += v; });
    uint32_t* w = reinterpret_cast<uint32_t*>(out + 2 * i);
    w[0] = o.e.conj;
    w[1] = o.e.packed;
    w[2] = o.g.conj;
    w[3] = o.g.packed;
  }
  return 0;
}
