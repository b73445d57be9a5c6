// C-ABI of gpc.h: context, control plane (compiler.cpp), epoch publish of the device image
// (image.cpp), data path (classify.hip). There is no CPU classification path: gpc_classify* fail
// with GPC_EDEV when no HIP device is usable.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "compiler.hpp"
#include "gpc.h"
#include "image.hpp"
#include "launch.hpp"

using namespace gpc;

struct DevEpoch {
  ImageHdr* d_hdr = nullptr;
  uint32_t* d_blob = nullptr;
  size_t bytes = 0;
  uint64_t epoch = 0;
};

struct gpc_ctx {
  gpc_config cfg;
  std::mutex ctl;    // control plane (conjMatchFlowLock + replayMutex role)
  std::mutex data;   // epoch pointer swap vs. kernel launch
  FeatureNP np;
  SlotMap slots;
  HostImage last;    // last committed host image: shadow state for device re-upload + debug export
  DevEpoch cur;
  unsigned long long* d_counters = nullptr;
  size_t counter_cap = 0;  // slots
  std::vector<uint32_t> released_slots;
  std::vector<uint32_t> slot_conj;
  uint64_t epoch = 0;
  explicit gpc_ctx(const gpc_config& c) : cfg(c), np(c) {}
};

static int hip_ok(hipError_t e) { return e == hipSuccess ? 0 : -GPC_EDEV; }

static void free_epoch(DevEpoch& e) {
  if (e.d_hdr) (void)hipFree(e.d_hdr);
  if (e.d_blob) (void)hipFree(e.d_blob);
  e = DevEpoch();
}

extern "C" {

int gpc_abi_version(void) { return GPC_ABI_VERSION; }

const char* gpc_strerror(int err) {
  switch (err < 0 ? -err : err) {
    case GPC_OK: return "ok";
    case GPC_ENOTFOUND: return "policyRuleConjunction not found";
    case GPC_EINVAL: return "invalid argument or unsupported flow shape";
    case GPC_ENOMEM: return "out of memory";
    case GPC_EDEV: return "HIP device error (no usable MI355X device?)";
    case GPC_ENOCLAUSE: return "no clause is using addrType";
    case GPC_EBUNDLE: return "flow bundle rejected";
    case GPC_ERANGE: return "output buffer too small";
  }
  return "unknown error";
}

int gpc_create(const gpc_config* cfg, gpc_ctx** out) {
  if (!cfg || !out) return -GPC_EINVAL;
  if (!cfg->ipv4_enabled && !cfg->ipv6_enabled) return -GPC_EINVAL;
  try {
    *out = new gpc_ctx(*cfg);
  } catch (...) {
    return -GPC_ENOMEM;
  }
  return GPC_OK;
}

void gpc_destroy(gpc_ctx* ctx) {
  if (!ctx) return;
  if (ctx->cur.d_blob || ctx->d_counters) {
    (void)hipSetDevice(ctx->cfg.device);
    (void)hipDeviceSynchronize();
    free_epoch(ctx->cur);
    if (ctx->d_counters) (void)hipFree(ctx->d_counters);
  }
  delete ctx;
}

int gpc_initialize(gpc_ctx* ctx) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  return ctx->np.initialize();
}

int gpc_install_rule(gpc_ctx* ctx, const gpc_rule* rule) {
  if (!ctx || !rule) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  try {
    return ctx->np.install_rule(*rule);
  } catch (...) {
    return -GPC_ENOMEM;
  }
}

int gpc_batch_install(gpc_ctx* ctx, const gpc_rule* rules, size_t n) {
  if (!ctx || (!rules && n)) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  try {
    return ctx->np.batch_install(rules, n);
  } catch (...) {
    return -GPC_ENOMEM;
  }
}

int gpc_uninstall_rule(gpc_ctx* ctx, uint32_t rule_id, uint16_t* stale, size_t cap, size_t* n_stale) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  std::vector<uint16_t> st;
  int rc = ctx->np.uninstall_rule(rule_id, &st);
  if (rc) return rc;
  ctx->slots.release(rule_id, &ctx->released_slots);
  if (n_stale) *n_stale = st.size();
  if (st.size() > cap && stale) return -GPC_ERANGE;
  if (stale)
    for (size_t i = 0; i < st.size(); i++) stale[i] = st[i];
  return GPC_OK;
}

int gpc_add_rule_addrs(gpc_ctx* ctx, uint32_t rule_id, int32_t addr_type, const gpc_addr* addrs, size_t n,
                       const uint16_t* prio, int32_t enable_logging, int32_t is_mcnp) {
  if (!ctx || (!addrs && n)) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  return ctx->np.add_rule_addrs(rule_id, addr_type, addrs, n, prio, enable_logging != 0, is_mcnp != 0);
}

int gpc_del_rule_addrs(gpc_ctx* ctx, uint32_t rule_id, int32_t addr_type, const gpc_addr* addrs, size_t n,
                       const uint16_t* prio) {
  if (!ctx || (!addrs && n)) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  return ctx->np.del_rule_addrs(rule_id, addr_type, addrs, n, prio);
}

int gpc_reassign_priorities(gpc_ctx* ctx, const uint16_t* from, const uint16_t* to, size_t n, uint8_t table) {
  if (!ctx || ((!from || !to) && n)) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  return ctx->np.reassign_priorities(from, to, n, table);
}

int gpc_get_policy_info(gpc_ctx* ctx, uint32_t rule_id, gpc_policy_info* out) {
  if (!ctx || !out) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  return ctx->np.policy_info(rule_id, out);
}

int gpc_dump_flows(gpc_ctx* ctx, char* buf, size_t cap, size_t* needed) {
  if (!ctx) return -GPC_EINVAL;
  std::string s;
  {
    std::lock_guard<std::mutex> g(ctx->ctl);
    s = ctx->np.dump();
  }
  if (needed) *needed = s.size() + 1;
  if (!buf || cap < s.size() + 1) return -GPC_ERANGE;
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return GPC_OK;
}

int gpc_commit(gpc_ctx* ctx) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  HostImage img;
  int rc;
  try {
    rc = build_image(ctx->np, ctx->slots, &img);
  } catch (...) {
    return -GPC_ENOMEM;
  }
  if (rc) return rc;
  ctx->slot_conj = ctx->slots.slot_conj();
  ctx->last = std::move(img);
  const HostImage& himg = ctx->last;
  if (hip_ok(hipSetDevice(ctx->cfg.device))) return -GPC_EDEV;
  DevEpoch ne;
  size_t bytes = himg.blob.size() * 4;
  if (hip_ok(hipMalloc(&ne.d_blob, bytes)) || hip_ok(hipMalloc(&ne.d_hdr, sizeof(ImageHdr)))) {
    free_epoch(ne);
    return -GPC_EDEV;
  }
  if (hip_ok(hipMemcpy(ne.d_blob, himg.blob.data(), bytes, hipMemcpyHostToDevice)) ||
      hip_ok(hipMemcpy(ne.d_hdr, &himg.hdr, sizeof(ImageHdr), hipMemcpyHostToDevice))) {
    free_epoch(ne);
    return -GPC_EDEV;
  }
  ne.bytes = bytes;
  ne.epoch = ++ctx->epoch;
  // counters: grow to the slot count, zero released slots (their Metric flows were deleted)
  size_t need = ctx->slots.size() ? ctx->slots.size() : 1;
  unsigned long long* nc = ctx->d_counters;
  bool grow = need > ctx->counter_cap;
  if (grow) {
    size_t cap = std::max(need, ctx->counter_cap * 2);
    if (hip_ok(hipMalloc(&nc, cap * kCounterBytes)) || hip_ok(hipMemset(nc, 0, cap * kCounterBytes))) {
      free_epoch(ne);
      return -GPC_EDEV;
    }
    if (ctx->d_counters) {
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(nc, ctx->d_counters, ctx->counter_cap * kCounterBytes, hipMemcpyDeviceToDevice);
    }
  }
  DevEpoch old;
  unsigned long long* old_counters = nullptr;
  {
    std::lock_guard<std::mutex> d(ctx->data);
    old = ctx->cur;
    ctx->cur = ne;
    if (grow) {
      old_counters = ctx->d_counters;
      ctx->d_counters = nc;
      ctx->counter_cap = std::max(need, ctx->counter_cap * 2);
    }
  }
  (void)hipDeviceSynchronize();  // in-flight launches of the previous epoch drain here
  free_epoch(old);
  if (old_counters) (void)hipFree(old_counters);
  for (uint32_t s : ctx->released_slots)
    if (s < ctx->counter_cap) (void)hipMemset(ctx->d_counters + kCounterWords * size_t(s), 0, kCounterBytes);
  ctx->released_slots.clear();
  return GPC_OK;
}

int gpc_classify(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, int32_t count, void* stream) {
  if (!ctx || !pk || (!out && n)) return -GPC_EINVAL;
  if (n && (!pk->src || !pk->dst || !pk->sport || !pk->dport || !pk->proto || !pk->out_port)) return -GPC_EINVAL;
  std::lock_guard<std::mutex> d(ctx->data);
  if (!ctx->cur.d_blob) return -GPC_EINVAL;  // nothing committed yet
  if (hip_ok(hipSetDevice(ctx->cfg.device))) return -GPC_EDEV;
  return launch_classify(ctx->cur.d_hdr, ctx->cur.d_blob, *pk, n, out, ctx->d_counters, count, (hipStream_t)stream);
}

int gpc_classify_host(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, int32_t count) {
  if (!ctx || !pk || (!out && n)) return -GPC_EINVAL;
  if (hip_ok(hipSetDevice(ctx->cfg.device))) return -GPC_EDEV;
  if (n == 0) return GPC_OK;
  gpc_pkt_soa d{};
  std::vector<void*> allocs;
  int rc = GPC_OK;
  auto up = [&](const void* h, size_t elem, const void** dst) {
    if (!h || rc) return;
    void* p = nullptr;
    if (hip_ok(hipMalloc(&p, n * elem)) || hip_ok(hipMemcpy(p, h, n * elem, hipMemcpyHostToDevice))) {
      rc = -GPC_EDEV;
      if (p) (void)hipFree(p);
      return;
    }
    allocs.push_back(p);
    *dst = p;
  };
  up(pk->src, 4, (const void**)&d.src);
  up(pk->dst, 4, (const void**)&d.dst);
  up(pk->sport, 2, (const void**)&d.sport);
  up(pk->dport, 2, (const void**)&d.dport);
  up(pk->proto, 1, (const void**)&d.proto);
  up(pk->out_port, 4, (const void**)&d.out_port);
  up(pk->in_port, 4, (const void**)&d.in_port);
  up(pk->svc_group, 4, (const void**)&d.svc_group);
  up(pk->tun_id, 4, (const void**)&d.tun_id);
  up(pk->ct_src, 4, (const void**)&d.ct_src);
  up(pk->ct_dst, 4, (const void**)&d.ct_dst);
  up(pk->ct_state, 1, (const void**)&d.ct_state);
  up(pk->dest, 1, (const void**)&d.dest);
  up(pk->len, 2, (const void**)&d.len);
  void* dout = nullptr;
  if (!rc && hip_ok(hipMalloc(&dout, n * 2 * sizeof(gpc_verdict)))) rc = -GPC_EDEV;
  if (!rc) rc = gpc_classify(ctx, &d, n, (gpc_verdict*)dout, count, nullptr);
  if (!rc && hip_ok(hipDeviceSynchronize())) rc = -GPC_EDEV;
  if (!rc && hip_ok(hipMemcpy(out, dout, n * 2 * sizeof(gpc_verdict), hipMemcpyDeviceToHost))) rc = -GPC_EDEV;
  if (dout) (void)hipFree(dout);
  for (void* p : allocs) (void)hipFree(p);
  return rc;
}

int gpc_counters(gpc_ctx* ctx, uint64_t** dev, const uint32_t** slot_conj, size_t* n_slots) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  if (dev) *dev = reinterpret_cast<uint64_t*>(ctx->d_counters);
  if (slot_conj) *slot_conj = ctx->slot_conj.data();
  if (n_slots) *n_slots = ctx->slot_conj.size();
  return GPC_OK;
}

int gpc_reset_counters(gpc_ctx* ctx) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  if (!ctx->d_counters) return GPC_OK;
  if (hip_ok(hipSetDevice(ctx->cfg.device))) return -GPC_EDEV;
  if (hip_ok(hipDeviceSynchronize()) || hip_ok(hipMemset(ctx->d_counters, 0, ctx->counter_cap * kCounterBytes))) return -GPC_EDEV;
  return GPC_OK;
}

int gpc_metrics(gpc_ctx* ctx, gpc_rule_metric* out, size_t cap, size_t* n) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  std::vector<unsigned long long> h(ctx->slot_conj.size() * kCounterWords, 0);
  if (ctx->d_counters && !h.empty()) {
    if (hip_ok(hipSetDevice(ctx->cfg.device)) || hip_ok(hipDeviceSynchronize()) ||
        hip_ok(hipMemcpy(h.data(), ctx->d_counters, h.size() * 8, hipMemcpyDeviceToHost)))
      return -GPC_EDEV;
  }
  size_t k = 0;
  for (size_t s = 0; s < ctx->slot_conj.size(); s++) {
    if (!ctx->slot_conj[s]) continue;
    if (out && k < cap) {
      out[k].conj_id = ctx->slot_conj[s];
      out[k].reserved = 0;
      out[k].packets = h[kCounterWords * s];
      out[k].bytes = h[kCounterWords * s + 1];
      out[k].sessions = h[kCounterWords * s + 2];
    }
    k++;
  }
  if (n) *n = k;
  return (out && k > cap) ? -GPC_ERANGE : GPC_OK;
}

int gpc_get_image_stats(gpc_ctx* ctx, gpc_image_stats* out) {
  if (!ctx || !out) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  std::memset(out, 0, sizeof *out);
  out->epoch = ctx->epoch;
  out->device_bytes = ctx->cur.bytes;
  for (int i = 0; i < 6; i++) {
    out->n_rules[i] = ctx->last.n_rules[i];
    out->n_hard[i] = ctx->last.n_hard[i];
  }
  out->n_flows = ctx->last.n_flows;
  out->n_counter_slots = uint32_t(ctx->slot_conj.size());
  out->bytes_records = ctx->last.bytes_records;
  out->bytes_ext = ctx->last.bytes_ext;
  out->bytes_bucket_offsets = ctx->last.bytes_bucket_offsets;
  out->bytes_entries = ctx->last.bytes_entries;
  out->bytes_hash = ctx->last.bytes_hash;
  return GPC_OK;
}

int gpc_debug_image(gpc_ctx* ctx, const uint32_t** blob, size_t* n_words, const void** hdr, size_t* hdr_bytes) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  if (blob) *blob = ctx->last.blob.data();
  if (n_words) *n_words = ctx->last.blob.size();
  if (hdr) *hdr = &ctx->last.hdr;
  if (hdr_bytes) *hdr_bytes = sizeof(ImageHdr);
  return GPC_OK;
}

}  // extern "C"
