// C-ABI of gpc.h: context, control plane (compiler.cpp), epoch publish of the device image
// (image.cpp), data path (classify.hip). There is no CPU classification path: gpc_classify* fail
// with GPC_EDEV when no HIP device is usable.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "compiler.hpp"
#include "gpc.h"
#include "image.hpp"
#include "launch.hpp"
#include "service.hpp"

using namespace gpc;

// Device memory of the epochs is allocated and freed stream-ordered on the context's upload stream
// (non-blocking), so a commit never waits for classification launches in flight on other streams.
static hipError_t dev_alloc(void** p, size_t bytes, hipStream_t s) {
  hipError_t e = hipMallocAsync(p, bytes, s);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    e = hipMalloc(p, bytes);
  }
  return e;
}
static void dev_free(void* p, hipStream_t s) {
  if (p && hipFreeAsync(p, s) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(p);
  }
}

struct DevImage {  // one uploaded image (freed when the last epoch using it retires)
  ImageHdr* d_hdr = nullptr;
  uint32_t* d_blob = nullptr;
  size_t bytes = 0;
  hipStream_t s = nullptr;
  ~DevImage() {
    dev_free(d_hdr, s);
    dev_free(d_blob, s);
  }
};

struct DevEpoch {
  std::shared_ptr<DevImage> base;       // shared by the delta epochs built on it
  std::shared_ptr<DevImage> pool;       // journal pool of that base (d_hdr unused; append-only)
  uint32_t jhdr = 0;                    // this epoch's JournalHdr in the pool (0: base only)
  std::shared_ptr<DevImage> svc;        // Service image (d_hdr unused), shared until Services change
  uint64_t epoch = 0;
  std::map<hipStream_t, hipEvent_t> last_use;  // last launch on each stream that used this epoch
};

struct RetiredEpoch {
  DevEpoch e;
  bool drained() const {
    for (auto& kv : e.last_use)
      if (hipEventQuery(kv.second) == hipErrorNotReady) return false;
    return true;
  }
  void release(hipStream_t s) {
    for (auto& kv : e.last_use) (void)hipEventDestroy(kv.second);
    (void)s;
    e = DevEpoch();
  }
};

// Delta commits append the changed rules to the journal of the current base (image.hpp Journal).
// A full rebuild (compaction) happens when the journal holds more than
// max(kDeltaMinRules, base rules / kDeltaFraction) live rules or its pool would pass its capacity.
constexpr size_t kDeltaMinRules = 16384;
constexpr size_t kDeltaFraction = 4;
constexpr size_t kPoolWords = size_t(256) << 20;  // 1 GiB journal pool per base (HBM is 288 GB)
constexpr size_t kMinUploadBytes = size_t(1) << 20;

struct gpc_ctx {
  gpc_config cfg;
  std::mutex ctl;    // control plane (conjMatchFlowLock + replayMutex role)
  std::mutex data;   // epoch pointer swap vs. kernel launch
  FeatureNP np;
  FeatureService svc;
  std::vector<uint32_t> svc_blob;        // host copy of the Service image (empty: no Services)
  uint64_t svc_gen = ~0ull;              // FeatureService generation the image was built from
  SlotMap slots;
  HostImage last;    // base image of the current epoch: shadow state for re-upload + debug export
  Journal journal;   // delta epochs over `last` (host mirror of the device pool)
  DevEpoch cur;
  std::vector<RetiredEpoch> retired;
  hipStream_t ustream = nullptr;         // uploads / frees (hipStreamNonBlocking)
  void* stage = nullptr;                 // pinned staging buffer of journal uploads
  size_t stage_bytes = 0;
  unsigned long long* d_counters = nullptr;
  size_t counter_cap = 0;  // slots
  std::vector<uint32_t> released_slots;
  std::vector<uint32_t> slot_conj;
  uint64_t epoch = 0, n_full = 0, n_delta = 0;
  explicit gpc_ctx(const gpc_config& c) : cfg(c), np(c), svc(c) {}
};

static int hip_ok(hipError_t e) { return e == hipSuccess ? 0 : -GPC_EDEV; }

static int upload_image(const HostImage& h, hipStream_t s, std::shared_ptr<DevImage>* out) {
  auto d = std::make_shared<DevImage>();
  d->s = s;
  d->bytes = h.blob.size() * 4;
  if (hip_ok(dev_alloc((void**)&d->d_blob, d->bytes, s)) || hip_ok(dev_alloc((void**)&d->d_hdr, sizeof(ImageHdr), s)) ||
      hip_ok(hipMemcpyAsync(d->d_blob, h.blob.data(), d->bytes, hipMemcpyHostToDevice, s)) ||
      hip_ok(hipMemcpyAsync(d->d_hdr, &h.hdr, sizeof(ImageHdr), hipMemcpyHostToDevice, s)))
    return -GPC_EDEV;
  *out = std::move(d);
  return GPC_OK;
}

static int upload_words(const std::vector<uint32_t>& w, hipStream_t s, std::shared_ptr<DevImage>* out) {
  auto d = std::make_shared<DevImage>();
  d->s = s;
  d->bytes = w.size() * 4;
  if (hip_ok(dev_alloc((void**)&d->d_blob, d->bytes, s)) ||
      hip_ok(hipMemcpyAsync(d->d_blob, w.data(), d->bytes, hipMemcpyHostToDevice, s)))
    return -GPC_EDEV;
  *out = std::move(d);
  return GPC_OK;
}

static void collect_retired(gpc_ctx* ctx, bool wait) {
  if (wait && !ctx->retired.empty()) (void)hipDeviceSynchronize();
  size_t k = 0;
  for (size_t i = 0; i < ctx->retired.size(); i++) {
    if (wait || ctx->retired[i].drained()) {
      ctx->retired[i].release(ctx->ustream);
    } else {
      if (k != i) ctx->retired[k] = std::move(ctx->retired[i]);
      k++;
    }
  }
  ctx->retired.resize(k);
}

static int commit_impl(gpc_ctx* ctx, bool force_full);

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
  if (ctx->cur.base || ctx->d_counters || !ctx->retired.empty()) {
    (void)hipSetDevice(ctx->cfg.device);
    (void)hipDeviceSynchronize();
    ctx->retired.push_back(RetiredEpoch{std::move(ctx->cur)});
    collect_retired(ctx, true);
    if (ctx->d_counters) (void)hipFree(ctx->d_counters);
    if (ctx->ustream) {
      (void)hipStreamSynchronize(ctx->ustream);
      (void)hipStreamDestroy(ctx->ustream);
    }
    if (ctx->stage) (void)hipHostFree(ctx->stage);
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

int gpc_load_flows(gpc_ctx* ctx, const char* text, size_t len, int32_t replace, size_t* n_loaded, size_t* n_skipped,
                   size_t* err_line) {
  if (!ctx || (!text && len)) return -GPC_EINVAL;
  std::vector<Flow> flows;
  size_t loaded = 0, skipped = 0, line_no = 0;
  size_t pos = 0;
  while (pos < len) {
    size_t e = pos;
    while (e < len && text[e] != '\n') e++;
    std::string line(text + pos, e - pos);
    pos = e + 1;
    line_no++;
    Flow f;
    std::string err;
    int r = parse_flow_text(line, &f, &err);
    if (r < 0) {
      if (err_line) *err_line = line_no;
      return r;
    }
    if (r == 0) {
      if (line.find_first_not_of(" \t\r") != std::string::npos) skipped++;
      continue;
    }
    flows.push_back(std::move(f));
    loaded++;
  }
  std::lock_guard<std::mutex> g(ctx->ctl);
  try {
    int rc = ctx->np.load_flows(flows, replace != 0);
    if (rc) return rc;
  } catch (...) {
    return -GPC_ENOMEM;
  }
  if (n_loaded) *n_loaded = loaded;
  if (n_skipped) *n_skipped = skipped;
  return GPC_OK;
}

#define GPC_SVC_CALL(expr)                       \
  do {                                           \
    if (!ctx) return -GPC_EINVAL;                \
    std::lock_guard<std::mutex> g(ctx->ctl);     \
    try {                                        \
      return (expr);                             \
    } catch (...) {                              \
      return -GPC_ENOMEM;                        \
    }                                            \
  } while (0)

int gpc_install_service_group(gpc_ctx* ctx, uint32_t group_id, int32_t aff, const gpc_endpoint* eps, size_t n) {
  if (!eps && n) return -GPC_EINVAL;
  GPC_SVC_CALL(ctx->svc.install_service_group(group_id, aff != 0, eps, n));
}
int gpc_uninstall_service_group(gpc_ctx* ctx, uint32_t group_id) { GPC_SVC_CALL(ctx->svc.uninstall_service_group(group_id)); }
int gpc_install_endpoint_flows(gpc_ctx* ctx, uint8_t protocol, uint8_t family, const gpc_endpoint* eps, size_t n) {
  if (!eps && n) return -GPC_EINVAL;
  GPC_SVC_CALL(ctx->svc.install_endpoint_flows(protocol, family, eps, n));
}
int gpc_uninstall_endpoint_flows(gpc_ctx* ctx, uint8_t protocol, uint8_t family, const gpc_endpoint* eps, size_t n) {
  if (!eps && n) return -GPC_EINVAL;
  GPC_SVC_CALL(ctx->svc.uninstall_endpoint_flows(protocol, family, eps, n));
}
int gpc_install_service_flows(gpc_ctx* ctx, const gpc_service_config* cfg) {
  if (!cfg) return -GPC_EINVAL;
  GPC_SVC_CALL(ctx->svc.install_service_flows(*cfg));
}
int gpc_uninstall_service_flows(gpc_ctx* ctx, const uint8_t* ip, uint8_t family, uint16_t port, uint8_t protocol) {
  if (!ip) return -GPC_EINVAL;
  GPC_SVC_CALL(ctx->svc.uninstall_service_flows(ip, family, port, protocol));
}
int gpc_install_pod(gpc_ctx* ctx, const uint8_t* ip, uint8_t family, uint32_t ofport) {
  if (!ip) return -GPC_EINVAL;
  GPC_SVC_CALL(ctx->svc.install_pod(ip, family, ofport));
}
int gpc_uninstall_pod(gpc_ctx* ctx, const uint8_t* ip, uint8_t family) {
  if (!ip) return -GPC_EINVAL;
  GPC_SVC_CALL(ctx->svc.uninstall_pod(ip, family));
}

int gpc_dump_groups(gpc_ctx* ctx, char* buf, size_t cap, size_t* needed) {
  if (!ctx) return -GPC_EINVAL;
  std::string s;
  {
    std::lock_guard<std::mutex> g(ctx->ctl);
    s = ctx->svc.dump_groups();
  }
  if (needed) *needed = s.size() + 1;
  if (!buf || cap < s.size() + 1) return -GPC_ERANGE;
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return GPC_OK;
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
    std::string sv = ctx->svc.dump_flows();
    if (!sv.empty()) {
      if (!s.empty() && s.back() != '\n') s += "\n";
      s += sv;
      if (!s.empty() && s.back() == '\n') s.pop_back();
    }
  }
  if (needed) *needed = s.size() + 1;
  if (!buf || cap < s.size() + 1) return -GPC_ERANGE;
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return GPC_OK;
}

int gpc_commit(gpc_ctx* ctx) { return commit_impl(ctx, false); }
int gpc_compact(gpc_ctx* ctx) { return commit_impl(ctx, true); }

int gpc_classify(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, int32_t count, void* stream) {
  return gpc_classify_lb(ctx, pk, n, out, nullptr, count, stream);
}

int gpc_classify_lb(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, gpc_lb_result* lb_out, int32_t count,
                    void* stream) {
  if (!ctx || !pk || (!out && n)) return -GPC_EINVAL;
  if (n && (!pk->src || !pk->dst || !pk->sport || !pk->dport || !pk->proto || !pk->out_port)) return -GPC_EINVAL;
  std::lock_guard<std::mutex> d(ctx->data);
  if (!ctx->cur.base) return -GPC_EINVAL;  // nothing committed yet
  if (hip_ok(hipSetDevice(ctx->cfg.device))) return -GPC_EDEV;
  EpochArgs ep{ctx->cur.base->d_hdr, ctx->cur.base->d_blob, ctx->cur.jhdr ? ctx->cur.pool->d_blob : nullptr, ctx->cur.jhdr,
               ctx->cur.svc ? ctx->cur.svc->d_blob : nullptr};
  hipStream_t st = (hipStream_t)stream;
  int rc = launch_classify(ep, *pk, n, out, reinterpret_cast<uint4*>(lb_out), ctx->d_counters, count, st);
  if (rc || n == 0) return rc;
  hipEvent_t& ev = ctx->cur.last_use[st];  // epoch lifetime: retired epochs are freed once drained
  if (!ev && hip_ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming))) return -GPC_EDEV;
  return hip_ok(hipEventRecord(ev, st));
}

int gpc_classify_host(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, int32_t count) {
  return gpc_classify_host_lb(ctx, pk, n, out, nullptr, count);
}

int gpc_classify_host_lb(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, gpc_lb_result* lb_out,
                         int32_t count) {
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
  void* dlb = nullptr;
  if (!rc && hip_ok(hipMalloc(&dout, n * 2 * sizeof(gpc_verdict)))) rc = -GPC_EDEV;
  if (!rc && lb_out && hip_ok(hipMalloc(&dlb, n * sizeof(gpc_lb_result)))) rc = -GPC_EDEV;
  if (!rc) rc = gpc_classify_lb(ctx, &d, n, (gpc_verdict*)dout, (gpc_lb_result*)dlb, count, nullptr);
  if (!rc && hip_ok(hipDeviceSynchronize())) rc = -GPC_EDEV;
  if (!rc && hip_ok(hipMemcpy(out, dout, n * 2 * sizeof(gpc_verdict), hipMemcpyDeviceToHost))) rc = -GPC_EDEV;
  if (!rc && lb_out && hip_ok(hipMemcpy(lb_out, dlb, n * sizeof(gpc_lb_result), hipMemcpyDeviceToHost))) rc = -GPC_EDEV;
  if (dout) (void)hipFree(dout);
  if (dlb) (void)hipFree(dlb);
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
  out->device_bytes = ctx->cur.base ? ctx->cur.base->bytes : 0;
  out->overlay_bytes = ctx->journal.active() ? ctx->journal.pool.size() * 4 : 0;
  out->n_overlay_rules = ctx->journal.n_live;
  out->n_tombstones = ctx->journal.n_tombstones();
  out->n_full_builds = ctx->n_full;
  out->n_delta_builds = ctx->n_delta;
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

int gpc_debug_service_image(gpc_ctx* ctx, const uint32_t** blob, size_t* n_words) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  if (blob) *blob = ctx->svc_blob.empty() ? nullptr : ctx->svc_blob.data();
  if (n_words) *n_words = ctx->svc_blob.size();
  return GPC_OK;
}

int gpc_debug_epoch(gpc_ctx* ctx, const uint32_t** pool, size_t* pool_words, uint32_t* jhdr) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  const bool has = ctx->journal.active();
  if (pool) *pool = has ? ctx->journal.pool.data() : nullptr;
  if (pool_words) *pool_words = has ? ctx->journal.pool.size() : 0;
  if (jhdr) *jhdr = has ? ctx->journal.hdr_off : 0;
  return GPC_OK;
}

}  // extern "C"

// Builds the next epoch (full or delta) on the host, uploads it and publishes it atomically.
// Host shadow state (last / ovl / dead) is updated before the upload, so tests on a host without a
// device still see the image (the call then returns GPC_EDEV).
static int commit_impl(gpc_ctx* ctx, bool force_full) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  FeatureNP::Dirty dirty = ctx->np.take_dirty();
  const bool have_base = !ctx->last.blob.empty();
  bool full = force_full || !have_base || ctx->last.any_noact || ctx->np.foreign() || ctx->journal.any_noact ||
              ctx->journal.n_live > std::max(kDeltaMinRules, ctx->last.conj_rid.size() / kDeltaFraction) ||
              ctx->journal.pool.size() > kPoolWords * 7 / 8;
  int rc = GPC_OK;
  try {
    if (!full && (!dirty.conj.empty() || dirty.hard_tables)) {
      std::string err;
      if (ctx->journal.apply(ctx->np, ctx->slots, dirty.conj, dirty.hard_tables, &err) != GPC_OK ||
          ctx->journal.pool.size() > kPoolWords)
        full = true;  // a shape the journal does not take (or it is full): rebuild everything
    }
    if (full) {
      HostImage img;
      rc = build_image(ctx->np, ctx->slots, &img);
      if (rc) return rc;
      ctx->last = std::move(img);
      ctx->journal.reset(&ctx->last);
    }
  } catch (...) {
    return -GPC_ENOMEM;
  }
  const bool svc_changed = ctx->svc.generation() != ctx->svc_gen;
  if (svc_changed) {
    std::string err;
    std::vector<uint32_t> sb;
    if (!ctx->svc.empty() && (rc = ctx->svc.build_image(&sb, &err))) return rc;
    ctx->svc_blob = std::move(sb);
    ctx->svc_gen = ctx->svc.generation();
  }
  ctx->slot_conj = ctx->slots.slot_conj();
  if (full) ctx->n_full++;
  else ctx->n_delta++;
  if (hip_ok(hipSetDevice(ctx->cfg.device))) return -GPC_EDEV;
  if (!ctx->ustream && hip_ok(hipStreamCreateWithFlags(&ctx->ustream, hipStreamNonBlocking))) return -GPC_EDEV;
  hipStream_t us = ctx->ustream;
  collect_retired(ctx, false);
  DevEpoch ne;
  if (full || !ctx->cur.base) {
    if ((rc = upload_image(ctx->last, us, &ne.base))) return rc;
    auto pool = std::make_shared<DevImage>();  // journal pool of the new base
    pool->s = us;
    pool->bytes = kPoolWords * 4;
    if (hip_ok(dev_alloc((void**)&pool->d_blob, pool->bytes, us))) return -GPC_EDEV;
    ne.pool = std::move(pool);
    ctx->journal.uploaded = 0;
  } else {
    ne.base = ctx->cur.base;
    ne.pool = ctx->cur.pool;
  }
  Journal& jn = ctx->journal;
  if (jn.active() && jn.pool.size() > jn.uploaded) {
    // Append-only: only the new tail travels, through a pinned buffer and padded to at least
    // kMinUploadBytes (the padding lands in not-yet-used pool space) so the runtime takes the DMA
    // path; a small copy may otherwise run as a blit kernel queued behind in-flight classification.
    const size_t tail = (jn.pool.size() - jn.uploaded) * 4;
    const size_t room = ne.pool->bytes - jn.uploaded * 4;
    const size_t bytes = std::min(std::max(tail, kMinUploadBytes), room);
    if (ctx->stage_bytes < bytes) {
      if (ctx->stage) (void)hipHostFree(ctx->stage);
      ctx->stage = nullptr;
      ctx->stage_bytes = 0;
      const size_t cap = std::max(bytes, size_t(4) << 20);
      if (hip_ok(hipHostMalloc(&ctx->stage, cap, hipHostMallocDefault))) return -GPC_EDEV;
      ctx->stage_bytes = cap;
    }
    std::memcpy(ctx->stage, jn.pool.data() + jn.uploaded, tail);
    if (hip_ok(hipMemcpyAsync(ne.pool->d_blob + jn.uploaded, ctx->stage, bytes, hipMemcpyHostToDevice, us)))
      return -GPC_EDEV;
    jn.uploaded = jn.pool.size();
  }
  ne.jhdr = jn.active() ? jn.hdr_off : 0;
  if (!svc_changed) ne.svc = ctx->cur.svc;
  else if (!ctx->svc_blob.empty() && (rc = upload_words(ctx->svc_blob, us, &ne.svc))) return rc;
  ne.epoch = ++ctx->epoch;
  // counters: grow to the slot count, zero released slots (their Metric flows were deleted)
  size_t need = ctx->slots.size() ? ctx->slots.size() : 1;
  unsigned long long* nc = ctx->d_counters;
  bool grow = need > ctx->counter_cap;
  if (grow) {
    size_t cap = std::max(need, ctx->counter_cap * 2);
    if (hip_ok(hipMalloc(&nc, cap * kCounterBytes)) || hip_ok(hipMemset(nc, 0, cap * kCounterBytes))) {
      RetiredEpoch{std::move(ne)}.release(us);
      return -GPC_EDEV;
    }
    if (ctx->d_counters) {
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(nc, ctx->d_counters, ctx->counter_cap * kCounterBytes, hipMemcpyDeviceToDevice);
    }
  }
  if (hip_ok(hipStreamSynchronize(us))) {  // the new epoch is resident before it is published
    RetiredEpoch{std::move(ne)}.release(us);
    return -GPC_EDEV;
  }
  DevEpoch old;
  unsigned long long* old_counters = nullptr;
  {
    std::lock_guard<std::mutex> d(ctx->data);
    old = std::move(ctx->cur);
    ctx->cur = std::move(ne);
    if (grow) {
      old_counters = ctx->d_counters;
      ctx->d_counters = nc;
      ctx->counter_cap = std::max(need, ctx->counter_cap * 2);
    }
  }
  // the previous epoch is freed once every stream that launched on it has passed that launch
  ctx->retired.push_back(RetiredEpoch{std::move(old)});
  if (old_counters) {
    (void)hipDeviceSynchronize();
    (void)hipFree(old_counters);
  }
  for (uint32_t s : ctx->released_slots)
    if (s < ctx->counter_cap) (void)hipMemsetAsync(ctx->d_counters + kCounterWords * size_t(s), 0, kCounterBytes, us);
  ctx->released_slots.clear();
  return GPC_OK;
}
