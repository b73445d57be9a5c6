// C-ABI of gpc.h: context, control plane (compiler.cpp), epoch publish of the device image
// (image.cpp), data path (classify.hip). There is no CPU classification path: gpc_classify* fail
// with GPC_EDEV when no HIP device is usable.
#include <hip/hip_runtime.h>

#include <atomic>
#include <deque>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <thread>
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
#include "oplog.hpp"
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

// Tuning knobs read once per context (documented in DESIGN.md §4); out-of-range values: default.
static uint32_t env_u32(const char* name, uint32_t dflt, uint32_t lo, uint32_t hi) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  const unsigned long x = std::strtoul(v, &end, 10);
  return (*end || x < lo || x > hi) ? dflt : uint32_t(x);
}

struct StreamScratch {  // device scratch of the packet grouping pre-pass on one stream
  uint8_t* p = nullptr;
  size_t bytes = 0;
  hipEvent_t done = nullptr;  // recorded after the last launch that used it
  uint32_t small = 0;         // consecutive calls that needed < 1/8 of it (shrink hysteresis)
};
constexpr uint32_t kScratchShrinkAfter = 64;  // that many small calls in a row release the buffer
constexpr size_t kScratchStreams = 8;  // idle buffers of other streams are released past this many

// Key of the per-stream state (grouping scratch, epoch lifetime events, gpc_stream_epoch). The
// hipStreamPerThread handle names a different stream on every host thread, so it is keyed by the
// calling thread too: two threads launching on it never share scratch or a lifetime event.
struct StreamKey {
  hipStream_t s;
  std::thread::id t;
  bool operator<(const StreamKey& o) const { return s != o.s ? s < o.s : t < o.t; }
};
// The epoch swap of a commit / replay: launches waiting for `data` let it go first.
struct PublishLock {
  std::atomic<uint32_t>& n;
  std::unique_lock<std::mutex> lk;
  PublishLock(std::mutex& m, std::atomic<uint32_t>& c) : n((c.fetch_add(1), c)), lk(m) {}
  ~PublishLock() {
    lk.unlock();
    n.fetch_sub(1);
  }
};
// Data-path entry: wait while a publisher is queued for `data`, then take it.
static std::unique_lock<std::mutex> launch_lock(std::mutex& m, const std::atomic<uint32_t>& publishers) {
  while (publishers.load(std::memory_order_acquire)) std::this_thread::yield();
  return std::unique_lock<std::mutex>(m);
}

static StreamKey stream_key(hipStream_t s) {
  return StreamKey{s, s == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id()};
}

struct DevImage {  // one uploaded image (freed when the last epoch using it retires)
  ImageHdr* d_hdr = nullptr;
  uint32_t* d_blob = nullptr;
  size_t bytes = 0;
  hipStream_t s = nullptr;
  int device = 0;                       // HIP ordinal the buffers live on
  uint8_t sort_table[2] = {0, 0};       // per policy stage: the table whose scan length orders lanes
  uint32_t axes = 0;                    // axes read by the sub-indexes (group_axes)
  bool composite = false;               // some table has a composite driver index (TableHdr n_cidx)
  ~DevImage() {
    int cur = 0;
    const bool swap = hipGetDevice(&cur) == hipSuccess && cur != device;
    if (swap) (void)hipSetDevice(device);
    dev_free(d_hdr, s);
    dev_free(d_blob, s);
    if (swap) (void)hipSetDevice(cur);
  }
};

struct DevEpoch {
  std::shared_ptr<DevImage> base;       // shared by the delta epochs built on it
  std::shared_ptr<DevImage> pool;       // journal pool of that base (d_hdr unused; append-only)
  uint32_t jhdr = 0;                    // this epoch's JournalHdr in the pool (0: base only)
  int jmode = kModeBase;                // what the kernel reads of it (Journal::mode: point extensions only, or the journal)
  std::shared_ptr<DevImage> svc;        // Service image (d_hdr unused), shared until Services change
  std::shared_ptr<DevImage> v6;         // IPv6 base image (ipv6_enabled), shared by its delta epochs
  std::shared_ptr<DevImage> v6_pool;    // journal pool of that base (append-only)
  uint32_t v6_jhdr = 0;                 // this epoch's IPv6 JournalHdr (0: base only)
  uint32_t v6_lpm = 0;                  // its ImageHdr.v6_lpm
  uint64_t base_gen = 0, v6_gen = 0;    // host base generation (gpc_ctx gen4 / gen6) base / v6 mirror
  uint64_t epoch = 0;
  std::map<StreamKey, hipEvent_t> last_use;  // last launch on each stream that used this epoch
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

// The data-path state of one device slot of a context (gpc_create_multi: one control plane, several
// devices). Every slot holds its own copy of each published epoch, counters, grouping scratch and
// upload stream; the host shadow (compiler, images, journal, counter slots) is shared.
struct DevState {
  int device = 0;
  DevEpoch cur;
  std::vector<RetiredEpoch> retired;
  hipStream_t ustream = nullptr;                 // uploads / frees (hipStreamNonBlocking)
  std::map<StreamKey, StreamScratch> scratch;    // packet grouping buffers per stream (data)
  std::map<StreamKey, uint64_t> launch_epoch;    // epoch of the last classify launch per stream (data)
  unsigned long long* d_counters = nullptr;
  size_t counter_cap = 0;                        // slots
  uint32_t counter_copies = 1;                   // striped copies of the counter array (counter_copies_for)
  std::vector<LaunchMarks> marks;                // gpc_set_launch_timing event sets (data)
  size_t marks_next = 0, marks_used = 0, marks_dropped = 0;
};

// Delta commits append the changed rules to the journal of the current base (image.hpp Journal).
// A full rebuild (compaction) happens when the journal holds more than
// max(kDeltaMinRules, base rules / kDeltaFraction) live rules or its pool would pass its capacity.
constexpr size_t kDeltaMinRules = 16384;
constexpr size_t kDeltaFraction = 4;
constexpr size_t kPendingCapFactor = 2;  // journal allowance while a background compaction is pending
constexpr size_t kPoolWords = size_t(256) << 20;  // 1 GiB journal pool per base (HBM is 288 GB)
// Pool collection bar: journal entries are chained by 24-bit entry indexes (32-B entries: the first
// 2^27 words of the pool), so the collection runs well before that; 3/8 of the pool (96 M words)
// rather than 1/4 makes C5 mixed collect every ~7 s instead of ~5 s (each collection is a 110-180 ms
// commit the ops due meanwhile wait for).
constexpr size_t kPoolGcWords = kPoolWords * 3 / 8;
static_assert(kPoolGcWords < (size_t(1) << 27), "collect before the 24-bit journal entry indexes run out");
constexpr size_t kMinUploadBytes = size_t(1) << 20;
constexpr size_t kExtCompactValues = size_t(1) << 16;  // live point-extension values that ask for a compaction
constexpr size_t kGcDeadMin = 2048;  // dead journal versions that ask for a pool collection (and 2x the live rules)

// Background compaction: a shadow compiler replays the control-plane log on its own thread; asked
// to compact, it builds a full image of its state at a commit boundary, catches up on the log by
// appending the rules changed meanwhile to a fresh journal (from its own state, no lock on the
// live compiler), uploads both and hands them over. The next gpc_commit installs them after
// appending the rules changed since the handover commit (from the live compiler) -- so the
// synchronous full rebuild is only a fallback when the journal outgrows its hard limit first.
struct Compactor {
  std::thread th;
  std::mutex mu;  // everything below
  std::condition_variable cv;
  std::vector<Op> log;       // operations the shadow has not replayed yet
  bool enabled = true, stop = false, busy = false;
  uint64_t want_commit = 0;  // compact once the shadow reaches this commit (0: not requested)
  bool ready = false;        // a result is waiting to be installed
  bool discard = false;      // gpc_replay ran while the result was being built: its device buffers are stale
  int rc = 0;
  std::unique_ptr<HostImage> base;
  std::unique_ptr<Journal> journal;
  std::vector<std::shared_ptr<DevImage>> dbase, dpool;  // per device slot (empty: not uploaded)
  size_t uploaded = 0;
  uint64_t at_commit = 0;
  // point extensions live at the requested commit: the new base leaves them out and the fresh
  // journal lists them as extensions again. Folding them into the base (round 5) made every later
  // delete of such a value a journaled rule (C5 mixed: 4-6 k journal rules, 25-70 ms per step).
  HeldExts hold;
};

struct gpc_ctx {
  gpc_config cfg;
  std::mutex ctl;    // control plane (conjMatchFlowLock + replayMutex role)
  std::mutex data;   // epoch pointer swap vs. kernel launch
  // Publishers waiting for `data`: launches yield to them. A caller that keeps its stream's queue
  // full holds `data` through every blocking launch and would otherwise re-take it ahead of a
  // waiting commit (std::mutex is not fair): measured 0.8-1.5 s per commit beside classification.
  std::atomic<uint32_t> publishers{0};
  std::atomic<int> fail_uploads{0};  // gpc_debug_fail_uploads: this context's next commit / replay uploads fail
  // Launch pacing (pace_take): per (slot, stream), the events after the last kPaceDepth calls.
  std::mutex pace_mu;
  std::map<std::pair<uint32_t, StreamKey>, std::deque<hipEvent_t>> pace;
  FeatureNP np;
  FeatureService svc;
  std::vector<uint32_t> svc_blob;        // host copy of the Service image (empty: no Services)
  uint64_t svc_gen = ~0ull;              // FeatureService generation the image was built from
  SlotMap slots;
  HostImage last;    // base image of the current epoch: shadow state for re-upload + debug export
  HostImage last6;   // IPv6 base image (ipv6_enabled)
  Journal journal;   // delta epochs over `last` (host mirror of the device pools)
  Journal journal6;  // IPv6 delta epochs over `last6`
  uint64_t n_full6 = 0, n_delta6 = 0;
  // Generation of the host base images (`last`, `last6`), bumped whenever one is replaced. A device
  // slot extends its published base with journal tails only while the base it holds is of the
  // current generation; otherwise (an earlier commit rebuilt the host base and then failed to
  // upload it) the slot re-uploads the base and the whole journal.
  uint64_t gen4 = 1, gen6 = 1;
  std::vector<DevState> dev;             // device slots (gpc_create: one, cfg.device)
  uint64_t cur_epoch = 0;                // epoch every slot currently publishes (0: nothing committed)
  uint32_t group_key = GPC_GROUP_KEY_AUTO;                            // gpc_group_key (gpc_create)
  uint32_t group_src_bits = env_u32("GPC_GROUP_SRC_BITS", 8, 0, 8);  // GPC_GROUP_KEY_ADDR key bits (classify.hip)
  // block order of grouped batches (classify.hip logical_block; 64M packets, ms per step for orders
  // 1 / 2 / 3: C2 16.04 / 15.66 / 15.77, C3 13.29 / 13.25 / 13.28, C4 14.57 / 14.16 / 14.06)
  uint32_t group_xcd = env_u32("GPC_GROUP_XCD", 2, 0, 3);
  // ingress verdicts of a grouped batch stored in grouped order, then put in caller order by
  // unpermute_kernel (1) or stored at the caller index by the ingress launch (0)
  uint32_t group_unpermute = env_u32("GPC_GROUP_UNPERMUTE", 1, 0, 1);
  // IPv6 batches are grouped like IPv4 ones, over their code columns (GPC_GROUP_V6=0: never)
  uint32_t group_v6 = env_u32("GPC_GROUP_V6", 1, 0, 1);
  // Service batches as two launches with the rewritten fields parked in between (GPC_SVC_SPLIT=1).
  // Off by default: measured slower than one launch doing the Service stage and both policy stages
  // (C4, 64M packets: 9.61 vs 9.10 ms; 12.24 vs 11.37 before the two-slot Service hash)
  uint32_t svc_split = env_u32("GPC_SVC_SPLIT", 0, 0, 1);
  void* stage = nullptr;                 // pinned staging buffer of journal uploads
  size_t stage_bytes = 0;
  std::vector<uint32_t> released_slots;
  std::vector<uint32_t> slot_conj;
  uint64_t epoch = 0, n_full = 0, n_delta = 0, n_bg = 0, n_pool_gc = 0;
  uint64_t commit_no = 0;                // commits so far (COMMIT markers in the log)
  bool comp_pending = false;             // a background compaction was requested, not installed yet
  std::vector<std::pair<uint64_t, FeatureNP::Dirty>> dirty_hist;  // per commit since the request
  Compactor comp;
  void* stage6 = nullptr;                // pinned staging buffer of IPv6 journal uploads
  size_t stage6_bytes = 0;
  gpc_ctx(const gpc_config& c, const std::vector<int>& devices) : cfg(c), np(c), svc(c), dev(devices.size()) {
    for (size_t k = 0; k < devices.size(); k++) dev[k].device = devices[k];
    journal6.set_family(6);
  }
};

// The event set of the next timed gpc_classify* call on a slot (ctx->data held), or null when
// timing is off.
static LaunchMarks* next_marks(DevState& D) {
  if (D.marks.empty()) return nullptr;
  LaunchMarks* m = &D.marks[D.marks_next];
  D.marks_next = (D.marks_next + 1) % D.marks.size();
  if (D.marks_used == D.marks.size()) D.marks_dropped++;
  else D.marks_used++;
  m->n = 0;
  return m;
}

static void free_marks(DevState& D) {
  for (auto& m : D.marks)
    for (auto& e : m.ev) (void)hipEventDestroy(e);
  D.marks.clear();
  D.marks_next = D.marks_used = D.marks_dropped = 0;
}

static void log_op(gpc_ctx* ctx, Op&& op) {
  {
    std::lock_guard<std::mutex> g(ctx->comp.mu);
    if (!ctx->comp.enabled) return;
    ctx->comp.log.push_back(std::move(op));
  }
  ctx->comp.cv.notify_one();
}

static int hip_ok(hipError_t e) { return e == hipSuccess ? 0 : -GPC_EDEV; }

// Per-rule counters are device-scope 64-bit atomics; with few rules (C1: 30 slots) every packet's
// update lands on a handful of addresses and serializes (64 M packets: 137 ms with counters vs
// 8.5 ms without). The array is therefore striped over `copies` replicas (block b updates copy
// b mod copies), sized so the replicas together span >= 64 K slots, and folded into copy 0 before
// anything reads it (gpc_counters, gpc_metrics). Large rule sets (C3: 89 k slots) keep one copy.
// The allocation holds copies + 1 arrays: the kernels' accumulators, then the published array
// that gpc_counters returns ({packets, bytes, sessions}; core.hpp count_stage).
static uint32_t counter_copies_for(size_t cap) {
  if (const char* e = std::getenv("GPC_COUNTER_COPIES")) {  // experiments: fixed power of two <= 64
    uint32_t r = 1;
    while (r < 64 && r * 2 <= uint32_t(std::atoi(e))) r <<= 1;
    return r;
  }
  uint32_t r = 1;
  while (r < 64 && cap * r < 65536) r <<= 1;
  return r;
}
static unsigned long long* published_counters(const DevState& D) {
  return D.d_counters ? D.d_counters + size_t(D.counter_copies) * D.counter_cap * kCounterWords : nullptr;
}
static int fold_counters(DevState& D) {  // caller holds ctl; device synchronized on return
  if (!D.d_counters) return GPC_OK;
  if (hip_ok(hipSetDevice(D.device)) || hip_ok(hipDeviceSynchronize())) return -GPC_EDEV;
  int rc = launch_fold_counters(D.d_counters, uint64_t(D.counter_cap) * kCounterWords, D.counter_copies, nullptr);
  if (!rc) rc = hip_ok(hipDeviceSynchronize());
  return rc;
}

// Lane regrouping (classify.hip sorted_index) pays when a stage's main table has long driver lists:
// it costs a second round of bucket lookups and a block barrier ahead of the table work, and saves
// the gap between a wave's longest and average scan. Per stage: the table with the most soft rules,
// if its entry-weighted mean bucket length (sum len^2 / sum len over the sub-index buckets of the
// shorter driver clause) reaches kLaneSortMinList. Measured on MI355X: C2 (statistic ~35) 33.4 -> 28.2 ms
// with it, C3 (statistic ~4: one clause has short lists) 14.6 -> 20.1 ms, so C3 runs without.
// Round 6: with combination lists and multi-interval exact entries C2g's statistic is 23-26 and it
// runs faster unsorted (one fused launch): 9.67 vs 10.91 ms per 64 M packets (r06h), so the bar is 32.
constexpr double kLaneSortMinList = 32.0;
static void lane_sort_tables(const HostImage& h, uint8_t* sort_table) {
  for (int st = 0; st < 2; st++) {
    sort_table[st] = 0;
    uint32_t best = 0, bt = 0;
    for (int t = 3 * st; t < 3 * st + 3; t++) {
      const uint32_t soft = h.hdr.t[t].n_rules - h.hdr.t[t].n_hard;
      if (soft > best) {
        best = soft;
        bt = uint32_t(t + 1);
      }
    }
    if (!bt) continue;
    const TableHdr& th = h.hdr.t[bt - 1];
    double mean[2];
    if (th.n_cidx) {  // the composite driver is the one scanned: its lists decide
      double s1 = th.always_n[th.cband], s2 = s1 * s1;
      for (uint32_t i = 0; i < th.n_cidx; i++) {
        const SubIdx& si = th.cidx[i];
        for (uint64_t b = 0; b < (1ull << si.bits); b++) {
          const double len = double(sub_bucket_len(h.blob.data(), si, uint32_t(b)));
          s1 += len;
          s2 += len * len;
        }
      }
      mean[0] = mean[1] = s1 > 0 ? s2 / s1 : 1e30;
    } else {
    for (int k = 0; k < 2; k++) {
      double s1 = th.always_n[k], s2 = double(th.always_n[k]) * th.always_n[k];
      for (uint32_t i = 0; i < th.n_idx[k]; i++) {
        const SubIdx& si = th.idx[k][i];
        const uint32_t* o = h.blob.data() + si.off;
        for (uint64_t b = 0; b < (1ull << si.bits); b++) {
          const double len = double(o[b + 1] - o[b]);
          s1 += len;
          s2 += len * len;
        }
      }
      mean[k] = s1 > 0 ? s2 / s1 : 1e30;
    }
    }
    const char* force = std::getenv("GPC_LANE_SORT");  // experiments: "1" forces regrouping on, "0" off
    if (force ? force[0] == '1' : std::min(mean[0], mean[1]) >= kLaneSortMinList) sort_table[st] = uint8_t(bt);
    if (std::getenv("GPC_IMAGE_DEBUG"))
      std::fprintf(stderr, "lane sort: stage %d table %u mean lists %.1f %.1f -> %s\n", st + 1, bt, mean[0], mean[1],
                   sort_table[st] ? "on" : "off");
  }
}

// Axes the driver sub-indexes of the image read: the packet columns the scan-length grouping key
// (classify.hip scan_key) needs.
static uint32_t group_axes(const HostImage& h) {
  uint32_t m = 0;
  for (const TableHdr& th : h.hdr.t) {
    for (int k = 0; k < 2; k++)
      for (uint32_t i = 0; i < th.n_idx[k] && i < uint32_t(kIdxPerClause); i++) m |= 1u << th.idx[k][i].axis;
    for (uint32_t i = 0; i < th.n_cidx && i < uint32_t(kIdxPerClause); i++) m |= 1u << th.cidx[i].axis | 1u << th.cx;
  }
  return m;
}


// Launch pacing. A caller that enqueues classify calls faster than the device runs them fills the
// stream's hardware queue, and its next launch then blocks -- inside the data lock, which a commit
// needs to publish its epoch (measured: commits waited 0.8-1.4 s beside a saturating caller). So a
// call first waits, outside every lock, until the call `depth` (gpc_config.launch_pacing, default
// kPaceDepth) calls before it on the same stream has finished; the device still has that many calls
// queued, and no launch blocks. The per-stream queues are bounded like the grouping scratch: past
// kPaceStreams streams, the queues whose events have all completed (idle streams, exited threads of
// hipStreamPerThread) are dropped and their events destroyed. The trim runs only when a call brings
// a new stream (not on every launch), and it queries one event per queue: events of a
// queue were recorded in stream order, so the newest one completing means the queue is idle.
constexpr size_t kPaceDepth = 8, kPaceStreams = 64;
static void pace_trim(gpc_ctx* ctx) {  // pace_mu held
  if (ctx->pace.size() <= kPaceStreams) return;
  for (auto it = ctx->pace.begin(); it != ctx->pace.end();) {
    const bool idle = it->second.empty() || hipEventQuery(it->second.back()) == hipSuccess;
    if (!idle) {
      (void)hipGetLastError();
      ++it;
      continue;
    }
    for (hipEvent_t e : it->second) (void)hipEventDestroy(e);
    it = ctx->pace.erase(it);
  }
}
struct Pace {
  gpc_ctx* ctx;
  uint32_t slot;
  hipStream_t st;
  hipEvent_t ev = nullptr;
  Pace(gpc_ctx* c, uint32_t sl, hipStream_t s, bool on) : ctx(c), slot(sl), st(s) {  // the slot's device is current
    const int32_t cfg = ctx->cfg.launch_pacing;
    if (!on || cfg < 0) return;
    const size_t depth = cfg > 0 ? size_t(cfg) : kPaceDepth;
    {
      std::lock_guard<std::mutex> p(ctx->pace_mu);
      const auto key = std::make_pair(slot, stream_key(st));
      if (!ctx->pace.count(key)) pace_trim(ctx);
      auto& q = ctx->pace[key];
      if (q.size() >= depth) {
        ev = q.front();
        q.pop_front();
      }
    }
    if (ev) {
      (void)hipEventSynchronize(ev);
    } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      ev = nullptr;
    }
  }
  void record() {  // after this call's launches, on its stream
    if (ev && hipEventRecord(ev, st) != hipSuccess) (void)hipGetLastError();
  }
  ~Pace() {
    if (!ev) return;
    std::lock_guard<std::mutex> p(ctx->pace_mu);
    ctx->pace[{slot, stream_key(st)}].push_back(ev);
  }
};

// fail: the context's gpc_debug_fail_uploads counter (commit / replay uploads only; the background
// compactor's uploads pass none)
static int upload_image(const HostImage& h, int device, hipStream_t s, std::shared_ptr<DevImage>* out,
                        std::atomic<int>* fail = nullptr) {
  if (fail && fail->load() > 0 && fail->fetch_sub(1) > 0) return -GPC_EDEV;
  auto d = std::make_shared<DevImage>();
  d->s = s;
  d->device = device;
  d->bytes = h.blob.size() * 4;
  if (hip_ok(dev_alloc((void**)&d->d_blob, d->bytes, s)) || hip_ok(dev_alloc((void**)&d->d_hdr, sizeof(ImageHdr), s)) ||
      hip_ok(hipMemcpyAsync(d->d_blob, h.blob.data(), d->bytes, hipMemcpyHostToDevice, s)) ||
      hip_ok(hipMemcpyAsync(d->d_hdr, &h.hdr, sizeof(ImageHdr), hipMemcpyHostToDevice, s)))
    return -GPC_EDEV;
  lane_sort_tables(h, d->sort_table);
  d->axes = group_axes(h);
  for (const TableHdr& th : h.hdr.t) d->composite = d->composite || th.n_cidx != 0;
  *out = std::move(d);
  return GPC_OK;
}

static int upload_words(const std::vector<uint32_t>& w, int device, hipStream_t s, std::shared_ptr<DevImage>* out) {
  auto d = std::make_shared<DevImage>();
  d->s = s;
  d->device = device;
  d->bytes = w.size() * 4;
  if (hip_ok(dev_alloc((void**)&d->d_blob, d->bytes, s)) ||
      hip_ok(hipMemcpyAsync(d->d_blob, w.data(), d->bytes, hipMemcpyHostToDevice, s)))
    return -GPC_EDEV;
  *out = std::move(d);
  return GPC_OK;
}

static void collect_retired(DevState& D, bool wait) {  // the slot's device is current
  if (wait && !D.retired.empty()) (void)hipDeviceSynchronize();
  size_t k = 0;
  for (size_t i = 0; i < D.retired.size(); i++) {
    if (wait || D.retired[i].drained()) {
      D.retired[i].release(D.ustream);
    } else {
      if (k != i) D.retired[k] = std::move(D.retired[i]);
      k++;
    }
  }
  D.retired.resize(k);
}

// A new journal pool on one slot (kPoolWords words, stream-ordered allocation).
static int alloc_pool(int device, hipStream_t s, std::shared_ptr<DevImage>* out) {
  auto pool = std::make_shared<DevImage>();
  pool->s = s;
  pool->device = device;
  pool->bytes = kPoolWords * 4;
  if (hip_ok(dev_alloc((void**)&pool->d_blob, pool->bytes, s))) return -GPC_EDEV;
  *out = std::move(pool);
  return GPC_OK;
}

static int commit_impl(gpc_ctx* ctx, bool force_full);

static void compactor_main(gpc_ctx* ctx) {
  Compactor& C = ctx->comp;
  FeatureNP shadow(ctx->cfg);
  uint64_t shadow_commit = 0;
  bool at_marker = true;
  std::vector<hipStream_t> bs(ctx->dev.size(), nullptr);  // one upload stream per device slot
  bool dev_ok = true;
  for (size_t k = 0; k < bs.size() && dev_ok; k++)
    dev_ok = hipSetDevice(ctx->dev[k].device) == hipSuccess &&
             hipStreamCreateWithFlags(&bs[k], hipStreamNonBlocking) == hipSuccess;
  if (!dev_ok) (void)hipGetLastError();
  auto grab = [&](std::vector<Op>* out, bool wait) {  // false: stop requested
    std::unique_lock<std::mutex> lk(C.mu);
    if (wait)
      C.cv.wait_for(lk, std::chrono::milliseconds(50), [&] { return C.stop || !C.log.empty() || C.want_commit; });
    if (C.stop) return false;
    out->swap(C.log);
    return true;
  };
  auto replay = [&](std::vector<Op>& ops) {
    for (auto& op : ops) {
      try {
        (void)op.apply(shadow);
      } catch (...) {
      }
      at_marker = op.kind == Op::COMMIT;
      if (at_marker) shadow_commit = op.commit_no;
    }
    size_t n = ops.size();
    ops.clear();
    return n;
  };
  std::vector<Op> ops;
  HeldExts hold;
  while (grab(&ops, true)) {
    replay(ops);
    uint64_t want;
    {
      std::lock_guard<std::mutex> g(C.mu);
      want = C.want_commit;
      if (want && at_marker && shadow_commit >= want) {
        C.want_commit = 0;
        C.busy = true;
        hold.swap(C.hold);
        C.hold.clear();
      } else {
        continue;
      }
    }
    // full image of the shadow's state, then catch up through a fresh journal
    const bool dbg = std::getenv("GPC_COMPACT_DEBUG") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto ms_since = [](std::chrono::steady_clock::time_point a) {
      return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    };
    double t_build = 0, t_catch = 0;
    auto base = std::make_unique<HostImage>();
    auto jn = std::make_unique<Journal>();
    int rc = GPC_OK;
    try {
      (void)shadow.take_dirty();
      rc = build_image(shadow, ctx->slots, base.get(), /*alloc=*/false, hold.empty() ? nullptr : &hold);
      t_build = ms_since(t0);
      jn->reset(base.get());
      for (int round = 0; rc == GPC_OK && round < 4; round++) {
        size_t n = 0;
        do {
          if (!grab(&ops, n > 0 || !at_marker)) {
            rc = -GPC_EINVAL;
            break;
          }
          n += replay(ops);
        } while (!at_marker);
        if (rc) break;
        FeatureNP::Dirty d = shadow.take_dirty();
        if (d.hard_tables & FeatureNP::kDirtyClassifier) {  // the base no longer matches: give up this round
          rc = -GPC_EINVAL;
          break;
        }
        if (round == 0)  // the held extensions become extensions of the new base
          for (auto& h : hold) d.conj.insert(h.first);
        std::string err;
        if ((!d.conj.empty() || d.hard_tables) && jn->apply(shadow, ctx->slots, d.conj, d.hard_tables, &err, false) != GPC_OK)
          rc = -GPC_EINVAL;
        if (n < 256) break;
      }
    } catch (...) {
      rc = -GPC_ENOMEM;
    }
    t_catch = ms_since(t0) - t_build;
    if (const char* d = std::getenv("GPC_TEST_COMPACT_DELAY_MS"))  // tests: widen the handover race window
      std::this_thread::sleep_for(std::chrono::milliseconds(std::atoi(d)));
    std::vector<std::shared_ptr<DevImage>> dbase, dpool;
    size_t up = 0;
    if (rc == GPC_OK && dev_ok) {  // the same base and journal on every device slot
      bool ok = true;
      dbase.resize(bs.size());
      dpool.resize(bs.size());
      for (size_t k = 0; k < bs.size() && ok; k++) {
        const int dv = ctx->dev[k].device;
        ok = hipSetDevice(dv) == hipSuccess && !upload_image(*base, dv, bs[k], &dbase[k]) &&
             !alloc_pool(dv, bs[k], &dpool[k]) &&
             !(jn->active() && hip_ok(hipMemcpyAsync(dpool[k]->d_blob, jn->pool.data(), jn->pool.size() * 4,
                                                     hipMemcpyHostToDevice, bs[k])));
      }
      for (size_t k = 0; k < bs.size() && ok; k++) ok = hipStreamSynchronize(bs[k]) == hipSuccess;
      if (!ok) {
        (void)hipGetLastError();
        dbase.clear();
        dpool.clear();
      } else {
        up = jn->active() ? jn->pool.size() : 0;
      }
    }
    if (dbg)
      std::fprintf(stderr, "compaction at commit %llu: build %.0f ms, catch-up %.0f ms (journal %zu words), upload %.0f ms\n",
                   (unsigned long long)shadow_commit, t_build, t_catch, jn->pool.size(), ms_since(t0) - t_build - t_catch);
    std::lock_guard<std::mutex> g(C.mu);
    C.busy = false;
    C.ready = true;
    C.rc = rc;
    C.base = std::move(base);
    C.journal = std::move(jn);
    C.dbase = std::move(dbase);
    C.dpool = std::move(dpool);
    C.uploaded = up;
    C.at_commit = shadow_commit;
  }
  {
    std::lock_guard<std::mutex> g(C.mu);  // results not installed are dropped with the context
    C.dbase.clear();
    C.dpool.clear();
  }
  for (size_t k = 0; k < bs.size(); k++)
    if (bs[k]) {
      (void)hipSetDevice(ctx->dev[k].device);
      (void)hipStreamSynchronize(bs[k]);
      (void)hipStreamDestroy(bs[k]);
    }
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
  if (!cfg) return -GPC_EINVAL;
  const int32_t d = cfg->device;
  return gpc_create_multi(cfg, &d, 1, out);
}

int gpc_create_multi(const gpc_config* cfg, const int32_t* devices, size_t n, gpc_ctx** out) {
  if (!cfg || !out || !devices || n == 0 || n > GPC_MAX_DEVICES) return -GPC_EINVAL;
  if (!cfg->ipv4_enabled && !cfg->ipv6_enabled) return -GPC_EINVAL;
  if (cfg->group_key < GPC_GROUP_KEY_AUTO || cfg->group_key > GPC_GROUP_KEY_SCAN) return -GPC_EINVAL;
  for (size_t k = 0; k < n; k++)
    if (devices[k] < 0) return -GPC_EINVAL;
  try {
    gpc_config c = *cfg;
    c.device = devices[0];
    *out = new gpc_ctx(c, std::vector<int>(devices, devices + n));
    // grouping key: the environment (experiments) overrides the config
    (*out)->group_key = env_u32("GPC_GROUP_KEY", uint32_t(cfg->group_key), GPC_GROUP_KEY_AUTO, GPC_GROUP_KEY_SCAN);
    if (cfg->compact_after >= 0) (*out)->comp.th = std::thread(compactor_main, *out);
    else (*out)->comp.enabled = false;
  } catch (...) {
    return -GPC_ENOMEM;
  }
  return GPC_OK;
}

// Drops every device buffer of a slot (the slot's device is current, launches drained).
static void drop_slot(DevState& D) {
  D.retired.push_back(RetiredEpoch{std::move(D.cur)});
  D.cur = DevEpoch();
  collect_retired(D, true);
  if (D.d_counters) (void)hipFree(D.d_counters);
  D.d_counters = nullptr;
  for (auto& kv : D.scratch) {
    (void)hipFree(kv.second.p);
    if (kv.second.done) (void)hipEventDestroy(kv.second.done);
  }
  D.scratch.clear();
  D.launch_epoch.clear();
}

int gpc_n_devices(gpc_ctx* ctx) { return ctx ? int(ctx->dev.size()) : -GPC_EINVAL; }

void gpc_destroy(gpc_ctx* ctx) {
  if (!ctx) return;
  {
    std::lock_guard<std::mutex> g(ctx->comp.mu);
    ctx->comp.stop = true;
  }
  ctx->comp.cv.notify_all();
  if (ctx->comp.th.joinable()) ctx->comp.th.join();
  for (DevState& D : ctx->dev) {
    if (D.cur.base || D.d_counters || !D.retired.empty() || D.ustream || !D.marks.empty()) {
      (void)hipSetDevice(D.device);
      (void)hipDeviceSynchronize();
      drop_slot(D);
      if (D.ustream) {
        (void)hipStreamSynchronize(D.ustream);
        (void)hipStreamDestroy(D.ustream);
      }
      free_marks(D);
    }
  }
  for (auto& kv : ctx->pace) {
    (void)hipSetDevice(ctx->dev[kv.first.first].device);
    for (hipEvent_t ev : kv.second) (void)hipEventDestroy(ev);
  }
  if (ctx->stage) (void)hipHostFree(ctx->stage);
  if (ctx->stage6) (void)hipHostFree(ctx->stage6);
  delete ctx;
}

int gpc_initialize(gpc_ctx* ctx) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  int rc = ctx->np.initialize();
  Op op;
  op.kind = Op::INIT;
  log_op(ctx, std::move(op));
  return rc;
}

int gpc_install_rule(gpc_ctx* ctx, const gpc_rule* rule) {
  if (!ctx || !rule) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  try {
    int rc = ctx->np.install_rule(*rule);
    Op op;
    op.kind = Op::INSTALL;
    op.rules.emplace_back(*rule);
    log_op(ctx, std::move(op));
    return rc;
  } catch (...) {
    return -GPC_ENOMEM;
  }
}

int gpc_batch_install(gpc_ctx* ctx, const gpc_rule* rules, size_t n) {
  if (!ctx || (!rules && n)) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  try {
    int rc = ctx->np.batch_install(rules, n);
    Op op;
    op.kind = Op::BATCH;
    op.rules.reserve(n);
    for (size_t i = 0; i < n; i++) op.rules.emplace_back(rules[i]);
    log_op(ctx, std::move(op));
    return rc;
  } catch (...) {
    return -GPC_ENOMEM;
  }
}

int gpc_uninstall_rule(gpc_ctx* ctx, uint32_t rule_id, uint16_t* stale, size_t cap, size_t* n_stale) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  std::vector<uint16_t> st;
  int rc = ctx->np.uninstall_rule(rule_id, &st);
  Op op;
  op.kind = Op::UNINSTALL;
  op.id = rule_id;
  log_op(ctx, std::move(op));
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
  int rc = ctx->np.add_rule_addrs(rule_id, addr_type, addrs, n, prio, enable_logging != 0, is_mcnp != 0);
  Op op;
  op.kind = Op::ADD;
  op.id = rule_id;
  op.addr_type = addr_type;
  op.addrs.assign(addrs, addrs + n);
  op.has_prio = prio != nullptr;
  op.prio = prio ? *prio : 0;
  op.logging = enable_logging != 0;
  op.mcnp = is_mcnp != 0;
  log_op(ctx, std::move(op));
  return rc;
}

int gpc_del_rule_addrs(gpc_ctx* ctx, uint32_t rule_id, int32_t addr_type, const gpc_addr* addrs, size_t n,
                       const uint16_t* prio) {
  if (!ctx || (!addrs && n)) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  int rc = ctx->np.del_rule_addrs(rule_id, addr_type, addrs, n, prio);
  Op op;
  op.kind = Op::DEL;
  op.id = rule_id;
  op.addr_type = addr_type;
  op.addrs.assign(addrs, addrs + n);
  op.has_prio = prio != nullptr;
  op.prio = prio ? *prio : 0;
  log_op(ctx, std::move(op));
  return rc;
}

int gpc_reassign_priorities(gpc_ctx* ctx, const uint16_t* from, const uint16_t* to, size_t n, uint8_t table) {
  if (!ctx || ((!from || !to) && n)) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  int rc = ctx->np.reassign_priorities(from, to, n, table);
  Op op;
  op.kind = Op::REASSIGN;
  op.from.assign(from, from + n);
  op.to.assign(to, to + n);
  op.table = table;
  log_op(ctx, std::move(op));
  return rc;
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
    {  // loaded flows always commit as full rebuilds: the shadow compiler is not needed any more
      std::lock_guard<std::mutex> c(ctx->comp.mu);
      ctx->comp.enabled = false;
      ctx->comp.log.clear();
    }
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
int gpc_set_node_port_addresses(gpc_ctx* ctx, const uint8_t* ips, uint8_t family, size_t n) {
  if ((!ips && n) || family != 4 || n > kSvcMaxNodePortAddrs - 1) return -GPC_EINVAL;
  std::vector<uint32_t> v4(n);
  for (size_t i = 0; i < n; i++) {
    const uint8_t* b = ips + 16 * i;
    v4[i] = (uint32_t(b[0]) << 24) | (uint32_t(b[1]) << 16) | (uint32_t(b[2]) << 8) | b[3];
  }
  GPC_SVC_CALL(ctx->svc.set_node_port_addresses(v4.data(), n));
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

int gpc_new_dns_conjunction(gpc_ctx* ctx, uint32_t id) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  try {
    int rc = ctx->np.new_dns_conjunction(id);
    Op op;
    op.kind = Op::DNS_NEW;
    op.id = id;
    log_op(ctx, std::move(op));
    return rc;
  } catch (...) {
    return -GPC_ENOMEM;
  }
}

// AddAddressToDNSConjunction / DeleteAddressFromDNSConjunction (network_policy.go:781-789): the
// Add/DeletePolicyRuleAddress of the DNS conjunction's to clause at priority 64991.
int gpc_add_dns_conj_addrs(gpc_ctx* ctx, uint32_t id, const gpc_addr* addrs, size_t n) {
  const uint16_t prio = kPriorityDNSIntercept;
  return gpc_add_rule_addrs(ctx, id, GPC_DST_ADDRESS, addrs, n, &prio, 0, 0);
}

int gpc_del_dns_conj_addrs(gpc_ctx* ctx, uint32_t id, const gpc_addr* addrs, size_t n) {
  const uint16_t prio = kPriorityDNSIntercept;
  return gpc_del_rule_addrs(ctx, id, GPC_DST_ADDRESS, addrs, n, &prio);
}

int gpc_network_policy_flow_keys(gpc_ctx* ctx, const char* name, const char* ns, uint8_t policy_type, char* buf,
                                 size_t cap, size_t* needed, size_t* n_keys) {
  if (!ctx || !name || !ns) return -GPC_EINVAL;
  std::string s;
  size_t n = 0;
  try {
    std::lock_guard<std::mutex> g(ctx->ctl);  // the replayMutex write lock of the reference
    for (auto& k : ctx->np.flow_keys(name, ns, policy_type)) {
      if (n++) s += "\n";
      s += k;
    }
  } catch (...) {
    return -GPC_ENOMEM;
  }
  if (needed) *needed = s.size() + 1;
  if (n_keys) *n_keys = n;
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

// ReplayFlows (client.go:1130-1152; NP part network_policy.go:1626-1657) for the device: after a
// device reset (or to move a context's data path to a freshly initialised device) every device
// buffer is rebuilt from the host shadow state -- base image, journal pool, IPv6 and Service
// images -- without compiler work; the realized flows, conj ids and counter slots are unchanged.
// Device counters restart from zero, as OVS flow counters do after the flows are replayed.
int gpc_debug_fail_uploads(gpc_ctx* ctx, int n) {
  if (!ctx) return -GPC_EINVAL;
  ctx->fail_uploads.store(n > 0 ? n : 0);
  return GPC_OK;
}

int gpc_replay(gpc_ctx* ctx) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  {  // a background compaction result built on the old device state is dropped
    std::lock_guard<std::mutex> c(ctx->comp.mu);
    if (ctx->comp.busy) ctx->comp.discard = true;
    ctx->comp.dbase.clear();
    ctx->comp.dpool.clear();
    if (ctx->comp.ready) ctx->comp.discard = true;
  }
  std::vector<DevState> old(ctx->dev.size());
  {
    std::lock_guard<std::mutex> d(ctx->data);
    for (size_t k = 0; k < ctx->dev.size(); k++) {
      DevState& D = ctx->dev[k];
      old[k].device = D.device;
      old[k].cur = std::move(D.cur);
      D.cur = DevEpoch();
      old[k].d_counters = D.d_counters;
      D.d_counters = nullptr;
      D.launch_epoch.clear();
      old[k].scratch.swap(D.scratch);
      old[k].retired.swap(D.retired);
      old[k].ustream = D.ustream;
    }
    ctx->cur_epoch = 0;
  }
  int drop_rc = GPC_OK;  // every old slot is dropped even when one of them fails
  for (DevState& O : old) {
    if (hip_ok(hipSetDevice(O.device))) drop_rc = -GPC_EDEV;
    (void)hipDeviceSynchronize();  // may fail after a reset: the old buffers are dropped regardless
    (void)hipGetLastError();
    drop_slot(O);
    (void)hipGetLastError();
  }
  if (drop_rc) return drop_rc;
  if (ctx->last.blob.empty()) return GPC_OK;  // nothing committed yet
  const size_t cap = std::max<size_t>(1, ctx->slots.size());
  const uint32_t copies = counter_copies_for(cap);
  std::vector<DevEpoch> ne(ctx->dev.size());
  std::vector<unsigned long long*> nc(ctx->dev.size(), nullptr);
  Journal& jn = ctx->journal;
  int rc = GPC_OK;
  for (size_t k = 0; k < ctx->dev.size() && !rc; k++) {
    DevState& D = ctx->dev[k];
    // (a failure leaves rc set: the cleanup below releases what earlier slots uploaded)
    if (hip_ok(hipSetDevice(D.device)) || (!D.ustream && hip_ok(hipStreamCreateWithFlags(&D.ustream, hipStreamNonBlocking)))) {
      rc = -GPC_EDEV;
      break;
    }
    hipStream_t us = D.ustream;
    ne[k].base_gen = ctx->gen4;
    ne[k].v6_gen = ctx->gen6;
    rc = upload_image(ctx->last, D.device, us, &ne[k].base, &ctx->fail_uploads);
    if (!rc && jn.active()) {
      rc = alloc_pool(D.device, us, &ne[k].pool);
      if (!rc && hip_ok(hipMemcpyAsync(ne[k].pool->d_blob, jn.pool.data(), jn.pool.size() * 4, hipMemcpyHostToDevice, us)))
        rc = -GPC_EDEV;
      ne[k].jhdr = jn.hdr_off;
      ne[k].jmode = jn.mode();
    }
    if (!rc && !ctx->last6.blob.empty()) {
      rc = upload_image(ctx->last6, D.device, us, &ne[k].v6, &ctx->fail_uploads);
      ne[k].v6_lpm = ctx->last6.hdr.v6_lpm;
      const Journal& j6 = ctx->journal6;
      if (!rc && j6.active()) {
        rc = alloc_pool(D.device, us, &ne[k].v6_pool);
        if (!rc && hip_ok(hipMemcpyAsync(ne[k].v6_pool->d_blob, j6.pool.data(), j6.pool.size() * 4,
                                         hipMemcpyHostToDevice, us)))
          rc = -GPC_EDEV;
        ne[k].v6_jhdr = j6.hdr_off;
      }
    }
    if (!rc && !ctx->svc_blob.empty()) rc = upload_words(ctx->svc_blob, D.device, us, &ne[k].svc);
    if (!rc && (hip_ok(hipMalloc(&nc[k], cap * kCounterBytes * (copies + 1))) ||
                hip_ok(hipMemset(nc[k], 0, cap * kCounterBytes * (copies + 1)))))
      rc = -GPC_EDEV;
    if (!rc) rc = hip_ok(hipStreamSynchronize(us));
  }
  if (rc) {
    for (size_t k = 0; k < ctx->dev.size(); k++) {
      (void)hipSetDevice(ctx->dev[k].device);
      RetiredEpoch{std::move(ne[k])}.release(ctx->dev[k].ustream);
      if (nc[k]) (void)hipFree(nc[k]);
    }
    return rc;
  }
  if (jn.active()) jn.uploaded = jn.pool.size();
  if (ctx->journal6.active()) ctx->journal6.uploaded = ctx->journal6.pool.size();
  const uint64_t epoch = ++ctx->epoch;
  PublishLock d(ctx->data, ctx->publishers);
  for (size_t k = 0; k < ctx->dev.size(); k++) {
    DevState& D = ctx->dev[k];
    ne[k].epoch = epoch;
    D.cur = std::move(ne[k]);
    D.d_counters = nc[k];
    D.counter_cap = cap;
    D.counter_copies = copies;
  }
  ctx->cur_epoch = epoch;
  return GPC_OK;
}
int gpc_compact(gpc_ctx* ctx) { return commit_impl(ctx, true); }

// gpc_config.group_packets = 0: batches from this size on are grouped by nw_src before the table
// walk when the image outgrows one XCD's L2 (4 MB); a smaller image stays L2-resident and grouping
// costs more than it saves (C1: 0.3 MB image, 10.87 -> 11.17 ms per 64M packets).
constexpr size_t kGroupMinPackets = size_t(1) << 18;
constexpr size_t kGroupMinImageBytes = size_t(4) << 20;

// Grouping scratch of stream st with at least `need` bytes (ctx->data held). A buffer held for a
// much larger earlier batch is given back when a batch needs less than an eighth of it.
static int group_scratch(DevState& D, hipStream_t s, size_t need, uint8_t** out) {
  const StreamKey st = stream_key(s);
  if (D.scratch.size() >= kScratchStreams && !D.scratch.count(st)) {
    for (auto it = D.scratch.begin(); it != D.scratch.end();) {  // streams whose last batch is done
      if (!it->second.done || hipEventQuery(it->second.done) == hipSuccess) {
        (void)hipFree(it->second.p);
        if (it->second.done) (void)hipEventDestroy(it->second.done);
        it = D.scratch.erase(it);
      } else {
        ++it;
      }
    }
    (void)hipGetLastError();
  }
  StreamScratch& sc = D.scratch[st];
  // Grow at once; shrink only after kScratchShrinkAfter consecutive small calls, so alternating
  // large and small batches on one stream never allocate on the data path.
  sc.small = sc.bytes / 8 > need ? sc.small + 1 : 0;
  if (sc.bytes < need || sc.small > kScratchShrinkAfter) {
    sc.small = 0;
    dev_free(sc.p, s);  // after the launches already queued on s
    sc.p = nullptr;
    sc.bytes = 0;
    if (hip_ok(hipMalloc((void**)&sc.p, need))) return -GPC_ENOMEM;
    sc.bytes = need;
  }
  *out = sc.p;
  return GPC_OK;
}

// The grouping scratch of stream st is in use until the launches just queued there have run.
static int group_scratch_used(DevState& D, hipStream_t st) {
  StreamScratch& sc = D.scratch[stream_key(st)];
  if (!sc.done && hip_ok(hipEventCreateWithFlags(&sc.done, hipEventDisableTiming))) return -GPC_EDEV;
  return hip_ok(hipEventRecord(sc.done, st));
}

// Grouping scratch for a batch the pre-pass would speed up. Grouping is a performance choice: when
// it was not forced (gpc_config.group_packets == 0) and its scratch cannot be had, the batch runs
// ungrouped instead of failing.
static int group_scratch_for(gpc_ctx* ctx, DevState& D, hipStream_t st, size_t need, uint8_t** out) {
  *out = nullptr;
  const int e = group_scratch(D, st, need, out);
  if (e == -GPC_ENOMEM && ctx->cfg.group_packets == 0) {
    (void)hipGetLastError();
    *out = nullptr;
    return GPC_OK;
  }
  return e;
}

// Auto mode leaves batches against a base-only image with composite driver indexes ungrouped: the
// short composite lists gain less from grouped lanes than the pre-pass and the un-permute cost (64M
// packets, profiles/r03q_grouping_ab.txt: C3 10.13 grouped vs 9.91 ms, C2 10.27 vs 9.79, C4 9.13
// vs 8.91). Delta epochs (journal walks) still gain from it (C5: 13.05 grouped vs 13.58 ms).
static bool group_batch(const gpc_ctx* ctx, size_t n, const DevImage& img, bool delta) {
  const int gm = ctx->cfg.group_packets;
  return n && (gm > 0 || (gm == 0 && n >= kGroupMinPackets && img.bytes >= kGroupMinImageBytes && (!img.composite || delta)));
}

// GPC_GROUP_KEY_AUTO: scan lengths where a wavefront's lanes scan very unequal driver lists (the
// lane_sort_tables statistic: C2, 26.4 -> 16.3 ms per 64M packets), address bits where the image
// lines a wave shares matter more (C3 13.2 ms by address vs 15.4 by scan length, C4 14.3 vs 16.4).
static uint32_t group_key(const gpc_ctx* ctx) {
  if (ctx->group_key != GPC_GROUP_KEY_AUTO) return ctx->group_key;
  const DevImage& b = *ctx->dev[0].cur.base;
  return (b.sort_table[0] || b.sort_table[1]) ? uint32_t(GPC_GROUP_KEY_SCAN) : uint32_t(GPC_GROUP_KEY_ADDR);
}

int gpc_classify(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, int32_t count, void* stream) {
  return gpc_classify_on(ctx, 0, pk, n, out, nullptr, count, stream);
}

int gpc_classify_lb(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, gpc_lb_result* lb_out, int32_t count,
                    void* stream) {
  return gpc_classify_on(ctx, 0, pk, n, out, lb_out, count, stream);
}

// Epoch lifetime bookkeeping after launches on stream st of slot D (ctx->data held).
static int note_launch(gpc_ctx* ctx, DevState& D, hipStream_t st) {
  D.launch_epoch[stream_key(st)] = D.cur.epoch;
  hipEvent_t& ev = D.cur.last_use[stream_key(st)];  // epoch lifetime: retired epochs are freed once drained
  if (!ev && hip_ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming))) return -GPC_EDEV;
  (void)ctx;
  return hip_ok(hipEventRecord(ev, st));
}

int gpc_classify_on(gpc_ctx* ctx, uint32_t slot, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out,
                    gpc_lb_result* lb_out, int32_t count, void* stream) {
  if (!ctx || !pk || (!out && n) || n > GPC_MAX_BATCH || slot >= ctx->dev.size()) return -GPC_EINVAL;
  if (n && (!pk->src || !pk->dst || !pk->sport || !pk->dport || !pk->proto || !pk->out_port)) return -GPC_EINVAL;
  if (hip_ok(hipSetDevice(ctx->dev[slot].device))) return -GPC_EDEV;
  Pace pace(ctx, slot, (hipStream_t)stream, n != 0);
  const auto d = launch_lock(ctx->data, ctx->publishers);
  DevState& D = ctx->dev[slot];
  if (!D.cur.base) return -GPC_EINVAL;  // nothing committed yet
  const bool jpool = D.cur.jhdr && D.cur.jmode != kModeBase;
  EpochArgs ep{D.cur.base->d_hdr, D.cur.base->d_blob, jpool ? D.cur.pool->d_blob : nullptr, D.cur.jhdr,
               D.cur.svc ? D.cur.svc->d_blob : nullptr, 0u, {D.cur.base->sort_table[0], D.cur.base->sort_table[1]},
               uint32_t(D.counter_cap * kCounterWords), D.counter_copies - 1, uint32_t(D.cur.jmode)};
  hipStream_t st = (hipStream_t)stream;
  // packet grouping (classify.hip group_*): one scratch buffer per stream, reused stream-ordered by
  // the next batch on that stream (launches of one stream run in order), so callers on different
  // streams never share one and the data path does no allocation once warm
  GroupArgs ga{nullptr, group_key(ctx), D.cur.base->axes, ctx->group_src_bits, ctx->group_xcd, ctx->group_unpermute,
               D.cur.svc && lb_out && ctx->group_unpermute};
  // Service batches: 16 B per packet to park the fields the Service stage rewrites between the
  // egress and the ingress launch (classify.hip launch); without it (no memory) one launch does both
  const size_t park_bytes = D.cur.svc && n && ctx->svc_split ? (16 * n + 255) & ~size_t(255) : 0;
  uint8_t* scratch = nullptr;
  if (group_batch(ctx, n, *D.cur.base, jpool && D.cur.jmode == kModeJournal)) {
    if (const int e = group_scratch_for(ctx, D, st, park_bytes + group_scratch_bytes(*pk, n, ga.lb), &scratch)) return e;
    if (scratch) ga.scratch = scratch + park_bytes;
  }
  if (park_bytes && !scratch && group_scratch(D, st, park_bytes, &scratch)) {
    (void)hipGetLastError();
    scratch = nullptr;  // a performance choice, never a data-path failure
  }
  int rc = launch_classify(ep, *pk, n, out, reinterpret_cast<uint4*>(lb_out), D.d_counters, count,
                           ga.scratch ? &ga : nullptr, st, n ? next_marks(D) : nullptr,
                           park_bytes && scratch ? reinterpret_cast<uint4*>(scratch) : nullptr);
  if (!rc && scratch) rc = group_scratch_used(D, st);
  if (rc || n == 0) return rc;
  pace.record();
  return note_launch(ctx, D, st);
}

int gpc_trace(gpc_ctx* ctx, const gpc_pkt_soa* pk, gpc_verdict* out, gpc_lb_result* lb_out, gpc_trace_step* steps,
              size_t cap, size_t* n_steps) {
  static_assert(sizeof(gpc_trace_step) == sizeof(TraceStep), "gpc_trace_step mirrors core.hpp TraceStep");
  if (!ctx || !pk || !out || !pk->src || !pk->dst || !pk->sport || !pk->dport || !pk->proto || !pk->out_port)
    return -GPC_EINVAL;
  if (hip_ok(hipSetDevice(ctx->dev[0].device))) return -GPC_EDEV;
  // one packet: every present column's element 0 goes into one small device buffer
  struct Col {
    const void* h;
    size_t elem;
    const void** d;
  };
  gpc_pkt_soa d{};
  Col cols[] = {{pk->src, 4, (const void**)&d.src},           {pk->dst, 4, (const void**)&d.dst},
                {pk->sport, 2, (const void**)&d.sport},       {pk->dport, 2, (const void**)&d.dport},
                {pk->proto, 1, (const void**)&d.proto},       {pk->out_port, 4, (const void**)&d.out_port},
                {pk->in_port, 4, (const void**)&d.in_port},   {pk->svc_group, 4, (const void**)&d.svc_group},
                {pk->tun_id, 4, (const void**)&d.tun_id},     {pk->ct_src, 4, (const void**)&d.ct_src},
                {pk->ct_dst, 4, (const void**)&d.ct_dst},     {pk->ct_state, 1, (const void**)&d.ct_state},
                {pk->dest, 1, (const void**)&d.dest},         {pk->len, 2, (const void**)&d.len},
                {pk->ct_mark, 1, (const void**)&d.ct_mark}};
  constexpr size_t kSlot = 16, kOut = 512;  // column slots, then verdicts / LB result / steps / count
  const size_t ncol = sizeof cols / sizeof cols[0];
  std::vector<uint8_t> h(kOut + ncol * kSlot, 0);
  for (size_t c = 0; c < ncol; c++)
    if (cols[c].h) std::memcpy(h.data() + kOut + c * kSlot, cols[c].h, cols[c].elem);
  uint8_t* buf = nullptr;
  if (hip_ok(hipMalloc(&buf, h.size()))) return -GPC_EDEV;
  for (size_t c = 0; c < ncol; c++)
    if (cols[c].h) *cols[c].d = buf + kOut + c * kSlot;
  int rc = hip_ok(hipMemcpy(buf, h.data(), h.size(), hipMemcpyHostToDevice));
  uint4* dout = reinterpret_cast<uint4*>(buf);
  uint4* dlb = reinterpret_cast<uint4*>(buf + 16);
  TraceStep* dsteps = reinterpret_cast<TraceStep*>(buf + 64);
  uint32_t* dn = reinterpret_cast<uint32_t*>(buf + 64 + kMaxTraceSteps * sizeof(TraceStep));
  if (!rc) {
    std::lock_guard<std::mutex> g(ctx->data);
    const DevEpoch& cur = ctx->dev[0].cur;
    if (!cur.base) {
      rc = -GPC_EINVAL;  // nothing committed yet
    } else {
      EpochArgs ep{cur.base->d_hdr, cur.base->d_blob, cur.jhdr ? cur.pool->d_blob : nullptr, cur.jhdr,
                   cur.svc ? cur.svc->d_blob : nullptr, 0u, {0, 0}, 0u, 0u};
      rc = launch_trace(ep, d, dout, dlb, dsteps, dn, nullptr);
      if (!rc) rc = hip_ok(hipDeviceSynchronize());  // the epoch stays alive while it is current
    }
  }
  if (!rc) rc = hip_ok(hipMemcpy(h.data(), buf, kOut, hipMemcpyDeviceToHost));
  (void)hipFree(buf);
  if (rc) return rc;
  std::memcpy(out, h.data(), 2 * sizeof(gpc_verdict));
  if (lb_out) std::memcpy(lb_out, h.data() + 16, sizeof(gpc_lb_result));
  uint32_t n = 0;
  std::memcpy(&n, h.data() + 64 + kMaxTraceSteps * sizeof(TraceStep), 4);
  if (n_steps) *n_steps = n;
  if (steps) std::memcpy(steps, h.data() + 64, std::min<size_t>(n, cap) * sizeof(TraceStep));
  return n > cap && steps ? -GPC_ERANGE : GPC_OK;
}

int gpc_classify_host(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, int32_t count) {
  return gpc_classify_host_lb(ctx, pk, n, out, nullptr, count);
}

int gpc_classify6(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, int32_t count, void* stream) {
  return gpc_classify6_on(ctx, 0, pk, n, out, count, stream);
}

int gpc_classify6_on(gpc_ctx* ctx, uint32_t slot, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, int32_t count,
                     void* stream) {
  if (!ctx || !pk || (!out && n) || n > GPC_MAX_BATCH || slot >= ctx->dev.size()) return -GPC_EINVAL;
  if (n && (!pk->src6 || !pk->dst6 || !pk->sport || !pk->dport || !pk->proto || !pk->out_port)) return -GPC_EINVAL;
  for (const void* c : {(const void*)pk->src6, (const void*)pk->dst6, (const void*)pk->ct_src6, (const void*)pk->ct_dst6})
    if (reinterpret_cast<uintptr_t>(c) % 16) return -GPC_EINVAL;  // one 128-bit load per address
  if (hip_ok(hipSetDevice(ctx->dev[slot].device))) return -GPC_EDEV;
  Pace pace(ctx, slot, (hipStream_t)stream, n != 0);
  const auto d = launch_lock(ctx->data, ctx->publishers);
  DevState& D = ctx->dev[slot];
  if (!D.cur.v6) return -GPC_EINVAL;  // IPv6 disabled or nothing committed yet
  EpochArgs ep{D.cur.v6->d_hdr, D.cur.v6->d_blob, D.cur.v6_jhdr ? D.cur.v6_pool->d_blob : nullptr, D.cur.v6_jhdr,
               nullptr, D.cur.v6_lpm, {0, 0}, uint32_t(D.counter_cap * kCounterWords), D.counter_copies - 1};
  hipStream_t st = (hipStream_t)stream;
  // per-stream scratch: the code columns of the batch (v6_code_kernel), then, for a grouped batch,
  // the grouping scratch of the IPv4-shaped batch over those columns (address key: the top byte of
  // the source code, i.e. the batch's source prefixes in tree order)
  GroupArgs ga{nullptr, GPC_GROUP_KEY_ADDR, 0u, 8u, ctx->group_xcd, ctx->group_unpermute, 0u};
  const size_t code_bytes = (size_t(v6_code_columns(*pk)) * n * 4 + 255) & ~size_t(255);
  gpc_pkt_soa shape = *pk;  // which columns the code batch has (group_scratch_bytes reads presence only)
  shape.src = shape.dst = reinterpret_cast<const uint32_t*>(pk->src6);
  shape.ct_src = pk->ct_src6 ? shape.src : nullptr;
  shape.ct_dst = pk->ct_dst6 ? shape.src : nullptr;
  uint8_t* scratch = nullptr;
  if (n && ctx->group_v6 && group_batch(ctx, n, *D.cur.v6, D.cur.v6_jhdr != 0)) {
    if (const int e = group_scratch_for(ctx, D, st, code_bytes + group_scratch_bytes(shape, n, false), &scratch)) return e;
    if (scratch) ga.scratch = scratch + code_bytes;
  }
  if (n && !scratch)
    if (const int e = group_scratch(D, st, code_bytes, &scratch)) return e;
  int rc = launch_classify6(ep, *pk, n, out, D.d_counters, count, ga.scratch ? &ga : nullptr,
                            reinterpret_cast<uint32_t*>(scratch), st, n ? next_marks(D) : nullptr);
  if (!rc && scratch) rc = group_scratch_used(D, st);
  if (rc || n == 0) return rc;
  pace.record();
  return note_launch(ctx, D, st);
}

int gpc_classify6_host(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, int32_t count) {
  if (!ctx || !pk || (!out && n)) return -GPC_EINVAL;
  if (hip_ok(hipSetDevice(ctx->dev[0].device))) return -GPC_EDEV;
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
  up(pk->src6, 16, (const void**)&d.src6);
  up(pk->dst6, 16, (const void**)&d.dst6);
  up(pk->ct_src6, 16, (const void**)&d.ct_src6);
  up(pk->ct_dst6, 16, (const void**)&d.ct_dst6);
  up(pk->sport, 2, (const void**)&d.sport);
  up(pk->dport, 2, (const void**)&d.dport);
  up(pk->proto, 1, (const void**)&d.proto);
  up(pk->out_port, 4, (const void**)&d.out_port);
  up(pk->in_port, 4, (const void**)&d.in_port);
  up(pk->svc_group, 4, (const void**)&d.svc_group);
  up(pk->tun_id, 4, (const void**)&d.tun_id);
  up(pk->ct_state, 1, (const void**)&d.ct_state);
  up(pk->dest, 1, (const void**)&d.dest);
  up(pk->len, 2, (const void**)&d.len);
  up(pk->ct_mark, 1, (const void**)&d.ct_mark);
  void* dout = nullptr;
  if (!rc && hip_ok(hipMalloc(&dout, n * 2 * sizeof(gpc_verdict)))) rc = -GPC_EDEV;
  if (!rc) rc = gpc_classify6(ctx, &d, n, (gpc_verdict*)dout, count, nullptr);
  if (!rc && hip_ok(hipDeviceSynchronize())) rc = -GPC_EDEV;
  if (!rc && hip_ok(hipMemcpy(out, dout, n * 2 * sizeof(gpc_verdict), hipMemcpyDeviceToHost))) rc = -GPC_EDEV;
  if (dout) (void)hipFree(dout);
  for (void* p : allocs) (void)hipFree(p);
  return rc;
}

int gpc_classify_host_lb(gpc_ctx* ctx, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out, gpc_lb_result* lb_out,
                         int32_t count) {
  return gpc_classify_host_on(ctx, 0, pk, n, out, lb_out, count);
}

int gpc_classify_host_on(gpc_ctx* ctx, uint32_t slot, const gpc_pkt_soa* pk, size_t n, gpc_verdict* out,
                         gpc_lb_result* lb_out, int32_t count) {
  if (!ctx || !pk || (!out && n) || slot >= ctx->dev.size()) return -GPC_EINVAL;
  if (hip_ok(hipSetDevice(ctx->dev[slot].device))) return -GPC_EDEV;
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
  up(pk->ct_mark, 1, (const void**)&d.ct_mark);
  void* dout = nullptr;
  void* dlb = nullptr;
  if (!rc && hip_ok(hipMalloc(&dout, n * 2 * sizeof(gpc_verdict)))) rc = -GPC_EDEV;
  if (!rc && lb_out && hip_ok(hipMalloc(&dlb, n * sizeof(gpc_lb_result)))) rc = -GPC_EDEV;
  if (!rc) rc = gpc_classify_on(ctx, slot, &d, n, (gpc_verdict*)dout, (gpc_lb_result*)dlb, count, nullptr);
  if (!rc && hip_ok(hipDeviceSynchronize())) rc = -GPC_EDEV;
  if (!rc && hip_ok(hipMemcpy(out, dout, n * 2 * sizeof(gpc_verdict), hipMemcpyDeviceToHost))) rc = -GPC_EDEV;
  if (!rc && lb_out && hip_ok(hipMemcpy(lb_out, dlb, n * sizeof(gpc_lb_result), hipMemcpyDeviceToHost))) rc = -GPC_EDEV;
  if (dout) (void)hipFree(dout);
  if (dlb) (void)hipFree(dlb);
  for (void* p : allocs) (void)hipFree(p);
  return rc;
}

int gpc_counters(gpc_ctx* ctx, uint64_t** dev, const uint32_t** slot_conj, size_t* n_slots) {
  return gpc_counters_on(ctx, 0, dev, slot_conj, n_slots);
}

int gpc_counters_on(gpc_ctx* ctx, uint32_t slot, uint64_t** dev, const uint32_t** slot_conj, size_t* n_slots) {
  if (!ctx || slot >= ctx->dev.size()) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  DevState& D = ctx->dev[slot];
  if (int rc = fold_counters(D)) return rc;  // the caller sees one array (the published one)
  if (dev) *dev = reinterpret_cast<uint64_t*>(published_counters(D));
  if (slot_conj) *slot_conj = ctx->slot_conj.data();
  if (n_slots) *n_slots = ctx->slot_conj.size();
  return GPC_OK;
}

int gpc_reset_counters(gpc_ctx* ctx) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  for (DevState& D : ctx->dev) {
    if (!D.d_counters) continue;
    if (hip_ok(hipSetDevice(D.device))) return -GPC_EDEV;
    if (hip_ok(hipDeviceSynchronize()) || hip_ok(hipMemset(D.d_counters, 0, D.counter_cap * kCounterBytes * (D.counter_copies + 1))))
      return -GPC_EDEV;
  }
  return GPC_OK;
}

// NetworkPolicyMetrics over every device slot of the context: each slot's counters are folded,
// copied back and summed per rule (the in-process counterpart of the RCCL all-reduce).
int gpc_metrics(gpc_ctx* ctx, gpc_rule_metric* out, size_t cap, size_t* n) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  std::vector<unsigned long long> h(ctx->slot_conj.size() * kCounterWords, 0), part(h.size());
  for (DevState& D : ctx->dev) {
    if (int rc = fold_counters(D)) return rc;
    if (!D.d_counters || h.empty()) continue;
    if (hip_ok(hipSetDevice(D.device)) || hip_ok(hipDeviceSynchronize()) ||
        hip_ok(hipMemcpy(part.data(), published_counters(D), part.size() * 8, hipMemcpyDeviceToHost)))
      return -GPC_EDEV;
    for (size_t i = 0; i < h.size(); i++) h[i] += part[i];
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
  const DevEpoch& cur = ctx->dev[0].cur;
  out->device_bytes = cur.base ? cur.base->bytes : 0;
  out->overlay_bytes = ctx->journal.active() ? ctx->journal.pool.size() * 4 : 0;
  out->n_overlay_rules = ctx->journal.n_live;
  out->n_tombstones = ctx->journal.n_tombstones();
  out->n_full_builds = ctx->n_full;
  out->n_delta_builds = ctx->n_delta;
  out->n_background_builds = ctx->n_bg;
  out->v6_full_builds = ctx->n_full6;
  out->v6_delta_builds = ctx->n_delta6;
  out->v6_overlay_rules = ctx->journal6.n_live;
  out->v6_prefixes = ctx->last6.v6_prefixes;
  out->n_ext_rules = ctx->journal.n_ext_rules();
  out->n_ext_values = ctx->journal.n_ext_values();
  out->n_pool_collections = ctx->n_pool_gc;
  if (cur.base) {
    out->group_key = group_key(ctx);
    out->lane_sort = cur.base->sort_table[0] | uint32_t(cur.base->sort_table[1]) << 8;
  }
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

int gpc_debug_image6(gpc_ctx* ctx, const uint32_t** blob, size_t* n_words, const void** hdr, size_t* hdr_bytes) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  const bool has = !ctx->last6.blob.empty();
  if (blob) *blob = has ? ctx->last6.blob.data() : nullptr;
  if (n_words) *n_words = ctx->last6.blob.size();
  if (hdr) *hdr = has ? &ctx->last6.hdr : nullptr;
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

int gpc_set_launch_timing(gpc_ctx* ctx, uint32_t slots) {
  if (!ctx || slots > 4096) return -GPC_EINVAL;
  std::lock_guard<std::mutex> d(ctx->data);
  for (DevState& D : ctx->dev) {
    if (hip_ok(hipSetDevice(D.device))) return -GPC_EDEV;
    (void)hipDeviceSynchronize();  // no recorded event is still pending when its set is destroyed
    free_marks(D);
    D.marks.resize(slots);
    for (auto& m : D.marks) {
      m.n = 0;
      for (auto& e : m.ev)
        if (hip_ok(hipEventCreate(&e))) {
          free_marks(D);
          return -GPC_EDEV;
        }
    }
  }
  return GPC_OK;
}

int gpc_launch_times(gpc_ctx* ctx, gpc_launch_time* out, size_t cap, size_t* n) {
  if (!ctx || !n || (!out && cap)) return -GPC_EINVAL;
  static const char* const names[kLaunchKinds] = {"group_tiles", "classify_egress", "classify_ingress", "classify_both",
                                                  "unpermute",   "v6_codes"};
  double ms[kLaunchKinds] = {};
  uint32_t cnt[kLaunchKinds] = {};
  size_t dropped = 0;
  {
    std::lock_guard<std::mutex> d(ctx->data);
    for (DevState& D : ctx->dev) {
      const size_t S = D.marks.size();
      if (S && hip_ok(hipSetDevice(D.device))) return -GPC_EDEV;
      for (size_t k = 0; k < D.marks_used; k++) {  // oldest first
        LaunchMarks& m = D.marks[(D.marks_next + S - D.marks_used + k) % S];
        if (m.n < 2 || hip_ok(hipEventSynchronize(m.ev[m.n - 1]))) continue;
        for (int i = 0; i + 1 < m.n; i++) {
          float t = 0.f;
          if (m.kind[i] < kLaunchKinds && !hip_ok(hipEventElapsedTime(&t, m.ev[i], m.ev[i + 1]))) {
            ms[m.kind[i]] += t;
            cnt[m.kind[i]]++;
          }
        }
      }
      dropped += D.marks_dropped;
      D.marks_used = D.marks_dropped = 0;
    }
  }
  size_t k = 0;
  for (int i = 0; i < kLaunchKinds; i++) {
    if (!cnt[i]) continue;
    if (k < cap) {
      std::memset(&out[k], 0, sizeof(gpc_launch_time));
      std::strncpy(out[k].kernel, names[i], sizeof(out[k].kernel) - 1);
      out[k].launches = cnt[i];
      out[k].dropped = uint32_t(dropped);
      out[k].total_ms = ms[i];
    }
    k++;
  }
  *n = k;
  return k > cap ? -GPC_ERANGE : GPC_OK;
}

int gpc_stream_epoch(gpc_ctx* ctx, void* stream, uint64_t* epoch) {
  if (!ctx || !epoch) return -GPC_EINVAL;
  std::lock_guard<std::mutex> d(ctx->data);
  for (DevState& D : ctx->dev) {
    auto it = D.launch_epoch.find(stream_key((hipStream_t)stream));
    if (it != D.launch_epoch.end()) {
      *epoch = it->second;
      return GPC_OK;
    }
  }
  return -GPC_ENOTFOUND;
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

int gpc_debug_epoch6(gpc_ctx* ctx, const uint32_t** pool, size_t* pool_words, uint32_t* jhdr) {
  if (!ctx) return -GPC_EINVAL;
  std::lock_guard<std::mutex> g(ctx->ctl);
  const bool has = ctx->journal6.active();
  if (pool) *pool = has ? ctx->journal6.pool.data() : nullptr;
  if (pool_words) *pool_words = has ? ctx->journal6.pool.size() : 0;
  if (jhdr) *jhdr = has ? ctx->journal6.hdr_off : 0;
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
  using clk = std::chrono::steady_clock;
  const clk::time_point tc0 = clk::now();
  // counter slots of the rules with Metric flows, allocated here in conj-id order before the commit
  // is logged: the compactor (which replays up to a commit marker) then only looks them up
  for (uint32_t conj : dirty.conj) {
    auto it = ctx->np.policies().find(conj);
    uint32_t slot;
    if (it != ctx->np.policies().end() && !it->second->metric_flows.empty()) (void)ctx->slots.lookup(conj, true, &slot);
  }
  const uint64_t commit_no = ++ctx->commit_no;
  {
    Op m;
    m.kind = Op::COMMIT;
    m.commit_no = commit_no;
    log_op(ctx, std::move(m));
  }
  // a background compaction result: install it, then append what changed after its commit
  bool installed = false;
  std::vector<std::shared_ptr<DevImage>> bg_base, bg_pool;  // per device slot
  size_t bg_uploaded = 0;
  {
    std::unique_lock<std::mutex> lk(ctx->comp.mu);
    if (ctx->comp.ready) {
      ctx->comp.ready = false;
      ctx->comp_pending = false;
      const bool discard = ctx->comp.discard;
      ctx->comp.discard = false;
      if (ctx->comp.rc == GPC_OK && !force_full && !ctx->np.foreign() && !discard) {
        ctx->last = std::move(*ctx->comp.base);
        ctx->gen4++;
        ctx->journal = std::move(*ctx->comp.journal);
        ctx->journal.set_base(&ctx->last);
        bg_base = std::move(ctx->comp.dbase);
        bg_pool = std::move(ctx->comp.dpool);
        bg_uploaded = ctx->comp.uploaded;
        for (auto& h : ctx->dirty_hist)
          if (h.first > ctx->comp.at_commit) {
            dirty.conj.insert(h.second.conj.begin(), h.second.conj.end());
            dirty.hard_tables |= h.second.hard_tables;
          }
        installed = true;
        ctx->n_bg++;
      }
      ctx->comp.base.reset();
      ctx->comp.journal.reset();
      ctx->comp.dbase.clear();
      ctx->comp.dpool.clear();
      ctx->dirty_hist.clear();
    }
  }
  if (ctx->comp_pending) ctx->dirty_hist.push_back({commit_no, dirty});
  const bool have_base = !ctx->last.blob.empty();
  const bool classifier_changed = (dirty.hard_tables & FeatureNP::kDirtyClassifier) != 0;
  dirty.hard_tables &= uint8_t(~FeatureNP::kDirtyClassifier);
  // Journal size bound: past it the next epoch is a full rebuild. While a background compaction is
  // in flight the journal takes up to every rule of the base instead: a synchronous rebuild here
  // would stall the control thread for a whole image build (C5 at 10 000 ops/s: commit p99 3.5 s,
  // 6 blocking rebuilds in 70 s) and discard the compaction it overtakes.
  // The allowance is a bounded multiple of the normal cap (a slow or failing compaction
  // must not leave the data path walking a base-sized journal).
  const size_t normal_cap = std::max(kDeltaMinRules, ctx->last.conj_rid.size() / kDeltaFraction);
  const size_t live_cap = ctx->comp_pending ? kPendingCapFactor * normal_cap : normal_cap;
  bool full = force_full || !have_base || classifier_changed || ctx->last.any_noact || ctx->np.foreign() || ctx->journal.any_noact ||
              ctx->journal.n_live > live_cap || ctx->journal.pool.size() > kPoolWords * 7 / 8;
  int rc = GPC_OK;
  bool pool_gc = false;
  try {
    if (!full && (!dirty.conj.empty() || dirty.hard_tables)) {
      std::string err;
      if (ctx->journal.apply(ctx->np, ctx->slots, dirty.conj, dirty.hard_tables, &err) != GPC_OK ||
          ctx->journal.pool.size() > kPoolWords)
        full = true;  // a shape the journal does not take (or it is full): rebuild everything
    }
    // Pool garbage collection: the journal's state again in a fresh pool once the old one holds
    // mostly superseded data -- extension indexes of earlier epochs (each epoch that moves an
    // extension appends one), dead journal versions (still walked by the chains that list them).
    // Cost ~ the rules touched since the base (C5 mixed: ~8 k); the alternative, a compaction, is
    // a whole image build (seconds) plus a base upload.
    if (!full && !installed && ctx->journal.active() && !std::getenv("GPC_NO_POOL_GC") &&
        (ctx->journal.pool.size() > kPoolGcWords ||
         ctx->journal.n_dead_versions() > std::max<size_t>(env_u32("GPC_GC_DEAD_MIN", kGcDeadMin, 1, 1u << 30),
                                                           2 * size_t(ctx->journal.n_live)))) {
      std::string err;
      const size_t was = ctx->journal.pool.size();
      const clk::time_point tg = clk::now();
      if (ctx->journal.rebuild(ctx->np, ctx->slots, &err) == GPC_OK) {
        pool_gc = true;
        ctx->n_pool_gc++;
        if (std::getenv("GPC_COMPACT_DEBUG"))
          std::fprintf(stderr, "commit %llu: pool collection %.1f -> %.1f MB in %.1f ms (%zu live rules, %u extended)\n",
                       (unsigned long long)commit_no, was * 4e-6, ctx->journal.pool.size() * 4e-6,
                       std::chrono::duration<double, std::milli>(clk::now() - tg).count(), ctx->journal.n_live,
                       ctx->journal.n_ext_rules());
      } else {
        full = true;
      }
    }
    if (full) {
      if (std::getenv("GPC_COMPACT_DEBUG"))
        std::fprintf(stderr, "commit %llu: full build (journal %zu live rules, %zu words, compaction %s)\n",
                     (unsigned long long)commit_no, ctx->journal.n_live, ctx->journal.pool.size(),
                     ctx->comp_pending ? "pending" : "idle");
      HostImage img;
      rc = build_image(ctx->np, ctx->slots, &img);
      if (rc) return rc;
      ctx->last = std::move(img);
      ctx->gen4++;
      ctx->journal.reset(&ctx->last);
      installed = false;
    }
  } catch (...) {
    return -GPC_ENOMEM;
  }
  // ask the compactor for a new base once the journal is large; commits continue meanwhile
  const int32_t ca = ctx->cfg.compact_after;
  // (default: max(512, base rules / 128) -- C3: 781; every live journal rule adds to the walk of the
  // packets its keys reach, and the pool collections keep everything else small)
  const size_t soft = ca > 0 ? size_t(ca) : std::max<size_t>(512, ctx->last.conj_rid.size() / 128);
  // (or once many point extensions are live, or the pool is a quarter full: epochs that only move
  // extensions append an index each, and the compactor folds them into a new base)
  // Live point extensions are held across the compaction (Compactor::hold) unless they are many
  // (kExtCompactValues), so they do not ask for one; their per-epoch index does, through the pool.
  const bool hold_ext = !std::getenv("GPC_COMPACT_FOLD_EXT") && ctx->journal.n_ext_values() <= kExtCompactValues;
  if (!full && ca >= 0 && !ctx->comp_pending &&
      (ctx->journal.n_live + (hold_ext ? 0u : ctx->journal.n_ext_rules()) > soft ||
       ctx->journal.n_ext_values() > kExtCompactValues || ctx->journal.pool.size() > kPoolGcWords)) {
    {
      std::lock_guard<std::mutex> c(ctx->comp.mu);
      if (ctx->comp.enabled && !ctx->comp.busy && !ctx->comp.ready) {
        ctx->comp.want_commit = commit_no;
        ctx->comp.hold = hold_ext ? ctx->journal.held_extensions() : HeldExts();
        ctx->comp_pending = true;
        ctx->dirty_hist.clear();
      }
    }
    ctx->comp.cv.notify_one();
  }
  // IPv6: a delta epoch over the IPv6 base (new prefixes interned in place, changed rules appended
  // to journal6) when possible, else a full rebuild. v6_full: a new base; v6_changed: a new epoch.
  bool v6_changed = false, v6_full = false;
  const bool rules_changed = !dirty.conj.empty() || dirty.hard_tables || classifier_changed;
  if (ctx->cfg.ipv6_enabled && (rules_changed || force_full || ctx->last6.blob.empty())) {
    Journal& j6 = ctx->journal6;
    v6_full = force_full || classifier_changed || ctx->np.foreign() || ctx->last6.blob.empty() || !ctx->last6.codes6 ||
              j6.any_noact || j6.n_live > std::max(kDeltaMinRules, ctx->last6.conj_rid.size() / kDeltaFraction) ||
              j6.pool.size() > kPoolWords * 7 / 8 ||
              // every epoch that interns a prefix re-emits the whole overflow table
              ctx->last6.v6_ovf.size() > std::max<size_t>(4096, size_t(ctx->last6.v6_prefixes) / 8);
    if (!v6_full) {
      std::string err;
      try {
        if (extend_image6(ctx->np, dirty.conj, dirty.hard_tables, &ctx->last6, &j6) != GPC_OK) err = "prefix not internable";
        else if (j6.apply(ctx->np, ctx->slots, dirty.conj, dirty.hard_tables, &err) != GPC_OK || j6.pool.size() > kPoolWords)
          err = err.empty() ? "journal full" : err;
      } catch (...) {
        err = "out of memory";
      }
      v6_full = !err.empty();
      if (v6_full && std::getenv("GPC_IMAGE_DEBUG")) std::fprintf(stderr, "IPv6 delta -> full build: %s\n", err.c_str());
    }
    if (v6_full) {  // an IPv6 rule set the image cannot take leaves IPv6 unpublished, not IPv4
      HostImage img6;
      int r6;
      try {
        r6 = build_image6(ctx->np, ctx->slots, &img6);
      } catch (...) {
        r6 = -GPC_ENOMEM;
      }
      if (r6) {
        std::string e = img6.error.empty() ? "IPv6 image build failed" : img6.error;
        img6 = HostImage();
        img6.error = e;
      }
      ctx->last6 = std::move(img6);
      ctx->gen6++;
      j6.reset(&ctx->last6);
      ctx->n_full6++;
    } else {
      ctx->n_delta6++;
    }
    v6_changed = true;
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
  // The new epoch goes to every device slot: uploads on each slot's stream, one synchronize per
  // slot, then all slots publish it under one data lock (no launch sees two epochs across slots).
  const size_t nd = ctx->dev.size();
  const clk::time_point tc1 = clk::now();
  std::vector<DevEpoch> ne(nd);
  std::vector<unsigned long long*> nc(nd, nullptr);
  std::vector<size_t> new_cap(nd, 0);
  std::vector<uint32_t> new_copies(nd, 1);
  auto fail = [&](int r) {  // releases what this commit allocated on every slot
    for (size_t k = 0; k < nd; k++) {
      (void)hipSetDevice(ctx->dev[k].device);
      if (ctx->dev[k].ustream) (void)hipStreamSynchronize(ctx->dev[k].ustream);
      RetiredEpoch{std::move(ne[k])}.release(ctx->dev[k].ustream);
      if (nc[k] && nc[k] != ctx->dev[k].d_counters) (void)hipFree(nc[k]);
    }
    return r;
  };
  const bool bg_ok = installed && bg_base.size() == nd && bg_pool.size() == nd;
  Journal& jn = ctx->journal;
  bool new_pool = false;
  bool resync4 = false;  // some slot holds a base of an older host generation: every slot re-uploads
  for (size_t k = 0; k < nd; k++) resync4 |= ctx->dev[k].cur.base && ctx->dev[k].cur.base_gen != ctx->gen4;
  for (size_t k = 0; k < nd; k++) {
    DevState& D = ctx->dev[k];
    if (hip_ok(hipSetDevice(D.device))) return fail(-GPC_EDEV);
    if (!D.ustream && hip_ok(hipStreamCreateWithFlags(&D.ustream, hipStreamNonBlocking))) return fail(-GPC_EDEV);
    hipStream_t us = D.ustream;
    collect_retired(D, false);
    if (bg_ok && bg_base[k] && bg_pool[k]) {  // uploaded by the compactor
      bg_base[k]->s = us;
      bg_pool[k]->s = us;
      ne[k].base = std::move(bg_base[k]);
      ne[k].pool = std::move(bg_pool[k]);
    } else if (full || installed || resync4 || !D.cur.base) {
      if ((rc = upload_image(ctx->last, D.device, us, &ne[k].base, &ctx->fail_uploads))) return fail(rc);
    } else {
      ne[k].base = D.cur.base;
      ne[k].pool = pool_gc ? nullptr : D.cur.pool;  // (a collected pool: a fresh one, uploaded whole)
    }
    ne[k].base_gen = ctx->gen4;
    if (jn.active() && !ne[k].pool) {  // the journal pool of a new base is allocated on first use
      if ((rc = alloc_pool(D.device, us, &ne[k].pool))) return fail(rc);
      new_pool = true;
    }
  }
  if (bg_ok) jn.uploaded = bg_uploaded;
  else if (full || installed || resync4 || !ctx->dev[0].cur.base) jn.uploaded = 0;
  if (new_pool) jn.uploaded = 0;
  // Append-only: only the new journal tail travels, staged once in a pinned buffer and padded to at
  // least kMinUploadBytes (the padding lands in not-yet-used pool space) so the runtime takes the
  // DMA path; a small copy may otherwise run as a blit kernel queued behind in-flight classification.
  const bool tail = jn.active() && jn.pool.size() > jn.uploaded;
  size_t tail_bytes = 0, copy_bytes = 0;
  if (tail) {
    tail_bytes = (jn.pool.size() - jn.uploaded) * 4;
    copy_bytes = std::min(std::max(tail_bytes, kMinUploadBytes), kPoolWords * 4 - jn.uploaded * 4);
    if (ctx->stage_bytes < copy_bytes) {
      // grown geometrically: hipHostFree waits for the device to drain, so a staging buffer
      // reallocated for every slightly larger tail stalled commits behind the classification queue
      // (C5 mixed: 260-340 ms per commit with 6-7 MB tails)
      if (ctx->stage) (void)hipHostFree(ctx->stage);
      ctx->stage = nullptr;
      ctx->stage_bytes = 0;
      const size_t cap = std::max(2 * copy_bytes, size_t(16) << 20);
      if (hip_ok(hipHostMalloc(&ctx->stage, cap, hipHostMallocPortable))) return fail(-GPC_EDEV);
      ctx->stage_bytes = cap;
    }
    std::memcpy(ctx->stage, jn.pool.data() + jn.uploaded, tail_bytes);
  }
  // the first delta commit after a full build would otherwise allocate the pinned staging buffer
  // (hipHostMalloc of 16 MB: ~0.3 s on the box, which every op queued behind it waited for: C5
  // op-latency p99 302 ms); allocated with the full build instead, outside the churn
  if (!tail && full && !ctx->stage && !std::getenv("GPC_LAZY_STAGE")) {
    const size_t cap = size_t(16) << 20;
    if (!hip_ok(hipHostMalloc(&ctx->stage, cap, hipHostMallocPortable))) ctx->stage_bytes = cap;
    else ctx->stage = nullptr;
  }
  const uint32_t jhdr = jn.active() ? jn.hdr_off : 0;
  // the IPv6 journal tail (delta epochs), staged the same way; a new pool on every slot when the
  // IPv6 base is new or its journal starts (lockstep: every slot has the same IPv6 base)
  Journal& j6 = ctx->journal6;
  // a slot whose IPv6 base is missing or of an older host generation gets the base and the whole
  // IPv6 journal again (a full IPv6 rebuild whose upload failed must not be extended)
  bool resync6 = false;
  if (ctx->cfg.ipv6_enabled && !v6_full && !ctx->last6.blob.empty())
    for (size_t k = 0; k < nd; k++) resync6 |= !ctx->dev[k].cur.v6 || ctx->dev[k].cur.v6_gen != ctx->gen6;
  if (resync6) v6_changed = true;
  const bool j6_active = v6_changed && !v6_full && j6.active();
  if (j6_active && (resync6 || !ctx->dev[0].cur.v6_pool)) j6.uploaded = 0;
  const size_t j6_from = j6.uploaded;
  const bool tail6 = j6_active && j6.pool.size() > j6.uploaded;
  size_t copy6_bytes = 0;
  if (tail6) {
    const size_t t6 = (j6.pool.size() - j6.uploaded) * 4;
    copy6_bytes = std::min(std::max(t6, kMinUploadBytes), kPoolWords * 4 - j6.uploaded * 4);
    if (ctx->stage6_bytes < copy6_bytes) {
      if (ctx->stage6) (void)hipHostFree(ctx->stage6);
      ctx->stage6 = nullptr;
      ctx->stage6_bytes = 0;
      const size_t cap = std::max(2 * copy6_bytes, size_t(16) << 20);
      if (hip_ok(hipHostMalloc(&ctx->stage6, cap, hipHostMallocPortable))) return fail(-GPC_EDEV);
      ctx->stage6_bytes = cap;
    }
    std::memcpy(ctx->stage6, j6.pool.data() + j6.uploaded, t6);
  }
  const uint64_t epoch = ctx->epoch + 1;
  const size_t need = ctx->slots.size() ? ctx->slots.size() : 1;
  for (size_t k = 0; k < nd; k++) {
    DevState& D = ctx->dev[k];
    hipStream_t us = D.ustream;
    if (hip_ok(hipSetDevice(D.device))) return fail(-GPC_EDEV);
    if (tail && hip_ok(hipMemcpyAsync(ne[k].pool->d_blob + jn.uploaded, ctx->stage, copy_bytes, hipMemcpyHostToDevice, us)))
      return fail(-GPC_EDEV);
    ne[k].jhdr = jhdr;
    ne[k].jmode = jhdr ? jn.mode() : kModeBase;
    if (resync6) {  // the current host IPv6 base, then the whole journal into a fresh pool
      if ((rc = upload_image(ctx->last6, D.device, us, &ne[k].v6, &ctx->fail_uploads))) return fail(rc);
      ne[k].v6_lpm = ctx->last6.hdr.v6_lpm;
      if (j6_active) {
        if ((rc = alloc_pool(D.device, us, &ne[k].v6_pool))) return fail(rc);
        if (tail6 && hip_ok(hipMemcpyAsync(ne[k].v6_pool->d_blob, ctx->stage6, copy6_bytes, hipMemcpyHostToDevice, us)))
          return fail(-GPC_EDEV);
        ne[k].v6_jhdr = ctx->journal6.hdr_off;
      }
      ne[k].v6_gen = ctx->gen6;
    } else if (!v6_full) {  // the IPv6 base stays; a delta extends its journal (new prefixes' LPM entries included)
      ne[k].v6 = D.cur.v6;
      ne[k].v6_lpm = D.cur.v6_lpm;
      ne[k].v6_pool = D.cur.v6_pool;
      ne[k].v6_jhdr = D.cur.v6_jhdr;
      ne[k].v6_gen = D.cur.v6_gen;
      if (v6_changed && ne[k].v6) {
        if (j6_active && !ne[k].v6_pool) {
          if ((rc = alloc_pool(D.device, us, &ne[k].v6_pool))) return fail(rc);
        }
        if (tail6 && hip_ok(hipMemcpyAsync(ne[k].v6_pool->d_blob + j6_from, ctx->stage6, copy6_bytes,
                                           hipMemcpyHostToDevice, us)))
          return fail(-GPC_EDEV);
        ne[k].v6_jhdr = j6_active ? ctx->journal6.hdr_off : 0u;
      }
    } else if (!ctx->last6.blob.empty()) {
      if ((rc = upload_image(ctx->last6, D.device, us, &ne[k].v6, &ctx->fail_uploads))) return fail(rc);
      ne[k].v6_lpm = ctx->last6.hdr.v6_lpm;
      ne[k].v6_gen = ctx->gen6;
    }
    if (!svc_changed) ne[k].svc = D.cur.svc;
    else if (!ctx->svc_blob.empty() && (rc = upload_words(ctx->svc_blob, D.device, us, &ne[k].svc))) return fail(rc);
    ne[k].epoch = epoch;
    // counters: grow to the slot count, zero released slots (their Metric flows were deleted)
    nc[k] = D.d_counters;
    new_cap[k] = D.counter_cap;
    new_copies[k] = D.counter_copies;
    if (need > D.counter_cap) {
      new_cap[k] = std::max(need, D.counter_cap * 2);
      new_copies[k] = counter_copies_for(new_cap[k]);
      const size_t bytes = new_cap[k] * kCounterBytes * (new_copies[k] + 1);
      nc[k] = nullptr;
      if (hip_ok(hipMalloc(&nc[k], bytes)) || hip_ok(hipMemset(nc[k], 0, bytes))) return fail(-GPC_EDEV);
    }
  }
  const clk::time_point tc2 = clk::now();
  for (size_t k = 0; k < nd; k++)  // the new epoch is resident on every slot before it is published
    if (hip_ok(hipSetDevice(ctx->dev[k].device)) || hip_ok(hipStreamSynchronize(ctx->dev[k].ustream)))
      return fail(-GPC_EDEV);
  const clk::time_point tc3 = clk::now();
  if (tail) jn.uploaded = jn.pool.size();
  if (tail6) j6.uploaded = j6.pool.size();
  ctx->epoch = epoch;
  std::vector<DevEpoch> old(nd);
  std::vector<unsigned long long*> old_counters(nd, nullptr);
  std::vector<size_t> old_cap(nd);
  std::vector<uint32_t> old_copies(nd);
  clk::time_point tc3b;
  {
    PublishLock d(ctx->data, ctx->publishers);
    tc3b = clk::now();
    for (size_t k = 0; k < nd; k++) {
      DevState& D = ctx->dev[k];
      old[k] = std::move(D.cur);
      D.cur = std::move(ne[k]);
      old_cap[k] = D.counter_cap;
      old_copies[k] = D.counter_copies;
      if (nc[k] != D.d_counters) {
        old_counters[k] = D.d_counters;
        D.d_counters = nc[k];
        D.counter_cap = new_cap[k];
        D.counter_copies = new_copies[k];
      }
    }
    ctx->cur_epoch = epoch;
  }
  for (size_t k = 0; k < nd; k++) {
    DevState& D = ctx->dev[k];
    (void)hipSetDevice(D.device);
    // the previous epoch is freed once every stream that launched on it has passed that launch
    D.retired.push_back(RetiredEpoch{std::move(old[k])});
    if (old_counters[k]) {
      // Every launch that could still add to the old array was queued before the swap: once the
      // device has drained them, all its replicas are merged into the new copy 0 (atomically: new
      // launches may already be adding to it), so no count is lost however the growth interleaves.
      (void)hipDeviceSynchronize();
      const uint64_t ow = uint64_t(old_cap[k]) * kCounterWords;
      (void)launch_merge_counters(D.d_counters, old_counters[k], ow, old_copies[k], ow, nullptr);
      (void)launch_merge_counters(published_counters(D), old_counters[k] + old_copies[k] * ow, ow, 1, ow, nullptr);
      (void)hipDeviceSynchronize();
      (void)hipFree(old_counters[k]);
    }
    for (uint32_t s : ctx->released_slots)
      if (s < D.counter_cap)
        for (uint32_t r = 0; r <= D.counter_copies; r++)  // (the published array too)
          (void)hipMemsetAsync(D.d_counters + kCounterWords * (size_t(r) * D.counter_cap + s), 0, kCounterBytes,
                               D.ustream);
  }
  ctx->released_slots.clear();
  if (std::getenv("GPC_COMPACT_DEBUG")) {
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const clk::time_point tc4 = clk::now();
    if (ms(tc0, tc4) > 50)
      std::fprintf(stderr,
                   "commit %llu: %.1f ms (host %.1f, upload enqueue %.1f, upload wait %.1f, data lock wait %.1f, publish %.1f; "
                   "tail %zu B, %s%s)\n",
                   (unsigned long long)commit_no, ms(tc0, tc4), ms(tc0, tc1), ms(tc1, tc2), ms(tc2, tc3), ms(tc3, tc3b),
                   ms(tc3b, tc4), tail_bytes, full ? "full" : installed ? "compacted base" : "delta",
                   old_counters[0] ? ", counters grew" : "");
  }
  return GPC_OK;
}
