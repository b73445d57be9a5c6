// Device image builder: realized OpenFlow flows -> core.hpp image (IPv4 packets).
//
// Flow classes handled (pipeline.go):
//   soft match flows  conjunction(id,k/n) actions       (conjunctiveMatchFlow :2019-2037)
//   conj action flows conj_id=id [+ ip/ipv6]           (:1718-1886) -> rule verdict, action priority
//   hard flows        drop / goto Metric                (defaultDropFlow :2040, MCNP :2068,
//                                                        skipPolicyRuleCheckFlows network_policy.go:2167)
//   metric flows      ct_label / reg3 counters          (:1604-1670) -> which rules are counted
#include "image.hpp"

#include <algorithm>
#include <cstring>
#include <random>

namespace gpc {

uint32_t SlotMap::get(uint32_t conj) {
  auto it = slot_.find(conj);
  if (it != slot_.end()) return it->second;
  uint32_t s;
  if (!free_.empty()) {
    s = free_.back();
    free_.pop_back();
    slot_conj_[s] = conj;
  } else {
    s = uint32_t(slot_conj_.size());
    slot_conj_.push_back(conj);
  }
  slot_[conj] = s;
  return s;
}

void SlotMap::release(uint32_t conj, std::vector<uint32_t>* freed) {
  auto it = slot_.find(conj);
  if (it == slot_.end()) return;
  free_.push_back(it->second);
  if (freed) freed->push_back(it->second);
  slot_conj_[it->second] = 0;
  slot_.erase(it);
}

namespace {

struct Term {
  uint8_t axis;
  uint32_t val, mask;
};
struct Atom {
  std::vector<Term> t;
};

struct RuleB {
  bool hard = false;
  uint32_t conj_id = 0;
  bool prio_set = false;
  uint16_t prio = 0;
  uint8_t n = 0;
  std::vector<Atom> clause[kMaxClauses];
  uint8_t verdict = RV_MISS;
  bool has_act = false;
  uint16_t act_prio = 0;
  bool counted = false;
  uint8_t tier = 0;
};

inline uint32_t prefix_mask(int plen) { return plen <= 0 ? 0u : plen >= 32 ? 0xffffffffu : ~((1u << (32 - plen)) - 1); }
inline bool is_prefix(uint32_t m) { return ((~m) & ((~m) + 1u)) == 0; }
inline int leading_ones(uint32_t m) {
  int n = 0;
  while (n < 32 && (m & (0x80000000u >> n))) n++;
  return n;
}

// Flow match -> atom over the IPv4 packet axes. Returns 0 ok, 1 never matches IPv4, -1 unsupported.
int atom_of(const Match& m, Atom* a) {
  a->t.clear();
  if (m.has_dl && m.dl_type != kEthIP) return 1;
  auto ip = [&](const IPMatch& f, uint8_t axis) -> int {
    if (!f.set) return 0;
    if (f.addr.fam != 4) return 1;
    int plen = f.plen < 0 ? 32 : f.plen;
    uint32_t mk = prefix_mask(plen);
    if (mk) a->t.push_back({axis, f.addr.v4() & mk, mk});
    return 0;
  };
  int r;
  if ((r = ip(m.nw_src, AX_SRC))) return r;
  if ((r = ip(m.nw_dst, AX_DST))) return r;
  if ((r = ip(m.ct_nw_src, AX_CTSRC))) return r;
  if ((r = ip(m.ct_nw_dst, AX_CTDST))) return r;
  for (int i = 0; i < 16; i++) {
    if (!(m.reg_present & (1u << i))) continue;
    uint8_t axis;
    if (i == 1) axis = AX_REG1;
    else if (i == 7) axis = AX_REG7;
    else return -1;
    if (m.reg_m[i]) a->t.push_back({axis, m.reg_v[i] & m.reg_m[i], m.reg_m[i]});
  }
  if (m.has_tun) {
    if (m.tun_id > 0xffffffffull) return 1;
    a->t.push_back({AX_TUN, uint32_t(m.tun_id), 0xffffffffu});
  }
  if (m.has_in_port) a->t.push_back({AX_INPORT, m.in_port, 0xffffffffu});
  if (m.has_ct_state && m.ct_mask) a->t.push_back({AX_CTST, uint32_t(m.ct_data & m.ct_mask), m.ct_mask});
  if (m.has_ct_label) return -1;
  if (m.has_proto) {
    uint32_t p = uint32_t(m.nw_proto) << 16;
    bool any = false;
    if (m.has_tp_dst) { a->t.push_back({AX_L4D, p | (m.tp_dst & m.tp_dst_m), 0xffff0000u | m.tp_dst_m}); any = true; }
    if (m.has_tp_src) { a->t.push_back({AX_L4S, p | (m.tp_src & m.tp_src_m), 0xffff0000u | m.tp_src_m}); any = true; }
    if (m.has_icmp_code) { a->t.push_back({AX_L4D, p | m.icmp_code, 0xffffffffu}); any = true; }
    if (m.has_icmp_type) { a->t.push_back({AX_L4S, p | m.icmp_type, 0xffffffffu}); any = true; }
    if (!any) a->t.push_back({AX_L4D, p, 0xffff0000u});
  } else if (m.has_tp_dst || m.has_tp_src || m.has_icmp_type || m.has_icmp_code) {
    return -1;
  }
  if (a->t.size() > 3) return -1;
  return 0;
}

uint8_t action_verdict(const Flow& f, bool* ok) {  // conj_id flows and hard flows
  *ok = true;
  bool deny = false, reject = false, ct = false, pass = false, metric = false, output = false;
  uint8_t table = f.table;
  uint8_t t2 = is_egress_table(table) ? TB_EGRESS : TB_INGRESS;
  uint8_t tm = is_egress_table(table) ? TB_EGRESS_METRIC : TB_INGRESS_METRIC;
  for (auto& a : f.acts) {
    switch (a.kind) {
      case ACT_SET_REG:
        if (a.a == 0 && (a.b & (a.has_mask ? a.c : 0xffffffffu) & 0x400)) deny = true;
        if (a.a == 0 && a.has_mask && a.c == 0xfe000000u && ((a.b >> 25) & 4)) reject = true;
        if (a.a == 0 && a.has_mask && a.c == 0x1800 && ((a.b >> 11) & 3) == 3) pass = true;
        break;
      case ACT_CT_COMMIT: ct = true; break;
      case ACT_GOTO:
        if (a.a == t2) pass = true;
        else if (a.a == tm) metric = true;
        else if (a.a == TB_OUTPUT) output = true;
        else *ok = false;
        break;
      case ACT_GROUP:
        if (a.a == t2) pass = true;
        else metric = true;  // logging / reject group resubmits to the metric table
        break;
      default: break;
    }
  }
  if (f.m.has_conj) {
    if (deny) return reject ? RV_REJECT : RV_DROP;
    if (ct) return RV_ALLOW;
    if (pass) return RV_PASS;
    if (metric) return RV_BYPASS;
    *ok = false;
    return RV_MISS;
  }
  if (ct || deny || pass) {
    *ok = false;
    return RV_MISS;
  }
  if (metric) return RV_BYPASS;
  return RV_ISO_DROP;  // drop, or logging drop (goto Output + packet-in, pipeline.go:2055-2062)
  (void)output;
}

// Segment builder ------------------------------------------------------------------------------
struct Blob {
  std::vector<uint32_t> w;
  uint32_t align(uint32_t words) {
    while (w.size() % words) w.push_back(0);
    return uint32_t(w.size());
  }
  template <class T>
  uint32_t put(const T* p, size_t n, uint32_t align_words) {
    uint32_t off = align(align_words);
    const uint32_t* s = reinterpret_cast<const uint32_t*>(p);
    w.insert(w.end(), s, s + n * sizeof(T) / 4);
    return off;
  }
};

constexpr uint32_t kHashMinPoints = 16;

struct PendingSeg {
  SegRec s;
  std::vector<uint32_t> ival;   // lo,hi pairs
  std::vector<BoxRec> boxes;
  std::vector<uint32_t> points;
};

void clause_segments(const std::vector<Atom>& atoms, uint8_t clause, std::vector<PendingSeg>* out) {
  for (auto& a : atoms)
    if (a.t.empty()) {
      PendingSeg ps{};
      ps.s.kind = SEG_ALWAYS;
      ps.s.clause = clause;
      out->push_back(ps);
      return;
    }
  std::map<uint8_t, std::vector<std::pair<uint32_t, uint32_t>>> by_axis;
  std::vector<BoxRec> boxes;
  for (auto& a : atoms) {
    if (a.t.size() == 1 && is_prefix(a.t[0].mask)) {
      uint32_t lo = a.t[0].val & a.t[0].mask, hi = lo | ~a.t[0].mask;
      by_axis[a.t[0].axis].push_back({lo, hi});
    } else {
      BoxRec b{};
      b.nterms = uint8_t(a.t.size());
      for (size_t i = 0; i < a.t.size(); i++) {
        b.axis[i] = a.t[i].axis;
        b.val[i] = a.t[i].val & a.t[i].mask;
        b.mask[i] = a.t[i].mask;
      }
      boxes.push_back(b);
    }
  }
  for (auto& kv : by_axis) {
    auto& iv = kv.second;
    std::sort(iv.begin(), iv.end());
    std::vector<std::pair<uint32_t, uint32_t>> merged;
    for (auto& x : iv) {
      if (!merged.empty() && (merged.back().second == 0xffffffffu || x.first <= merged.back().second + 1)) {
        merged.back().second = std::max(merged.back().second, x.second);
      } else {
        merged.push_back(x);
      }
    }
    bool points = true;
    for (auto& x : merged) points &= x.first == x.second;
    PendingSeg ps{};
    ps.s.axis = kv.first;
    ps.s.clause = clause;
    if (points && merged.size() > kHashMinPoints) {
      ps.s.kind = SEG_HASH;
      ps.s.n = uint32_t(merged.size());
      for (auto& x : merged) ps.points.push_back(x.first);
    } else {
      ps.s.kind = SEG_IVAL;
      ps.s.n = uint32_t(merged.size());
      for (auto& x : merged) {
        ps.ival.push_back(x.first);
        ps.ival.push_back(x.second);
      }
    }
    out->push_back(std::move(ps));
  }
  if (!boxes.empty()) {
    PendingSeg ps{};
    ps.s.kind = SEG_BOX;
    ps.s.clause = clause;
    ps.s.n = uint32_t(boxes.size());
    ps.boxes = std::move(boxes);
    out->push_back(std::move(ps));
  }
}

// Driver index -----------------------------------------------------------------------------------
constexpr uint32_t kMaxBucketsPerAtom = 1024;
const uint8_t kAxisPref[AX_N] = {AX_SRC, AX_DST, AX_CTSRC, AX_CTDST, AX_REG1, AX_INPORT, AX_REG7, AX_TUN, AX_L4D, AX_L4S, AX_CTST};

// Buckets of one atom for the driver index; false = index it in the always list.
bool atom_buckets(const Atom& a, uint8_t* axis, uint8_t* band, std::vector<uint32_t>* bks) {
  if (a.t.empty()) return false;
  const Term* pt = nullptr;
  for (uint8_t ax : kAxisPref) {
    for (auto& t : a.t)
      if (t.axis == ax) { pt = &t; break; }
    if (pt) break;
  }
  if (!pt || pt->axis == AX_CTST) return false;
  uint32_t mk = pt->mask;
  int L = leading_ones(mk);
  uint32_t cov_mask = prefix_mask(L);
  uint32_t lo = pt->val & cov_mask, hi = lo | ~cov_mask;
  *axis = pt->axis;
  bks->clear();
  if (pt->axis <= AX_CTDST) {
    if (L <= 16) {
      *band = 0;
      uint64_t n = (uint64_t(hi >> 16) - (lo >> 16)) + 1;
      if (n > kMaxBucketsPerAtom) return false;
      for (uint32_t b = lo >> 16; b <= (hi >> 16); b++) bks->push_back(b);
    } else if (L <= 24) {
      *band = 1;
      for (uint32_t t = lo >> 8; t <= (hi >> 8); t++) bks->push_back(mix32(t) & 0xffffu);
    } else {
      *band = 2;
      for (uint64_t v = lo; v <= hi; v++) bks->push_back(mix32(uint32_t(v)) & 0xffffu);
    }
  } else if (pt->axis == AX_L4D || pt->axis == AX_L4S) {
    *band = 0;
    if ((lo >> 16) != (hi >> 16)) return false;
    uint32_t pc = proto_class(lo >> 16) << 13;
    uint32_t b0 = pc | ((lo & 0xffffu) >> 3), b1 = pc | ((hi & 0xffffu) >> 3);
    if (b1 - b0 + 1 > kMaxBucketsPerAtom) return false;
    for (uint32_t b = b0; b <= b1; b++) bks->push_back(b);
  } else {
    *band = 0;
    if (uint64_t(hi) - lo >= 128) return false;
    for (uint64_t v = lo; v <= hi; v++) bks->push_back(mix32(uint32_t(v)) & 0xffffu);
  }
  return true;
}

bool build_hash(const std::vector<uint64_t>& keys, uint32_t* log2_out, std::vector<uint64_t>* tab) {
  uint32_t lg = 0;
  while ((8ull << lg) * 3 / 4 < keys.size() + 1) lg++;
  for (int attempt = 0; attempt < 8; attempt++, lg++) {
    uint32_t nb = 1u << lg, mask = nb - 1;
    tab->assign(size_t(nb) * 8, ~0ull);
    std::mt19937 rng(1234 + attempt);
    bool ok = true;
    for (uint64_t k : keys) {
      uint64_t cur = k;
      bool placed = false;
      for (int kick = 0; kick < 500 && !placed; kick++) {
        uint32_t bs[2] = {hash_b1(cur, mask), hash_b2(cur, mask)};
        for (uint32_t b : bs) {
          uint64_t* slot = tab->data() + size_t(b) * 8;
          for (int i = 0; i < 8; i++)
            if (slot[i] == ~0ull || slot[i] == cur) {
              slot[i] = cur;
              placed = true;
              break;
            }
          if (placed) break;
        }
        if (!placed) {
          uint32_t b = bs[rng() & 1];
          int i = int(rng() & 7);
          std::swap(cur, (*tab)[size_t(b) * 8 + i]);
        }
      }
      if (!placed) {
        ok = false;
        break;
      }
    }
    if (ok) {
      *log2_out = lg;
      return true;
    }
  }
  return false;
}

}  // namespace

int build_image(const FeatureNP& np, SlotMap& slots, HostImage* out) {
  *out = HostImage();
  // ---- 1. gather rules per table
  std::map<uint32_t, RuleB> soft[7];
  std::map<std::pair<int, int>, RuleB> hard[7];  // key (-priority, verdict)
  std::set<uint32_t> counted_allow, counted_deny;
  for (auto& kv : np.installed()) {
    const Flow& f = kv.second;
    out->n_flows++;
    if (f.table == TB_EGRESS_METRIC || f.table == TB_INGRESS_METRIC) {
      const Match& m = f.m;
      if (m.has_ct_label && m.has_ct_state && (m.ct_mask & 1) && (m.ct_data & 1) && (!m.has_dl || m.dl_type == kEthIP)) {
        uint32_t id = f.table == TB_INGRESS_METRIC ? uint32_t(m.label_v & 0xffffffffu) : uint32_t(m.label_v >> 32);
        counted_allow.insert(id);
      } else if ((m.reg_present & (1u << 3)) && (m.reg_present & 1) && (m.reg_v[0] & 0x400)) {
        counted_deny.insert(m.reg_v[3]);
      }
      continue;
    }
    if (f.table < TB_AP_EGRESS || f.table > TB_INGRESS_DEFAULT) continue;
    if (f.m.has_conj) {  // conj action flow
      Match rest = f.m;
      rest.has_conj = false;
      bool fam_ok = !rest.has_dl || rest.dl_type == kEthIP;
      rest.has_dl = false;
      if (rest.str(0) != "priority=0") {
        out->error = "unsupported conj_id flow: " + f.str();
        return -GPC_EINVAL;
      }
      bool ok;
      uint8_t v = action_verdict(f, &ok);
      if (!ok) {
        out->error = "unsupported conj_id flow actions: " + f.str();
        return -GPC_EINVAL;
      }
      RuleB& r = soft[f.table][f.m.conj_id];
      r.conj_id = f.m.conj_id;
      r.verdict = v;
      if (fam_ok) {
        if (!r.has_act || f.priority > r.act_prio) r.act_prio = f.priority;
        r.has_act = true;
      }
      continue;
    }
    Atom a;
    int ar = atom_of(f.m, &a);
    if (ar < 0) {
      out->error = "unsupported match: " + f.str();
      return -GPC_EINVAL;
    }
    if (f.is_soft()) {
      for (auto& act : f.acts) {
        RuleB& r = soft[f.table][act.a];
        r.conj_id = act.a;
        if (act.c < 2 || act.c > kMaxClauses || act.b < 1 || act.b > act.c) {
          out->error = "unsupported conjunction shape: " + f.str();
          return -GPC_EINVAL;
        }
        if ((r.prio_set && r.prio != f.priority) || (r.n && r.n != act.c)) {
          out->error = "conjunction clauses at different priorities / clause counts: " + f.str();
          return -GPC_EINVAL;
        }
        r.prio_set = true;
        r.prio = f.priority;
        r.n = uint8_t(act.c);
        if (ar == 0) r.clause[act.b - 1].push_back(a);
      }
    } else {
      bool ok;
      uint8_t v = action_verdict(f, &ok);
      if (!ok) {
        out->error = "unsupported flow actions: " + f.str();
        return -GPC_EINVAL;
      }
      RuleB& r = hard[f.table][{-int(f.priority), int(v)}];
      r.hard = true;
      r.prio_set = true;
      r.prio = f.priority;
      r.n = 1;
      r.verdict = v;
      if (ar == 0) r.clause[0].push_back(a);
    }
  }
  // ---- 2. per table: rank, emit
  Blob B;
  B.w.reserve(1 << 20);
  B.w.push_back(0);  // keep offset 0 unused
  std::vector<uint64_t> hash_keys;
  for (int t = 1; t <= 6; t++) {
    std::vector<RuleB*> rs;
    for (auto& kv : hard[t])
      if (!kv.second.clause[0].empty()) rs.push_back(&kv.second);
    for (auto& kv : soft[t]) {
      RuleB& r = kv.second;
      if (!r.prio_set) continue;  // action flow without match flows
      bool complete = true;
      for (int k = 0; k < r.n; k++) complete &= !r.clause[k].empty();
      if (!complete) continue;  // a clause without atoms (e.g. To = []) never completes
      auto pit = np.policies().find(r.conj_id);
      r.tier = pit != np.policies().end() ? uint8_t(std::max(0, std::min(255, pit->second->tier))) : 0;
      bool is_deny = r.verdict == RV_DROP || r.verdict == RV_REJECT;
      r.counted = r.has_act && ((r.verdict == RV_ALLOW && counted_allow.count(r.conj_id)) || (is_deny && counted_deny.count(r.conj_id)));
      rs.push_back(&r);
    }
    std::stable_sort(rs.begin(), rs.end(), [](const RuleB* a, const RuleB* b) {
      if (a->prio != b->prio) return a->prio > b->prio;
      if (a->hard != b->hard) return a->hard;
      if (a->hard) return a->verdict < b->verdict;
      return a->conj_id < b->conj_id;
    });
    TableHdr& th = out->hdr.t[t - 1];
    th.n_rules = uint32_t(rs.size());
    std::vector<RuleRec> recs(rs.size());
    std::vector<SegRec> segs;
    std::vector<uint32_t> hard_ranks;
    for (size_t rank = 0; rank < rs.size(); rank++) {
      RuleB& r = *rs[rank];
      RuleRec& rec = recs[rank];
      std::memset(&rec, 0, sizeof rec);
      rec.conj_id = r.hard ? 0 : r.conj_id;
      rec.priority = r.prio;
      rec.act_priority = r.act_prio;
      rec.kind = r.hard ? RK_HARD : RK_SOFT;
      rec.n_clauses = r.n;
      rec.verdict = r.verdict;
      rec.flags = uint8_t((r.has_act ? RF_ACT : 0) | (r.counted ? RF_COUNTED : 0));
      rec.tier = r.tier;
      rec.slot = (!r.hard && r.counted) ? slots.get(r.conj_id) : 0;
      rec.seg_begin = uint32_t(segs.size());
      if (r.hard) hard_ranks.push_back(uint32_t(rank));
      uint8_t* nseg[3] = {&rec.nseg0, &rec.nseg1, &rec.nseg2};
      for (int k = 0; k < r.n; k++) {
        std::vector<PendingSeg> ps;
        clause_segments(r.clause[k], uint8_t(k), &ps);
        std::stable_sort(ps.begin(), ps.end(), [](const PendingSeg& a, const PendingSeg& b) {
          static const int order[4] = {1, 2, 3, 0};  // ALWAYS first, then IVAL, HASH, BOX
          return order[a.s.kind] < order[b.s.kind];
        });
        if (ps.size() > 255) {
          out->error = "too many segments in a clause";
          return -GPC_EINVAL;
        }
        *nseg[k] = uint8_t(ps.size());
        for (auto& p : ps) {
          SegRec s = p.s;
          if (p.s.kind == SEG_IVAL) s.off = B.put(p.ival.data(), p.ival.size(), 2);
          else if (p.s.kind == SEG_BOX) s.off = B.put(p.boxes.data(), p.boxes.size(), 8);
          else if (p.s.kind == SEG_HASH)
            for (uint32_t v : p.points) hash_keys.push_back(point_key(uint32_t(t), uint32_t(k), p.s.axis, uint32_t(rank), v));
          segs.push_back(s);
        }
      }
    }
    th.n_hard = uint32_t(hard_ranks.size());
    th.rules_off = recs.empty() ? 0 : B.put(recs.data(), recs.size(), 8);
    th.hard_off = hard_ranks.empty() ? 0 : B.put(hard_ranks.data(), hard_ranks.size(), 1);
    th.seg_off = segs.empty() ? 0 : B.put(segs.data(), segs.size(), 4);
    // driver indexes for clauses 0 and 1 of the soft rules
    for (int k = 0; k < 2; k++) {
      std::vector<uint32_t> always;
      std::map<std::pair<uint8_t, uint8_t>, std::vector<std::pair<uint32_t, uint32_t>>> sub;  // (axis,band) -> (bucket, rank)
      std::vector<uint32_t> bks;
      for (size_t rank = 0; rank < rs.size(); rank++) {
        RuleB& r = *rs[rank];
        if (r.hard) continue;
        for (auto& a : r.clause[k]) {
          uint8_t axis = 0, band = 0;
          if (!atom_buckets(a, &axis, &band, &bks)) {
            always.push_back(uint32_t(rank));
            continue;
          }
          auto& v = sub[{axis, band}];
          for (uint32_t b : bks) v.push_back({b, uint32_t(rank)});
        }
      }
      // the largest sub-indexes keep their index; extras fold into the always list
      std::vector<std::pair<size_t, std::pair<uint8_t, uint8_t>>> order;
      for (auto& kv : sub) order.push_back({kv.second.size(), kv.first});
      std::sort(order.rbegin(), order.rend());
      th.n_idx[k] = 0;
      for (size_t i = 0; i < order.size(); i++) {
        auto& v = sub[order[i].second];
        if (i >= size_t(kIdxPerClause)) {
          for (auto& e : v) always.push_back(e.second);
          continue;
        }
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        std::vector<uint32_t> offs(kBuckets + 1, 0), ents(v.size());
        for (auto& e : v) offs[e.first + 1]++;
        for (uint32_t b = 0; b < kBuckets; b++) offs[b + 1] += offs[b];
        for (size_t j = 0; j < v.size(); j++) ents[j] = v[j].second;  // sorted by (bucket, rank)
        SubIdx& si = th.idx[k][th.n_idx[k]++];
        si.axis = order[i].second.first;
        si.band = order[i].second.second;
        si.off = B.put(offs.data(), offs.size(), 16);
        si.ent = ents.empty() ? si.off : B.put(ents.data(), ents.size(), 16);
      }
      std::sort(always.begin(), always.end());
      always.erase(std::unique(always.begin(), always.end()), always.end());
      th.always_n[k] = uint32_t(always.size());
      th.always_off[k] = always.empty() ? 0 : B.put(always.data(), always.size(), 16);
    }
    out->n_rules[t - 1] = th.n_rules;
    out->n_hard[t - 1] = th.n_hard;
  }
  // ---- 3. point hash
  std::sort(hash_keys.begin(), hash_keys.end());
  hash_keys.erase(std::unique(hash_keys.begin(), hash_keys.end()), hash_keys.end());
  std::vector<uint64_t> tab;
  uint32_t lg = 0;
  if (!build_hash(hash_keys, &lg, &tab)) {
    out->error = "point hash construction failed";
    return -GPC_ENOMEM;
  }
  out->hdr.hash_log2 = lg;
  out->hdr.hash_off = B.put(tab.data(), tab.size(), 16);
  out->hdr.n_slots = slots.size();
  B.align(16);
  out->blob = std::move(B.w);
  return GPC_OK;
}

}  // namespace gpc
