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
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <cstring>
#include <random>
#include <queue>
#include <set>
#include <thread>
#include <tuple>

namespace gpc {

uint32_t SlotMap::get(uint32_t conj) {
  std::lock_guard<std::mutex> g(mu_);
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

bool SlotMap::lookup(uint32_t conj, bool alloc, uint32_t* slot) {
  if (alloc) {
    *slot = get(conj);
    return true;
  }
  std::lock_guard<std::mutex> g(mu_);
  auto it = slot_.find(conj);
  if (it == slot_.end()) return false;
  *slot = it->second;
  return true;
}

void SlotMap::release(uint32_t conj, std::vector<uint32_t>* freed) {
  std::lock_guard<std::mutex> g(mu_);
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
  bool pin = false;  // the action flow sends the packet to the controller (DNS interception)
  uint32_t set_hi[kMaxClauses] = {0, 0, 0};  // base images: key word of a point-hash clause's set
};

// Point extensions (core.hpp ExtHdr, Journal::apply): an atom's identity and a rule's record
// fields other than its atoms, as 64-bit hashes.
uint64_t atom_hash(const Atom& a) {
  uint64_t h = 0x9ae16a3b2f90404full ^ a.t.size();
  for (const Term& t : a.t) h = mix64(mix64(h ^ ((uint64_t(t.val) << 32) | t.mask)) ^ t.axis);
  return h;
}
uint64_t rule_sig(const RuleB& r, bool counted, uint32_t slot) {
  uint64_t h = mix64(uint64_t(r.prio) | uint64_t(r.act_prio) << 16 | uint64_t(r.verdict) << 32 | uint64_t(r.n) << 40 |
                     uint64_t(r.tier) << 48);
  return mix64(h ^ (uint64_t(r.has_act) | uint64_t(r.pin) << 1 | uint64_t(counted) << 2 | uint64_t(slot) << 8));
}
// One copy per distinct sorted hash list (BaseRule::atoms).
struct AtomSetInterner {
  std::unordered_map<uint64_t, std::vector<std::shared_ptr<const std::vector<uint64_t>>>> by_digest;
  std::shared_ptr<const std::vector<uint64_t>> intern(std::vector<uint64_t>&& v) {
    uint64_t d = 0xcbf29ce484222325ull ^ v.size();
    for (uint64_t x : v) d = (d ^ x) * 0x100000001b3ull;
    auto& bucket = by_digest[d];
    for (const auto& p : bucket)
      if (*p == v) return p;
    bucket.push_back(std::make_shared<const std::vector<uint64_t>>(std::move(v)));
    return bucket.back();
  }
};

std::vector<uint64_t> clause_hashes(const std::vector<Atom>& atoms) {
  std::vector<uint64_t> v;
  v.reserve(atoms.size());
  for (const Atom& a : atoms) v.push_back(atom_hash(a));
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  return v;
}

inline uint32_t prefix_mask(int plen) { return plen <= 0 ? 0u : plen >= 32 ? 0xffffffffu : ~((1u << (32 - plen)) - 1); }
inline bool is_prefix(uint32_t m) { return ((~m) & ((~m) + 1u)) == 0; }
inline int leading_ones(uint32_t m) {
  int n = 0;
  while (n < 32 && (m & (0x80000000u >> n))) n++;
  return n;
}

// IPv6 interning (core.hpp "IPv6 interning"): the prefix tree of every IPv6 prefix the realized
// flows match on, each node's 32-bit code prefix, and the device LPM table that maps an address to
// the code of its deepest prefix.
using u128 = unsigned __int128;
inline u128 v6_value(const IPAddr& a) {
  u128 v = 0;
  for (int i = 0; i < 16; i++) v = (v << 8) | a.b[i];
  return v;
}
inline u128 v6_prefix_mask(int len) { return len <= 0 ? u128(0) : len >= 128 ? ~u128(0) : ~((u128(1) << (128 - len)) - 1); }

}  // namespace

class V6Codes {
 public:
  struct Node {
    u128 v;
    int len;
    int parent = -1;
    uint32_t code = 0;
    int clen = 0;
    std::vector<int> kids;
    // Free code space for prefixes added after the build (add_leaf): the "none" leaf of the node
    // (addresses in no child) is its code padded with zeros, at depth none_clen; every other code
    // of that all-zero subtree, [code + 1, code + 2^(32 - none_clen)), is unused. -1: no room.
    int none_clen = -1;
    uint64_t next_free = 1;
  };
  std::vector<Node> nodes;  // nodes[0] = ::/0
  int max_clen = 0;
  std::set<int> lens;       // distinct node lengths (root excluded)
  // lengths first seen in delta epochs (add_leaf), at most kV6MaxNewLens: their leaves are probed
  // in the journal's overflow table after the binary search (core.hpp v6_codes), not searched
  std::set<int> new_lens;

  int build(const FeatureNP& np, std::string* err) {
    std::vector<std::pair<u128, int>> pf;
    auto take = [&](const IPMatch& f) {
      if (!f.set || f.addr.fam != 6) return;
      const int len = f.plen < 0 ? 128 : f.plen;
      if (len > 0) pf.push_back({v6_value(f.addr) & v6_prefix_mask(len), len});
    };
    for (auto& kv : np.installed()) {
      const Flow& f = kv.second;
      if (f.table < TB_AP_EGRESS || f.table > TB_INGRESS_DEFAULT) continue;
      take(f.m.nw_src);
      take(f.m.nw_dst);
      take(f.m.ct_nw_src);
      take(f.m.ct_nw_dst);
    }
    std::sort(pf.begin(), pf.end());  // parents (shorter, same start) before children
    pf.erase(std::unique(pf.begin(), pf.end()), pf.end());
    nodes.assign(1, Node{0, 0});
    index_.clear();
    lens.clear();
    new_lens.clear();
    std::vector<int> st{0};
    for (auto& p : pf) {
      while (st.size() > 1) {
        const Node& t = nodes[st.back()];
        if (p.second > t.len && (p.first & v6_prefix_mask(t.len)) == t.v) break;
        st.pop_back();
      }
      const int id = int(nodes.size());
      nodes.push_back(Node{p.first, p.second});
      nodes.back().parent = st.back();
      nodes[st.back()].kids.push_back(id);
      st.push_back(id);
      index_[{p.first, p.second}] = id;
      lens.insert(p.second);
    }
    // Codes. The children of a node (plus a "none of them" leaf unless they tile the node) get a
    // prefix-free code built like a minimax Huffman tree: merge the two leaves / subtrees needing
    // the fewest bits below them, repeatedly (optimal for the deepest code). Codes need not keep
    // address order -- only containment along tree paths matters -- but the "none" leaf must be
    // the all-zero path: addresses in no child keep the node's code padded with zeros.
    const size_t nn = nodes.size();
    std::vector<int> req(nn, 0);
    for (size_t n = nn; n-- > 0;) {
      std::vector<MergeNode> mt;
      req[n] = merge_children(n, req, &mt);
    }
    if (req[0] > 32) {
      *err = "IPv6 prefix set needs more than 32 code bits";
      return -GPC_EINVAL;
    }
    for (size_t n = 0; n < nn; n++) {
      const Node& N = nodes[n];
      if (N.kids.empty()) continue;
      std::vector<MergeNode> mt;
      merge_children(n, req, &mt);
      std::vector<std::tuple<int, uint32_t, int>> st{{int(mt.size()) - 1, 0u, 0}};  // (merge node, path, depth)
      while (!st.empty()) {
        auto [m, path, depth] = st.back();
        st.pop_back();
        const MergeNode& M = mt[size_t(m)];
        if (M.leaf == kInternal) {
          int zero = M.a, one = M.b;
          if (mt[size_t(one)].has_none) std::swap(zero, one);
          st.push_back({zero, path << 1, depth + 1});
          st.push_back({one, (path << 1) | 1u, depth + 1});
        } else if (M.leaf != kNone) {
          Node& K = nodes[size_t(M.leaf)];
          K.clen = N.clen + depth;
          K.code = N.code | (depth ? path << (32 - K.clen) : 0u);
          max_clen = std::max(max_clen, K.clen);
        } else {
          nodes[n].none_clen = N.clen + depth;
        }
      }
    }
    for (Node& N : nodes)
      if (N.kids.empty()) N.none_clen = N.len < 128 ? N.clen : -1;  // a /128 has no sub-prefixes
    return GPC_OK;
  }

  // Interns a prefix that appeared after the build (a delta commit) without changing any existing
  // code: it must be a leaf (no interned prefix below it) and gets an exact code from the free
  // space of its deepest containing node. Every rule term of that node (a code prefix) and of its
  // ancestors still covers it, so no other rule changes. A length the base LPM does not search is
  // taken as one of at most kV6MaxNewLens new lengths (probed directly: a leaf is the deepest match
  // of every address in it). Returns the node id, or -1 when the tree has to be rebuilt (not a
  // leaf, below a leaf added since the build, no free code, or too many new lengths).
  int add_leaf(u128 v, int len) {
    if (len <= 0) return -1;
    const bool fresh = !lens.count(len) && !new_lens.count(len);
    if (fresh && new_lens.size() >= kV6MaxNewLens) return -1;
    v &= v6_prefix_mask(len);
    auto hit = index_.find({v, len});
    if (hit != index_.end()) return hit->second;
    const u128 last = len >= 128 ? v : v | ~v6_prefix_mask(len);
    auto it = index_.upper_bound({v, len});
    if (it != index_.end() && it->first.first <= last) return -1;  // an interned prefix lies below it
    int P = 0, plen = 0;  // deepest containing node, over the searched and the new lengths
    for (const std::set<int>* ls : {&lens, &new_lens})
      for (int l : *ls) {
        if (l >= len || l <= plen) continue;
        auto a = index_.find({v & v6_prefix_mask(l), l});
        if (a != index_.end()) P = a->second, plen = l;
      }
    Node& p = nodes[size_t(P)];
    if (p.none_clen < 0 || p.none_clen >= 32 || p.next_free >= (uint64_t(1) << (32 - p.none_clen))) return -1;
    if (fresh) new_lens.insert(len);
    Node k{v, len};
    k.parent = P;
    k.code = p.code + uint32_t(p.next_free++);
    k.clen = 32;  // exact: nothing can be added below it without a rebuild
    const int id = int(nodes.size());
    nodes.push_back(k);
    nodes[size_t(P)].kids.push_back(id);
    index_[{v, len}] = id;
    n_added++;
    return id;
  }
  uint32_t n_added = 0;  // prefixes interned by add_leaf since the build
  const char* why_not(u128 v, int len) const {  // the reason add_leaf refused (debug output)
    if (!lens.count(len) && !new_lens.count(len) && new_lens.size() >= kV6MaxNewLens) return "too many new prefix lengths";
    const u128 last = len >= 128 ? v : v | ~v6_prefix_mask(len);
    auto it = index_.upper_bound({v, len});
    if (it != index_.end() && it->first.first <= last) return "an interned prefix lies below it";
    return "no free code in its containing prefix";
  }
  static constexpr int kInternal = -1, kNone = -2;
  struct MergeNode {
    int leaf;      // child node id, kNone, or kInternal
    int a, b;      // merged subtrees (internal)
    bool has_none;
  };
  // Minimax merge of node n's children (+ the none leaf); returns the bits the node needs below
  // its own code; *mt ends with the merge tree's root.
  int merge_children(size_t n, const std::vector<int>& req, std::vector<MergeNode>* mt) const {
    const Node& N = nodes[n];
    if (N.kids.empty()) return 0;
    bool tiles = false;
    if (N.len > 0) {
      u128 sum = 0;
      for (int k : N.kids) sum += u128(1) << (128 - nodes[size_t(k)].len);
      tiles = sum == (u128(1) << (128 - N.len));
    }
    using E = std::tuple<int, int, int>;  // (bits needed, sequence, merge node)
    std::priority_queue<E, std::vector<E>, std::greater<E>> pq;
    int seq = 0;
    for (int k : N.kids) {
      mt->push_back({k, 0, 0, false});
      pq.push({req[size_t(k)], seq++, int(mt->size()) - 1});
    }
    if (!tiles) {
      mt->push_back({kNone, 0, 0, true});
      pq.push({0, seq++, int(mt->size()) - 1});
    }
    while (pq.size() > 1) {
      E x = pq.top();
      pq.pop();
      E y = pq.top();
      pq.pop();
      const int a = std::get<2>(x), b = std::get<2>(y);
      mt->push_back({kInternal, a, b, (*mt)[size_t(a)].has_none || (*mt)[size_t(b)].has_none});
      pq.push({std::max(std::get<0>(x), std::get<0>(y)) + 1, seq++, int(mt->size()) - 1});
    }
    return std::get<0>(pq.top());
  }

  // code prefix of the flow prefix (a, len): false if unknown (not collected)
  bool term(const IPAddr& a, int len, uint32_t* val, uint32_t* mask) const {
    if (len <= 0) {
      *val = *mask = 0;
      return true;
    }
    auto it = index_.find({v6_value(a) & v6_prefix_mask(len), len});
    if (it == index_.end()) return false;
    const Node& N = nodes[it->second];
    // a /128 (no prefix can lie below it): every address in it has exactly the code N.code, so
    // the term is an exact value (host addresses stay points: exact band, point hash); any other
    // prefix is its code prefix, so a leaf added below it later (add_leaf) is still covered
    *mask = (N.kids.empty() && N.len >= 128) || N.clen >= 32 ? 0xffffffffu : prefix_mask(N.clen);
    *val = N.code & *mask;
    return true;
  }
  int find(u128 v, int len) const {
    auto it = index_.find({v & v6_prefix_mask(len), len});
    return it == index_.end() ? -1 : it->second;
  }

 private:
  std::map<std::pair<u128, int>, int> index_;
};

namespace {

// Flow match -> atom over the packet axes of a `fam` image (IPv6: addresses as V6Codes codes).
// Returns 0 ok, 1 never matches a packet of that family, -1 unsupported.
int atom_of(const Match& m, Atom* a, int fam = 4, const V6Codes* codes = nullptr) {
  a->t.clear();
  if (m.has_dl && m.dl_type != (fam == 4 ? kEthIP : kEthIPv6)) return 1;
  auto ip = [&](const IPMatch& f, uint8_t axis) -> int {
    if (!f.set) return 0;
    if (f.addr.fam != fam) return 1;
    if (fam == 6) {
      uint32_t v, mk;
      if (!codes || !codes->term(f.addr, f.plen < 0 ? 128 : f.plen, &v, &mk)) return -1;
      if (mk) a->t.push_back({axis, v, mk});
      return 0;
    }
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
      case ACT_GROUP:  // logging-and-resubmit group (pipeline.go:1739-1760, 1874-1881): the group id is
        // the agent's allocation, so it is not read; a logged Pass flow also loads
        // DispositionPassRegMark (reg0[11..12] = 3, detected above), every other one resubmits to Metric
        metric = true;
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
constexpr uint32_t kHashMinPoints = 24;   // > 24 exact values on one axis: image-wide point hash
constexpr uint32_t kInlinePoints = 16;    // <= 16 points inline in the record
constexpr uint32_t kInlineIvals = 6;      // <= 6 intervals inline
constexpr uint32_t kInlineBoxes = 2;

struct PendingSeg {
  uint8_t kind = SK_ALWAYS, axis = 0;
  std::vector<uint32_t> data;  // IVAL: lo,hi pairs ; PTS / HASH: points ; BOX: 7 words per box
  uint32_t n = 0;
  uint32_t key_hi = 0;         // HASH: the interned point set's key word (core.hpp set_key_hi)
};

// A clause that is a large set of exact values on one axis (AddressGroup members as /32s, Pod
// ofports): its values go to the point hash (SK_HASH) and driver entries of the rule's other
// clauses probe it (core.hpp Ent). Axes 0-6 only (the probe marker is Bloom axis 8 + axis).
bool hash_clause(const std::vector<Atom>& atoms, uint8_t* axis, std::vector<uint32_t>* pts) {
  if (atoms.size() <= kHashMinPoints) return false;
  const uint8_t ax = atoms[0].t.empty() ? 0xff : atoms[0].t[0].axis;
  if (ax > AX_REG7) return false;
  std::vector<uint32_t> v;
  v.reserve(atoms.size());
  for (auto& a : atoms) {
    if (a.t.size() != 1 || a.t[0].axis != ax || a.t[0].mask != 0xffffffffu) return false;
    v.push_back(a.t[0].val);
  }
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  if (v.size() <= kHashMinPoints) return false;
  *axis = ax;
  if (pts) *pts = std::move(v);
  return true;
}

void clause_segments(const std::vector<Atom>& atoms, std::vector<PendingSeg>* out) {
  for (auto& a : atoms)
    if (a.t.empty()) {
      out->push_back(PendingSeg());  // SK_ALWAYS
      return;
    }
  {
    PendingSeg hs;
    if (hash_clause(atoms, &hs.axis, &hs.data)) {
      hs.kind = SK_HASH;
      hs.n = uint32_t(hs.data.size());
      out->push_back(std::move(hs));
      return;
    }
  }
  std::map<uint8_t, std::vector<std::pair<uint32_t, uint32_t>>> by_axis;
  PendingSeg boxes;
  boxes.kind = SK_BOX;
  for (auto& a : atoms) {
    if (a.t.size() == 1 && is_prefix(a.t[0].mask)) {
      uint32_t lo = a.t[0].val & a.t[0].mask, hi = lo | ~a.t[0].mask;
      by_axis[a.t[0].axis].push_back({lo, hi});
    } else {
      uint32_t w[kBoxWords] = {0, 0, 0, 0, 0, 0, 0};
      for (size_t i = 0; i < a.t.size(); i++) {
        w[i] = a.t[i].val & a.t[i].mask;
        w[3 + i] = a.t[i].mask;
        w[6] |= uint32_t(a.t[i].axis) << (8 * i);
      }
      w[6] |= uint32_t(a.t.size()) << 24;
      boxes.data.insert(boxes.data.end(), w, w + kBoxWords);
      boxes.n++;
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
    PendingSeg ps;
    ps.axis = kv.first;
    ps.n = uint32_t(merged.size());
    if (points) {
      ps.kind = SK_PTS;
      for (auto& x : merged) ps.data.push_back(x.first);
    } else {
      ps.kind = SK_IVAL;
      for (auto& x : merged) {
        ps.data.push_back(x.first);
        ps.data.push_back(x.second);
      }
    }
    out->push_back(std::move(ps));
  }
  if (boxes.n) out->push_back(std::move(boxes));
  std::stable_sort(out->begin(), out->end(), [](const PendingSeg& a, const PendingSeg& b) {
    return a.data.size() < b.data.size();  // cheapest segment first
  });
}

// Encodes one clause: returns its words; external data goes to `ext` with its patch positions
// (word index inside the clause) recorded in `patches` (clause-relative position, ext offset).
std::vector<uint32_t> encode_clause(const std::vector<PendingSeg>& segs, std::vector<uint32_t>* ext,
                                    std::vector<std::pair<uint32_t, uint32_t>>* patches) {
  std::vector<uint32_t> w;
  w.push_back(uint32_t(segs.size()));
  for (auto& s : segs) {
    uint32_t kind = s.kind;
    bool external = (kind == SK_IVAL && s.n > kInlineIvals) || (kind == SK_PTS && s.n > kInlinePoints) ||
                    (kind == SK_BOX && s.n > kInlineBoxes);
    if (external) kind = kind == SK_IVAL ? SK_XIVAL : kind == SK_PTS ? SK_XPTS : SK_XBOX;
    w.push_back(kind | (uint32_t(s.axis) << 4) | (s.n << 8));
    if (kind == SK_HASH) w.push_back(s.key_hi);
    if (kind == SK_ALWAYS || kind == SK_HASH) continue;
    if (external) {
      while (ext->size() % 16) ext->push_back(0);
      patches->push_back({uint32_t(w.size()), uint32_t(ext->size())});
      w.push_back(0);
      ext->insert(ext->end(), s.data.begin(), s.data.end());
    } else {
      w.insert(w.end(), s.data.begin(), s.data.end());
    }
  }
  return w;
}

// Fast descriptor (core.hpp FastKind) of a clause encoded by encode_clause. `data` tells where word
// B must point: -1 nowhere (B holds a value), 0 the first data word of the clause's single inline
// segment (clause-relative word 2), 1 its external data (B is patched like the clause's pointer).
struct Fcd {
  uint32_t a = FK_GENERIC, b = 0, c = 0;
  int data = -1;
};
Fcd fast_clause(const std::vector<PendingSeg>& segs) {
  Fcd f;
  if (segs.size() != 1) return f;  // several segments: the interpreter
  const PendingSeg& s = segs[0];
  const uint32_t ax = uint32_t(s.axis) << 4;
  const bool external = (s.kind == SK_IVAL && s.n > kInlineIvals) || (s.kind == SK_PTS && s.n > kInlinePoints) ||
                        (s.kind == SK_BOX && s.n > kInlineBoxes);
  switch (s.kind) {
    case SK_ALWAYS:
      f.a = FK_ALWAYS;
      return f;
    case SK_HASH:
      f.a = FK_HASH | ax;
      f.b = s.key_hi;
      return f;
    case SK_IVAL:
    case SK_PTS:
      if (s.n == 1) {
        f.a = FK_IV1 | ax;
        f.b = s.data[0];
        f.c = s.kind == SK_IVAL ? s.data[1] : s.data[0];
        return f;
      }
      f.a = (s.kind == SK_IVAL ? FK_IVN : FK_PTN) | ax | (s.n << 8);
      f.data = external ? 1 : 0;
      return f;
    case SK_BOX: {
      // single-term boxes on one axis only (the ct_state bypass flows, masked tun_id / ports)
      uint32_t axis0 = 0xffu;
      for (uint32_t i = 0; i < s.n; i++) {
        const uint32_t meta = s.data[kBoxWords * i + 6];
        if ((meta >> 24) != 1u) return f;
        if (axis0 != 0xffu && (meta & 0xffu) != axis0) return f;
        axis0 = meta & 0xffu;
      }
      if (s.n == 1) {
        f.a = FK_MK1 | (axis0 << 4);
        f.b = s.data[0];
        f.c = s.data[3];
        return f;
      }
      f.a = FK_MKN | (axis0 << 4) | (s.n << 8);
      f.data = external ? 1 : 0;
      return f;
    }
    default:
      return f;
  }
}

// Image blob (uint32 words) ------------------------------------------------------------------------
struct Blob {
  std::vector<uint32_t> w;
  void align(size_t words) {
    while (w.size() % words) w.push_back(0);
  }
  template <typename T>
  uint32_t put(const T* p, size_t n, size_t align_words) {
    static_assert(sizeof(T) % 4 == 0, "word-sized elements");
    align(align_words);
    uint32_t off = uint32_t(w.size());
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
    w.insert(w.end(), q, q + n * (sizeof(T) / 4));
    return off;
  }
};

// Driver index -----------------------------------------------------------------------------------
constexpr uint64_t kMaxBucketsPerAtom = 1024;
const uint8_t kAxisPref[AX_N] = {AX_SRC, AX_DST, AX_CTSRC, AX_CTDST, AX_REG1, AX_INPORT, AX_REG7, AX_TUN, AX_L4D, AX_L4S, AX_CTST};

struct AtomKey {  // an atom's primary term as seen by the driver index
  uint8_t axis, band;
  uint32_t lo, hi;
};

// false = index it in the always list
bool atom_key(const Atom& a, AtomKey* k) {
  if (a.t.empty()) return false;
  const Term* pt = nullptr;
  for (uint8_t ax : kAxisPref) {
    for (auto& t : a.t)
      if (t.axis == ax) { pt = &t; break; }
    if (pt) break;
  }
  if (!pt || pt->axis == AX_CTST) return false;
  int L = leading_ones(pt->mask);
  uint32_t cov = prefix_mask(L);
  k->axis = pt->axis;
  k->lo = pt->val & cov;
  k->hi = k->lo | ~cov;
  if (pt->axis <= AX_CTDST) {
    if (L < 4) return false;  // /0../3: always list
    k->band = L <= 12 ? 0 : L <= 16 ? 1 : L <= 24 ? 2 : L <= 31 ? 3 : 4;
  } else if (pt->axis == AX_L4D || pt->axis == AX_L4S) {
    k->band = 0;
    if ((k->lo >> 16) != (k->hi >> 16)) return false;
    if ((((k->hi & 0xffffu) >> 3) - ((k->lo & 0xffffu) >> 3) + 1) > kMaxBucketsPerAtom) return false;
  } else {
    k->band = 0;
    if (uint64_t(k->hi) - k->lo >= 128) return false;
  }
  return true;
}

uint64_t atom_span(const AtomKey& k) {  // number of bucket-key values the atom covers
  if (k.axis <= AX_CTDST) {
    const uint32_t sh = ip_band_shift(k.band);
    return uint64_t(k.hi >> sh) - (k.lo >> sh) + 1;
  }
  if (k.axis == AX_L4D || k.axis == AX_L4S) return ((k.hi & 0xffffu) >> 3) - ((k.lo & 0xffffu) >> 3) + 1;
  return uint64_t(k.hi) - k.lo + 1;
}

void atom_bucket_list(const AtomKey& k, uint32_t bits, std::vector<uint32_t>* out) {
  out->clear();
  if (k.axis <= AX_CTDST) {
    const uint32_t sh = ip_band_shift(k.band);
    for (uint64_t t = k.lo >> sh; t <= (k.hi >> sh); t++) out->push_back(bucket_of(k.axis, k.band, bits, uint32_t(t << sh)));
  } else if (k.axis == AX_L4D || k.axis == AX_L4S) {
    uint32_t b0 = bucket_of(k.axis, 0, 16, k.lo), b1 = bucket_of(k.axis, 0, 16, k.hi);
    for (uint32_t b = b0; b <= b1; b++) out->push_back(b);
  } else {
    for (uint64_t v = k.lo; v <= k.hi; v++) out->push_back(bucket_of(k.axis, 0, bits, uint32_t(v)));
  }
  std::sort(out->begin(), out->end());
  out->erase(std::unique(out->begin(), out->end()), out->end());
}

// Entry filter (core.hpp Ent): Bloom bits of the rule's non-driver clauses -------------------------
// An IP / exact-axis term usable by the filter: returns false when it cannot be represented.
bool filt_term_ip(const Term& t, uint32_t* bit) {
  if (t.axis <= AX_CTDST) {
    if (!is_prefix(t.mask)) return false;
    int L = leading_ones(t.mask);
    if (L < 8) return false;
    uint32_t band = L < 16 ? 1 : L < 24 ? 2 : L < 32 ? 3 : 4;
    uint32_t shift = band == 1 ? 24 : band == 2 ? 16 : band == 3 ? 8 : 0;
    *bit = filt_ip_bit(t.axis, band, t.val >> shift);
    return true;
  }
  if (t.axis >= AX_INPORT && t.axis <= AX_TUN) {
    if (t.mask != 0xffffffffu) return false;
    *bit = filt_ip_bit(t.axis, 4, t.val);
    return true;
  }
  return false;
}

// IP part of one clause: all atoms must carry a usable term on one common axis.
bool filt_clause_ip(const std::vector<Atom>& atoms, uint32_t* axis, uint32_t* bits) {
  if (atoms.empty()) return false;
  int ax = -1;
  for (auto& t : atoms[0].t) {
    uint32_t b;
    if (filt_term_ip(t, &b)) {
      ax = t.axis;
      break;
    }
  }
  if (ax < 0) return false;
  uint32_t m = 0;
  for (auto& a : atoms) {
    bool found = false;
    for (auto& t : a.t) {
      uint32_t b;
      if (t.axis == ax && filt_term_ip(t, &b)) {
        m |= b;
        found = true;
        break;
      }
    }
    if (!found) return false;
  }
  *axis = uint32_t(ax);
  *bits = m;
  return true;
}

// Service part of one clause: every atom needs a tp_dst (L4D) term.
bool filt_clause_l4(const std::vector<Atom>& atoms, uint32_t* bits) {
  if (atoms.empty()) return false;
  uint32_t m = 0;
  for (auto& a : atoms) {
    const Term* l4 = nullptr;
    for (auto& t : a.t)
      if (t.axis == AX_L4D) l4 = &t;
    if (!l4 || (l4->mask >> 16) != 0xffffu) return false;
    uint32_t pc = proto_class(l4->val >> 16);
    uint32_t pm = l4->mask & 0xffffu;
    uint32_t lo = l4->val & pm & 0xffffu, hi = lo | (~pm & 0xffffu);
    if (!is_prefix(l4->mask)) lo = 0, hi = 0xffffu;
    if (lo == hi) {
      m |= filt_l4x_bit(pc, lo);
      continue;
    }
    for (uint32_t blk = lo >> 12; blk <= (hi >> 12); blk++) m |= filt_l4_bit(pc, blk);
  }
  *bits = m;
  return true;
}

// Hull of one clause on `axis` (every atom needs a term on it): any value matching v/m lies in
// [v & m, (v & m) | ~m], so the hull is a necessary condition of the clause.
bool clause_hull(const std::vector<Atom>& atoms, uint8_t axis, uint32_t* lo, uint32_t* hi) {
  if (atoms.empty()) return false;
  uint32_t l = 0xffffffffu, h = 0;
  for (auto& a : atoms) {
    const Term* tm = nullptr;
    for (auto& t : a.t)
      if (t.axis == axis) tm = &t;
    if (!tm) return false;
    l = std::min(l, tm->val & tm->mask);
    h = std::max(h, (tm->val & tm->mask) | ~tm->mask);
  }
  *lo = l;
  *hi = h;
  return true;
}

// Fraction of the axis' value space the hull covers (the interval prefilter keeps the smallest).
double hull_coverage(uint8_t axis, uint32_t lo, uint32_t hi, const uint64_t* span) {
  double len = double(hi) - double(lo) + 1.0;
  if (axis == AX_L4D || axis == AX_L4S) return (lo >> 16) == (hi >> 16) ? len / 65536.0 : 1.0;
  if (axis <= AX_TUN) return span[axis] ? std::min(1.0, len / double(span[axis])) : 1.0;  // IP and exact axes
  return 1.0;
}

// True if the clause's match set is exactly [lo, hi] on `axis` (single-term atoms whose ranges
// merge into one interval), so a passing interval test decides the clause.
bool clause_is_interval(const std::vector<Atom>& atoms, uint8_t axis, uint32_t lo, uint32_t hi) {
  std::vector<std::pair<uint32_t, uint32_t>> iv;
  for (auto& a : atoms) {
    if (a.t.size() != 1 || a.t[0].axis != axis || !is_prefix(a.t[0].mask)) return false;
    uint32_t l = a.t[0].val & a.t[0].mask;
    iv.push_back({l, l | ~a.t[0].mask});
  }
  std::sort(iv.begin(), iv.end());
  uint32_t cur = iv[0].first;
  if (cur != lo) return false;
  uint64_t reach = iv[0].second;
  for (auto& x : iv) {
    if (uint64_t(x.first) > reach + 1) return false;
    reach = std::max<uint64_t>(reach, x.second);
  }
  return reach == hi;
}

// The clause's match set on `axis` as sorted disjoint intervals (single-term prefix atoms, merged
// where they touch); false if some atom is not such a term.
bool clause_intervals(const std::vector<Atom>& atoms, uint8_t axis, std::vector<std::pair<uint32_t, uint32_t>>* out) {
  std::vector<std::pair<uint32_t, uint32_t>> iv;
  for (auto& a : atoms) {
    if (a.t.size() != 1 || a.t[0].axis != axis || !is_prefix(a.t[0].mask)) return false;
    const uint32_t l = a.t[0].val & a.t[0].mask;
    iv.push_back({l, l | ~a.t[0].mask});
  }
  if (iv.empty()) return false;
  std::sort(iv.begin(), iv.end());
  out->clear();
  for (auto& x : iv) {
    if (!out->empty() && uint64_t(x.first) <= uint64_t(out->back().second) + 1)
      out->back().second = std::max(out->back().second, x.second);
    else
      out->push_back(x);
  }
  return true;
}

struct IvalChoice {
  int clause = -1;
  uint32_t axis = kFiltNoAxis, lo = 0, hi = 0;
  bool exact = false;
};

// The non-driver clause whose hull covers the smallest fraction of its axis (entry interval test).
IvalChoice choose_interval(const RuleB& r, int d, const uint64_t* span) {
  IvalChoice ch;
  double best = 0.5;  // an interval covering more than half of its axis is not worth a check
  for (int c = 0; c < r.n; c++) {
    if (c == d || r.clause[c].empty()) continue;
    for (auto& t : r.clause[c][0].t) {
      if (t.axis >= AX_CTST) continue;
      uint32_t lo, hi;
      if (!clause_hull(r.clause[c], t.axis, &lo, &hi)) continue;
      double cov = hull_coverage(t.axis, lo, hi, span);
      if (cov < best) {
        best = cov;
        ch.clause = c;
        ch.axis = t.axis;
        ch.lo = lo;
        ch.hi = hi;
      }
    }
  }
  if (ch.clause >= 0) ch.exact = clause_is_interval(r.clause[ch.clause], uint8_t(ch.axis), ch.lo, ch.hi);
  return ch;
}

// The non-driver clause driver-d entries probe in the point hash (the largest hash clause), or -1.
int probe_clause(const RuleB& r, int d, uint8_t* axis) {
  int best = -1;
  size_t most = 0;
  for (int c = 0; c < r.n; c++) {
    uint8_t ax;
    uint32_t fax, fbits;
    if (c == d || r.clause[c].size() <= most || !hash_clause(r.clause[c], &ax, nullptr)) continue;
    if (!filt_clause_ip(r.clause[c], &fax, &fbits) || fax != ax) continue;
    best = c;
    most = r.clause[c].size();
    *axis = ax;
  }
  return best;
}

// Clauses a passing entry of driver d has already decided (record word 5, core.hpp): the exact
// interval test, and the probed point-set clause.
uint32_t skip_mask(const RuleB& r, int d, const uint64_t* span) {
  if (d >= r.n) return 0;
  IvalChoice ch = choose_interval(r, d, span);
  uint8_t pax;
  const int pc = probe_clause(r, d, &pax);
  return (ch.exact ? (1u << ch.clause) : 0u) | (pc >= 0 ? (1u << pc) : 0u);
}

// Driver entry (core.hpp Ent) of rule r for driver clause d at record offset `off`; `span` = value
// span of each IP / exact axis over the table's atoms.
std::array<uint32_t, 4> entry_of(const RuleB& r, int d, uint32_t off, const uint64_t* span) {
  uint32_t axis = kFiltNoAxis, ipbits = 0, l4bits = kFiltL4All;
  bool have_ip = false, have_l4 = false;
  uint8_t pax;
  const int pc = probe_clause(r, d, &pax);
  if (pc >= 0) {  // probe entry: the probed set's id in base images (core.hpp entry_pass), else
                   // the Bloom bits of the probed clause (probe_clause checked them)
    filt_clause_ip(r.clause[pc], &axis, &ipbits);
    if (r.set_hi[pc]) ipbits = (r.set_hi[pc] >> 4) & (kPointSetMax - 1u);
    axis = 8u + pax;
    have_ip = true;
  }
  for (int c = 0; c < r.n; c++) {
    if (c == d || c == pc) continue;
    uint32_t ax, b;
    if (!have_l4 && filt_clause_l4(r.clause[c], &b)) {
      l4bits = b;
      have_l4 = true;
    } else if (!have_ip && filt_clause_ip(r.clause[c], &ax, &b)) {
      axis = ax;
      ipbits = b;
      have_ip = true;
    }
  }
  IvalChoice ch = choose_interval(r, d, span);
  return {((off >> 4) << 8) | (ch.axis << 4) | axis, ipbits | l4bits, ch.lo, ch.hi};
}

// ImageHdr / JournalHdr bloom_axes bit of an entry's Bloom axis (core.hpp entry_pass reads
// fm[x & 7] unless the axis field is kFiltNoAxis).
uint32_t bloom_axis_bit(uint32_t x) { return (x & 15u) == kFiltNoAxis ? 0u : 1u << (x & 7u); }

// Point hash (core.hpp hash_contains): 2-choice cuckoo hash of kHashSlots-slot 16-B buckets,
// sized to <= 70 % load (random-walk insertion; a failed build retries with twice the buckets).
bool build_hash(const std::vector<uint64_t>& keys, uint32_t* log2_out, std::vector<uint64_t>* tab) {
  constexpr uint32_t S = kHashSlots;
  uint32_t lg = 0;
  while (double(S << lg) * 0.7 < double(keys.size() + 1)) lg++;
  for (int attempt = 0; attempt < 8; attempt++, lg++) {
    uint32_t nb = 1u << lg, mask = nb - 1;
    tab->assign(size_t(nb) * S, ~0ull);
    std::mt19937 rng(1234 + attempt);
    bool ok = true;
    for (uint64_t k : keys) {
      uint64_t cur = k;
      bool placed = false;
      for (int kick = 0; kick < 1000 && !placed; kick++) {
        uint32_t bs[2] = {hash_b1(cur, mask), hash_b2(cur, mask)};
        for (uint32_t b : bs) {
          uint64_t* slot = tab->data() + size_t(b) * S;
          for (uint32_t i = 0; i < S; i++)
            if (slot[i] == ~0ull || slot[i] == cur) {
              slot[i] = cur;
              placed = true;
              break;
            }
          if (placed) break;
        }
        if (!placed) {
          uint32_t b = bs[rng() & 1];
          uint32_t i = rng() % S;
          std::swap(cur, (*tab)[size_t(b) * S + i]);
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

// Bit-parallel table (core.hpp BitTable): built when the table has 1..kBitRules soft rules, all with
// conj_id action flows, whose atoms are single terms on at most kBitProbes (axis, mask, clause)
// triples, and every hard rule is inline. The driver indexes stay (delta epochs with tombstones
// scan them). GPC_NO_BITSET=1 turns it off.
void build_bits(const std::vector<RuleB*>& rs, const std::vector<uint32_t>& rec_off, TableHdr& th, Blob& B) {
  th.bits_off = 0;
  if (std::getenv("GPC_NO_BITSET")) return;
  if (th.n_hard != th.n_hfast) return;
  std::vector<size_t> soft;  // rank indexes of the soft rules
  std::vector<uint32_t> hard_prefix;
  for (size_t r = 0; r < rs.size(); r++) {
    if (rs[r]->hard) hard_prefix.push_back(uint32_t(soft.size()));
    else soft.push_back(r);
  }
  if (soft.empty() || soft.size() > kBitRules || hard_prefix.size() > kHardFast) return;
  BitTable bt{};
  std::map<std::array<uint32_t, 3>, std::map<uint32_t, uint32_t>> probes;  // (axis, mask, clause) -> key -> rule mask
  for (size_t i = 0; i < soft.size(); i++) {
    const RuleB& r = *rs[soft[i]];
    if (!r.has_act) return;
    for (int k = 0; k < kMaxClauses; k++) {
      if (k >= r.n) {
        bt.absent[k] |= 1u << i;
        continue;
      }
      for (const Atom& a : r.clause[k]) {
        if (a.t.size() != 1 || a.t[0].axis >= AX_N) return;
        const Term& t = a.t[0];
        probes[{t.axis, t.mask, uint32_t(k)}][t.val & t.mask] |= 1u << i;
      }
    }
  }
  if (probes.empty() || probes.size() > kBitProbes) return;
  for (size_t h = 0; h < hard_prefix.size(); h++) bt.hard_prefix[h] = hard_prefix[h];
  for (size_t i = 0; i < soft.size(); i++) {
    size_t end = i + 1;
    while (end < soft.size() && rs[soft[end]]->prio == rs[soft[i]]->prio) end++;
    bt.info[2 * i] = rec_off[soft[i]];
    bt.info[2 * i + 1] = uint32_t(rs[soft[i]]->prio) | (uint32_t(end) << 16);
  }
  uint32_t q = 0;
  std::vector<std::pair<uint32_t, std::vector<uint32_t>>> tabs;  // (probe, slots) emitted after the header
  for (auto& kv : probes) {
    const auto& keys = kv.second;
    uint32_t lg = 4;
    while ((uint64_t(1) << lg) < 2 * keys.size()) lg++;
    bool placed_all = false;
    std::vector<uint32_t> slots;
    for (; lg <= 16 && !placed_all; lg++) {
      const uint32_t m = (1u << lg) - 1u;
      slots.assign(size_t(2) << lg, 0u);
      std::vector<bool> used(size_t(1) << lg, false);
      placed_all = true;
      std::mt19937 rng(7 + lg);
      for (auto& e : keys) {
        uint32_t key = e.first, val = e.second;
        bool done = false;
        for (int kick = 0; kick < 500 && !done; kick++) {
          const uint32_t h = bit_hash(q, key), b[2] = {h & m, (h >> 16) & m};
          for (uint32_t bb : b)
            if (!used[bb]) {
              used[bb] = true;
              slots[2 * bb] = key;
              slots[2 * bb + 1] = val;
              done = true;
              break;
            }
          if (done) break;
          const uint32_t v = b[rng() & 1];  // evict and re-place the resident
          std::swap(key, slots[2 * v]);
          std::swap(val, slots[2 * v + 1]);
        }
        if (!done) {
          placed_all = false;
          break;
        }
      }
      if (placed_all) break;
    }
    if (!placed_all) return;
    // an empty slot {0, 0} whose key equals a packet's masked value contributes no rule bit
    BitProbe& pr = bt.probe[q];
    pr.ak = kv.first[0] | (kv.first[2] << 8);
    pr.mask = kv.first[1];
    pr.lg = lg;
    tabs.push_back({q, std::move(slots)});
    q++;
  }
  bt.n_probe = q;
  for (auto& tb : tabs) bt.probe[tb.first].off = B.put(tb.second.data(), tb.second.size(), 16);
  th.bits_off = B.put(reinterpret_cast<const uint32_t*>(&bt), sizeof bt / 4, 16);
  if (std::getenv("GPC_IMAGE_DEBUG"))
    std::fprintf(stderr, "bit-parallel table: %zu soft rules, %u probes\n", soft.size(), bt.n_probe);
}

// Composite driver (core.hpp TableHdr cidx): built when every soft rule of the table has, in clause
// 1 - cb, at most kCompositeMaxValues exact values on one common axis (AppliedTo ofports, Pod IPs)
// and, in clause cb, only IP atoms the driver index can key. Each rule is listed under (band key,
// value) for every band key its clause-cb atoms cover and every value of its other clause, with the
// same entry (prefilter) as clause cb's plain index. GPC_COMPOSITE=0 turns it off. Measured on
// MI355X (64M packets, profiles/r03h_*): C1 8.73 -> 8.51 ms, C2 14.00 -> 10.25, C3 10.66 -> 10.12,
// C4 12.18 -> 11.38.
constexpr size_t kCompositeMaxValues = 16;
// An exact-value entry decides a third clause of up to this many intervals (one entry per interval;
// C2 / C2g services: 1-3 single ports), so candidates need no record read to verify it.
constexpr size_t kExactMaxIntervals = 4;
// Entries of a composite index at most (GPC_COMPOSITE_MAX_ENTRIES overrides, experiments)
constexpr uint64_t kCompositeMaxEntries = uint64_t(1) << 24;  // 256 MB of entries at most
uint64_t composite_max_entries() {
  static const uint64_t v = std::getenv("GPC_COMPOSITE_MAX_ENTRIES")
                                ? std::strtoull(std::getenv("GPC_COMPOSITE_MAX_ENTRIES"), nullptr, 0) : kCompositeMaxEntries;
  return v;
}
// Band merging (round 5). Every sub-index is a probe -- a dependent bucket-offset load and an entry
// load, lines of 25-30 MB arrays that miss L2 -- so a packet pays per band, not per entry. Per IP
// axis of the band clause, the atoms of bands m.. are keyed at band m's granularity (one sub-index)
// for the coarsest m whose (key, value) lists stay short: the entry-weighted mean list length
// sum(len^2) / sum(len) over the exact (band-m key, value) pairs at most kMergeListMax -- and only
// when the index's entries exceed kMergeMinBytes (an L2-resident index pays little per probe and
// much per scanned entry). Measured (64M packets, profiles/r05e, r05f; the statistic in brackets):
// C3 (CIDRs /8-/32 spread over the address space) 7.98 ms unmerged, 6.11 with m = 1 [6.2], 5.58
// with m = 0 [11]; C4 7.58 -> 5.41 (m = 0); C2 (AddressGroup /32s inside a few /16s) 7.94 unmerged,
// 29.2 with m = 3 [29-34], 73.5 with m = 1; C1 (0.08 MB image) 5.80 unmerged, 7.38 with m = 3 [3-4],
// 8.07 with m = 0.
constexpr double kMergeListMax = 16.0;
constexpr uint32_t kV6DefaultTags = 4;
// Sub-region tables (kV6L1Child) cost 4 KB per split and a block keeps splitting while it holds
// more than kV6LeafLens lengths, so rule sets mixing many long prefix lengths under distinct blocks
// could grow them without bound (a /64 holding a /96 and a /128 under c = 48 costs
// 16 KB). Budget: 1 KB per prefix of the tree, at least 128 MB, at most 1 GB (C3: 245 k prefixes,
// 94.5 MB of sub-tables). Past it a block keeps its length list (or the global search), which is
// the unsplit round-5 layout: exact, only slower for the addresses under it.
constexpr size_t kV6SubBytesPerPrefix = 1024, kV6SubMinBudget = size_t(128) << 20, kV6SubMaxBudget = size_t(1) << 30;
constexpr uint64_t kMergeMinBytes = uint64_t(16) << 20;
// Host-set combinations (build_composite, core.hpp kBandCombo): applied to a host-address band
// of at least kComboMinEntries (member, value) entries that at least halves them, with at most
// kComboMax combinations (ids fit the entries' 16 spare bits).
constexpr uint64_t kComboMinEntries = 1u << 16;
constexpr size_t kComboMax = 65535;
// Membership hash of a combination sub-index (core.hpp combo_of): {lg, 0, 0, 0}, then 2^lg buckets
// of two {host value, combination id} slots, two choices, load <= 1/2 (combination 0: empty slot).
uint32_t put_combo_members(const std::vector<std::pair<uint32_t, uint32_t>>& members, Blob& B, HostImage* out) {
  uint32_t lg = 4;
  while ((1ull << lg) < members.size()) lg++;
  std::mt19937 rng(0xC0B0u);
  for (;; lg++) {
    const uint32_t mask = (1u << lg) - 1u;
    std::vector<uint32_t> tab(4 + (size_t(4) << lg), 0u);
    tab[0] = lg;
    bool ok = true;
    for (auto m : members) {
      uint32_t v = m.first, c = m.second;
      for (int kick = 0; kick < 500 && c; kick++) {
        const uint64_t k = combo_key64(v);
        const uint32_t b[2] = {hash_b1(k, mask), hash_b2(k, mask)};
        for (int j = 0; j < 2 && c; j++)
          for (int sl = 0; sl < 2 && c; sl++) {
            uint32_t* q = &tab[4 + 4 * size_t(b[j]) + 2 * sl];
            if (q[1] == 0) q[0] = v, q[1] = c, c = 0;
          }
        if (!c) break;
        uint32_t* q = &tab[4 + 4 * size_t(b[rng() & 1u]) + 2 * (rng() & 1u)];  // evict, retry the victim
        std::swap(q[0], v);
        std::swap(q[1], c);
      }
      if (c) {
        ok = false;
        break;
      }
    }
    if (!ok) continue;
    out->bytes_hash += 4ull * tab.size();
    return B.put(tab.data(), tab.size(), 16);
  }
}

template <typename CE>
void merge_bands(std::map<std::pair<uint8_t, uint8_t>, std::vector<CE>>& sub, const std::vector<std::vector<uint32_t>>& xsets) {
  std::set<uint8_t> axes;
  uint64_t entries = 0;
  for (auto& kv : sub) {
    axes.insert(kv.first.first);
    for (auto& e : kv.second) entries += atom_span(e.key) * xsets[e.xi].size();
  }
  if (entries * sizeof(Ent) < kMergeMinBytes) return;
  for (uint8_t ax : axes) {
    for (uint32_t m = 0; m + 1 < kIpBands; m++) {
      const uint32_t sh = ip_band_shift(m);
      std::vector<uint64_t> combos;
      bool big = false;
      for (auto& kv : sub) {
        if (kv.first.first != ax || kv.first.second < m || big) continue;
        for (auto& e : kv.second) {
          for (uint64_t k = e.key.lo >> sh; k <= (e.key.hi >> sh) && !big; k++)
            for (uint32_t x : xsets[e.xi]) combos.push_back((k << 32) | x);
          big = combos.size() > composite_max_entries();
        }
      }
      if (big || combos.empty()) continue;
      std::sort(combos.begin(), combos.end());
      double s1 = 0, s2 = 0;
      for (size_t i = 0; i < combos.size();) {
        size_t j = i;
        while (j < combos.size() && combos[j] == combos[i]) j++;
        const double c = double(j - i);
        s1 += c;
        s2 += c * c;
        i = j;
      }
      const bool merge = s2 / s1 <= kMergeListMax;
      if (std::getenv("GPC_IMAGE_DEBUG"))
        std::fprintf(stderr, "composite axis %u: bands >= %u at band %u: %zu entries, mean list %.2f -> %s\n", ax, m, m,
                     combos.size(), s2 / s1, merge ? "merged" : "kept");
      if (!merge) continue;
      std::vector<CE> moved;
      for (auto it = sub.begin(); it != sub.end();) {
        if (it->first.first == ax && it->first.second > m) {
          for (auto& e : it->second) {
            e.key.band = uint8_t(m);
            moved.push_back(e);
          }
          it = sub.erase(it);
        } else {
          ++it;
        }
      }
      auto& dst = sub[{ax, uint8_t(m)}];
      dst.insert(dst.end(), moved.begin(), moved.end());
      break;
    }
  }
}
void build_composite(const std::vector<RuleB*>& rs, const std::vector<uint32_t>& rec_off, const uint64_t* span, int t,
                     TableHdr& th, Blob& B, HostImage* out) {
  th.n_cidx = 0;
  th.cband = th.cx = 0;
  th.xmap_off = 0;
  const char* on = std::getenv("GPC_COMPOSITE");  // GPC_COMPOSITE=0 turns it off (read at every build)
  if (on && on[0] == '0') return;
  struct CE {
    AtomKey key;
    uint32_t xi;  // index of the rule's value list in xsets
    std::array<uint32_t, 4> ent;
  };
  // GPC_CBAND_MERGE=m (experiments): key every band above m at band m's granularity, instead of the
  // adaptive choice below
  const char* mb = std::getenv("GPC_CBAND_MERGE");
  const int merge_to = mb ? std::min(int(kIpBands) - 1, std::max(0, std::atoi(mb))) : int(kIpBands) - 1;
  for (int cb = 0; cb < 2; cb++) {
    const int ce = 1 - cb;
    int X = -1;
    bool ok = true;
    size_t nsoft = 0;
    std::vector<std::vector<uint32_t>> xsets;
    std::map<std::pair<uint8_t, uint8_t>, std::vector<CE>> sub;
    std::vector<std::pair<uint32_t, uint32_t>> xpatch;  // (record word 5 offset, skip bits) of exact-value rules
    std::vector<uint32_t> xi_rank;                      // rule of each value list (rank in rs)
    // exact-value rules whose third clause is 2..kExactMaxIntervals intervals: one entry per interval
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> xivs;
    const bool exact_ok = !std::getenv("GPC_NO_EXACT_X");  // (experiments)
    const bool multi_ok = !std::getenv("GPC_NO_EXACT_MULTI");  // (experiments)
    for (size_t rank = 0; rank < rs.size() && ok; rank++) {
      const RuleB& r = *rs[rank];
      if (r.hard) continue;
      nsoft++;
      if (r.n < 2 || r.clause[ce].empty() || r.clause[ce].size() > kCompositeMaxValues) {
        ok = false;
        break;
      }
      std::vector<uint32_t> xs;
      for (auto& a : r.clause[ce]) {
        if (a.t.size() != 1 || a.t[0].mask != 0xffffffffu || a.t[0].axis > AX_TUN || (X >= 0 && a.t[0].axis != X)) {
          ok = false;
          break;
        }
        X = a.t[0].axis;
        xs.push_back(a.t[0].val);
      }
      if (!ok) break;
      std::sort(xs.begin(), xs.end());
      xs.erase(std::unique(xs.begin(), xs.end()), xs.end());
      std::array<uint32_t, 4> ent = entry_of(r, cb, rec_off[rank], span);
      // exact-value entry (core.hpp kEntExactX) when the rule's remaining clause, if any, is one
      // interval: the entry then decides every clause but the band clause (record word 5 skips them)
      int sc = -1;
      uint32_t sax = kFiltNoAxis, slo = 0, shi = 0;
      bool exact = exact_ok && r.n <= 3 && rec_off[rank] < (1u << 27);
      std::vector<std::pair<uint32_t, uint32_t>> ivs;
      if (exact && r.n == 3) {
        sc = 3 - cb - ce;
        const auto& cl = r.clause[sc];
        exact = !cl.empty() && cl[0].t.size() == 1 && cl[0].t[0].axis < AX_N &&
                clause_intervals(cl, cl[0].t[0].axis, &ivs) && (ivs.size() == 1 || (multi_ok && ivs.size() <= kExactMaxIntervals));
        if (exact) {
          sax = cl[0].t[0].axis;
          slo = ivs[0].first;
          shi = ivs[0].second;
        }
      }
      if (ivs.size() < 2) ivs.clear();
      if (exact) {
        ent = {((rec_off[rank] >> 4) << 8) | (sax << 4) | kFiltNoAxis | kEntExactX, 0u, slo, shi};
        xpatch.push_back({rec_off[rank] + 5, ((1u << ce) | (sc >= 0 ? 1u << sc : 0u)) << (3 * cb)});
      }
      for (auto& a : r.clause[cb]) {
        AtomKey key;
        if (!atom_key(a, &key) || key.axis > AX_CTDST) {
          ok = false;
          break;
        }
        if (key.band > merge_to) key.band = uint8_t(merge_to);  // keyed coarser: fewer probes per packet
        sub[{key.axis, key.band}].push_back({key, uint32_t(xsets.size()), ent});
      }
      xsets.push_back(std::move(xs));
      xi_rank.push_back(uint32_t(rank));
      xivs.push_back(exact ? std::move(ivs) : std::vector<std::pair<uint32_t, uint32_t>>());
    }
    if (!ok || nsoft == 0 || X < 0) continue;
    if (!mb) merge_bands(sub, xsets);
    if (sub.size() > size_t(kIdxPerClause)) continue;
    // Host-set combinations (round 6, core.hpp kBandCombo): the host-address band of an IP axis
    // whose atoms are large shared sets (AddressGroups of Pod IPs) is keyed by the packet's
    // combination -- the interned set of those host sets that contain its address (a membership
    // hash, value -> combination id) -- instead of by the address. Each rule is listed once per
    // (combination holding its set, value of its other clause), not once per (member, value): C2g
    // (16 groups of 10 000 Pod IPs) 24 M entries -> far fewer, each list the few rules whose group
    // holds the packet's source AND whose AppliedTo holds its value. The entries are exact-value
    // entries that also carry the combination id (16 bits in the top bytes of lo / hi), so the
    // band clause is decided by the entry too (record word 5 skips it for rules keyed only here).
    std::pair<uint8_t, uint8_t> combo_key{0xff, 0xff};
    std::vector<std::pair<uint64_t, std::array<uint32_t, 4>>> combo_ents;  // (combo << 32 | x, entry)
    std::vector<std::pair<uint32_t, uint32_t>> combo_members;               // (host value, combo id)
    std::map<uint32_t, uint32_t> combo_rules;  // rules keyed only by combinations: (record word 5, skip bits)
    if (!std::getenv("GPC_NO_COMBO")) {  // (experiments)
      for (auto& kv : sub) {
        if (kv.first.second != 4 || kv.first.first > AX_CTDST || combo_key.first != 0xff) continue;
        std::map<uint32_t, std::vector<uint32_t>> hosts;  // rule (xi) -> its host values in this band
        std::map<uint32_t, std::vector<std::array<uint32_t, 4>>> tmpl;  // rule (xi) -> its combination entries
        std::map<uint32_t, uint32_t> skips;                // rule (xi) -> clauses its entry decides
        bool elig = true;
        uint64_t old_n = 0;
        for (auto& e : kv.second) {
          elig = elig && e.key.lo == e.key.hi && rec_off[xi_rank[e.xi]] < (1u << 27);
          if (!elig) break;
          hosts[e.xi].push_back(e.key.lo);
          old_n += xsets[e.xi].size() * std::max<size_t>(1, xivs[e.xi].size());
          if (tmpl.count(e.xi)) continue;
          // the entry decides the value clause (y) and the band clause (combination id); the rule's
          // third clause, if any, must be on a port axis: its hull is the entry's interval, decided
          // when it is one interval, else verified from the record
          const RuleB& r = *rs[xi_rank[e.xi]];
          uint32_t sax = kFiltNoAxis, slo = 0, shi = 0, skip = (1u << ce) | (1u << cb);
          std::vector<std::pair<uint32_t, uint32_t>> ivs{{0u, 0u}};
          if (r.n == 3) {
            const int sc = 3 - cb - ce;
            const auto& cl = r.clause[sc];
            const uint32_t a0 = cl.empty() || cl[0].t.size() != 1 ? uint32_t(AX_N) : cl[0].t[0].axis;
            elig = (a0 == AX_L4D || a0 == AX_L4S) && clause_hull(cl, a0, &slo, &shi) && shi <= 0xffffffu;
            if (!elig) break;
            sax = a0;
            std::vector<std::pair<uint32_t, uint32_t>> exact_ivs;
            if (clause_intervals(cl, a0, &exact_ivs) && exact_ivs.size() <= (multi_ok ? kExactMaxIntervals : 1u)) {
              skip |= 1u << sc;  // decided by the entry: one entry per interval
              ivs = exact_ivs;
            } else {
              ivs = {{slo, shi}};  // the hull, verified from the record
            }
          } else if (r.n != 2) {
            elig = false;
            break;
          }
          for (auto& iv : ivs)
            tmpl[e.xi].push_back({((rec_off[xi_rank[e.xi]] >> 4) << 8) | (sax << 4) | kFiltCombo | kEntExactX, 0u,
                                  iv.first, iv.second});
          skips[e.xi] = skip;
        }
        if (!elig || old_n < kComboMinEntries) continue;
        std::map<std::vector<uint32_t>, uint32_t> set_ids;
        std::vector<std::vector<uint32_t>> set_rules;  // set id -> rules (xi)
        for (auto& h : hosts) {
          std::sort(h.second.begin(), h.second.end());
          h.second.erase(std::unique(h.second.begin(), h.second.end()), h.second.end());
          auto ins = set_ids.emplace(h.second, uint32_t(set_ids.size()));
          if (ins.second) set_rules.emplace_back();
          set_rules[ins.first->second].push_back(h.first);
        }
        std::unordered_map<uint32_t, std::vector<uint32_t>> pat;  // host value -> set ids (ascending)
        for (auto& si : set_ids)
          for (uint32_t v : si.first) pat[v].push_back(si.second);
        std::map<std::vector<uint32_t>, uint32_t> combos;
        std::vector<std::pair<uint32_t, uint32_t>> members;
        members.reserve(pat.size());
        for (auto& pv : pat) {
          auto ins = combos.emplace(pv.second, uint32_t(combos.size() + 1));
          members.push_back({pv.first, ins.first->second});
        }
        if (combos.size() > kComboMax) continue;
        uint64_t new_n = 0;
        for (auto& c : combos)
          for (uint32_t sid : c.first)
            for (uint32_t xi : set_rules[sid]) new_n += xsets[xi].size() * tmpl[xi].size();
        if (new_n * 2 > old_n) continue;  // not worth a dependent membership load
        std::vector<std::pair<uint64_t, std::array<uint32_t, 4>>> ents;
        ents.reserve(new_n);
        for (auto& c : combos)
          for (uint32_t sid : c.first)
            for (uint32_t xi : set_rules[sid])
              for (uint32_t x : xsets[xi])
                for (const auto& t0 : tmpl[xi]) {
                  std::array<uint32_t, 4> en = t0;
                  en[1] = x;
                  en[2] = (en[2] & 0xffffffu) | ((c.second & 0xffu) << 24);
                  en[3] = (en[3] & 0xffffffu) | (((c.second >> 8) & 0xffu) << 24);
                  ents.push_back({(uint64_t(c.second) << 32) | x, en});
                }
        // rules whose every band-clause entry is in this band: the combination decides the clause
        std::map<uint32_t, size_t> n_all, n_here;
        for (auto& kv2 : sub)
          for (auto& e : kv2.second) (kv2.first == kv.first ? n_here : n_all)[e.xi]++;
        for (auto& h : tmpl)
          if (!n_all.count(h.first)) combo_rules[rec_off[xi_rank[h.first]] + 5] = skips[h.first] << (3 * cb);
        (void)n_here;
        if (std::getenv("GPC_IMAGE_DEBUG"))
          std::fprintf(stderr, "table %d composite axis %u: %zu host sets, %zu combinations over %zu hosts: %llu -> %llu entries\n",
                       t, kv.first.first, set_ids.size(), combos.size(), members.size(), (unsigned long long)old_n,
                       (unsigned long long)new_n);
        combo_key = kv.first;
        combo_ents.swap(ents);
        combo_members.swap(members);
      }
    }
    auto n_ent = [&](uint32_t xi) -> uint64_t { return std::max<size_t>(1, xivs[xi].size()); };
    uint64_t total = 0;
    for (auto& kv : sub)
      if (kv.first == combo_key) total += combo_ents.size();
      else
        for (auto& e : kv.second) total += atom_span(e.key) * xsets[e.xi].size() * n_ent(e.xi);
    if (total > composite_max_entries()) continue;
    std::vector<std::pair<uint32_t, std::array<uint32_t, 4>>> be;
    // 2^extra buckets per entry: fewer hash collisions per probe. Round 4 (offset pairs, C3 / C2):
    // extra 0 -> 10.48 / 10.98 ms, 1 -> 10.12 / 10.25 ms, 2 -> 10.10 / 10.05 ms with 40 % more image.
    // Round 5 (bucket directories: a bucket costs 0.5 B of directory, not 4 B of offsets): 1 -> 4.756
    // / 7.402 ms, 2 -> 4.718 / 7.193 ms for 2-4 MB more image (profiles/r05zd_extra_bits.txt).
    // GPC_COMPOSITE_EXTRA_BITS overrides (experiments)
    const char* xe = std::getenv("GPC_COMPOSITE_EXTRA_BITS");
    const uint32_t extra = xe ? uint32_t(std::min(3, std::max(0, std::atoi(xe)))) : 2u;
    // core.hpp SubIdx fmt: bucket directories (1: read in the value-map word's round, where the map
    // cannot filter -- an exact non-IP value axis; 2: after it, an IP value axis). GPC_COMPOSITE_DIR
    // overrides (experiments): 0 = offset pairs (+ presence maps), 1 or 2 for every table
    const char* de = std::getenv("GPC_COMPOSITE_DIR");
    const int dir_fmt = de ? std::min(2, std::max(0, std::atoi(de))) : (X > AX_CTDST ? 1 : 2);
    for (auto& kv : sub) {
      const bool combo = kv.first == combo_key;
      const uint8_t axis = kv.first.first, band = combo ? uint8_t(kBandCombo) : kv.first.second;
      uint64_t n = 0;
      if (combo) n = combo_ents.size();
      else
        for (auto& e : kv.second) n += atom_span(e.key) * xsets[e.xi].size() * n_ent(e.xi);
      uint32_t bits = 10;
      while (bits < 24 && (1ull << bits) < n) bits++;
      bits = std::min(26u, bits + extra);
      const uint32_t sh = ip_band_shift(band);
      be.clear();
      if (combo) {
        for (auto& ce : combo_ents)
          be.push_back({cbucket_of(band, bits, uint32_t(ce.first >> 32), uint32_t(ce.first)), ce.second});
      } else {
        for (auto& e : kv.second)
          for (uint64_t k = e.key.lo >> sh; k <= (e.key.hi >> sh); k++)
            for (uint32_t x : xsets[e.xi]) {
              std::array<uint32_t, 4> en = e.ent;
              if (en[0] & kEntExactX) en[1] = x;
              else out->hdr.bloom_axes |= bloom_axis_bit(en[0]) | kBloomL4;
              const uint32_t bk = cbucket_of(band, bits, uint32_t(k << sh), x);
              if (xivs[e.xi].size() > 1) {  // one exact entry per interval of the third clause
                for (auto& iv : xivs[e.xi]) {
                  en[2] = iv.first;
                  en[3] = iv.second;
                  be.push_back({bk, en});
                }
              } else {
                be.push_back({bk, en});
              }
            }
      }
      std::sort(be.begin(), be.end());
      be.erase(std::unique(be.begin(), be.end()), be.end());
      const uint32_t nb = 1u << bits;
      std::vector<uint32_t> offs(size_t(nb) + 1, 0), ents;
      ents.reserve(4 * be.size());
      for (auto& e : be) offs[e.first + 1]++;
      for (uint32_t b = 0; b < nb; b++) offs[b + 1] += offs[b];
      SubIdx& si = th.cidx[th.n_cidx++];
      si.axis = axis;
      si.band = band;
      si.bits = uint8_t(bits);
      si.pres = combo ? put_combo_members(combo_members, B, out) : 0u;
      si.fmt = uint8_t(dir_fmt);
      if (dir_fmt) {
        // core.hpp dir_list: a 16-B block per 32 buckets; lists of kDirCountMax or more entries
        // move behind the main ones, their bucket holding a pointer entry and 6 inert zero entries
        std::vector<uint32_t> dir(size_t(nb) / 8, 0u), ovf;
        uint32_t main_n = 0;
        for (uint32_t b = 0; b < nb; b++)
          main_n += std::min(offs[b + 1] - offs[b], kDirCountMax);
        ents.assign(size_t(4) * main_n, 0u);
        uint32_t slot = 0;
        for (uint32_t b = 0; b < nb; b++) {
          uint32_t* d = &dir[4 * (b >> 5)];
          if ((b & 31u) == 0) d[3] = slot;
          const uint32_t n = offs[b + 1] - offs[b], c = std::min(n, kDirCountMax);
          for (int k = 0; k < 3; k++) d[k] |= ((c >> k) & 1u) << (b & 31u);
          if (n < kDirCountMax) {
            for (uint32_t e = offs[b]; e < offs[b + 1]; e++, slot++)
              std::copy(be[e].second.begin(), be[e].second.end(), &ents[4 * size_t(slot)]);
          } else {
            const uint32_t at = main_n + uint32_t(ovf.size() / 4);
            ents[4 * size_t(slot) + 1] = at;  // {0, overflow index, count, 0}
            ents[4 * size_t(slot) + 2] = n;
            slot += kDirCountMax;
            for (uint32_t e = offs[b]; e < offs[b + 1]; e++) ovf.insert(ovf.end(), be[e].second.begin(), be[e].second.end());
          }
        }
        ents.insert(ents.end(), ovf.begin(), ovf.end());
        si.off = B.put(dir.data(), dir.size(), 16);
        si.ent = ents.empty() ? si.off : B.put(ents.data(), ents.size(), 16);
        out->bytes_bucket_offsets += 4ull * dir.size();
        out->bytes_entries += 4ull * ents.size();
        if (std::getenv("GPC_IMAGE_DEBUG"))
          std::fprintf(stderr, "table %d composite clause %d x axis %d: axis %u band %u bits %u entries %zu dir fmt %d (%zu overflow)\n",
                       t, cb, X, axis, band, bits, be.size(), dir_fmt, ovf.size() / 4);
        continue;
      }
      for (auto& e : be) ents.insert(ents.end(), e.second.begin(), e.second.end());
      si.off = B.put(offs.data(), offs.size(), 16);
      si.ent = ents.empty() ? si.off : B.put(ents.data(), ents.size(), 16);
      // core.hpp SubIdx.pres, where the value map cannot filter and several bands are probed: an
      // exact non-IP axis (AppliedTo ofports: every ingress packet goes to a local Pod, so its value
      // is always in the map) with >= 2 sub-indexes. With an IP value axis (egress: the Pod IPs) the
      // map already drops most packets, and the bitmaps only take L2 room: C3 egress 3.57 -> 3.98 ms
      // with them, ingress 5.56 -> 5.01 ms; C2 (one sub-index) unchanged (profiles/r04g_*).
      const bool want_pres = X > AX_CTDST && sub.size() >= 2;
      if (want_pres && !std::getenv("GPC_NO_PRESENCE")) {  // (GPC_NO_PRESENCE: experiments)
        std::vector<uint32_t> pres(nb / 32, 0u);
        for (uint32_t b = 0; b < nb; b++)
          if (offs[b + 1] > offs[b]) pres[b >> 5] |= 1u << (b & 31u);
        si.pres = B.put(pres.data(), pres.size(), 16);
        out->bytes_bucket_offsets += 4ull * pres.size();
      }
      out->bytes_bucket_offsets += 4ull * offs.size();
      out->bytes_entries += 4ull * ents.size();
      if (std::getenv("GPC_IMAGE_DEBUG"))
        std::fprintf(stderr, "table %d composite clause %d x axis %d: axis %u band %u bits %u entries %zu\n", t, cb, X, axis,
                     band, bits, be.size());
    }
    std::vector<uint32_t> xmap(1u << 11, 0u);  // 2^16 bits
    for (auto& xs : xsets)
      for (uint32_t x : xs) xmap[cx_bit(x) >> 5] |= 1u << (cx_bit(x) & 31u);
    th.xmap_off = B.put(xmap.data(), xmap.size(), 16);
    th.cband = uint8_t(cb);
    th.cx = uint8_t(X);
    for (auto& pt : xpatch) B.w[pt.first] |= pt.second;
    for (auto& pt : combo_rules) B.w[pt.first] |= pt.second;
    return;
  }
}

}  // namespace

namespace {

// GPC_IMAGE_TIMING=1: per-phase build times on stderr (rank/span, records, indexes, hash).
struct PhaseTimer {
  bool on = std::getenv("GPC_IMAGE_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  double acc[4] = {0, 0, 0, 0};
  void lap(int i) {
    if (!on) return;
    auto n = std::chrono::steady_clock::now();
    acc[i] += std::chrono::duration<double, std::milli>(n - t).count();
    t = n;
  }
  void report(const char* what) {
    if (on) std::fprintf(stderr, "%s ms: rank %.3f records %.3f index %.3f hash %.3f\n", what, acc[0], acc[1], acc[2], acc[3]);
  }
};

// Flow -> rule gathering (step 1 of an image build).
struct Gather {
  int fam = 4;                      // image family: 4, or 6 (addresses through `codes`)
  const V6Codes* codes = nullptr;
  std::map<uint32_t, RuleB> soft[7];
  std::map<std::pair<int, int>, RuleB> hard[7];  // key (-priority, verdict)
  std::set<uint32_t> counted_allow, counted_deny;
  uint32_t isc = 0;  // ImageHdr.isc: the IngressSecurityClassifier bypasses the installed flows define
  uint32_t n_flows = 0;
  std::string error;
  // only_conj != 0: take only that conjunction's actions of a soft flow (delta builds gather per rule).
  int add(const Flow& f, uint32_t only_conj = 0);
  int add_isc(const Flow& f);
  uint16_t isc_prio = 0;
  uint16_t eth() const { return fam == 4 ? kEthIP : kEthIPv6; }
  // One conjunction(id, k/n) action of soft flow f (delta builds: the action comes from the
  // context's action map, not from a scan of the flow's possibly long action list).
  int add_soft(const Flow& f, uint32_t id, uint32_t k, uint32_t n) {
    n_flows++;
    Atom a;
    int ar = atom_of(f.m, &a, fam, codes);
    if (ar < 0) {
      error = "unsupported match: " + f.str();
      return -GPC_EINVAL;
    }
    return add_clause_atom(f, ar == 0 ? &a : nullptr, id, k, n);
  }
  int add_clause_atom(const Flow& f, const Atom* a, uint32_t id, uint32_t k, uint32_t n) {
    RuleB& r = soft[f.table][id];
    r.conj_id = id;
    if (n < 2 || n > uint32_t(kMaxClauses) || k < 1 || k > n) {
      error = "unsupported conjunction shape: " + f.str();
      return -GPC_EINVAL;
    }
    if ((r.prio_set && r.prio != f.priority) || (r.n && r.n != n)) {
      error = "conjunction clauses at different priorities / clause counts: " + f.str();
      return -GPC_EINVAL;
    }
    r.prio_set = true;
    r.prio = f.priority;
    r.n = uint8_t(n);
    if (a) r.clause[k - 1].push_back(*a);
    return GPC_OK;
  }
};

int Gather::add(const Flow& f, uint32_t only_conj) {
  n_flows++;
  if (f.table == TB_EGRESS_METRIC || f.table == TB_INGRESS_METRIC) {
    const Match& m = f.m;
    if (m.has_ct_label && m.has_ct_state && (m.ct_mask & 1) && (m.ct_data & 1) && (!m.has_dl || m.dl_type == eth())) {
      uint32_t id = f.table == TB_INGRESS_METRIC ? uint32_t(m.label_v & 0xffffffffu) : uint32_t(m.label_v >> 32);
      counted_allow.insert(id);
    } else if ((m.reg_present & (1u << 3)) && (m.reg_present & 1) && (m.reg_v[0] & 0x400)) {
      counted_deny.insert(m.reg_v[3]);
    }
    return GPC_OK;
  }
  if (f.table == TB_INGRESS_CLASSIFIER) return add_isc(f);
  if (f.table < TB_AP_EGRESS || f.table > TB_INGRESS_DEFAULT) return GPC_OK;
  if (f.m.has_conj) {  // conj action flow
    Match rest = f.m;
    rest.has_conj = false;
    bool fam_ok = !rest.has_dl || rest.dl_type == eth();
    rest.has_dl = false;
    if (rest.str(0) != "priority=0") {
      error = "unsupported conj_id flow: " + f.str();
      return -GPC_EINVAL;
    }
    bool ok;
    uint8_t v = action_verdict(f, &ok);
    if (!ok) {
      error = "unsupported conj_id flow actions: " + f.str();
      return -GPC_EINVAL;
    }
    RuleB& r = soft[f.table][f.m.conj_id];
    r.conj_id = f.m.conj_id;
    r.verdict = v;
    for (auto& act : f.acts)
      if (act.kind == ACT_CONTROLLER) r.pin = true;
    if (fam_ok) {
      if (!r.has_act || f.priority > r.act_prio) r.act_prio = f.priority;
      r.has_act = true;
    }
    return GPC_OK;
  }
  Atom a;
  int ar = atom_of(f.m, &a, fam, codes);
  if (ar < 0) {
    error = "unsupported match: " + f.str();
    return -GPC_EINVAL;
  }
  if (f.is_soft()) {
    for (auto& act : f.acts) {
      if (only_conj && act.a != only_conj) continue;
      int rc = add_clause_atom(f, ar == 0 ? &a : nullptr, act.a, act.b, act.c);
      if (rc) return rc;
    }
  } else {
    bool ok;
    uint8_t v = action_verdict(f, &ok);
    if (!ok) {
      error = "unsupported flow actions: " + f.str();
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
  return GPC_OK;
}

// IngressSecurityClassifier flows (pipeline.go:2144-2182) -> ImageHdr.isc. Supported: the shapes
// ingressClassifierFlows installs, at one priority: reg0=<PktDestinationField mark>/0xf0 and
// ct_mark=0x40/0x40 (HairpinCTMark), each going to IngressMetric or ConntrackCommit (out of the
// policy tables). Anything else is rejected: the kernel could not honour it.
int Gather::add_isc(const Flow& f) {
  const Match& m = f.m;
  const bool out = f.acts.size() == 1 && f.acts[0].kind == ACT_GOTO &&
                   (f.acts[0].a == TB_INGRESS_METRIC || f.acts[0].a == TB_CONNTRACK_COMMIT);
  const uint16_t only_reg0 = 1u;
  uint32_t bit = 0;
  if (out && m.reg_present == only_reg0 && m.reg_m[0] == 0xf0u && !m.has_ct_mark) {
    switch (m.reg_v[0]) {
      case kToGatewayMark: bit = kIscGateway; break;
      case kToTunnelMark: bit = kIscTunnel; break;
      case kToUplinkMark: bit = kIscUplink; break;
    }
  } else if (out && m.reg_present == 0 && m.has_ct_mark && m.ct_mark_v == kHairpinCTMark && m.ct_mark_m == kHairpinCTMark) {
    bit = kIscHairpin;
  }
  const bool rest = !m.has_conj && !m.has_ct_state && !m.has_ct_label && !m.has_dl && !m.has_tun && !m.has_in_port &&
                    !m.nw_src.set && !m.nw_dst.set && !m.ct_nw_src.set && !m.ct_nw_dst.set && !m.has_tp_src && !m.has_tp_dst;
  if (!bit || !rest || (isc_prio && isc_prio != f.priority)) {
    error = "unsupported IngressSecurityClassifier flow: " + f.str();
    return -GPC_EINVAL;
  }
  isc_prio = f.priority;
  isc |= bit;
  return GPC_OK;
}

int emit(Gather& G, const FeatureNP& np, SlotMap& slots, HostImage* out, bool alloc);

}  // namespace

int build_image(const FeatureNP& np, SlotMap& slots, HostImage* out, bool alloc, const HeldExts* hold) {
  *out = HostImage();
  Gather G;
  for (auto& kv : np.installed()) {
    int rc = G.add(kv.second);
    if (rc) {
      out->error = G.error;
      return rc;
    }
  }
  // Held point extensions: the base gets the rule without those exact values (never an emptied
  // clause: such a rule keeps all its atoms, and Journal::apply then journals it as it would any).
  if (hold)
    for (auto& h : *hold) {
      RuleB* r = nullptr;
      for (int t = 1; t <= 6 && !r; t++) {
        auto it = G.soft[t].find(h.first);
        if (it != G.soft[t].end()) r = &it->second;
      }
      if (!r || h.second.clause >= uint32_t(r->n)) continue;
      std::vector<Atom>& cl = r->clause[h.second.clause];
      auto held = [&](const Atom& a) {
        return a.t.size() == 1 && a.t[0].mask == 0xffffffffu &&
               std::binary_search(h.second.values.begin(), h.second.values.end(),
                                  std::make_pair(uint32_t(a.t[0].axis), a.t[0].val));
      };
      const size_t keep = size_t(std::count_if(cl.begin(), cl.end(), [&](const Atom& a) { return !held(a); }));
      if (keep && keep < cl.size()) cl.erase(std::remove_if(cl.begin(), cl.end(), held), cl.end());
    }
  return emit(G, np, slots, out, alloc);
}

HeldExts Journal::held_extensions() const {
  HeldExts h;
  for (auto& kv : ext_) {
    HeldExt& e = h[kv.first];
    e.clause = kv.second.clause;
    e.values = kv.second.values;
  }
  return h;
}

// A 2-choice hash of V6Lpm slots (core.hpp v6_codes) at most `load` full: 2^lg buckets of
// kV6BucketSlots slots; cuckoo placement, a larger table when it does not converge.
static bool v6_hash_build(const std::vector<std::array<uint32_t, 8>>& slots6, double load, std::vector<uint32_t>* tab,
                          uint32_t* lg_out) {
  const size_t nk = slots6.size();
  const uint32_t S = kV6BucketSlots, W = kV6SlotWords;
  uint32_t lg = 0;
  while (double(S << lg) * load < double(nk + 1)) lg++;
  for (int attempt = 0; attempt < 8; attempt++, lg++) {
    const uint32_t nb = 1u << lg, mask = nb - 1;
    tab->assign(size_t(nb) * S * W, 0u);
    std::mt19937 rng(4321 + attempt);
    bool ok = true;
    for (size_t n = 0; n < slots6.size() && ok; n++) {
      uint32_t cur[8];
      std::memcpy(cur, slots6[n].data(), sizeof cur);
      bool placed = false;
      for (int kick = 0; kick < 1000 && !placed; kick++) {
        const uint64_t hk = v6_hkey(cur, cur[4] & 0xffu);
        const uint32_t bs[2] = {hash_b1(hk, mask), hash_b2(hk, mask)};
        for (uint32_t b : bs) {
          for (uint32_t i = 0; i < S && !placed; i++) {
            uint32_t* sl = tab->data() + (size_t(b) * S + i) * W;
            if (!(sl[4] & kV6Valid)) {
              std::memcpy(sl, cur, sizeof cur);
              placed = true;
            }
          }
          if (placed) break;
        }
        if (!placed) {
          uint32_t* sl = tab->data() + (size_t(bs[rng() & 1]) * S + rng() % S) * W;
          for (uint32_t w = 0; w < W; w++) std::swap(cur[w], sl[w]);
        }
      }
      ok = placed;
    }
    if (ok) {
      *lg_out = lg;
      return true;
    }
  }
  return false;
}

// The LPM table of one prefix length (core.hpp V6Len): entries (kv = prefix right-aligned, code).
// Key words kw = the fewest of 1 / 2 / 4 whose complement (the tag) all entries share; the empty-slot
// key is one no entry has. 2-choice cuckoo placement over buckets of two slots, a larger table when
// it does not converge. Fills d (except tab_off) and tab.
// kw = 1: line buckets (core.hpp kV6LineSlots): each key in its first choice while that has room,
// else in its second choice with the first one's flag set; the table doubles until every key fits.
static bool v6_line_table_build(uint32_t len, const std::vector<std::pair<std::array<uint32_t, 4>, uint32_t>>& ents,
                                V6Len* d, std::vector<uint32_t>* tab) {
  std::set<uint32_t> used;
  for (auto& e : ents) used.insert(e.first[3]);
  uint32_t empty = ~0u;
  while (used.count(empty)) empty--;
  for (uint32_t w = 0; w < 3; w++) d->pat[w] = ents.empty() ? 0u : ents[0].first[w];
  d->pat[3] = empty;
  d->seed = v6_seed(len, 1, d->pat);
  uint32_t lg = 0;
  while (double(kV6LineSlots << lg) * 0.4 < double(ents.size() + 1)) lg++;
  for (int attempt = 0; attempt < 8; attempt++, lg++) {
    const uint32_t nb = 1u << lg;
    d->meta = len | 1u << 8 | lg << 16;
    tab->assign(size_t(nb) * 16, 0u);
    std::vector<uint8_t> n_in(nb, 0);
    for (size_t b = 0; b < nb; b++)
      for (uint32_t s = 0; s < kV6LineSlots; s++) (*tab)[b * 16 + 1 + 2 * s] = empty;
    bool ok = true;
    for (size_t n = 0; n < ents.size() && ok; n++) {
      uint32_t bs[2];
      v6_buckets(*d, ents[n].first.data(), &bs[0], &bs[1]);
      uint32_t b = bs[0];
      if (n_in[b] >= kV6LineSlots) {
        (*tab)[size_t(bs[0]) * 16] = 1u;  // flag: look at the second choice too
        b = bs[1];
      }
      if (n_in[b] >= kV6LineSlots) {
        ok = false;
        break;
      }
      (*tab)[size_t(b) * 16 + 1 + 2 * n_in[b]] = ents[n].first[3];
      (*tab)[size_t(b) * 16 + 2 + 2 * n_in[b]] = ents[n].second;
      n_in[b]++;
    }
    if (ok) return true;
  }
  return false;
}

static bool v6_len_table_build(uint32_t len, const std::vector<std::pair<std::array<uint32_t, 4>, uint32_t>>& ents,
                               V6Len* d, std::vector<uint32_t>* tab) {
  *d = V6Len{};
  uint32_t kw = 4;
  for (uint32_t k : {1u, 2u}) {
    bool same = true;
    for (auto& e : ents)
      for (uint32_t w = 0; w + k < 4 && same; w++) same = e.first[w] == ents[0].first[w];
    if (same) {
      kw = k;
      break;
    }
  }
  if (kw == 1u) return v6_line_table_build(len, ents, d, tab);
  const uint32_t sw = v6_slot_words(kw), ns = 2, bw = v6_bucket_words(kw);
  std::set<std::array<uint32_t, 4>> used;
  for (auto& e : ents) {
    std::array<uint32_t, 4> k = e.first;
    for (uint32_t w = 0; w + kw < 4; w++) k[w] = 0;
    used.insert(k);
  }
  std::array<uint32_t, 4> empty{0u, 0u, 0u, 0u};
  for (uint32_t w = 4 - kw; w < 4; w++) empty[w] = ~0u;
  while (used.count(empty)) empty[3]--;  // at most |ents| tries
  for (uint32_t w = 0; w < 4; w++) d->pat[w] = w + kw < 4 ? (ents.empty() ? 0u : ents[0].first[w]) : empty[w];
  d->seed = v6_seed(len, kw, d->pat);
  const double load = 0.7;
  uint32_t lg = 0;
  while (double(ns << lg) * load < double(ents.size() + 1)) lg++;
  for (int attempt = 0; attempt < 8; attempt++, lg++) {
    const uint32_t nb = 1u << lg;
    d->meta = len | kw << 8 | lg << 16;
    tab->assign(size_t(nb) * bw, 0u);
    std::vector<uint8_t> full(size_t(nb) * ns, 0);
    for (size_t s = 0; s < size_t(nb) * ns; s++)
      for (uint32_t w = 0; w < kw; w++) (*tab)[s * sw + w] = empty[4 - kw + w];
    std::mt19937 rng(4321 + attempt);
    bool ok = true;
    for (size_t n = 0; n < ents.size() && ok; n++) {
      std::array<uint32_t, 4> cur = ents[n].first;
      uint32_t code = ents[n].second;
      bool placed = false;
      for (int kick = 0; kick < 1000 && !placed; kick++) {
        uint32_t bs[2];
        v6_buckets(*d, cur.data(), &bs[0], &bs[1]);
        for (uint32_t bk : bs) {
          for (uint32_t i = 0; i < ns && !placed; i++) {
            const size_t s = size_t(bk) * ns + i;
            if (!full[s]) {
              for (uint32_t w = 0; w < kw; w++) (*tab)[s * sw + w] = cur[4 - kw + w];
              (*tab)[s * sw + kw] = code;
              full[s] = 1;
              placed = true;
            }
          }
          if (placed) break;
        }
        if (!placed) {  // evict a random resident of one of the two buckets
          const size_t s = size_t(bs[rng() & 1]) * ns + rng() % ns;
          for (uint32_t w = 0; w < kw; w++) std::swap(cur[4 - kw + w], (*tab)[s * sw + w]);
          std::swap(code, (*tab)[s * sw + kw]);
        }
      }
      ok = placed;
    }
    if (ok) return true;
  }
  return false;
}

// IPv6 image: the same build over the IPv6 half of the flows (addresses interned as codes), plus
// the LPM tables the kernel maps packet addresses through (appended to the blob, hdr.v6_lpm).
int build_image6(const FeatureNP& np, SlotMap& slots, HostImage* out, bool alloc) {
  *out = HostImage();
  out->codes6 = std::make_shared<V6Codes>();
  V6Codes& codes = *out->codes6;
  int rc = codes.build(np, &out->error);
  if (rc) return rc;
  Gather G;
  G.fam = 6;
  G.codes = &codes;
  for (auto& kv : np.installed()) {
    if ((rc = G.add(kv.second))) {
      out->error = G.error;
      return rc;
    }
  }
  if ((rc = emit(G, np, slots, out, alloc))) return rc;
  // LPM by binary search on prefix lengths (Waldvogel et al.): the table holds every tree node
  // (root excluded: a miss everywhere means code 0) plus, for each node, a marker at every shorter
  // length its binary search passes through, carrying the best matching prefix's code there.
  std::vector<uint32_t> lens;
  for (size_t n = 1; n < codes.nodes.size(); n++) lens.push_back(uint32_t(codes.nodes[n].len));
  std::sort(lens.begin(), lens.end());
  lens.erase(std::unique(lens.begin(), lens.end()), lens.end());
  if (lens.size() > kV6MaxLens) {
    out->error = "too many distinct IPv6 prefix lengths";
    return -GPC_EINVAL;
  }
  auto pad = [](const V6Codes::Node& N) { return N.kids.empty() || N.clen == 0 ? N.code : N.code & prefix_mask(N.clen); };
  std::map<std::pair<u128, uint32_t>, uint32_t> lpm_map;  // (value, len) -> code
  for (size_t n = 1; n < codes.nodes.size(); n++) lpm_map[{codes.nodes[n].v, uint32_t(codes.nodes[n].len)}] = pad(codes.nodes[n]);
  for (size_t n = 1; n < codes.nodes.size(); n++) {
    const auto& P = codes.nodes[n];
    const int t = int(std::lower_bound(lens.begin(), lens.end(), uint32_t(P.len)) - lens.begin());
    int lo = 0, hi = int(lens.size()) - 1;
    while (lo <= hi) {
      const int mid = (lo + hi) / 2;
      if (mid == t) break;
      if (mid > t) {
        hi = mid - 1;
        continue;
      }
      const uint32_t M = lens[size_t(mid)];
      const std::pair<u128, uint32_t> key{P.v & v6_prefix_mask(int(M)), M};
      if (!lpm_map.count(key)) {  // marker: code of the deepest ancestor of P no longer than M
        int a = P.parent;
        while (a > 0 && codes.nodes[size_t(a)].len > int(M)) a = codes.nodes[size_t(a)].parent;
        lpm_map[key] = a > 0 ? pad(codes.nodes[size_t(a)]) : 0u;
      }
      lo = mid + 1;
    }
  }
  // Region tables (core.hpp kV6L1Bits): the tag length c is the longest (c + 16 <= 128) at which the
  // prefixes no shorter than c fall under at most kV6DefaultTags distinct /c blocks (GPC_V6_MAX_TAGS:
  // 1..kV6MaxTags). More tags mean finer regions (shorter searches) and more region-table bytes:
  // C3 in IPv6 (64M packets, profiles/r05j) code launch 3.90 ms with one tag (c = 96), 3.26 ms with
  // four (c = 98), 3.46 ms with sixteen (c = 100). Per tag, every /c+16 region gets the best match no longer than c + 16 (prefixes
  // shorter than c cover whole tags) and the list of longer lengths present under it, plus the
  // markers of that shorter search.
  uint32_t l1_c = 0, n_short = 0;
  bool l1 = codes.nodes.size() > 1;
  std::vector<uint32_t> l1_tab;
  std::vector<u128> tags;
  std::map<u128, uint32_t> tag_ix;
  uint32_t max_tags = kV6DefaultTags;
  if (const char* e = std::getenv("GPC_V6_MAX_TAGS")) max_tags = uint32_t(std::min<long>(kV6MaxTags, std::max<long>(1, std::atol(e))));
  if (l1) {
    int maxlen = 0;
    for (size_t n = 1; n < codes.nodes.size(); n++) maxlen = std::max(maxlen, codes.nodes[n].len);
    l1 = false;
    for (int c = std::min(maxlen, 128 - int(kV6L1Bits)); c >= 1 && !l1; c--) {
      std::set<u128> ts;
      for (size_t n = 1; n < codes.nodes.size() && ts.size() <= max_tags; n++)
        if (codes.nodes[n].len >= c) ts.insert(codes.nodes[n].v & v6_prefix_mask(c));
      if (ts.empty() || ts.size() > max_tags) continue;
      l1 = true;
      l1_c = uint32_t(c);
      tags.assign(ts.begin(), ts.end());
    }
    for (size_t t = 0; t < tags.size(); t++) tag_ix[tags[t]] = uint32_t(t);
  }
  if (l1) {
    const uint32_t s_len = l1_c + kV6L1Bits, nreg = 1u << kV6L1Bits, nt = uint32_t(tags.size());
    auto region = [&](u128 v) { return uint32_t(v >> (128 - s_len)) & (nreg - 1u); };
    auto tag_of = [&](u128 v) { return tag_ix.at(v & v6_prefix_mask(int(l1_c))); };
    std::vector<uint32_t> base(size_t(nt) * nreg, 0u), base_len(size_t(nt) * nreg, 0u);
    std::vector<std::vector<uint32_t>> reg_nodes(size_t(nt) * nreg);  // nodes longer than s_len, per region
    // prefixes shorter than c: the deepest one covering each tag is every region's starting base
    for (uint32_t t = 0; t < nt; t++) {
      uint32_t bc = 0, bl = 0;
      for (size_t n = 1; n < codes.nodes.size(); n++) {
        const auto& N = codes.nodes[n];
        if (uint32_t(N.len) < l1_c && (tags[t] & v6_prefix_mask(N.len)) == N.v && uint32_t(N.len) >= bl) {
          bc = pad(N);
          bl = uint32_t(N.len);
        }
      }
      std::fill(base.begin() + size_t(t) * nreg, base.begin() + size_t(t + 1) * nreg, bc);
      std::fill(base_len.begin() + size_t(t) * nreg, base_len.begin() + size_t(t + 1) * nreg, bl);
    }
    for (size_t n = 1; n < codes.nodes.size(); n++) {
      const auto& N = codes.nodes[n];
      if (uint32_t(N.len) < l1_c) continue;
      const size_t tb = size_t(tag_of(N.v)) * nreg;
      if (uint32_t(N.len) > s_len) {
        reg_nodes[tb + region(N.v)].push_back(uint32_t(n));
        continue;
      }
      // a prefix no longer than c + 16 covers 2^(c+16-len) whole regions of its tag: the deepest wins
      const uint32_t r0 = region(N.v), span = 1u << (s_len - uint32_t(N.len));
      for (uint32_t r = r0; r < r0 + span; r++)
        if (uint32_t(N.len) >= base_len[tb + r]) {
          base[tb + r] = pad(N);
          base_len[tb + r] = uint32_t(N.len);
        }
    }
    // Entries (core.hpp v6_codes): a leaf carries its base and the list of longer lengths present
    // (kV6L1Global past kV6L1MaxLens); a block whose list exceeds kV6LeafLens is split into 256
    // sub-blocks (kV6L1Child) while it is shorter than /128. GPC_V6_LEAF_LENS overrides the split
    // threshold (experiments; 8 = round-5 regions without sub-tables).
    uint32_t leaf_max = kV6LeafLens;
    if (const char* e = std::getenv("GPC_V6_LEAF_LENS")) leaf_max = uint32_t(std::min<long>(kV6L1MaxLens, std::max<long>(0, std::atol(e))));
    l1_tab.assign(size_t(nt) * nreg * 4, 0u);
    std::vector<std::vector<uint32_t>> leaf_L(size_t(nt) * nreg);  // per entry: its search list (leaves)
    size_t n_sub = 0, sub_bytes = 0, n_unsplit = 0;
    size_t sub_budget = std::min(kV6SubMaxBudget, std::max(kV6SubMinBudget, kV6SubBytesPerPrefix * codes.nodes.size()));
    if (const char* e = std::getenv("GPC_V6_SUB_BUDGET_KB")) sub_budget = size_t(std::max<long>(0, std::atol(e))) << 10;
    auto len_ix = [&](uint32_t len) { return uint32_t(std::lower_bound(lens.begin(), lens.end(), len) - lens.begin()); };
    std::function<void(size_t, uint32_t, uint32_t, uint32_t, std::vector<uint32_t>&)> fill =
        [&](size_t ei, uint32_t ll, uint32_t bc, uint32_t bl, std::vector<uint32_t>& ns) {
          std::vector<uint32_t> L;
          for (uint32_t n : ns) L.push_back(len_ix(uint32_t(codes.nodes[n].len)));
          std::sort(L.begin(), L.end());
          L.erase(std::unique(L.begin(), L.end()), L.end());
          const bool over = L.size() > leaf_max && ll < 128u &&
                            sub_bytes + 16ull * (1ull << v6_sub_bits(ll)) > sub_budget;
          n_unsplit += over;
          if (L.size() > leaf_max && ll < 128u && !over) {
            const uint32_t st = v6_sub_bits(ll), sl = ll + st, nsub = 1u << st;
            const size_t child = l1_tab.size() / 4;
            l1_tab.resize(l1_tab.size() + 4 * size_t(nsub), 0u);
            leaf_L.resize(l1_tab.size() / 4);
            n_sub++;
            sub_bytes += 16ull * nsub;
            l1_tab[4 * ei + 1] = kV6L1Child;
            l1_tab[4 * ei + 2] = uint32_t(4 * child);
            std::vector<uint32_t> sb(nsub, bc), sbl(nsub, bl);
            std::vector<std::vector<uint32_t>> sn(nsub);
            auto sub = [&](u128 v) { return uint32_t(v >> (128 - sl)) & (nsub - 1u); };
            for (uint32_t n : ns) {
              const auto& N = codes.nodes[n];
              if (uint32_t(N.len) > sl) {
                sn[sub(N.v)].push_back(n);
                continue;
              }
              const uint32_t s0 = sub(N.v), span = 1u << (sl - uint32_t(N.len));
              for (uint32_t q = s0; q < s0 + span; q++)
                if (uint32_t(N.len) >= sbl[q]) {
                  sb[q] = pad(N);
                  sbl[q] = uint32_t(N.len);
                }
            }
            for (uint32_t q = 0; q < nsub; q++) fill(child + q, sl, sb[q], sbl[q], sn[q]);
            return;
          }
          l1_tab[4 * ei] = bc;
          if (L.size() > kV6L1MaxLens) {
            l1_tab[4 * ei + 1] = kV6L1Global;
            return;
          }
          l1_tab[4 * ei + 1] = uint32_t(L.size());
          for (size_t q = 0; q < L.size(); q++) l1_tab[4 * ei + 2 + q / 4] |= L[q] << (8 * (q % 4));
          leaf_L[ei] = std::move(L);
        };
    for (size_t r = 0; r < size_t(nt) * nreg; r++) fill(r, s_len, base[r], base_len[r], reg_nodes[r]);
    // markers of the regional searches: each node longer than its leaf's block, along the leaf's list
    for (size_t n = 1; n < codes.nodes.size(); n++) {
      const auto& P = codes.nodes[n];
      if (uint32_t(P.len) <= s_len) continue;
      size_t ei = size_t(tag_of(P.v)) * nreg + region(P.v);
      uint32_t ll = s_len;
      while (l1_tab[4 * ei + 1] & kV6L1Child) {
        const uint32_t st = v6_sub_bits(ll);
        ll += st;
        ei = l1_tab[4 * ei + 2] / 4 + (uint32_t(P.v >> (128 - ll)) & ((1u << st) - 1u));
      }
      if (uint32_t(P.len) <= ll || (l1_tab[4 * ei + 1] & kV6L1Global)) continue;  // folded into the base / global search
      const auto& L = leaf_L[ei];
      const uint32_t li = len_ix(uint32_t(P.len));
      const int t = int(std::lower_bound(L.begin(), L.end(), li) - L.begin());
      int lo = 0, hi = int(L.size()) - 1;
      while (lo <= hi) {
        const int mid = (lo + hi) / 2;
        if (mid == t) break;
        if (mid > t) {
          hi = mid - 1;
          continue;
        }
        const uint32_t M = lens[L[size_t(mid)]];
        const std::pair<u128, uint32_t> key{P.v & v6_prefix_mask(int(M)), M};
        if (!lpm_map.count(key)) {
          int a = P.parent;
          while (a > 0 && codes.nodes[size_t(a)].len > int(M)) a = codes.nodes[size_t(a)].parent;
          lpm_map[key] = a > 0 ? pad(codes.nodes[size_t(a)]) : 0u;
        }
        lo = mid + 1;
      }
    }
    // markers of the searches of addresses under no tag: over the lengths shorter than c only
    n_short = uint32_t(std::lower_bound(lens.begin(), lens.end(), l1_c) - lens.begin());
    for (size_t n = 1; n < codes.nodes.size(); n++) {
      const auto& P = codes.nodes[n];
      if (uint32_t(P.len) >= l1_c) continue;
      const int t = int(len_ix(uint32_t(P.len)));
      int lo = 0, hi = int(n_short) - 1;
      while (lo <= hi) {
        const int mid = (lo + hi) / 2;
        if (mid == t) break;
        if (mid > t) {
          hi = mid - 1;
          continue;
        }
        const uint32_t M = lens[size_t(mid)];
        const std::pair<u128, uint32_t> key{P.v & v6_prefix_mask(int(M)), M};
        if (!lpm_map.count(key)) {
          int a = P.parent;
          while (a > 0 && codes.nodes[size_t(a)].len > int(M)) a = codes.nodes[size_t(a)].parent;
          lpm_map[key] = a > 0 ? pad(codes.nodes[size_t(a)]) : 0u;
        }
        lo = mid + 1;
      }
    }
    if (std::getenv("GPC_IMAGE_DEBUG"))
      std::fprintf(stderr, "IPv6 sub-region tables: %zu (%.1f MB of a %.1f MB budget; %zu blocks left unsplit)\n", n_sub,
                   double(sub_bytes) / 1e6, double(sub_budget) / 1e6, n_unsplit);
    if (std::getenv("GPC_IMAGE_DEBUG"))
      std::fprintf(stderr, "IPv6 region tables: c = %u, %u tags\n", l1_c, nt);
  }
  // one table per length (core.hpp V6Len), appended after the V6Lpm block
  std::vector<std::vector<std::pair<std::array<uint32_t, 4>, uint32_t>>> per_len(lens.size());
  for (auto& kv : lpm_map) {
    const u128 v = kv.first.first;
    const uint32_t a[4] = {uint32_t(v >> 96), uint32_t(v >> 64), uint32_t(v >> 32), uint32_t(v)};
    const size_t li = size_t(std::lower_bound(lens.begin(), lens.end(), kv.first.second) - lens.begin());
    std::array<uint32_t, 4> r;
    v6_key(a, kv.first.second, r.data());
    per_len[li].push_back({r, kv.second});
  }
  auto& b = out->blob;
  while (b.size() % 16) b.push_back(0u);
  const uint32_t lpm = uint32_t(b.size());
  V6Lpm L{};
  L.n_lens = uint32_t(lens.size());
  const size_t lw = (sizeof(V6Lpm) / 4 + 15) / 16 * 16;
  b.resize(b.size() + lw, 0u);
  size_t tab_words = 0;
  for (size_t i = 0; i < lens.size(); i++) {
    L.lens[i] = lens[i];
    std::vector<uint32_t> tab;
    if (!v6_len_table_build(lens[i], per_len[i], &L.d[i], &tab)) {
      out->error = "IPv6 LPM table construction failed";
      return -GPC_ENOMEM;
    }
    L.d[i].tab_off = uint32_t(b.size());
    b.insert(b.end(), tab.begin(), tab.end());
    tab_words += tab.size();
  }
  if (l1) {
    while (b.size() % 16) b.push_back(0u);
    L.l1_off = uint32_t(b.size());
    L.l1_c = l1_c;
    L.n_tags = uint32_t(tags.size());
    L.n_short = n_short;
    for (size_t t = 0; t < tags.size(); t++) {
      const u128 tv = tags[t];
      const uint32_t tg[4] = {uint32_t(tv >> 96), uint32_t(tv >> 64), uint32_t(tv >> 32), uint32_t(tv)};
      if (l1_c) v6_key(tg, l1_c, L.l1_tag[t]);
    }
    b.insert(b.end(), l1_tab.begin(), l1_tab.end());
    tab_words += l1_tab.size();
  }
  std::memcpy(b.data() + lpm, &L, sizeof L);
  out->hdr.v6_lpm = lpm;
  out->bytes_hash += 4ull * tab_words;
  out->v6_code_bits = uint32_t(codes.max_clen);
  out->v6_prefixes = uint32_t(codes.nodes.size() - 1);
  return GPC_OK;
}

int extend_image6(const FeatureNP& np, const std::set<uint32_t>& conj, uint8_t hard_tables, HostImage* img, Journal* j6) {
  if (!img->codes6 || !img->hdr.v6_lpm) return -GPC_EINVAL;
  V6Codes& codes = *img->codes6;
  const std::vector<uint32_t>& b = img->blob;
  const V6Lpm& L = *reinterpret_cast<const V6Lpm*>(b.data() + img->hdr.v6_lpm);
  auto words = [](u128 v, uint32_t len, uint32_t* m) {
    const uint32_t a[4] = {uint32_t(v >> 96), uint32_t(v >> 64), uint32_t(v >> 32), uint32_t(v)};
    v6_mask(a, len, m);
  };
  auto in_base = [&](const uint32_t* m, uint32_t len) { return v6_base_has(b.data(), img->hdr.v6_lpm, m, len); };
  // new LPM entries go to the overflow table of the IPv6 journal (never into the published base)
  const size_t before = img->v6_ovf.size();
  auto put = [&](u128 v, uint32_t len, uint32_t code) {
    std::array<uint32_t, 5> key;
    words(v, len, key.data());
    key[4] = len;
    if (in_base(key.data(), len) || img->v6_ovf.count(key)) return;
    img->v6_ovf[key] = code;
  };
  std::vector<uint32_t> lens(L.lens, L.lens + L.n_lens);
  auto take = [&](const IPMatch& f) -> int {
    if (!f.set || f.addr.fam != 6) return GPC_OK;
    const int len = f.plen < 0 ? 128 : f.plen;
    if (len <= 0) return GPC_OK;
    const u128 v = v6_value(f.addr) & v6_prefix_mask(len);
    if (codes.find(v, len) >= 0) return GPC_OK;
    const int id = codes.add_leaf(v, len);
    if (id < 0) {
      if (std::getenv("GPC_IMAGE_DEBUG"))
        std::fprintf(stderr, "IPv6 prefix %016llx%016llx/%d: %s\n", (unsigned long long)(v >> 64), (unsigned long long)v, len,
                     codes.why_not(v, len));
      return -GPC_EINVAL;
    }
    const V6Codes::Node& N = codes.nodes[size_t(id)];
    // the prefix itself, then a marker at every shorter length its binary search passes through
    // (build_image6), carrying the code of its deepest ancestor no longer than that length; a new
    // length is probed directly after the search (no markers)
    const int t = int(std::lower_bound(lens.begin(), lens.end(), uint32_t(len)) - lens.begin());
    put(v, uint32_t(len), N.code);
    if (codes.new_lens.count(len)) return GPC_OK;
    if (t >= int(lens.size()) || lens[size_t(t)] != uint32_t(len)) return -GPC_EINVAL;
    int lo = 0, hi = int(lens.size()) - 1;
    while (lo <= hi) {
      const int mid = (lo + hi) / 2;
      if (mid == t) break;
      if (mid > t) {
        hi = mid - 1;
        continue;
      }
      const uint32_t M = lens[size_t(mid)];
      int a = N.parent;
      while (a > 0 && codes.nodes[size_t(a)].len > int(M)) a = codes.nodes[size_t(a)].parent;
      put(v & v6_prefix_mask(int(M)), M, a > 0 ? codes.nodes[size_t(a)].code : 0u);
      lo = mid + 1;
    }
    return GPC_OK;
  };
  int rc = GPC_OK;
  auto scan = [&](const Flow& f) {
    if (f.table < TB_AP_EGRESS || f.table > TB_INGRESS_DEFAULT || rc) return;
    for (const IPMatch* m : {&f.m.nw_src, &f.m.nw_dst, &f.m.ct_nw_src, &f.m.ct_nw_dst})
      if (!rc) rc = take(*m);
  };
  for (uint32_t c : conj) {
    auto it = np.policies().find(c);
    if (it == np.policies().end()) continue;
    for (Clause* cl : it->second->clauses())
      for (auto& kv : cl->matches)
        if (kv.second->flow) scan(*kv.second->flow);
  }
  for (auto& kv : np.hard_flows())
    if ((hard_tables >> (kv.second.table - 1)) & 1u) scan(kv.second);
  if (rc) return rc;
  img->v6_prefixes = uint32_t(codes.nodes.size() - 1);
  if (img->v6_ovf.size() != before) {  // a new overflow table for this epoch's journal header
    std::vector<std::array<uint32_t, 8>> sl;
    sl.reserve(img->v6_ovf.size());
    for (auto& kv : img->v6_ovf)
      sl.push_back({kv.first[0], kv.first[1], kv.first[2], kv.first[3], kv.first[4] | kV6Valid, kv.second, 0u, 0u});
    std::vector<uint32_t> tab;
    uint32_t lg = 0;
    if (!v6_hash_build(sl, 0.5, &tab, &lg)) return -GPC_ENOMEM;
    uint32_t packed = 0, k = 0;  // JournalHdr.v6_ovf_log2: the new lengths above the log2 byte
    for (int l : codes.new_lens) packed |= uint32_t(l) << (8 * ++k);
    j6->set_v6_overflow(std::move(tab), lg | packed);
  }
  return GPC_OK;
}

// Rule-centric gather of the current versions of `conj` (uninstalled ones are skipped) plus every
// hard flow of the tables in `hard_tables` (bit t-1 = table t).
static int gather_rules(const FeatureNP& np, const std::set<uint32_t>& conj, uint8_t hard_tables, Gather* G) {
  int rc = GPC_OK;
  for (uint32_t c : conj) {
    auto it = np.policies().find(c);
    if (it == np.policies().end()) continue;  // uninstalled: tombstone only
    const Conjunction& cj = *it->second;
    for (Clause* cl : cj.clauses())
      for (auto& kv : cl->matches)
        if (kv.second->flow && !rc) {
          auto act = kv.second->actions.find(c);
          if (act != kv.second->actions.end())
            rc = G->add_soft(*kv.second->flow, c, act->second.clause_id, act->second.n_clause);
        }
    for (auto& f : cj.action_flows)
      if (!rc) rc = G->add(f);
    for (auto& f : cj.metric_flows)
      if (!rc) rc = G->add(f);
  }
  for (auto& kv : np.hard_flows())
    if (!rc && ((hard_tables >> (kv.second.table - 1)) & 1u)) rc = G->add(kv.second);
  return rc;
}

// ------------------------------------------------------------------------------------- journal
namespace {

void set_bit(std::vector<uint32_t>& bm, uint32_t i, std::set<uint32_t>* dirty_pages) {
  if (bm.size() <= i / 32) bm.resize(i / 32 + 1, 0u);
  bm[i / 32] |= 1u << (i % 32);
  dirty_pages->insert(i >> kDeadPageShift);
}

// Bucket key values an atom covers in the journal (core.hpp jkey); false = always chain.
bool journal_keys(const AtomKey& k, std::vector<uint32_t>* out) {
  out->clear();
  if (k.axis <= AX_CTDST) {
    const uint32_t sh = ip_band_shift(k.band);
    if ((uint64_t(k.hi >> sh) - (k.lo >> sh)) >= kMaxBucketsPerAtom) return false;
    for (uint64_t t = k.lo >> sh; t <= (k.hi >> sh); t++) out->push_back(uint32_t(t));
  } else if (k.axis == AX_L4D || k.axis == AX_L4S) {
    const uint32_t a = jkey(k.axis, 0, k.lo), b = jkey(k.axis, 0, k.hi);
    for (uint32_t t = a; t <= b; t++) out->push_back(t);
  } else {
    for (uint64_t v = k.lo; v <= k.hi; v++) out->push_back(uint32_t(v));
  }
  return true;
}

}  // namespace

// Chain-head table size: chains are per head bucket, so a journal of many entries needs many heads
// (a composite-keyed journal lists a rule once per key and value). 16 bits for small bases, up to 21
// (1 M heads, 16 K head pages; the page table travels with every epoch: 64 KB) for C3-sized ones.
constexpr uint32_t kJournalLgMin = 16, kJournalLgMax = 20;

void Journal::reset(const HostImage* base, uint32_t lg) {
  base_ = base;
  if (!lg) {
    uint32_t mx = kJournalLgMax;
    if (const char* e = std::getenv("GPC_JOURNAL_LG_MAX"))  // (experiments)
      mx = uint32_t(std::min(24, std::max(int(kJournalLgMin), std::atoi(e))));
    lg = kJournalLgMin;
    while (lg < mx && base && (uint64_t(1) << lg) < uint64_t(base->n_rids) * 16) lg++;
  }
  lg_ = lg;
  pool.assign(16, 0u);  // offset 0 is "none"
  uploaded = 0;
  hdr_off = 0;
  n_versions = n_live = 0;
  any_noact = false;
  bloom_axes_ = 0;
  heads_.assign(size_t(1) << lg_, 0u);
  pt_.assign((size_t(1) << lg_) / kJPageHeads, 0u);
  bdead_.clear();
  odead_.clear();
  bpt_.clear();
  opt_.clear();
  bdirty_.clear();
  odirty_.clear();
  live_.clear();
  for (int t = 0; t < 6; t++) {
    hard_orids_[t].clear();
    hard_offs_[t].clear();
  }
  std::memset(tables_, 0, sizeof tables_);
  ovf_table_.clear();
  ovf_off_ = ovf_log2_ = 0;
  ovf_dirty_ = false;
  ext_.clear();
  ext_values_ = ext_off_ = 0;
  ext_entries_ = 0;
  touched_.clear();
  touched_hard_ = 0;
  ext_force_ = false;
  ext_dirty_.clear();
  extd_.clear();
  extb_ = ExtHdr{};
  extb_ents_.clear();
  extb_tomb_.clear();
  extb_pres_.clear();
  extb_dead_ = 0;
  journaled_ = false;
  pt_off_ = bdead_pt_off_ = odead_pt_off_ = 0;
}

int Journal::rebuild(const FeatureNP& np, SlotMap& slots, std::string* err) {
  if (fam_ != 4) return -GPC_EINVAL;  // (the IPv6 journal's overflow tables are not carried over)
  Journal j;
  j.fam_ = fam_;
  j.reset(base_, lg_);
  // Extensions and base tombstones carry over as they are (their base records did not change):
  // only the journaled rules are gathered and written again -- hundreds, not the ~8 k rules C5
  // mixed touches (re-applying every touched rule took 170-230 ms per collection).
  j.ext_ = ext_;
  j.ext_values_ = ext_values_;
  j.ext_entries_ = ext_entries_;
  j.ext_force_ = !ext_.empty();
  j.bdead_ = bdead_;
  for (size_t w = 0; w < bdead_.size(); w++)
    if (bdead_[w]) {
      j.bdirty_.insert(uint32_t((w * 32) >> kDeadPageShift));
      j.journaled_ = true;
    }
  j.any_noact = any_noact;
  j.touched_ = touched_;
  j.touched_hard_ = touched_hard_;
  std::set<uint32_t> live;
  for (auto& kv : live_) live.insert(kv.first);
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = j.apply(np, slots, live, touched_hard_, err);
  if (rc) return rc;
  if (std::getenv("GPC_COMPACT_DEBUG"))
    std::fprintf(stderr, "pool collection: apply of %zu live rules + extension index %.1f ms\n", live.size(),
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  // the old host mirror (hundreds of MB) is released off the control thread: unmapping it took
  // tens of ms of the collection's commit
  std::thread([old = std::move(pool)]() mutable { std::vector<uint32_t>().swap(old); }).detach();
  *this = std::move(j);
  return GPC_OK;
}

uint32_t Journal::n_dead_versions() const {
  uint32_t n = 0;
  for (uint32_t w : odead_) n += uint32_t(__builtin_popcount(w));
  return n;
}

uint32_t Journal::n_tombstones() const {
  uint32_t n = 0;
  for (uint32_t w : bdead_) n += uint32_t(__builtin_popcount(w));
  for (uint32_t w : odead_) n += uint32_t(__builtin_popcount(w));
  return n;
}

uint32_t Journal::append(const uint32_t* w, size_t n, size_t align) {
  while (pool.size() % align) pool.push_back(0u);
  const uint32_t off = uint32_t(pool.size());
  pool.insert(pool.end(), w, w + n);
  return off;
}

// Point extensions per rule (core.hpp ExtHdr): at most kExtMaxRuleValues added values per rule and
// kExtMaxValues in all (past them a rule takes the journal; the compactor folds them into a base).
constexpr size_t kExtMaxRuleValues = 256, kExtMaxValues = size_t(1) << 20;
constexpr size_t kExtMaxXValues = 64, kExtPresBits = 8, kExtMaxIntervals = 4;
// index entries of one extended rule (emit_ext): per value, one per x (composite) and interval (exact)
template <class R>
static size_t ext_entries_of(const R& e) {
  return e.values.size() * std::max<size_t>(1, e.xv.size()) * std::max<size_t>(1, e.ivs.size());
}  // composite keys up to this many x values per rule (else plain)

// The index of every live point extension, appended to the pool per epoch in two levels (nothing
// published is rewritten). The bulk level B holds every extended rule's entries as of its last
// rebuild and is appended only then; the delta level D holds the entries of the rules changed since
// (re-appended every epoch, small), and a bitmap over B's entries tombstones those rules' B entries.
// B is rebuilt once D passes max(kExtDeltaMin, B / kExtDeltaFrac) entries or half of B is dead.
// Per epoch: the presence bitmap of B and D (one bitmap: a packet still settles with one load),
// D, the tombstones and the header. C5 mixed (80 k entries with composite keys): ~0.3 MB per commit
// instead of 1.3 MB re-emitting everything. Returns the ExtHdr offset (0: no extensions).
constexpr size_t kExtDeltaMin = 4096, kExtDeltaFrac = 8;
uint32_t Journal::emit_ext() {
  const auto te0 = std::chrono::steady_clock::now();
  struct Report {
    std::chrono::steady_clock::time_point t;
    const Journal* j;
    ~Report() {
      if (std::getenv("GPC_EXT_TIMING"))
        std::fprintf(stderr, "emit_ext: %.2f ms (%zu entries)\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count(), j->ext_entries_);
    }
  } report{te0, this};
  for (uint32_t c : ext_dirty_) {  // the changed rules leave B (their entries go to D, if any)
    auto it = extb_ents_.find(c);
    if (it != extb_ents_.end()) {
      for (uint32_t i : it->second) extb_tomb_[i >> 5] |= 1u << (i & 31u);
      extb_dead_ += uint32_t(it->second.size());
      extb_ents_.erase(it);
    }
    if (ext_.count(c)) extd_.insert(c);
    else extd_.erase(c);
  }
  ext_dirty_.clear();
  if (ext_.empty()) {
    extb_ = ExtHdr{};
    extb_ents_.clear();
    extb_tomb_.clear();
    extb_pres_.clear();
    extd_.clear();
    extb_dead_ = 0;
    return 0;
  }
  struct E {
    uint32_t hs, w[kExtEntWords], conj;
  };
  auto entries_of = [](uint32_t c, const ExtRule& e, uint32_t* axes, std::vector<E>* out) {
    for (auto& av : e.values) {
      const uint32_t meta = ext_meta(e.table, av.first, e.clause);
      if (e.xv.empty()) {
        out->push_back({ext_hash(e.table, av.first, av.second), {av.second, meta, e.rec_off, e.prio, 0u, 0u, 0u, c}, c});
        axes[e.table - 1] |= 1u << av.first;
      } else if (e.ivs.empty()) {  // composite, the record verifies the third clause
        for (uint32_t x : e.xv)
          out->push_back({ext_hash_x(e.table, av.first, av.second, x),
                          {av.second, meta | kExtComposite, e.rec_off, e.prio, x, 0u, 0u, c}, c});
        axes[e.table - 1] |= 1u << (16 + av.first);
      } else {  // composite and exact: one entry per (x, interval)
        const uint32_t m = meta | kExtComposite | kExtExact | (e.iax << 11);
        for (uint32_t x : e.xv)
          for (auto& iv : e.ivs)
            out->push_back({ext_hash_x(e.table, av.first, av.second, x), {av.second, m, e.rec_off, e.prio, x, iv.first, iv.second, c}, c});
        axes[e.table - 1] |= 1u << (16 + av.first);
      }
    }
  };
  // one level: entries bucket-sorted (half a bucket per entry); returns offsets / entries in the pool
  auto put_level = [&](std::vector<E>& es, uint32_t* bkt_off, uint32_t* bkt_log2, uint32_t* ent_off) {
    uint32_t lg = 6;
    while (lg < 22 && (uint64_t(2) << lg) < uint64_t(es.size())) lg++;
    const uint32_t mask = (1u << lg) - 1u;
    std::stable_sort(es.begin(), es.end(), [mask](const E& a, const E& b) { return (a.hs & mask) < (b.hs & mask); });
    std::vector<uint32_t> offs((size_t(1) << lg) + 1, 0u), ents;
    for (const E& e : es) offs[(e.hs & mask) + 1]++;
    for (size_t b = 0; b + 1 < offs.size(); b++) offs[b + 1] += offs[b];
    ents.reserve(es.size() * kExtEntWords);
    for (const E& e : es) ents.insert(ents.end(), e.w, e.w + kExtEntWords);
    *bkt_log2 = lg;
    *bkt_off = append(offs.data(), offs.size(), 16);
    *ent_off = ents.empty() ? *bkt_off : append(ents.data(), ents.size(), 16);
  };
  size_t dn = 0;
  for (uint32_t c : extd_) {
    dn += ext_entries_of(ext_.at(c));
  }
  const char* dmin_env = std::getenv("GPC_EXT_DELTA_MIN");  // (tests: rebuild B often)
  const size_t dmin = dmin_env ? size_t(std::strtoul(dmin_env, nullptr, 10)) : kExtDeltaMin;
  const bool rebase = std::getenv("GPC_EXT_ONE_LEVEL") || !extb_.b_n ||
                      dn > std::max(dmin, size_t(extb_.b_n) / kExtDeltaFrac) || extb_dead_ * 2 > extb_.b_n;
  if (rebase) {  // B := every extended rule; D empty
    std::vector<E> es;
    es.reserve(ext_entries_);
    ExtHdr b{};
    for (auto& kv : ext_) entries_of(kv.first, kv.second, b.axes, &es);
    // presence sized for B and the D it may grow before the next rebuild
    b.pres_log2 = 12;
    const uint64_t cap = es.size() + std::max(dmin, es.size() / kExtDeltaFrac);
    while (b.pres_log2 < 24 && (uint64_t(1) << b.pres_log2) < cap * kExtPresBits) b.pres_log2++;
    extb_pres_.assign(size_t(1) << (b.pres_log2 - 5), 0u);
    for (const E& e : es) {
      const uint32_t pb = e.hs >> (32u - b.pres_log2);
      extb_pres_[pb >> 5] |= 1u << (pb & 31u);
    }
    put_level(es, &b.b_bkt_off, &b.b_bkt_log2, &b.b_ent_off);
    b.b_n = uint32_t(es.size());
    extb_ents_.clear();
    for (uint32_t i = 0; i < uint32_t(es.size()); i++) extb_ents_[es[i].conj].push_back(i);
    extb_tomb_.assign((es.size() + 31) / 32 + 1, 0u);
    extb_dead_ = 0;
    extd_.clear();
    extb_ = b;
  }
  ExtHdr h = extb_;  // B's level, presence size and axes
  std::vector<E> ds;
  ds.reserve(dn);
  for (uint32_t c : extd_) entries_of(c, ext_.at(c), h.axes, &ds);
  std::vector<uint32_t> pres = extb_pres_;
  for (const E& e : ds) {
    const uint32_t pb = e.hs >> (32u - h.pres_log2);
    pres[pb >> 5] |= 1u << (pb & 31u);
  }
  h.n = uint32_t(ds.size());
  if (h.n) put_level(ds, &h.bkt_off, &h.bkt_log2, &h.ent_off);
  h.pres_off = append(pres.data(), pres.size(), 16);
  h.b_tomb_off = append(extb_tomb_.data(), extb_tomb_.size(), 16);
  return append(reinterpret_cast<const uint32_t*>(&h), sizeof h / 4, 16);
}

int Journal::apply(const FeatureNP& np, SlotMap& slots, const std::set<uint32_t>& conj, uint8_t hard_tables,
                   std::string* err, bool alloc) {
  // 0. current versions of the changed rules
  Gather G;
  G.fam = fam_;
  G.codes = fam_ == 6 ? base_->codes6.get() : nullptr;
  if (fam_ == 6 && !G.codes) {
    *err = "IPv6 journal without a prefix tree";
    return -GPC_EINVAL;
  }
  touched_.insert(conj.begin(), conj.end());
  touched_hard_ |= hard_tables;
  int rc = gather_rules(np, conj, hard_tables, &G);
  if (rc) {
    *err = G.error;
    return rc;
  }
  // 1. point extensions: a rule whose new version is its base record plus exact values on one
  // clause keeps the base record (core.hpp ExtHdr); a rule back at its base version drops its
  // extension. Every other changed rule takes the journal (jconj).
  const bool ext_off = std::getenv("GPC_NO_EXTENSIONS") != nullptr;  // (experiments, A/B tests)
  bool ext_changed = false;
  std::set<uint32_t> jconj;
  auto extend = [&](uint32_t c) {
    if (fam_ != 4 || ext_off || live_.count(c)) return false;
    auto b = base_->base_rules.find(c);
    if (b == base_->base_rules.end()) return false;
    auto rid = base_->conj_rid.find(c);  // a tombstoned base record (an earlier uninstall) stays dead
    if (rid == base_->conj_rid.end() ||
        (rid->second / 32 < bdead_.size() && ((bdead_[rid->second / 32] >> (rid->second % 32)) & 1u)))
      return false;
    const BaseRule& br = b->second;
    auto it = G.soft[br.table].find(c);
    if (it == G.soft[br.table].end()) return false;
    for (int t = 1; t <= 6; t++)
      if (t != int(br.table) && G.soft[t].count(c)) return false;
    RuleB& r = it->second;
    if (!r.prio_set || !r.has_act) return false;
    for (int k = 0; k < r.n; k++)
      if (r.clause[k].empty()) return false;
    auto pit = np.policies().find(c);
    r.tier = pit != np.policies().end() ? uint8_t(std::max(0, std::min(255, pit->second->tier))) : 0;
    const bool is_deny = r.verdict == RV_DROP || r.verdict == RV_REJECT;
    r.counted = r.has_act && ((r.verdict == RV_ALLOW && G.counted_allow.count(c)) || (is_deny && G.counted_deny.count(c)));
    uint32_t slot = 0;
    const bool counted = r.counted && slots.lookup(c, alloc, &slot);
    if (rule_sig(r, counted, slot) != br.sig) return false;
    ExtRule e;
    e.table = br.table;
    e.rec_off = br.rec_off;
    e.prio = r.prio;
    int kx = -1;
    for (int k = 0; k < r.n; k++) {
      std::vector<std::pair<uint64_t, const Atom*>> now;
      now.reserve(r.clause[k].size());
      for (const Atom& a : r.clause[k]) now.push_back({atom_hash(a), &a});
      std::sort(now.begin(), now.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
      static const std::vector<uint64_t> kNone;
      const std::vector<uint64_t>& was = br.atoms[k] ? *br.atoms[k] : kNone;
      size_t j = 0;
      for (size_t i = 0; i < now.size(); i++) {
        if (i && now[i].first == now[i - 1].first) continue;
        while (j < was.size() && was[j] < now[i].first) return false;  // a base atom is gone
        if (j < was.size() && was[j] == now[i].first) {
          j++;
          continue;
        }
        const Atom& a = *now[i].second;  // added: must be one exact value on one axis
        if (a.t.size() != 1 || a.t[0].mask != 0xffffffffu || a.t[0].axis >= AX_N || (kx >= 0 && kx != k)) return false;
        kx = k;
        e.values.push_back({a.t[0].axis, a.t[0].val});
      }
      if (j != was.size()) return false;
    }
    std::sort(e.values.begin(), e.values.end());
    auto old = ext_.find(c);
    const size_t had = old == ext_.end() ? 0 : old->second.values.size();
    if (kx < 0) {  // the base version again
      if (old != ext_.end()) {
        ext_values_ -= uint32_t(had);
        ext_entries_ -= ext_entries_of(old->second);
        ext_.erase(old);
        ext_dirty_.insert(c);
        ext_changed = true;
      }
      return true;
    }
    e.clause = uint32_t(kx);
    const TableHdr& th = base_->hdr.t[e.table - 1];
    if (th.n_cidx && uint32_t(kx) == th.cband && !std::getenv("GPC_EXT_PLAIN")) {  // composite keys
      for (const Atom& a : r.clause[1 - th.cband]) {
        if (a.t.size() != 1 || a.t[0].axis != th.cx || a.t[0].mask != 0xffffffffu) {
          e.xv.clear();
          break;
        }
        e.xv.push_back(a.t[0].val);
      }
      std::sort(e.xv.begin(), e.xv.end());
      e.xv.erase(std::unique(e.xv.begin(), e.xv.end()), e.xv.end());
      if (e.xv.size() > kExtMaxXValues) e.xv.clear();
      // exact entries: nothing else to verify, or a third clause of at most kExtMaxIntervals
      // intervals on one axis (one entry per interval)
      e.conj = c;
      if (!e.xv.empty() && r.n == 2) {
        e.ivs = {{0u, 0u}};
      } else if (!e.xv.empty() && r.n == 3 && !std::getenv("GPC_EXT_NO_EXACT")) {
        const auto& cl = r.clause[2];
        std::vector<std::pair<uint32_t, uint32_t>> ivs;
        if (!cl.empty() && cl[0].t.size() == 1 && cl[0].t[0].axis < AX_N &&
            clause_intervals(cl, cl[0].t[0].axis, &ivs) && ivs.size() <= kExtMaxIntervals) {
          e.iax = cl[0].t[0].axis;
          e.ivs = std::move(ivs);
        }
      }
    }
    if (e.values.size() > kExtMaxRuleValues || ext_values_ - had + e.values.size() > kExtMaxValues) return false;
    if (old != ext_.end() && old->second == e) return true;
    ext_values_ = uint32_t(ext_values_ - had + e.values.size());
    if (old != ext_.end()) ext_entries_ -= ext_entries_of(old->second);
    ext_entries_ += ext_entries_of(e);
    ext_[c] = std::move(e);
    ext_dirty_.insert(c);
    ext_changed = true;
    return true;
  };
  for (uint32_t c : conj) {
    if (extend(c)) continue;
    jconj.insert(c);
    auto old = ext_.find(c);
    if (old != ext_.end()) {
      ext_values_ -= uint32_t(old->second.values.size());
      ext_entries_ -= ext_entries_of(old->second);
      ext_.erase(old);
      ext_dirty_.insert(c);
      ext_changed = true;
    }
  }
  if (hard_tables) journaled_ = true;  // (rules: once a tombstone or a record is written, below)
  if (std::getenv("GPC_IMAGE_DEBUG") && (!jconj.empty() || hard_tables)) {
    std::fprintf(stderr, "journal: %zu rules, hard tables 0x%x:", jconj.size(), unsigned(hard_tables));
    for (uint32_t c : jconj) {
      int in_t = 0;
      for (int t = 1; t <= 6; t++)
        if (G.soft[t].count(c)) in_t = t;
      std::fprintf(stderr, " %u(table %d, base %d)", c, in_t, int(base_->base_rules.count(c)));
    }
    std::fprintf(stderr, "\n");
  }
  // 2. tombstones: every earlier copy of a rule that takes the journal (base or journal)
  for (uint32_t c : jconj) {
    auto it = live_.find(c);
    if (it != live_.end()) {
      set_bit(odead_, it->second, &odirty_);
      live_.erase(it);
      n_live--;
      journaled_ = true;
    }
    auto b = base_->conj_rid.find(c);
    if (b != base_->conj_rid.end()) {
      set_bit(bdead_, b->second, &bdirty_);
      journaled_ = true;
    }
  }
  for (int t = 0; t < 6; t++) {
    if (!((hard_tables >> t) & 1u)) continue;
    for (uint32_t o : hard_orids_[t]) set_bit(odead_, o, &odirty_);
    hard_orids_[t].clear();
    hard_offs_[t].clear();
    for (uint32_t rid : base_->hard_rids[t]) set_bit(bdead_, rid, &bdirty_);
  }
  // 3. current versions of the journal's rules
  uint64_t span[AX_N];  // interval prefilter choice: price hulls against the whole axis
  for (int a = 0; a < AX_N; a++) span[a] = 1ull << 32;
  std::set<uint32_t> dirty_pages;
  std::vector<uint32_t> keys;
  for (int t = 1; t <= 6; t++) {
    std::vector<RuleB*> rs;
    for (auto& kv : G.soft[t]) {
      RuleB& r = kv.second;
      if (!r.prio_set || !jconj.count(r.conj_id)) continue;
      bool complete = true;
      for (int k = 0; k < r.n; k++) complete &= !r.clause[k].empty();
      if (!complete) continue;
      auto pit = np.policies().find(r.conj_id);
      r.tier = pit != np.policies().end() ? uint8_t(std::max(0, std::min(255, pit->second->tier))) : 0;
      const bool is_deny = r.verdict == RV_DROP || r.verdict == RV_REJECT;
      r.counted = r.has_act && ((r.verdict == RV_ALLOW && G.counted_allow.count(r.conj_id)) ||
                                (is_deny && G.counted_deny.count(r.conj_id)));
      if (!r.has_act) {
        any_noact = true;
        *err = "rule without an IPv4 conj_id flow";
        return -GPC_EINVAL;
      }
      rs.push_back(&r);
    }
    if ((hard_tables >> (t - 1)) & 1u)
      for (auto& kv : G.hard[t])
        if (!kv.second.clause[0].empty()) rs.push_back(&kv.second);
    std::stable_sort(rs.begin(), rs.end(), [](const RuleB* a, const RuleB* b) {  // hard list in rank order
      if (a->prio != b->prio) return a->prio > b->prio;
      if (a->hard != b->hard) return a->hard;
      if (a->hard) return a->verdict < b->verdict;
      return a->conj_id < b->conj_id;
    });
    for (RuleB* rp : rs) {
      RuleB& r = *rp;
      if (n_versions >= (1u << (32 - kJOridShift))) {
        *err = "journal rule ids exhausted";
        return -GPC_ENOMEM;
      }
      const uint32_t orid = n_versions++;
      journaled_ = true;
      // record: header, clauses, then this record's out-of-line segment data
      std::vector<uint32_t> rec(kRecLine, 0u), ext;
      std::vector<std::pair<uint32_t, uint32_t>> patches;  // (record word, ext offset)
      std::vector<std::pair<uint32_t, uint32_t>> inl;      // (record word, record word of the data)
      uint32_t offs[3] = {0, 0, 0};
      for (int k = 0; k < r.n; k++) {
        std::vector<PendingSeg> ps;
        clause_segments(r.clause[k], &ps);
        for (auto& sg : ps)
          if (sg.kind == SK_HASH) sg.kind = SK_PTS;  // no point hash in the journal (sorted points)
        std::vector<std::pair<uint32_t, uint32_t>> cp;
        std::vector<uint32_t> cw = encode_clause(ps, &ext, &cp);
        if (rec.size() > 255) {
          *err = "rule record too large";
          return -GPC_EINVAL;
        }
        offs[k] = uint32_t(rec.size());
        for (auto& pt : cp) patches.push_back({uint32_t(rec.size()) + pt.first, pt.second});
        const Fcd f = fast_clause(ps);  // fast descriptor (core.hpp FastKind)
        rec[kRecFcd + 3 * k] = f.a;
        rec[kRecFcd + 3 * k + 1] = f.b;
        rec[kRecFcd + 3 * k + 2] = f.c;
        if (f.data == 0) inl.push_back({kRecFcd + 3 * uint32_t(k) + 1, offs[k] + 2});
        if (f.data == 1) {
          if (cp.size() != 1) {
            *err = "fast clause descriptor: external segment without its patch";
            return -GPC_EINVAL;
          }
          patches.push_back({kRecFcd + 3 * uint32_t(k) + 1, cp[0].second});
        }
        rec.insert(rec.end(), cw.begin(), cw.end());
      }
      while (rec.size() % 16) rec.push_back(0u);
      const uint32_t ext_at = uint32_t(rec.size());
      rec.insert(rec.end(), ext.begin(), ext.end());
      for (int i = 0; i < 16; i++) rec.push_back(0u);  // chunk reads past the last array (core.hpp rule_match)
      while (pool.size() % 16) pool.push_back(0u);
      const uint32_t base_off = uint32_t(pool.size());
      for (auto& pt : patches) rec[pt.first] = base_off + ext_at + pt.second;
      for (auto& pt : inl) rec[pt.first] = base_off + pt.second;
      rec[0] = r.hard ? 0u : r.conj_id;
      rec[1] = uint32_t(r.prio) | (uint32_t(r.act_prio) << 16);
      uint32_t slot = 0;
      const bool counted = !r.hard && r.counted && slots.lookup(r.conj_id, alloc, &slot);
      rec[2] = (r.verdict & 7u) | ((r.hard ? 1u : 0u) << 3) | ((r.has_act ? 1u : 0u) << 4) | ((counted ? 1u : 0u) << 5) |
               (uint32_t(r.n & 3) << 6) | (offs[0] << 8) | (offs[1] << 16) | (offs[2] << 24);
      rec[3] = slot;
      rec[4] = uint32_t(r.tier) | (orid << 8);
      rec[5] = (!r.hard && r.pin) ? kRecPacketIn : 0u;
      const uint32_t off = append(rec.data(), rec.size(), 16);
      if (r.hard) {
        hard_orids_[t - 1].push_back(orid);
        hard_offs_[t - 1].push_back(off);
        continue;
      }
      live_[r.conj_id] = orid;
      n_live++;
      // driver entries for clauses 0 and 1. A table with a composite base index walks only its band
      // clause, keyed by (band key, composite value) (core.hpp jxkey): one entry per key and value of
      // the rule's other clause; a rule whose other clause is not such a value set goes to the always
      // list of the band clause.
      JournalTable& jt = tables_[t - 1];
      const TableHdr& bt = base_->hdr.t[t - 1];
      std::vector<uint32_t> xs;
      bool xok = false;
      if (bt.n_cidx && r.n >= 2) {
        xok = r.clause[1 - bt.cband].size() <= kCompositeMaxValues;
        for (auto& a : r.clause[1 - bt.cband]) {
          xok = xok && a.t.size() == 1 && a.t[0].mask == 0xffffffffu && a.t[0].axis == bt.cx;
          if (xok) xs.push_back(a.t[0].val);
        }
      }
      for (int k = 0; k < 2 && k < r.n; k++) {
        if (bt.n_cidx && k != bt.cband) continue;  // the kernel never walks the other clause's chains
        const std::array<uint32_t, 4> pf = entry_of(r, k, 0u, span);
        bloom_axes_ |= bloom_axis_bit(pf[0]) | kBloomL4;
        for (auto& a : r.clause[k]) {
          AtomKey key;
          bool keyed = (!bt.n_cidx || xok) && atom_key(a, &key);
          // a composite base that merged its IP bands (build_composite merge_bands: C3 / C4 key
          // every prefix at band 0) keys the journal the same way: one chain per (band key, value)
          // for the packet to walk instead of one per band. Single addresses (band kIpBands - 1:
          // the Pod IPs AddPolicyRuleAddress adds) keep their own band: merged, every /32 of a Pod
          // subnet shared one chain per value (C5 mixed: 6.9 matching entries per packet, 0.1 apart)
          if (keyed && bt.n_cidx && key.axis <= AX_CTDST && key.band + 1u < kIpBands && !std::getenv("GPC_JOURNAL_NO_MERGE"))
            for (uint32_t i = 0; i < bt.n_cidx && i < uint32_t(kIdxPerClause); i++)
              if (bt.cidx[i].axis == key.axis && bt.cidx[i].band < key.band) key.band = bt.cidx[i].band;
          keyed = keyed && journal_keys(key, &keys);
          if (!keyed) {
            const uint32_t e[kJEntWords] = {jt.always[k], 0u, (orid << kJOridShift), off, pf[0] & 0xffu, pf[1], pf[2], pf[3]};
            const uint32_t eo = append(e, kJEntWords, kJEntWords);
            if (eo / kJEntWords >= (1u << 24)) {
              *err = "journal pool exceeds 24-bit entry offsets";
              return -GPC_ENOMEM;
            }
            jt.always[k] = (eo / kJEntWords) | (std::min(255u, (jt.always[k] >> 24) + 1u) << 24);
            continue;
          }
          const uint32_t kind = uint32_t(key.axis) | (uint32_t(key.band) << 4);
          bool have = false;
          for (uint32_t i = 0; i < jt.n_kinds[k]; i++) have |= jt.kinds[k][i] == kind;
          if (!have) {
            if (jt.n_kinds[k] >= 8) {
              *err = "too many journal bucket kinds";
              return -GPC_EINVAL;
            }
            jt.kinds[k][jt.n_kinds[k]++] = uint8_t(kind);
          }
          const uint32_t meta = jmeta(uint32_t(t), uint32_t(k), key.axis, key.band);
          if (bt.n_cidx) {  // (band key, value) keys
            std::vector<uint32_t> kx;
            kx.reserve(keys.size() * xs.size());
            for (uint32_t kv : keys)
              for (uint32_t x : xs) kx.push_back(jxkey(kv, x));
            keys.swap(kx);
          }
          for (uint32_t kv : keys) {
            const uint32_t bkt = jbucket(meta, kv, lg_);
            const uint32_t e[kJEntWords] = {heads_[bkt], kv, meta | (orid << kJOridShift), off, pf[0] & 0xffu, pf[1], pf[2], pf[3]};
            const uint32_t eo = append(e, kJEntWords, kJEntWords);
            if (eo / kJEntWords >= (1u << 24)) {
              *err = "journal pool exceeds 24-bit entry offsets";
              return -GPC_ENOMEM;
            }
            heads_[bkt] = (eo / kJEntWords) | (std::min(255u, (heads_[bkt] >> 24) + 1u) << 24);
            dirty_pages.insert(bkt / kJPageHeads);
          }
        }
      }
    }
  }
  // 4. copy-on-write head pages, then this epoch's page table (the previous one when no head page
  // changed: an epoch that only moves point extensions appends no 64-KB page table), bitmaps, the
  // extension index and the header
  for (uint32_t pg : dirty_pages) pt_[pg] = append(&heads_[size_t(pg) * kJPageHeads], kJPageHeads, kJPageHeads);
  JournalHdr h{};
  h.lg = lg_;
  if (!dirty_pages.empty() || !pt_off_) pt_off_ = append(pt_.data(), pt_.size(), 16);
  h.pt_off = pt_off_;
  // tombstone bitmaps: changed 8192-bit pages copied on write, then this epoch's page tables
  auto publish = [&](std::vector<uint32_t>& bm, std::vector<uint32_t>& pt, std::set<uint32_t>& dirty, uint32_t n_ids,
                     uint32_t* last) {
    if (bm.empty()) return 0u;
    const size_t n_pages = size_t(n_ids >> kDeadPageShift) + 1;
    if (dirty.empty() && *last && pt.size() >= n_pages) return *last;
    if (pt.size() < n_pages) pt.resize(n_pages, 0u);
    bm.resize(std::max(bm.size(), n_pages * kDeadPageWords), 0u);
    for (uint32_t pg : dirty) pt[pg] = append(&bm[size_t(pg) * kDeadPageWords], kDeadPageWords, kDeadPageWords);
    dirty.clear();
    *last = append(pt.data(), pt.size(), 16);
    return *last;
  };
  if (ext_changed || ext_force_) {
    ext_force_ = false;
    ext_off_ = emit_ext();
  }
  h.ext_off = std::getenv("GPC_DEBUG_HIDE_EXT") ? 0u : ext_off_;  // (timing experiments only: wrong verdicts)
  h.jflags = journaled_ ? kJUsed : 0u;
  h.bloom_axes = bloom_axes_;
  if (ovf_dirty_) {
    ovf_off_ = append(ovf_table_.data(), ovf_table_.size(), 16);
    ovf_dirty_ = false;
  }
  h.v6_ovf_off = ovf_off_;
  h.v6_ovf_log2 = ovf_log2_;
  h.bdead_off = publish(bdead_, bpt_, bdirty_, base_->n_rids, &bdead_pt_off_);
  h.odead_off = publish(odead_, opt_, odirty_, n_versions, &odead_pt_off_);
  for (int t = 0; t < 6; t++) {
    h.t[t] = tables_[t];
    if (!hard_offs_[t].empty()) {
      h.t[t].hard_off = append(hard_offs_[t].data(), hard_offs_[t].size(), 4);
      h.t[t].n_hard = uint32_t(hard_offs_[t].size());
    }
    const JournalTable& jt = h.t[t];
    if (jt.n_kinds[0] || jt.n_kinds[1] || (jt.always[0] & 0xffffffu) || (jt.always[1] & 0xffffffu) || jt.n_hard)
      h.live |= 1u << t;
  }
  if (std::getenv("GPC_DEBUG_HIDE_JOURNAL")) {  // (timing experiments only: wrong verdicts)
    h.live = 0;
    h.bdead_off = h.odead_off = 0;
  }
  hdr_off = append(reinterpret_cast<const uint32_t*>(&h), sizeof h / 4, 16);
  return GPC_OK;
}

namespace {

int emit(Gather& G, const FeatureNP& np, SlotMap& slots, HostImage* out, bool alloc) {
  PhaseTimer T_;
  auto& soft = G.soft;
  auto& hard = G.hard;
  auto& counted_allow = G.counted_allow;
  auto& counted_deny = G.counted_deny;
  out->n_flows = G.n_flows;
  out->hdr.live = 0;
  AtomSetInterner atom_sets;
  // ---- 2. per table: rank, emit records, driver indexes
  Blob B;
  B.w.reserve(1 << 20);
  for (int i = 0; i < 16; i++) B.w.push_back(0);  // keep offset 0 unused
  std::vector<uint64_t> hash_keys;
  // point sets (core.hpp set_key), interned over the image: rules sharing an AddressGroup share keys
  std::map<std::pair<uint8_t, std::vector<uint32_t>>, uint32_t> point_sets;
  auto intern_set = [&](uint8_t axis, const std::vector<uint32_t>& pts) -> uint32_t {
    auto it = point_sets.find({axis, pts});
    if (it != point_sets.end()) return it->second;
    const uint32_t sid = uint32_t(point_sets.size());
    if (sid >= kPointSetMax) return 0u;
    const uint32_t hi = set_key_hi(sid, axis);
    point_sets.emplace(std::make_pair(axis, pts), hi);
    for (uint32_t v : pts) hash_keys.push_back(set_key(hi, v));
    return hi;
  };
  uint32_t next_rid = 0;
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
    if (!rs.empty()) out->hdr.live |= 1u << (t - 1);
    // value span of the exact axes over this table's soft rules (interval prefilter selectivity)
    uint64_t span[AX_N] = {0};
    {
      uint32_t mn[AX_N], mx[AX_N];
      for (int a = 0; a < AX_N; a++) mn[a] = 0xffffffffu, mx[a] = 0;
      for (RuleB* rp : rs)
        if (!rp->hard)
          for (int c = 0; c < rp->n; c++)
            for (auto& at : rp->clause[c])
              for (auto& t : at.t) {
                mn[t.axis] = std::min(mn[t.axis], t.val & t.mask);
                mx[t.axis] = std::max(mx[t.axis], (t.val & t.mask) | ~t.mask);
              }
      for (int a = 0; a < AX_N; a++) span[a] = mx[a] >= mn[a] ? uint64_t(mx[a]) - mn[a] + 1 : 0;
    }

    T_.lap(0);
    // records (rank order), then this table's external data
    std::vector<uint32_t> rec_off(rs.size());
    const uint32_t tbl_start = uint32_t(B.w.size());
    std::vector<uint32_t> ext;
    std::vector<std::pair<uint32_t, uint32_t>> abs_patches;  // (absolute record word, ext offset)
    std::vector<uint32_t> hard_offs;
    std::vector<HardFast> hard_fast;
    bool hard_fits = true;
    for (size_t rank = 0; rank < rs.size(); rank++) {
      RuleB& r = *rs[rank];
      uint32_t rid = next_rid++;
      if (rid >= (1u << 23)) {
        out->error = "too many rules for the point-hash key";
        return -GPC_EINVAL;
      }
      // encode clauses, smallest first in the record
      std::vector<std::vector<uint32_t>> cw(r.n);
      std::vector<std::vector<std::pair<uint32_t, uint32_t>>> cp(r.n);
      Fcd fcd[3];
      uint32_t mk2[3][4] = {};  // FK_MKN with two boxes: their (value, mask) terms (inline hard rules)
      for (int k = 0; k < r.n; k++) {
        std::vector<PendingSeg> ps;
        clause_segments(r.clause[k], &ps);
        r.set_hi[k] = 0;
        for (auto& sg : ps)
          if (sg.kind == SK_HASH) {
            sg.key_hi = intern_set(sg.axis, sg.data);
            if (!sg.key_hi) {
              out->error = "too many distinct point sets";
              return -GPC_EINVAL;
            }
            r.set_hi[k] = sg.key_hi;
          }
        cw[k] = encode_clause(ps, &ext, &cp[k]);
        fcd[k] = fast_clause(ps);
        if ((fcd[k].a & 15u) == FK_MKN && (fcd[k].a >> 8) == 2u) {
          const std::vector<uint32_t>& bx = ps[0].data;
          mk2[k][0] = bx[0], mk2[k][1] = bx[3], mk2[k][2] = bx[kBoxWords], mk2[k][3] = bx[kBoxWords + 3];
        }
      }
      std::vector<int> order(r.n);
      for (int k = 0; k < r.n; k++) order[k] = k;
      std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cw[a].size() < cw[b].size(); });
      B.align(16);
      uint32_t base = uint32_t(B.w.size());
      std::vector<uint32_t> rec(kRecLine, 0);
      uint32_t offs[3] = {0, 0, 0};
      for (int k : order) {
        if (rec.size() > 255) {
          out->error = "rule record too large";
          return -GPC_EINVAL;
        }
        offs[k] = uint32_t(rec.size());
        for (auto& pt : cp[k]) abs_patches.push_back({base + uint32_t(rec.size()) + pt.first, pt.second});
        rec.insert(rec.end(), cw[k].begin(), cw[k].end());
      }
      for (int k = 0; k < r.n; k++) {  // fast descriptors (core.hpp FastKind)
        rec[kRecFcd + 3 * k] = fcd[k].a;
        rec[kRecFcd + 3 * k + 1] = fcd[k].data == 0 ? base + offs[k] + 2 : fcd[k].b;
        rec[kRecFcd + 3 * k + 2] = fcd[k].c;
        if (fcd[k].data == 1) {
          if (cp[k].size() != 1) {
            out->error = "fast clause descriptor: external segment without its patch";
            return -GPC_EINVAL;
          }
          abs_patches.push_back({base + kRecFcd + 3 * uint32_t(k) + 1, cp[k][0].second});
        }
      }
      rec[0] = r.hard ? 0 : r.conj_id;
      rec[1] = uint32_t(r.prio) | (uint32_t(r.act_prio) << 16);
      uint32_t slot = 0;
      const bool counted = !r.hard && r.counted && slots.lookup(r.conj_id, alloc, &slot);
      uint32_t flags = (r.verdict & 7u) | ((r.hard ? 1u : 0u) << 3) | ((r.has_act ? 1u : 0u) << 4) | ((counted ? 1u : 0u) << 5) |
                       (uint32_t(r.n & 3) << 6);
      rec[2] = flags | (offs[0] << 8) | (offs[1] << 16) | (offs[2] << 24);
      rec[3] = slot;
      rec[4] = uint32_t(r.tier) | (rid << 8);
      rec[5] = r.hard ? 0u : (skip_mask(r, 0, span) | (skip_mask(r, 1, span) << 3) | (r.pin ? kRecPacketIn : 0u));
      if (base >= (1u << 28)) {  // Ent.x holds record offset / 16 in 24 bits
        out->error = "rule records exceed 1 GiB";
        return -GPC_ENOMEM;
      }
      rec_off[rank] = base;
      B.w.insert(B.w.end(), rec.begin(), rec.end());
      if (r.hard) {
        // inline copy for TableHdr.hf (core.hpp HardFast), if every clause has a one-word kind
        HardFast hf{};
        bool fits = true;
        int n_mk2 = 0;
        hf.pv = uint32_t(r.prio) | ((uint32_t(r.verdict) & 0xffu) << 16) | (uint32_t(r.n) << 24);
        hf.roff = base;
        hf.rid = rid;
        for (int k = 0; k < r.n; k++) {
          const uint32_t kind = fcd[k].a & 15u;
          hf.d[3 * k] = fcd[k].a, hf.d[3 * k + 1] = fcd[k].b, hf.d[3 * k + 2] = fcd[k].c;
          if (kind == FK_MKN && (fcd[k].a >> 8) == 2u && n_mk2++ == 0) {
            hf.d[3 * k] = (fcd[k].a & 0xf0u) | FK_MK2;
            for (int j = 0; j < 4; j++) hf.mk[j] = mk2[k][j];
          } else if (kind != FK_ALWAYS && kind != FK_IV1 && kind != FK_MK1 && kind != FK_HASH) {
            fits = false;
          }
        }
        hard_fast.push_back(hf);
        hard_fits = hard_fits && fits;
        hard_offs.push_back(base);
        out->hard_rids[t - 1].push_back(rid);
      } else {
        out->conj_rid[r.conj_id] = rid;
        if (!r.has_act) out->any_noact = true;
        if (G.fam == 4) {  // what a later point extension of this rule is checked against
          BaseRule& br = out->base_rules[r.conj_id];
          br.table = uint32_t(t);
          br.rec_off = base;
          br.sig = rule_sig(r, counted, slot);
          for (int k = 0; k < r.n; k++) br.atoms[k] = atom_sets.intern(clause_hashes(r.clause[k]));
        }
      }
    }
    B.align(16);
    th.end_off = uint32_t(B.w.size()) + 1;
    uint32_t ext_base = uint32_t(B.w.size());
    out->bytes_records += 4ull * (ext_base - tbl_start);
    out->bytes_ext += 4ull * ext.size();
    B.w.insert(B.w.end(), ext.begin(), ext.end());
    for (auto& pt : abs_patches) B.w[pt.first] = ext_base + pt.second;
    th.n_hard = uint32_t(hard_offs.size());
    th.hard_off = hard_offs.empty() ? 0 : B.put(hard_offs.data(), hard_offs.size(), 1);
    th.n_hfast = 0;
    if (hard_fits && !hard_fast.empty() && hard_fast.size() <= kHardFast && !std::getenv("GPC_NO_HARD_INLINE")) {
      th.n_hfast = uint32_t(hard_fast.size());
      for (size_t h = 0; h < hard_fast.size(); h++) th.hf[h] = hard_fast[h];
    }
    build_bits(rs, rec_off, th, B);
    if (std::getenv("GPC_IMAGE_DEBUG"))
      std::fprintf(stderr, "table %d: %zu rules, %u hard (%u inline)\n", t, rs.size(), th.n_hard, th.n_hfast);
    T_.lap(1);
    // composite driver first: a table that has one never scans the plain sub-indexes, so they are
    // not emitted (only the always lists, which the composite driver scans too)
    build_composite(rs, rec_off, span, t, th, B, out);
    const bool composite = th.n_cidx != 0;
    // driver indexes for clauses 0 and 1 of the soft rules; entries carry the non-driver filter
    for (int k = 0; k < 2; k++) {
      std::vector<std::array<uint32_t, 4>> always;
      std::map<std::pair<uint8_t, uint8_t>, std::vector<std::pair<AtomKey, std::array<uint32_t, 4>>>> sub;
      for (size_t rank = 0; rank < rs.size(); rank++) {
        RuleB& r = *rs[rank];
        if (r.hard || k >= r.n) continue;
        std::array<uint32_t, 4> ent = entry_of(r, k, rec_off[rank], span);
        for (auto& a : r.clause[k]) {
          AtomKey key;
          if (!atom_key(a, &key)) {
            always.push_back(ent);
            out->hdr.bloom_axes |= bloom_axis_bit(ent[0]) | kBloomL4;
            continue;
          }
          sub[{key.axis, key.band}].push_back({key, ent});
          // (a composite table emits no plain sub-index entry: only what it emits needs filter bits)
          if (!composite) out->hdr.bloom_axes |= bloom_axis_bit(ent[0]) | kBloomL4;
        }
      }
      // Host addresses get the exact band only where they dominate the axis (Pod / AddressGroup
      // members); a few /32 among CIDRs ride in band 3 (/28 keys) and save the packet a lookup.
      for (uint8_t ax = 0; ax <= AX_CTDST; ax++) {
        auto h = sub.find({ax, uint8_t(4)});
        if (h == sub.end()) continue;
        size_t on_axis = 0;
        for (uint8_t b = 0; b < kIpBands; b++) {
          auto it = sub.find({ax, b});
          if (it != sub.end()) on_axis += it->second.size();
        }
        if (h->second.size() * 4 >= on_axis) continue;
        auto& b3 = sub[{ax, uint8_t(3)}];
        for (auto& e : h->second) {
          e.first.band = 3;
          b3.push_back(e);
        }
        sub.erase(h);
      }
      std::vector<std::pair<size_t, std::pair<uint8_t, uint8_t>>> order;
      if (composite) sub.clear();  // keyed atoms are all in the composite sub-indexes
      for (auto& kv : sub) order.push_back({kv.second.size(), kv.first});
      std::sort(order.rbegin(), order.rend());
      th.n_idx[k] = 0;
      std::vector<uint32_t> bks;
      for (size_t i = 0; i < order.size(); i++) {
        auto& v = sub[order[i].second];
        if (i >= size_t(kIdxPerClause)) {
          for (auto& e : v) always.push_back(e.second);
          continue;
        }
        uint8_t axis = order[i].second.first, band = order[i].second.second;
        uint32_t bits = 16;
        if (axis <= AX_CTDST) {
          if (band == 0) bits = 12;
          if (band >= 2) {  // hashed bands: about one bucket per entry
            uint64_t ent = 0;
            for (auto& e : v) ent += atom_span(e.first);
            bits = 10;
            while (bits < 22 && (1ull << bits) < ent) bits++;
          }
        }
        std::vector<std::pair<uint32_t, std::array<uint32_t, 4>>> be;  // (bucket, entry)
        for (auto& e : v) {
          atom_bucket_list(e.first, bits, &bks);
          for (uint32_t b : bks) be.push_back({b, e.second});
        }
        std::sort(be.begin(), be.end());
        be.erase(std::unique(be.begin(), be.end()), be.end());
        uint32_t nb = 1u << bits;
        std::vector<uint32_t> offs(size_t(nb) + 1, 0), ents;
        ents.reserve(4 * be.size());
        for (auto& e : be) offs[e.first + 1]++;
        for (uint32_t b = 0; b < nb; b++) offs[b + 1] += offs[b];
        for (auto& e : be) ents.insert(ents.end(), e.second.begin(), e.second.end());
        SubIdx& si = th.idx[k][th.n_idx[k]++];
        si.axis = axis;
        si.band = band;
        si.bits = uint8_t(bits);
        si.fmt = 0;  // offset pairs (bucket directories: composite sub-indexes)
        si.off = B.put(offs.data(), offs.size(), 16);
        si.ent = ents.empty() ? si.off : B.put(ents.data(), ents.size(), 16);
        si.pres = 0;
        out->bytes_bucket_offsets += 4ull * offs.size();
        if (std::getenv("GPC_IMAGE_DEBUG"))
          std::fprintf(stderr, "table %d clause %d axis %u band %u bits %u atoms %zu entries %zu\n", t, k, axis, band, bits,
                       v.size(), be.size());
        out->bytes_entries += 4ull * ents.size();
      }
      std::sort(always.begin(), always.end());
      always.erase(std::unique(always.begin(), always.end()), always.end());
      std::vector<uint32_t> aw;
      for (auto& e : always) aw.insert(aw.end(), e.begin(), e.end());
      th.always_n[k] = uint32_t(always.size());
      th.always_off[k] = always.empty() ? 0 : B.put(aw.data(), aw.size(), 16);
      out->bytes_entries += 4ull * aw.size();
    }
    out->n_rules[t - 1] = th.n_rules;
    out->n_hard[t - 1] = th.n_hard;
  }
  T_.lap(2);
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
  out->bytes_hash = 8ull * tab.size();
  out->hdr.n_slots = slots.size();
  out->hdr.isc = G.isc;
  out->n_rids = next_rid;
  T_.lap(3);
  T_.report("emit");
  B.align(16);
  for (int i = 0; i < 16; i++) B.w.push_back(0);  // core.hpp rule_match reads 4 words per clause
  out->blob = std::move(B.w);
  return GPC_OK;
}

}  // namespace

}  // namespace gpc
