// Device classification image + per-packet evaluation (shared by the gfx950 kernel and the
// test-only host emulation in tests/csrc). See DESIGN.md §3 for the algorithm.
//
// Semantics restated (per rule table, per packet): OVS classifier_lookup__ with conjunctive
// matches (lib/classifier.c, OVS 2.17.7): H = best hard (non-conjunctive) flow; a conjunction can
// win only at a priority strictly above H; the highest completed conjunction (lowest conj id on a
// tie) wins, and its conj_id action flow (or H, if H has a higher priority) is the table verdict.
// Antrea's compile invariant -- every clause flow of conjunction `id` has the rule's priority
// (network_policy.go:866-889) -- lets the image store one record per conjunction ("rule") whose
// clauses are OR-lists of match atoms, instead of per-priority flow lists.
//
// Image = one uint32 blob. Per rule table: RuleRec[] sorted by (priority desc, hard first, id asc),
// clause segments (sorted interval lists, point-hash references, generic masked boxes) and a
// driver index per clause 0/1: bucket -> ranks, so a packet only visits rules that can match.
#pragma once

#include <stdint.h>

#include "gpc.h"

#if defined(__HIPCC__)
#define GPC_HD __host__ __device__ __forceinline__
#else
#define GPC_HD inline
#endif
// Wave-uniform loop condition: any lane of the wavefront still has work (host emulation: this lane).
#if defined(__HIP_DEVICE_COMPILE__)
#define GPC_WAVE_ANY(c) __any(c)
#else
#define GPC_WAVE_ANY(c) (c)
#endif

// Image words read at wave-uniform addresses (the hard pseudo-rules of a table: the same records for
// every lane) go through the constant address space, so the compiler issues scalar loads (K$, the
// scalar-memory counter) that overlap the lanes' vector loads instead of queueing behind them.
#if defined(__HIP_DEVICE_COMPILE__)
#define GPC_CONST_AS __attribute__((address_space(4)))
#else
#define GPC_CONST_AS
#endif

namespace gpc {

typedef GPC_CONST_AS uint32_t cword;  // an image word read at a wave-uniform address

// Packet axes (all 32-bit; IPv4 image).
enum Axis : uint8_t {
  AX_SRC = 0,    // nw_src
  AX_DST = 1,    // nw_dst
  AX_CTSRC = 2,  // ct_nw_src
  AX_CTDST = 3,  // ct_nw_dst
  AX_INPORT = 4, // in_port
  AX_REG1 = 5,   // reg1 TargetOFPortField
  AX_REG7 = 6,   // reg7 ServiceGroupIDField
  AX_TUN = 7,    // tun_id (label identity)
  AX_L4D = 8,    // nw_proto << 16 | tp_dst   (ICMP: code)
  AX_L4S = 9,    // nw_proto << 16 | tp_src   (ICMP: type)
  AX_CTST = 10,  // ct_state bits
  AX_N = 11
};

// Per-rule record: uint32 words, 16-word (64-B) aligned, laid out in rank order, so a record's
// word offset orders rules exactly like their rank (priority desc, hard first, conj id asc).
//   w0 conj_id (0 for hard pseudo-rules)
//   w1 priority | act_priority << 16
//   w2 flags byte (RecFlags) | off0 << 8 | off1 << 16 | off2 << 24   (word offsets of the clauses)
//   w3 counter slot
//   w4 tier | rid << 8                                               (rid: image-wide rule id)
//   w5 clauses decided exactly by a passing driver entry: bits 0-2 (driver clause 0), 3-5 (1);
//      bit 8 (kRecPacketIn): the action flow sends the packet to the controller (GPC_VFLAG_PACKETIN)
// clause k at word off_k: nseg, then nseg segments, each a tag word kind | axis << 4 | n << 8
// followed by its data:
//   SK_IVAL  2n words, sorted disjoint [lo,hi]     SK_XIVAL  1 word: offset of the 2n words
//   SK_PTS   n words, sorted points                SK_XPTS   1 word: offset of the n words
//   SK_BOX   7n words (val[3], mask[3], axes|nt)   SK_XBOX   1 word: offset of the 7n words
//   SK_HASH  1 word: the high word of the clause's point-set keys (set_key). The clause's values on
//            `axis` live in the image-wide point hash -- clauses that are large sets of exact values
//            (AddressGroup members, Pod ofports); driver entries probe it during the candidate scan
//   SK_ALWAYS
enum SegKind : uint8_t { SK_ALWAYS = 0, SK_IVAL = 1, SK_PTS = 2, SK_HASH = 3, SK_BOX = 4, SK_XIVAL = 5, SK_XPTS = 6, SK_XBOX = 7 };
enum RuleKind : uint8_t { RK_SOFT = 0, RK_HARD = 1 };
// What the table walk does with a rule's verdict.
enum RVerdict : uint8_t { RV_MISS = 1, RV_ALLOW = 2, RV_DROP = 3, RV_REJECT = 4, RV_ISO_DROP = 5, RV_BYPASS = 6, RV_PASS = 7 };
// w2 flag byte: verdict (bits 0-2) | kind (3) | has action flow (4) | counted (5) | n_clauses (6-7)
GPC_HD uint32_t rec_verdict(uint32_t w2) { return w2 & 7u; }
GPC_HD uint32_t rec_hard(uint32_t w2) { return (w2 >> 3) & 1u; }
GPC_HD uint32_t rec_has_act(uint32_t w2) { return (w2 >> 4) & 1u; }
GPC_HD uint32_t rec_counted(uint32_t w2) { return (w2 >> 5) & 1u; }
GPC_HD uint32_t rec_nclauses(uint32_t w2) { return (w2 >> 6) & 3u; }
GPC_HD uint32_t rec_off(uint32_t w2, uint32_t k) { return (w2 >> (8 + 8 * k)) & 0xffu; }
constexpr uint32_t kRecHdrWords = 6;
constexpr uint32_t kRecPacketIn = 1u << 8;
constexpr uint32_t kBoxWords = 7;
// Fast clause descriptors (round 4): words kRecFcd + 3k .. + 2 of the record's first 64-B line
// describe clause k in a shape the kernel checks with straight-line code instead of interpreting
// its segment list (image.cpp fast_clause). A = kind | axis << 4 | n << 8, then B, C by kind:
//   FK_GENERIC  several segments or multi-field boxes: clause_match at the clause offset
//   FK_ALWAYS   every packet
//   FK_IV1      B <= v <= C (one interval, a CIDR, a port range, one point)
//   FK_MK1      (v & C) == B (one masked term: ct_state, masked tun_id)
//   FK_HASH     the image-wide point hash holds (record, axis, v)
//   FK_IVN      n >= 2 sorted disjoint intervals (lo, hi) at word B of the blob
//   FK_PTN      n >= 2 sorted points at word B
//   FK_MKN      n single-term boxes (kBoxWords each: value at +0, mask at +3) at word B
// Clause data (the segment lists) starts at word kRecLine. Arrays a descriptor points at are
// followed by at least 16 readable words (a final chunk reads up to kChunkQuads x 16 B from its
// window start).
enum FastKind : uint32_t { FK_GENERIC = 0, FK_ALWAYS = 1, FK_IV1 = 2, FK_MK1 = 3, FK_HASH = 4, FK_IVN = 5, FK_PTN = 6, FK_MKN = 7 };
constexpr uint32_t kRecFcd = 6;
constexpr uint32_t kRecLine = 16;

constexpr int kMaxClauses = 3;
constexpr int kIdxPerClause = 5;  // sub-indexes (axis, band) per driver clause (more -> always list)

// Driver-index entry (16 B): a prefilter of the rule's NON-driver clauses, so that most candidates
// are rejected without reading the record.
//   x  = record offset / 16 << 8 | interval axis << 4 | Bloom axis          (15 = none)
//        Bloom axis 8 + a (a < 7): "probe" entry -- the non-driver clause on axis a is an SK_HASH
//        point set, so the scan probes the point hash for (record, a, packet value) and the
//        Bloom bits are those of axis a
//   y  = Bloom bits: 0-19 one IP / exact-axis clause on the Bloom axis, 20-31 the service clause
//        (protocol class x tp_dst for single ports, protocol class x 4096-port block for ranges)
//   lo, hi = hull of the most selective non-driver clause on the interval axis
// Both tests are necessary conditions of the clauses, so skipping never changes a verdict.
struct alignas(16) Ent {
  uint32_t x, y, lo, hi;
};
// Exact-value entries (composite driver, round 4): bit 31 of x set -> y is the exact value of the
// table's composite axis cx the entry was listed under (not Bloom bits), and the interval test is
// the rule's service clause when that is one interval; together they decide both non-band
// clauses exactly (record word 5 skips them), so a candidate is verified from its first line alone.
// Record offsets are then < 2^27 words (23 bits of x).
constexpr uint32_t kEntExactX = 1u << 31;
GPC_HD uint32_t ent_off(uint32_t x) { return ((x & ~kEntExactX) >> 8) << 4; }

struct SubIdx {  // one (axis, band) bucket index of a driver clause
  uint8_t axis, band, bits, fmt;
  uint32_t off;   // fmt 0: word offset of 2^bits + 1 bucket offsets (in entries, relative to `ent`);
                  // fmt 1 (composite sub-indexes, round 5): word offset of the bucket directory
  uint32_t ent;   // word offset (multiple of 4) of the Ent entries, ascending record offset per bucket
  uint32_t pres;  // fmt 0 composite sub-indexes: word offset of a 2^bits-bit map of the non-empty
                  // buckets (0: none): the offset pair -- a random line of a 25 MB array -- is
                  // fetched only for the probes that can list a rule.
};
// Bucket directory (SubIdx fmt 1, round 5): per 32 buckets one 16-B block {count bit 0, count bit 1,
// count bit 2, first entry}: bucket b's list starts at first + the counts of the block's earlier
// buckets (three popcounts) and holds its 3-bit count of entries. So one load -- a line of an array
// 1/8 the size of the offset pairs it replaces (C3: ~1 MB per table, L2-resident) -- settles both
// "empty?" and "where", and a probe of a non-empty bucket costs one line miss (its entries) instead
// of two (offset pair, then entries). Count 7: the bucket's first slot is a pointer entry
// {0, overflow index, count, 0} to a list kept after the main entries (lists of 7 or more rules
// under one (key, value): a rare, second dependent load). A zero entry is inert in the scan.
constexpr uint32_t kDirCountMax = 7;  // dir_list below

// An inline hard pseudo-rule (TableHdr.hf): its record's fast descriptors, plus the two (value,
// mask) terms of an FK_MK2 clause (two single-term boxes, e.g. the ct_state bypass flows
// ct_state=-new+est / -new+rel).
constexpr uint32_t kHardFast = 2;
constexpr uint32_t FK_MK2 = 8;  // HardFast only: (v & mk[1]) == mk[0] || (v & mk[3]) == mk[2]
struct HardFast {
  uint32_t pv;    // priority | verdict << 16 | n_clauses << 24
  uint32_t roff;  // record offset (rank bound of the soft scan; point-hash key)
  uint32_t rid;   // rule id (tombstones of delta epochs)
  uint32_t d[3 * kMaxClauses];
  uint32_t mk[4];
};
struct TableHdr {
  uint32_t n_rules, n_hard;
  uint32_t hard_off;  // record offsets of the hard pseudo-rules (ascending)
  uint32_t end_off;   // larger than every record offset of this table ("no hard match")
  uint32_t always_off[2], always_n[2];
  uint32_t n_idx[2];
  SubIdx idx[2][kIdxPerClause];
  // Composite driver (image.cpp build_composite): when every soft rule's clause 1 - cband is a small
  // set of exact values on one axis cx (AppliedTo ofports, Pod IPs), the driver lists of clause cband
  // are also kept keyed by (band key, exact value): sub-index i lists the rules whose clause cband
  // covers the packet's band key AND whose clause 1 - cband holds its cx value. A packet then scans
  // only those (plus clause cband's always list) -- a subset of either plain driver's candidates
  // (up to hash collisions). n_cidx = 0: none.
  uint32_t n_cidx;
  uint8_t cband, cx, pad[2];
  uint32_t xmap_off;  // 2^16-bit map of the cx values any soft rule holds (cx_bit): a packet whose
                      // value is absent has no soft candidate at all (one load, L2-resident)
  SubIdx cidx[kIdxPerClause];
  // Hard pseudo-rules inline (round 4): when the table has at most kHardFast of them and every
  // clause has a one-word fast kind, their descriptors live here and the hard match is decided
  // from the header (scalar loads) without reading any record; n_hfast = 0: the record loop.
  uint32_t n_hfast;
  HardFast hf[kHardFast];
  uint32_t bits_off;  // BitTable of the table's soft rules (0: none), see below
};

// Bit-parallel tables (round 5; north_star piece 4, "clause matches as bitsets ANDed across
// dimensions"): a table of at most kBitRules soft rules whose atoms are single (axis, value, mask)
// terms, on at most kBitProbes distinct (axis, mask, clause) triples, with every hard rule inline.
// Per triple a 2-choice hash maps the packet's masked value to a 32-bit rule mask -- bit i: clause
// k of soft rule i (rank order) holds an atom with that value -- so clause k of rule i holds iff
// bit i of the OR over its triples (or of absent[k]: the rule has no clause k) is set. completed =
// the AND over the clauses, restricted to the rules ranked above the hard match; the best-ranked
// completed rule is the lowest set bit, a tie a second one in its priority level. One round of
// independent 8-B loads replaces the driver lookup, candidate scan and verification rounds.
constexpr uint32_t kBitRules = 32, kBitProbes = 6;
struct BitProbe {
  uint32_t ak;    // axis | clause << 8
  uint32_t mask;  // term mask (key = value & mask)
  uint32_t off;   // word offset of 2^lg slots {key, rule mask} (8 B; an empty slot is {0, 0})
  uint32_t lg;    // <= 16
};
struct BitTable {
  uint32_t n_probe;
  uint32_t absent[kMaxClauses];     // rules without clause k
  uint32_t hard_prefix[kHardFast];  // soft rules ranked above inline hard rule h
  uint32_t pad[2];
  BitProbe probe[kBitProbes];
  uint32_t info[2 * kBitRules];     // soft rule i: record offset, priority | (last index of its level + 1) << 16
};
struct alignas(8) BitSlot {  // {key, rule mask}: one 8-B load
  uint32_t x, y;
};

struct ImageHdr {
  TableHdr t[6];        // AP egress, egress, egress default, AP ingress, ingress, ingress default
  uint32_t hash_off;    // point hash: 2^hash_log2 buckets x kHashSlots uint64 keys (16 B)
  uint32_t hash_log2;
  uint32_t n_slots;
  uint32_t v6_lpm;      // IPv6 image: word offset of its V6Lpm block (0 in IPv4 images)
  uint32_t isc;         // IngressSecurityClassifier bypasses installed (kIsc* bits)
  uint32_t bloom_axes;  // bit a: some driver entry tests the Bloom bits of axis a (Pkt::fm[a] is needed);
                        // kBloomL4: some entry is not an exact-value entry (Pkt::l4m is needed)
  uint32_t live;        // bit t - 1: table t has rules (hard or soft); an empty table is a miss
};
// IngressSecurityClassifier (pipeline.go:2144-2182), from the installed flows: bit d (gpc_dest d =
// gateway 1, tunnel 2, uplink 3) -- packets to that destination skip to IngressMetric; kIscHairpin
// -- ct_mark HairpinCTMark skips to ConntrackCommit. All at one priority, so a packet hitting two of
// them is an overlap of different actions (TIE).
constexpr uint32_t kIscGateway = 1u << GPC_DEST_GATEWAY, kIscTunnel = 1u << GPC_DEST_TUNNEL,
                   kIscUplink = 1u << GPC_DEST_UPLINK, kIscHairpin = 1u << 4;
// 0: the packet takes the ingress policy tables; else RV_BYPASS, | kHTie when two bypasses overlap.
GPC_HD uint32_t ingress_bypass(uint32_t isc, uint32_t dest, uint32_t ct_mark) {
  const bool d = dest != 0 && dest < 4 && ((isc >> dest) & 1u);
  const bool h = (ct_mark & GPC_CT_MARK_HAIRPIN) && (isc & kIscHairpin);
  return (d || h) ? (uint32_t(RV_BYPASS) | ((d && h) ? (1u << 8) : 0u)) : 0u;
}

// Per-packet values the evaluation indexes at run time (axis numbers come from the image): the 11
// axes and the Bloom filter bits of axes 0..7. They live in caller-provided storage, strided: the
// kernel gives each lane a column of a block-wide LDS table laid out [word][lane] (conflict-free,
// explicitly sized, no scratch), the host emulation a plain array (stride 1).
constexpr uint32_t kPktWords = AX_N + 8;
struct PktRef {
  uint32_t* v;
  uint32_t s;
  GPC_HD uint32_t& operator[](uint32_t i) const { return v[size_t(i) * s]; }
};
struct Pkt {
  PktRef ax;     // ax[a]: axis a
  PktRef fm;     // fm[a]: filter bits of axis a < 8 (bits 0-19)
  uint32_t l4m;  // filter bit of (proto class, tp_dst block) (bits 20-31)
  GPC_HD Pkt(uint32_t* store, uint32_t stride) : ax{store, stride}, fm{store + AX_N * stride, stride}, l4m(0) {}
};
// Compiler barrier: values stored to LDS before it are reloaded after it, not forwarded from the
// registers they were stored from (so those registers are free during the code in between).
GPC_HD void lds_reload() { asm volatile("" ::: "memory"); }

// Partial decision of one image for one table, packed (it is live across the table loop):
//   h   = best hard match: priority | verdict << 16 | found << 24 | tie << 25
//   s   = decided soft level: priority | have << 16 | noact << 17 | tie << 18 | image << 19
//         (noact: decided by a completion without an IPv4 conj_id flow, so the hard match wins;
//          tie: more than one completion at the level)
//   win = record offset of the soft winner (have && !noact)
struct TablePart {
  uint32_t h, s, win;
};
constexpr uint32_t kHFound = 1u << 24, kHTie = 1u << 25;
constexpr uint32_t kSHave = 1u << 16, kSNoAct = 1u << 17, kSTie = 1u << 18, kSImg = 1u << 19;

struct TableResult {
  uint8_t verdict;  // RVerdict
  uint8_t tie;
  uint8_t tier;
  uint8_t counted;
  uint32_t conj;
  uint32_t slot;
  uint32_t pin;     // GPC_VFLAG_PACKETIN or 0
  uint32_t prio;    // priority of the deciding flow (action flow of a soft winner, the hard flow; 0: miss)
};

// ------------------------------------------------------------------------------ hashing / buckets
GPC_HD uint32_t mix32(uint32_t x) {  // murmur3 finalizer
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}
GPC_HD uint64_t mix64(uint64_t x) {  // splitmix64 finalizer
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}
GPC_HD uint32_t bit_hash(uint32_t q, uint32_t key) { return mix32(key ^ (q * 0x9e3779b1u + 0x51ed270bu)); }  // BitTable slots
GPC_HD uint32_t proto_class(uint32_t proto) {
  switch (proto) {
    case 6: return 1;
    case 17: return 2;
    case 132: return 3;
    case 1: return 4;
    case 2: return 5;
    case 58: return 6;
    default: return 0;
  }
}
// Bands of the IP axes, by prefix length L: 0 = L 4..12 keyed by the top 12 bits (direct),
// 1 = L 13..16 by the top 16 (direct), 2 = L 17..24 by a hash of the top 20, 3 = L 25..31 by a
// hash of the top 28, 4 = host addresses (L 32) by a hash of the address. An atom is listed under
// every key its prefix covers (at most 2^8, 2^3, 2^3, 2^3, 1 keys); longer prefixes than the key
// share their key's bucket and are checked on verification. Host addresses get their own exact
// band so AddressGroup / Pod members do not share /28 buckets. Exact axes (in_port, reg1, reg7,
// tun) band 0 = low `bits` bits of the value; L4 axes band 0 = proto class x port/8.
constexpr uint32_t kIpBands = 5;
GPC_HD uint32_t ip_band_shift(uint32_t band) {
  return band == 0 ? 20u : band == 1 ? 16u : band == 2 ? 12u : band == 3 ? 4u : 0u;
}
GPC_HD uint32_t bucket_of(uint32_t axis, uint32_t band, uint32_t bits, uint32_t v) {
  if (axis <= AX_CTDST) {
    const uint32_t key = v >> ip_band_shift(band);
    return band < 2 ? key : mix32(key) >> (32 - bits);
  }
  if (axis == AX_L4D || axis == AX_L4S) return (proto_class(v >> 16) << 13) | ((v & 0xffffu) >> 3);
  return v & ((1u << bits) - 1u);
}
// Hash of a composite table's exact value x: the value-map bit and every sub-index bucket of the
// packet derive from this one mix (the compiler computes it once per table: two multiplies, then
// one mix per sub-index -- 32-bit multiplies issue at a quarter of the VALU rate).
GPC_HD uint32_t cx_hash(uint32_t x) { return mix32(x ^ 0x2545f491u); }
// Bit of exact value x in a composite table's value map (TableHdr xmap_off, 2^16 bits).
GPC_HD uint32_t cx_bit(uint32_t x) { return cx_hash(x) >> 16; }
// Composite driver bucket (TableHdr cidx): IP band key of v on (axis, band) with the exact value x.
GPC_HD uint32_t cbucket_of(uint32_t band, uint32_t bits, uint32_t v, uint32_t x) {
  const uint32_t key = v >> ip_band_shift(band);
  return mix32((key * 0x9e3779b1u) ^ cx_hash(x) ^ (band * 0x68e31da4u)) >> (32 - bits);
}
// Point-hash key of value v in point set `sid` on `axis` (round 5: sets are interned per image, so
// the rules that share an AddressGroup share its keys -- C2g: 16 sets of 10 000 members instead of
// 10 M (record, value) keys): high word 1 << 31 | sid << 4 | axis. ~0 (empty slot) is never a key.
constexpr uint32_t kPointSetMax = 1u << 20;  // set ids fit the 20 filter bits of a probe entry
GPC_HD uint32_t set_key_hi(uint32_t sid, uint32_t axis) { return 0x80000000u | (sid << 4) | axis; }
GPC_HD uint64_t set_key(uint32_t hi, uint32_t v) { return (uint64_t(hi) << 32) | v; }
constexpr uint32_t kHashSlots = 2;  // 16-B buckets, two choices: one 16-B load per choice
// The two cuckoo choices take the low and the high half of one mix (one 64-bit mix per probe).
GPC_HD uint32_t hash_b1(uint64_t k, uint32_t mask) { return uint32_t(mix64(k)) & mask; }
GPC_HD uint32_t hash_b2(uint64_t k, uint32_t mask) { return uint32_t(mix64(k) >> 32) & mask; }


// Entry filter bits. IP axes: band 1/2/3/4 = prefix length 8-15 / 16-23 / 24-31 / 32 keyed by the
// top 8 / 16 / 24 / 32 address bits; exact axes (in_port, reg1, reg7, tun_id): band 4 keyed by the value.
constexpr uint32_t kFiltIpBits = 20, kFiltL4Shift = 20, kFiltL4Bits = 12;
constexpr uint32_t kFiltNoAxis = 15u;
constexpr uint32_t kBloomL4 = 1u << 8;  // ImageHdr / JournalHdr bloom_axes: the service bits are tested
constexpr uint32_t kFiltL4All = 0xfff00000u;
GPC_HD uint32_t filt_ip_bit(uint32_t axis, uint32_t band, uint32_t key) {
  return 1u << uint32_t((uint64_t(mix32(key ^ (axis << 24) ^ (band << 28))) * kFiltIpBits) >> 32);
}
GPC_HD uint32_t filt_l4_bit(uint32_t pclass, uint32_t block) {  // a port range: its 4096-port blocks
  return 1u << (kFiltL4Shift + uint32_t((uint64_t(mix32(((pclass << 4) | block) + 0x3c6ef372u)) * kFiltL4Bits) >> 32));
}
GPC_HD uint32_t filt_l4x_bit(uint32_t pclass, uint32_t port) {  // a single port (most Services)
  return 1u << (kFiltL4Shift + uint32_t((uint64_t(mix32(((pclass << 16) | port) ^ 0xa54ff53au)) * kFiltL4Bits) >> 32));
}
GPC_HD uint32_t filt_pkt_axis(uint32_t axis, uint32_t v) {
  if (axis <= 3u)
    return filt_ip_bit(axis, 1, v >> 24) | filt_ip_bit(axis, 2, v >> 16) | filt_ip_bit(axis, 3, v >> 8) |
           filt_ip_bit(axis, 4, v);
  return filt_ip_bit(axis, 4, v);
}

// ------------------------------------------------------------------------------ evaluation
#ifdef GPC_EMU_STATS  // test-only instrumentation (tests/csrc/emu.cpp); never defined in the product build
extern "C" unsigned long long gpc_emu_stats[16];
extern "C" void gpc_emu_touch(const void* p, unsigned bytes, int line);
#define GPC_STAT(i, v) (gpc_emu_stats[i] += (v))
#define GPC_TOUCH(p, n) gpc_emu_touch((p), (n), __LINE__)
#else
#define GPC_STAT(i, v) ((void)0)
#define GPC_TOUCH(p, n) ((void)0)
#endif

// core.hpp SubIdx fmt 1: bucket b's entry range [lo, hi) from its directory block
GPC_HD void dir_list(const uint32_t* blob, const SubIdx& si, uint32_t b, uint32_t* lo, uint32_t* hi) {
  const uint32_t* d = blob + si.off + 4u * (b >> 5);
  GPC_TOUCH(d, 16);
#if defined(__HIPCC__)
  const uint4 q = *reinterpret_cast<const uint4*>(d);
#else
  const struct { uint32_t x, y, z, w; } q = {d[0], d[1], d[2], d[3]};
#endif
  const uint32_t sh = b & 31u, m = (1u << sh) - 1u;
  const uint32_t c = ((q.x >> sh) & 1u) | (((q.y >> sh) & 1u) << 1) | (((q.z >> sh) & 1u) << 2);
  const uint32_t start = q.w + uint32_t(__builtin_popcount(q.x & m)) + 2u * uint32_t(__builtin_popcount(q.y & m)) +
                         4u * uint32_t(__builtin_popcount(q.z & m));
  *lo = si.ent / 4u + start;
  *hi = *lo + c;
}
// Host-set combinations (round 6, image.cpp build_composite): a composite sub-index with band
// kBandCombo is keyed by the packet's combination id -- from the membership hash at word SubIdx.pres
// (combo_of) -- instead of by its address; its entries are exact-value entries whose Bloom axis
// field is kFiltCombo and whose lo / hi carry the combination id in their top bytes.
constexpr uint32_t kBandCombo = 5, kFiltCombo = 14u;
GPC_HD uint64_t combo_key64(uint32_t v) { return (uint64_t(0xC0B0u) << 32) | v; }
// Combination id of host value v (0: in no set of the sub-index): both 16-B buckets loaded together.
GPC_HD uint32_t combo_of(const uint32_t* blob, uint32_t off, uint32_t v) {
  const uint32_t* t = blob + off;
  const uint32_t mask = (1u << t[0]) - 1u;
  const uint64_t k = combo_key64(v);
  const uint32_t* b1 = t + 4 + 4 * size_t(hash_b1(k, mask));
  const uint32_t* b2 = t + 4 + 4 * size_t(hash_b2(k, mask));
  GPC_TOUCH(b1, 16);
  GPC_TOUCH(b2, 16);
#if defined(__HIPCC__)
  const uint4 q1 = *reinterpret_cast<const uint4*>(b1), q2 = *reinterpret_cast<const uint4*>(b2);
#else
  const struct { uint32_t x, y, z, w; } q1 = {b1[0], b1[1], b1[2], b1[3]}, q2 = {b2[0], b2[1], b2[2], b2[3]};
#endif
  return (q1.x == v ? q1.y : 0u) | (q1.z == v ? q1.w : 0u) | (q2.x == v ? q2.y : 0u) | (q2.z == v ? q2.w : 0u);
}
// Bucket key of a composite sub-index for the packet: its band key, or its combination id.
GPC_HD uint32_t ckey_of(const uint32_t* blob, const SubIdx& si, uint32_t v) {
  return si.band == kBandCombo ? combo_of(blob, si.pres, v) : v;
}
// Entries listed under bucket b of a sub-index (either format; host statistics).
GPC_HD uint32_t sub_bucket_len(const uint32_t* blob, const SubIdx& si, uint32_t b) {
  if (!si.fmt) return blob[si.off + b + 1] - blob[si.off + b];
  uint32_t lo, hi;
  dir_list(blob, si, b, &lo, &hi);
  return hi - lo == kDirCountMax ? blob[4 * lo + 2] : hi - lo;
}

// Region stamps (diagnostic builds only, -DGPC_STAMPS; tools/stamps.py): from GPC_MARK(r) on, the
// wave's s_memtime cycles are charged to region r; the kernel adds each wave's totals to
// gpc_stamp_acc. Never defined in the product build.
enum StampRegion : uint32_t { ST_PRE = 0, ST_HARD, ST_DRV, ST_SCAN, ST_VER, ST_TAIL, ST_FIN, ST_WALK, ST_POST, ST_N };
#if defined(GPC_STAMPS) && defined(__HIPCC__)
extern __device__ unsigned long long gpc_stamp_acc[32];
__device__ __forceinline__ uint32_t* gpc_stamp_lds() {
  __shared__ uint32_t st[ST_N + 3];  // per region cycles, current region, last time (lo, hi)
  return st;
}
__device__ __forceinline__ void gpc_mark(uint32_t r) {
  const uint64_t now = __builtin_amdgcn_s_memtime();
  const unsigned long long act = __ballot(1);
  if (__lane_id() == uint32_t(__ffsll((long long)act) - 1)) {
    uint32_t* st = gpc_stamp_lds();
    const uint64_t last = uint64_t(st[ST_N + 1]) | (uint64_t(st[ST_N + 2]) << 32);
    st[st[ST_N]] += uint32_t(now - last);
    st[ST_N] = r;
    st[ST_N + 1] = uint32_t(now);
    st[ST_N + 2] = uint32_t(now >> 32);
  }
}
#endif
#if defined(GPC_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
#define GPC_MARK(r) gpc_mark(r)
#else
#define GPC_MARK(r) ((void)0)
#endif

// ------------------------------------------------------------------------------ IPv6 interning
// An IPv6 image is an ordinary image over 32-bit *codes* of the IPv6 address axes. Every IPv6
// prefix of the rule set (ipv6_src / ipv6_dst / ct_ipv6_* matches) is a node of the prefix tree
// (prefixes are nested or disjoint); node codes are 32-bit prefixes: the children of a node with
// code c/l get c.i/(l + w), w = ceil(log2(m + 1)) bits for m children (i = 1..m; 0 = "in the
// node, in none of its children"), or ceil(log2 m) with i = 0..m-1 when the children tile the
// node. Then "a in P" <=> "code(a) in code(P)", where code(a) = code of the deepest prefix holding
// a (its longest matching prefix) padded with zeros, so the flows keep their prefix shape and the
// whole IPv4 machinery (bands, Bloom bits, intervals) applies unchanged. code(a) is found on the
// device by a longest-prefix match: binary search on the distinct prefix lengths (Waldvogel), one
// hash probe per step -- prefixes and markers, each carrying the code of its best matching prefix.
//
// One hash table per prefix length, keyed by the prefix right-aligned: kv = a >> (128 - L) (4 words,
// [0] most significant). Its slots hold only the low kw words of kv (kw = 1, 2 or 4) and the code:
// the other 4 - kw words are the same for every entry of the length (the tag, kept in the length's
// descriptor), so an address whose tag differs misses without a load. Rule sets whose prefixes of
// one length share their upper bits (C3 in fd00:10::/96: every length) get 8-B slots: a bucket of
// two slots is one 16-B load, so a probe of both choices is two 128-bit loads per lane (the table
// is a quarter of a 32-B-slot table with the length in every slot: C3 29 MB -> 5 MB, mostly
// L2-resident instead of Infinity-Cache traffic).
constexpr uint32_t kV6MaxLens = 64;
struct V6Len {
  uint32_t meta;     // prefix length | key words kw << 8 | log2(buckets) << 16
  uint32_t tab_off;  // word offset of its buckets
  uint32_t seed;     // hash state after the length and the tag (v6_seed)
  uint32_t reserved;
  uint32_t pat[4];  // kv words 0 .. 3 - kw: the tag every entry shares; words 4 - kw .. 3: the key of an
                    // empty slot (no entry of the length has it)
};
GPC_HD uint32_t v6_len(const V6Len& d) { return d.meta & 0xffu; }
GPC_HD uint32_t v6_kw(const V6Len& d) { return (d.meta >> 8) & 0xffu; }
GPC_HD uint32_t v6_log2(const V6Len& d) { return d.meta >> 16; }
constexpr uint32_t kV6MaxTags = 16;
struct V6Lpm {
  uint32_t n_lens;
  uint32_t l1_off;            // region tables (0: none): per tag 2^16 entries of 4 words, see v6_codes
  uint32_t l1_c;              // the tag length c: regions are the /c+16 blocks under a tag
  uint32_t n_tags;            // tags (1..kV6MaxTags) with a region table each, in l1_tag order
  uint32_t n_short;           // lengths shorter than l1_c (lens[0 .. n_short)): every prefix no shorter
                              // than c lies under a tag, so an address under none searches only these
  uint32_t lens[kV6MaxLens];  // distinct prefix lengths of the tree (root excluded), ascending
  V6Len d[kV6MaxLens];        // d[i]: the table of lens[i]
  uint32_t l1_tag[kV6MaxTags][4];  // the top c bits of the prefixes of length >= c, right-aligned (v6_key(a, c))
};
// Region tables (image.cpp build_image6): when every prefix of the tree no shorter than c lies under
// one of at most kV6MaxTags /c blocks (the tags; C3 in fd00:10::/96: one tag, c = 96; rule sets over
// several /48s: c = 48, a tag per /48), an address under a tag is first looked up by its next 16
// bits in that tag's table (one 16-B load, 1 MB per tag; shorter prefixes are folded into the
// entries as region bases): entry {code of the deepest prefix no longer than c + 16 holding the region,
// number n of the lengths longer than c + 16 present in the region | kV6L1Global, the indexes of
// those lengths, 8 bits each}; the binary search then runs over those n lengths only (regional
// markers are in the per-length tables; a marker carries the best match at its length whatever
// search tree placed it, so extra markers never mislead the global search). kV6L1Global: more
// than 8 lengths, search them all.
constexpr uint32_t kV6L1Bits = 16, kV6L1Global = 16u, kV6L1MaxLens = 8;
// Sub-region tables (round 5): a region whose search would span more than kV6LeafLens lengths is
// split instead -- its entry is {0, kV6L1Child, child, 0}, child = word offset (from l1_off) of 2^st
// entries of the same format for its /+st sub-blocks (st = v6_sub_bits: 8, or what is left to /128;
// prefixes up to that length folded into their bases), recursively while the block is not a /128. A wave's search then costs one dependent load
// per level it descends and at most ceil(log2(kV6LeafLens + 1)) probe rounds below, instead of up to
// four rounds of a list of 8 or a global search (C3 in IPv6: 2.2 % of the addresses, in ~3 of 4 waves).
constexpr uint32_t kV6L1Child = 32u, kV6LeafLens = 1, kV6SubBits = 8;
// bits a sub-region table of a /ll block resolves (the last one of a tree may be narrower)
GPC_HD uint32_t v6_sub_bits(uint32_t ll) { return 128u - ll < kV6SubBits ? 128u - ll : kV6SubBits; }
// Bucket (kw 2 / 4): two slots; slot = key (kw words), code, padding to 4 / 8 words: 32 / 64-B
// buckets, both choices loaded in one step. kw = 1 (round 5, "line buckets"): one 64-B line per
// bucket -- word 0 a flag (some key whose first choice is this bucket lives in its second choice),
// then 7 slots {key, code} -- so a step reads the first choice's line only, and the second choice
// only where the flag says a key may be there (rare: the builder places keys in their first choice
// whenever it has room). Halves the lines a step reads (C3 in IPv6: every table is kw = 1).
constexpr uint32_t kV6BucketWords = 16;  // the largest bucket (and the overflow table's)
constexpr uint32_t kV6LineSlots = 7;
GPC_HD uint32_t v6_slot_words(uint32_t kw) { return kw == 4u ? 8u : 2u * kw; }
GPC_HD uint32_t v6_bucket_words(uint32_t kw) { return kw == 1u ? 16u : 2u * v6_slot_words(kw); }
// Wide slot of the delta epochs' overflow table (journal): masked address (4 words), len | kV6Valid,
// code, 2 pad; 2 slots per 64-B bucket, two choices.
constexpr uint32_t kV6SlotWords = 8, kV6BucketSlots = 2, kV6Valid = 0x100u;
constexpr uint32_t kV6MaxNewLens = 3;  // prefix lengths a delta epoch may add (JournalHdr.v6_ovf_log2)
GPC_HD void v6_mask(const uint32_t* a, uint32_t len, uint32_t* m) {
  for (int w = 0; w < 4; w++) {
    const int bits = int(len) - 32 * w;
    m[w] = bits >= 32 ? a[w] : bits <= 0 ? 0u : (a[w] & ~((1u << (32 - bits)) - 1u));
  }
}
GPC_HD uint64_t v6_hkey(const uint32_t* m, uint32_t len) {
  const uint64_t h = mix64(((uint64_t(m[0]) << 32) | m[1]) ^ (uint64_t(len + 1) * 0x9e3779b97f4a7c15ull));
  return mix64(h ^ ((uint64_t(m[2]) << 32) | m[3]));
}
// kv = a >> (128 - len): the top len bits of a, right-aligned (len 1..128).
GPC_HD void v6_key(const uint32_t* a, uint32_t len, uint32_t* r) {
  const uint64_t hi = (uint64_t(a[0]) << 32) | a[1], lo = (uint64_t(a[2]) << 32) | a[3];
  const uint32_t s = 128u - len;
  uint64_t rh, rl;
  if (s >= 64u) {
    rh = 0;
    rl = hi >> (s - 64u);
  } else if (s == 0u) {
    rh = hi;
    rl = lo;
  } else {
    rh = hi >> s;
    rl = (lo >> s) | (hi << (64u - s));
  }
  r[0] = uint32_t(rh >> 32);
  r[1] = uint32_t(rh);
  r[2] = uint32_t(rl >> 32);
  r[3] = uint32_t(rl);
}
// Bucket hash of a per-length table: 32-bit mixing only (no 64-bit multiplies: the hash is a
// large part of a step's ALU work). seed = hash of the length and of the tag words (the same for
// every key of the table, so kept in its descriptor); then one mix per key word.
GPC_HD uint32_t v6_seed(uint32_t len, uint32_t kw, const uint32_t* r) {
  uint32_t h = mix32(len * 0x9e3779b9u + 0x7f4a7c15u);
  for (uint32_t w = 0; w + kw < 4u; w++) h = mix32(h ^ r[w]);
  return h;
}
GPC_HD void v6_buckets(const V6Len& d, const uint32_t* r, uint32_t* b1, uint32_t* b2) {
  const uint32_t kw = v6_kw(d);
  uint32_t h = d.seed;
  if (kw == 1u) {
    h = mix32(h ^ r[3]);
  } else {
#pragma unroll
    for (uint32_t w = 0; w < 4; w++)
      if (w + kw >= 4u) h = mix32(h ^ r[w]);
  }
  const uint32_t mask = (1u << v6_log2(d)) - 1u;
  *b1 = h & mask;
  *b2 = mix32(h ^ 0x85ebca6bu) & mask;
}
// Does the length's table have to be probed for key kv: its tag matches and it is not the empty key.
GPC_HD bool v6_probe_needed(const V6Len& d, const uint32_t* r) {
  bool tag = true, empty = true;
#pragma unroll
  for (uint32_t w = 0; w < 4; w++) {
    if (w + v6_kw(d) < 4u) tag = tag && r[w] == d.pat[w];
    else empty = empty && r[w] == d.pat[w];
  }
  return tag && !empty;
}
// Key kv in one bucket (16 words): slot s of a kw-word table holds kv's low kw words, then the code.
// Keys are unique in a table, so at most one slot matches: its code is OR-accumulated under a mask
// (no data-dependent slot index, which the compiler would turn into a private-memory array).
GPC_HD bool v6_bucket_find(const uint32_t* w, uint32_t kw, const uint32_t* r, uint32_t* code) {
  uint32_t c = 0, any = 0;
  if (kw == 1u) {  // a line bucket: flag word, then kV6LineSlots slots
#pragma unroll
    for (uint32_t s = 0; s < kV6LineSlots; s++) {
      const uint32_t mt = 0u - uint32_t(w[1 + 2 * s] == r[3]);
      c |= w[2 + 2 * s] & mt;
      any |= mt;
    }
  } else if (kw == 2u) {
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const uint32_t mt = 0u - uint32_t(w[4 * s] == r[2] && w[4 * s + 1] == r[3]);
      c |= w[4 * s + 2] & mt;
      any |= mt;
    }
  } else {
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const uint32_t mt = 0u - uint32_t(w[8 * s] == r[0] && w[8 * s + 1] == r[1] && w[8 * s + 2] == r[2] && w[8 * s + 3] == r[3]);
      c |= w[8 * s + 4] & mt;
      any |= mt;
    }
  }
  if (any) *code = c;
  return any != 0;
}
// A wide (overflow-table) bucket: masked address m of length len.
GPC_HD bool v6_wide_find(const uint32_t* w, const uint32_t* m, uint32_t len, uint32_t* code) {
  uint32_t c = 0, any = 0;
#pragma unroll
  for (int s = 0; s < 2; s++) {
    const uint32_t* x = w + s * kV6SlotWords;
    const uint32_t mt = 0u - uint32_t(x[4] == (len | kV6Valid) && x[0] == m[0] && x[1] == m[1] && x[2] == m[2] && x[3] == m[3]);
    c |= x[5] & mt;
    any |= mt;
  }
  if (any) *code = c;
  return any != 0;
}
// The first `words` (4, 8 or 16) words of a bucket (128-bit loads; w is 16 words).
GPC_HD void v6_load_bucket(const uint32_t* p, uint32_t words, uint32_t* w) {
#if defined(__HIPCC__)
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    if (4u * j < words) {
      const uint4 v = q[j];
      w[4 * j] = v.x;
      w[4 * j + 1] = v.y;
      w[4 * j + 2] = v.z;
      w[4 * j + 3] = v.w;
    }
  }
#else
  for (uint32_t j = 0; j < words; j++) w[j] = p[j];
#endif
}
// code(a_k) for K addresses at once (a[k][0..3], [0] = most significant): the K binary searches run
// in lock step, so each step issues every bucket load before any compare. `desc`: the length
// descriptors (the kernel's LDS copy; null: those of the image). kOvf (IPv6 delta epochs): the
// journal's overflow table `ovf` (2^ovf_log2 wide buckets, the LPM entries of prefixes interned since
// the base) is probed in the same step, its loads issued with the base's: no extra dependent round.
// ovf_log2: JournalHdr.v6_ovf_log2 (log2 in the low byte, new prefix lengths above it): a prefix of a
// new length is a leaf interned since the base with an exact code and nothing below it, so when the
// address is in one it is the address's deepest match: after the search, one probe per new length
// (at most kV6MaxNewLens; wave-uniform, only in epochs that have them) replaces the code on a hit.
template <int K, bool kOvf = false>
GPC_HD void v6_codes(const uint32_t* blob, uint32_t lpm_off, const uint32_t (*a)[4], uint32_t* code,
                     const uint32_t* ovf = nullptr, uint32_t ovf_log2 = 0, const V6Len* desc = nullptr) {
  const V6Lpm* L = reinterpret_cast<const V6Lpm*>(blob + lpm_off);
  const V6Len* D = desc ? desc : L->d;
  const uint32_t omask = (1u << (ovf_log2 & 0xffu)) - 1u;
  int lo[K], hi[K];
  uint32_t rl[K][2];  // regional search: the length indexes (8 bits each); all-ones: global
#pragma unroll
  for (int k = 0; k < K; k++) {
    code[k] = 0;
    lo[k] = 0;
    hi[k] = int(L->n_lens) - 1;
    rl[k][0] = rl[k][1] = 0xffffffffu;
    // (a delta epoch's overflow entries may sit at lengths a region's list omits: global search)
    if (!kOvf && L->l1_off) {
      const uint32_t c = L->l1_c;
      uint32_t t[4] = {0u, 0u, 0u, 0u}, x[4];
      if (c) v6_key(a[k], c, t);
      uint32_t ti = 0xffffffffu;  // the address's tag (uniform loop over the few tags, scalar operands)
      for (uint32_t j = 0; j < L->n_tags; j++)
        if (t[0] == L->l1_tag[j][0] && t[1] == L->l1_tag[j][1] && t[2] == L->l1_tag[j][2] && t[3] == L->l1_tag[j][3])
          ti = j;
      if (ti == 0xffffffffu) hi[k] = int(L->n_short) - 1;
      if (ti != 0xffffffffu) {
        v6_key(a[k], c + kV6L1Bits, x);
        const uint32_t* e = blob + L->l1_off + (size_t(ti) << (kV6L1Bits + 2)) + 4 * size_t(x[3] & ((1u << kV6L1Bits) - 1u));
        GPC_TOUCH(e, 16);
#if defined(__HIPCC__)
        uint4 ev = *reinterpret_cast<const uint4*>(e);
#else
        struct { uint32_t x, y, z, w; } ev = {e[0], e[1], e[2], e[3]};
#endif
        for (uint32_t ll = c + kV6L1Bits; ev.y & kV6L1Child;) {  // sub-region tables
          const uint32_t st = v6_sub_bits(ll);
          ll += st;
          v6_key(a[k], ll, x);
          e = blob + L->l1_off + ev.z + 4 * (x[3] & ((1u << st) - 1u));
          GPC_TOUCH(e, 16);
          GPC_STAT(14, 1);
#if defined(__HIPCC__)
          ev = *reinterpret_cast<const uint4*>(e);
#else
          ev = {e[0], e[1], e[2], e[3]};
#endif
        }
        if (!(ev.y & kV6L1Global)) {
          code[k] = ev.x;
          hi[k] = int(ev.y & 15u) - 1;
          rl[k][0] = ev.z;
          rl[k][1] = ev.w;
          GPC_STAT(12, ev.y & 15u);  // lengths the regional search spans
        } else {
          GPC_STAT(13, 1);  // global searches
        }
      }
    }
  }
  while (true) {
    bool any = false;
#pragma unroll
    for (int k = 0; k < K; k++) any |= lo[k] <= hi[k];
    if (!any) break;
    GPC_STAT(11, 1);  // dependent search rounds of the K-address group
    uint32_t r[K][4], kw[K], w[K][2][kV6BucketWords];
    const uint32_t* b2[K];  // the second choice's bucket (line buckets: loaded only when flagged)
    bool probe[K];
    uint32_t m[K][kOvf ? 4 : 1], len[K], ow[K][kOvf ? 2 : 1][kOvf ? kV6BucketWords : 1];
#pragma unroll
    for (int k = 0; k < K; k++) {
      const bool live = lo[k] <= hi[k];
      const uint32_t mid = live ? uint32_t(lo[k] + hi[k]) >> 1 : 0u;
      const uint32_t li = rl[k][0] == 0xffffffffu ? mid : ((mid < 4u ? rl[k][0] >> (8u * mid) : rl[k][1] >> (8u * (mid - 4u))) & 0xffu);
      const V6Len& d = D[li];
      len[k] = v6_len(d);
      kw[k] = v6_kw(d);
      v6_key(a[k], len[k], r[k]);
      probe[k] = live && v6_probe_needed(d, r[k]);
      uint32_t bk[2];
      v6_buckets(d, r[k], &bk[0], &bk[1]);
      b2[k] = blob + d.tab_off + size_t(bk[1]) * v6_bucket_words(kw[k]);
#pragma unroll
      for (int c = 0; c < 2; c++) {
        const uint32_t bw = v6_bucket_words(kw[k]);
        const uint32_t* b = blob + d.tab_off + size_t(bk[c]) * bw;
        if (probe[k] && (c == 0 || kw[k] != 1u)) {  // line buckets: the first choice only
          GPC_TOUCH(b, bw * 4);
          v6_load_bucket(b, bw, w[k][c]);
        }
      }
      if constexpr (kOvf) {
        v6_mask(a[k], len[k], m[k]);
        const uint64_t ok = v6_hkey(m[k], len[k]);
#pragma unroll
        for (int c = 0; c < 2; c++) {
          const uint32_t* b = ovf + size_t(c ? hash_b2(ok, omask) : hash_b1(ok, omask)) * (kV6SlotWords * kV6BucketSlots);
          if (live) v6_load_bucket(b, kV6BucketWords, ow[k][c]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
      if (lo[k] > hi[k]) continue;
      const int mid = (lo[k] + hi[k]) >> 1;
      bool hit = false;
      if (probe[k]) {
        hit = v6_bucket_find(w[k][0], kw[k], r[k], &code[k]);
        if (kw[k] != 1u) {
          hit = v6_bucket_find(w[k][1], kw[k], r[k], &code[k]) || hit;
        } else if (GPC_WAVE_ANY(!hit && w[k][0][0] != 0u)) {  // flagged line bucket: the second choice
          if (!hit && w[k][0][0] != 0u) {
            GPC_TOUCH(b2[k], 64);
            v6_load_bucket(b2[k], 16u, w[k][1]);
            hit = v6_bucket_find(w[k][1], 1u, r[k], &code[k]);
          }
        }
      }
      if constexpr (kOvf) {
        hit = v6_wide_find(ow[k][0], m[k], len[k], &code[k]) || hit;
        hit = v6_wide_find(ow[k][1], m[k], len[k], &code[k]) || hit;
      }
      if (hit) lo[k] = mid + 1;
      else hi[k] = mid - 1;
    }
  }
  if constexpr (kOvf) {
    for (uint32_t nl = ovf_log2 >> 8; nl; nl >>= 8) {
      const uint32_t len = nl & 0xffu;
      if (!len) continue;
      uint32_t m[K][4], ow[K][2][kV6BucketWords];
#pragma unroll
      for (int k = 0; k < K; k++) {  // both choices of every address loaded before any compare
        v6_mask(a[k], len, m[k]);
        const uint64_t ok = v6_hkey(m[k], len);
#pragma unroll
        for (int c = 0; c < 2; c++)
          v6_load_bucket(ovf + size_t(c ? hash_b2(ok, omask) : hash_b1(ok, omask)) * (kV6SlotWords * kV6BucketSlots),
                         kV6BucketWords, ow[k][c]);
      }
#pragma unroll
      for (int k = 0; k < K; k++) {
        if (!v6_wide_find(ow[k][0], m[k], len, &code[k])) (void)v6_wide_find(ow[k][1], m[k], len, &code[k]);
      }
    }
  }
}
GPC_HD uint32_t v6_code(const uint32_t* blob, uint32_t lpm_off, const uint32_t* a, const uint32_t* ovf = nullptr,
                        uint32_t ovf_log2 = 0) {
  uint32_t aa[1][4] = {{a[0], a[1], a[2], a[3]}}, c;
  if (ovf) v6_codes<1, true>(blob, lpm_off, aa, &c, ovf, ovf_log2);
  else v6_codes<1>(blob, lpm_off, aa, &c);
  return c;
}
// Is the (masked address m, len) entry in the base LPM (host: which delta entries go to the overflow).
GPC_HD bool v6_base_has(const uint32_t* blob, uint32_t lpm_off, const uint32_t* m, uint32_t len) {
  const V6Lpm* L = reinterpret_cast<const V6Lpm*>(blob + lpm_off);
  for (uint32_t i = 0; i < L->n_lens; i++) {
    const V6Len& d = L->d[i];
    if (v6_len(d) != len) continue;
    uint32_t r[4], w[kV6BucketWords], c = 0, bk[2];
    v6_key(m, len, r);
    if (!v6_probe_needed(d, r)) return false;
    v6_buckets(d, r, &bk[0], &bk[1]);
    const uint32_t bw = v6_bucket_words(v6_kw(d));
    for (int j = 0; j < 2; j++) {
      v6_load_bucket(blob + d.tab_off + size_t(bk[j]) * bw, bw, w);
      if (v6_bucket_find(w, v6_kw(d), r, &c)) return true;
    }
    return false;
  }
  return false;
}
// 16 network-order bytes -> 4 host words, most significant first.
GPC_HD void v6_words(const uint8_t* p, uint32_t* a) {
  for (int w = 0; w < 4; w++)
    a[w] = (uint32_t(p[4 * w]) << 24) | (uint32_t(p[4 * w + 1]) << 16) | (uint32_t(p[4 * w + 2]) << 8) | p[4 * w + 3];
}

struct Img {
  const uint32_t* blob;
  const ImageHdr* hdr;
  const uint32_t* dead;   // tombstones over this image's rule ids (delta epochs), or null: a page table
  const uint32_t* dpool;  // of journal-pool word offsets, one 256-word (8192-bit) bitmap page each
};
constexpr uint32_t kDeadPageWords = 256, kDeadPageShift = 13;
GPC_HD bool rule_dead(const Img& im, uint32_t rid) {
  if (!im.dead) return false;
  const uint32_t pg = im.dead[rid >> kDeadPageShift];
  return pg && ((im.dpool[pg + ((rid >> 5) & (kDeadPageWords - 1u))] >> (rid & 31u)) & 1u);
}

// One published epoch: the base image and, after delta commits, the journal (ovl.blob = journal
// pool, jhdr = this epoch's JournalHdr word offset in it) holding the current version of every
// rule changed since the base was built (the base copies are tombstoned). Table verdict = the OVS
// decision over the union of both rule sets.
struct View {
  Img base, ovl;
  uint32_t n_img;  // 1 or 2
  uint32_t jhdr;
  uint32_t ext;    // ExtHdr word offset in the pool (ovl.blob), 0: no point extensions
};

// Epoch modes (kernel instantiations): the base image alone; the base plus point extensions (no
// journal walk, no tombstones); the base with tombstones, the journal and point extensions.
constexpr int kModeBase = 0, kModeExt = 1, kModeJournal = 2;

// ------------------------------------------------------------------------------ journal
// Append-only delta store (journal.cpp). Every commit appends, never rewrites, so launches of
// older epochs keep reading consistent data while a new epoch is written:
//   rule records   same format as the base image (no point-hash segments), rid = journal id;
//   entries        8 words {next head word, key value, meta, record offset, prefilter x, y, lo, hi}
//                  chained per hash bucket (newest first); meta = table | clause << 3 | axis << 5 |
//                  band << 9 | orid << 12;
//   head pages     64 head words each, copied on write; a head word = entry offset / 8 | chain
//                  length (saturating) << 24, 0 = empty;
//   JournalHdr     per epoch: the page table, both tombstone bitmaps (base rids, journal rids) and
//                  per table the bucket kinds (axis, band) per driver clause, the always chains and
//                  the hard pseudo-rule list (rank order).
struct JournalTable {
  uint8_t n_kinds[2], pad[2];
  uint8_t kinds[2][8];     // axis | band << 4
  uint32_t always[2];      // head word of the clause's always chain
  uint32_t hard_off, n_hard;
};
struct JournalHdr {
  uint32_t lg;             // 2^lg buckets
  uint32_t pt_off;         // page table: 2^(lg-8) words, word offset of each head page (0: empty)
  uint32_t bdead_off;      // base tombstones: page table (0: none), see rule_dead
  uint32_t odead_off;      // journal tombstones: page table (0: none)
  uint32_t bloom_axes;     // as ImageHdr.bloom_axes, over every journal entry so far
  // IPv6 journals: LPM entries of the prefixes interned since the base (image.cpp extend_image6),
  // a hash laid out like V6Lpm's (2^(v6_ovf_log2 & 0xff) buckets) probed next to the base's; 0:
  // none. Bytes 1..3 of v6_ovf_log2: prefix lengths the base does not search (0: none), whose
  // leaves are probed in that hash after the binary search (v6_codes)
  uint32_t v6_ovf_off, v6_ovf_log2;
  uint32_t ext_off;        // ExtHdr of this epoch's point extensions (0: none)
  uint32_t jflags;         // kJUsed: the journal holds records, tombstones or hard rules (else only extensions)
  uint32_t live;           // bit t-1: table t has journal chains, always entries or hard rules
  JournalTable t[6];
};
constexpr uint32_t kJUsed = 1u;
constexpr uint32_t kJEntWords = 8;
constexpr uint32_t kJOridShift = 12, kJMetaMask = (1u << kJOridShift) - 1u;  // meta: 12 bits, orid: 20
constexpr uint32_t kJPageHeads = 64;
GPC_HD uint32_t jkey(uint32_t axis, uint32_t band, uint32_t v) {  // bucket key value of a packet
  if (axis <= AX_CTDST) return v >> ip_band_shift(band);
  if (axis == AX_L4D || axis == AX_L4S) return (proto_class(v >> 16) << 13) | ((v & 0xffffu) >> 3);
  return v;
}
// Journal key of a table with a composite base index (TableHdr n_cidx): the band key of the band
// clause combined with the packet's value x of the composite axis, so a chain lists only the changed
// rules that hold both (as the base's composite buckets do); a collision costs a verification.
GPC_HD uint32_t jxkey(uint32_t key, uint32_t x) { return mix32((key * 0x9e3779b1u) ^ cx_hash(x)); }
GPC_HD uint32_t jmeta(uint32_t table, uint32_t clause, uint32_t axis, uint32_t band) {
  return table | (clause << 3) | (axis << 5) | (band << 9);
}
GPC_HD uint32_t jbucket(uint32_t meta, uint32_t key, uint32_t lg) {
  return mix32(key ^ mix32(meta * 0x9e3779b1u + 0x7f4a7c15u)) >> (32 - lg);
}
GPC_HD uint32_t jhead(const uint32_t* pool, const JournalHdr* jh, uint32_t b) {
  GPC_TOUCH(pool + jh->pt_off + (b / kJPageHeads), 4);
  const uint32_t page = pool[jh->pt_off + (b / kJPageHeads)];
  if (page) GPC_TOUCH(pool + page + (b % kJPageHeads), 4);
  return page ? pool[page + (b % kJPageHeads)] : 0u;
}

// Two consecutive words (a bucket's begin / end offsets) as one 8-B load: dword-aligned multi-dword
// global loads are legal on gfx950, so the pair costs one vector memory instruction, not two.
GPC_HD void load_pair(const uint32_t* p, uint32_t* a, uint32_t* b) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  *a = uint32_t(v);
  *b = uint32_t(v >> 32);
}

// A rule record's 6 header words (records are 64-B aligned): one 16-B and one 8-B load.
struct RecHdr {
  uint32_t w[kRecHdrWords];
};
GPC_HD RecHdr load_rec_hdr(const uint32_t* rec) {
  RecHdr h;
#if defined(__HIPCC__)
  const uint4 a = *reinterpret_cast<const uint4*>(rec);
  const uint2 b = *reinterpret_cast<const uint2*>(rec + 4);
  h.w[0] = a.x, h.w[1] = a.y, h.w[2] = a.z, h.w[3] = a.w, h.w[4] = b.x, h.w[5] = b.y;
#else
  for (uint32_t i = 0; i < kRecHdrWords; i++) h.w[i] = rec[i];
#endif
  return h;
}
// A record's first line: header and fast descriptors (words 0-14) in one round of 16-B loads, so
// the verification needs no further dependent load for its one-word clause kinds.
struct RecLine {
  uint32_t w[kRecLine];
};
GPC_HD RecLine load_rec_line(const uint32_t* rec) {
  RecLine h;
#if defined(__HIPCC__)
  const uint4* q = reinterpret_cast<const uint4*>(rec);
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint4 a = q[j];
    h.w[4 * j] = a.x, h.w[4 * j + 1] = a.y, h.w[4 * j + 2] = a.z, h.w[4 * j + 3] = a.w;
  }
#else
  for (uint32_t i = 0; i < kRecLine; i++) h.w[i] = rec[i];
#endif
  return h;
}

// Both buckets are loaded before either is compared (two independent 16-B loads).
GPC_HD bool hash_contains(const Img& im, uint64_t key) {
  const uint64_t* tab = reinterpret_cast<const uint64_t*>(im.blob + im.hdr->hash_off);
  const uint32_t mask = (1u << im.hdr->hash_log2) - 1;
  const uint64_t* b1 = tab + size_t(hash_b1(key, mask)) * kHashSlots;
  const uint64_t* b2 = tab + size_t(hash_b2(key, mask)) * kHashSlots;
  GPC_TOUCH(b1, 16);
  GPC_TOUCH(b2, 16);
  const uint64_t k0 = b1[0], k1 = b1[1], k2 = b2[0], k3 = b2[1];
  return (k0 == key) | (k1 == key) | (k2 == key) | (k3 == key);
}

template <typename W = uint32_t>
GPC_HD bool ival_hit(const W* iv, uint32_t n, uint32_t v) {
  if (n <= 8) {
    for (uint32_t i = 0; i < n; i++) {
      GPC_TOUCH(iv + 2 * i, 8);
      if (v < iv[2 * i]) return false;
      if (v <= iv[2 * i + 1]) return true;
    }
    return false;
  }
  uint32_t lo = 0, hi = n;  // first interval with lo > v
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    GPC_TOUCH(iv + 2 * mid, 8);
    if (iv[2 * mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return lo > 0 && v <= iv[2 * (lo - 1) + 1];
}

template <typename W = uint32_t>
GPC_HD bool pts_hit(const W* pt, uint32_t n, uint32_t v) {
  if (n <= 16) {
    for (uint32_t i = 0; i < n; i++) {
      GPC_TOUCH(pt + i, 4);
      if (pt[i] >= v) return pt[i] == v;
    }
    return false;
  }
  uint32_t lo = 0, hi = n;  // first point >= v
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    GPC_TOUCH(pt + mid, 4);
    if (pt[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && pt[lo] == v;
}

template <typename W = uint32_t>
GPC_HD bool box_hit(const W* bx, uint32_t n, const Pkt& p) {
  for (uint32_t i = 0; i < n; i++, bx += kBoxWords) {
    GPC_TOUCH(bx, kBoxWords * 4);
    const uint32_t meta = bx[6];
    const uint32_t nt = meta >> 24;
    bool ok = true;
    for (uint32_t t = 0; t < nt; t++) ok &= (p.ax[(meta >> (8 * t)) & 0xffu] & bx[3 + t]) == bx[t];
    if (ok) return true;
  }
  return false;
}

// One clause of the record at word offset `roff` (OR of its segments). W: uint32_t, or cword when
// the record is read at a wave-uniform address (hard pseudo-rules).
template <typename W = uint32_t>
GPC_HD bool clause_match(const Img& im, uint32_t roff, const W* c, const Pkt& p) {
  const W* blob = (const W*)im.blob;
  GPC_TOUCH(c, 4);
  const uint32_t nseg = c[0];
  const W* w = c + 1;
  for (uint32_t s = 0; s < nseg; s++) {
    GPC_TOUCH(w, 4);
    const uint32_t tag = *w++;
    const uint32_t kind = tag & 0xfu, axis = (tag >> 4) & 0xfu, n = tag >> 8;
    bool hit;
    switch (kind) {
      case SK_ALWAYS: return true;
      case SK_IVAL: hit = ival_hit(w, n, p.ax[axis]); w += 2 * n; break;
      case SK_PTS: hit = pts_hit(w, n, p.ax[axis]); w += n; break;
      case SK_HASH: GPC_TOUCH(w, 4); hit = hash_contains(im, set_key(*w, p.ax[axis])); w++; break;
      case SK_BOX: hit = box_hit(w, n, p); w += kBoxWords * n; break;
      case SK_XIVAL: GPC_TOUCH(w, 4); hit = ival_hit(blob + *w, n, p.ax[axis]); w++; break;
      case SK_XPTS: GPC_TOUCH(w, 4); hit = pts_hit(blob + *w, n, p.ax[axis]); w++; break;
      case SK_XBOX: GPC_TOUCH(w, 4); hit = box_hit(blob + *w, n, p); w++; break;
      default: hit = false; break;
    }
    if (hit) return true;
  }
  return false;
}

// Four consecutive words at a dword-aligned address as one 16-B load (gfx950 allows dword-aligned
// multi-dword global loads).
#ifndef GPC_CHUNK_QUADS
#define GPC_CHUNK_QUADS 2
#endif
constexpr int kChunkQuads = GPC_CHUNK_QUADS;  // 16-B loads of a final chunk in rule_match's search

template <typename W>
GPC_HD void load_quad(const W* p, uint32_t* w) {
#if defined(__HIPCC__)
  struct Q {
    uint32_t a, b, c, d;
  } q;
  __builtin_memcpy(&q, (const void*)p, 16);
  w[0] = q.a, w[1] = q.b, w[2] = q.c, w[3] = q.d;
#else
  for (int i = 0; i < 4; i++) w[i] = p[i];
#endif
}

// All clauses of a record (AND), from the fast descriptors of its first line: the one-word kinds
// are decided with compares, the array kinds by one lock-step search over the (at most three)
// clauses -- binary steps while a clause's window is longer than one 16-B chunk, then one chunk
// compare -- so a verification is one round of descriptor loads plus a few rounds of 16-B loads,
// with loop trip counts uniform over the wavefront and branch-free bodies (the round-3 segment
// interpreter spent most of C1's time on exec-mask bookkeeping). FK_GENERIC clauses (rare) fall
// back to clause_match. `dsc`: the record's nine descriptor words (already loaded with its first
// line); `skip`: clauses already decided by the driver entry. W: uint32_t, or cword for records
// read at a wave-uniform address (hard pseudo-rules).
template <typename W = uint32_t>
GPC_HD bool rule_match(const Img& im, const W* rec, uint32_t w2, const uint32_t* dsc, uint32_t skip, const Pkt& p) {
  const W* blob = (const W*)im.blob;
  const uint32_t ncl = rec_nclauses(w2);
  bool ok = true;
  uint32_t gen = 0, hsh = 0;
  uint32_t x[kMaxClauses], l[kMaxClauses], h[kMaxClauses], base[kMaxClauses], kd[kMaxClauses];
#pragma unroll
  for (int k = 0; k < kMaxClauses; k++) {
    const uint32_t A = dsc[3 * k], B = dsc[3 * k + 1], C = dsc[3 * k + 2];
    const bool need = uint32_t(k) < ncl && !((skip >> k) & 1u);
    const uint32_t kind = need ? (A & 15u) : uint32_t(FK_ALWAYS);
    const uint32_t v = p.ax[(A >> 4) & 15u];
    x[k] = v;
    kd[k] = kind;
    base[k] = B;
    l[k] = 0;
    h[k] = kind >= FK_IVN ? (A >> 8) : 0u;
    const bool r = kind == FK_IV1 ? (B <= v) & (v <= C) : kind == FK_MK1 ? (v & C) == B : true;
    ok = ok & r;
    gen |= kind == FK_GENERIC ? 1u << k : 0u;
    hsh |= kind == FK_HASH ? 1u << k : 0u;
  }
  // point-hash clauses (large exact-value sets): both buckets loaded before either compare
  if (GPC_WAVE_ANY(ok & (hsh != 0u))) {
    const uint32_t roff = uint32_t(rec - blob);
#pragma unroll
    for (int k = 0; k < kMaxClauses; k++)
      if (ok & ((hsh >> k) & 1u)) ok = hash_contains(im, set_key(dsc[3 * k + 1], x[k]));
  }
  // array clauses: window [l, h) of elements still to look at, per clause, in lock step
  while (GPC_WAVE_ANY(ok & ((h[0] > l[0]) | (h[1] > l[1]) | (h[2] > l[2])))) {
    GPC_STAT(9, 1);
#pragma unroll
    for (int k = 0; k < kMaxClauses; k++) {
      const bool live = ok & (h[k] > l[k]);
      const uint32_t kind = kd[k];
      const uint32_t stride = kind == FK_IVN ? 2u : kind == FK_PTN ? 1u : kBoxWords;
      // elements one final chunk covers: kChunkQuads 16-B loads issued together (all but the first
      // only by lanes whose window needs them), one box for FK_MKN
      const uint32_t cap = kind == FK_IVN ? 2u * kChunkQuads : kind == FK_PTN ? 4u * kChunkQuads : 1u;
      const uint32_t n = h[k] - l[k];
      const bool bin = live & (kind != FK_MKN) & (n > cap);
      const uint32_t mid = (l[k] + h[k]) >> 1;
      const uint32_t pos = bin ? mid : l[k];
      const W* q = blob + (live ? base[k] + stride * pos : 0u);  // idle lanes read word 0 (a valid line)
      const uint32_t words = bin ? 1u : n * stride;  // words of the window
      uint32_t w[4 * kChunkQuads];
      GPC_TOUCH(q, 16);
      load_quad(q, w);
#pragma unroll
      for (int j = 1; j < kChunkQuads; j++) {
        w[4 * j] = w[4 * j + 1] = w[4 * j + 2] = w[4 * j + 3] = 0u;
        if (live & (words > 4u * j) & (kind != FK_MKN)) {
          GPC_TOUCH(q + 4 * j, 16);
          load_quad(q + 4 * j, &w[4 * j]);
        }
      }
      const uint32_t v = x[k];
      // binary step: the last element whose low end is <= v stays in the window
      const bool le = w[0] <= v;
      // chunk compare over the window (at most cap elements)
      bool hit = false;
      if (kind == FK_IVN) {
#pragma unroll
        for (uint32_t j = 0; j < 2u * kChunkQuads; j++) hit = hit | ((n > j) & (w[2 * j] <= v) & (v <= w[2 * j + 1]));
      } else if (kind == FK_PTN) {
#pragma unroll
        for (uint32_t j = 0; j < 4u * kChunkQuads; j++) hit = hit | ((n > j) & (w[j] == v));
      } else {
        hit = (v & w[3]) == w[0];
      }
      const bool fin = live & !bin & (hit | (kind != FK_MKN) | (n <= 1u));  // this clause is settled
      if (bin) {
        l[k] = le ? mid : l[k];
        h[k] = le ? h[k] : mid;
      }
      if (live & !bin) {
        ok = ok & (hit | !fin);
        l[k] = fin ? h[k] : l[k] + 1u;  // MKN without a hit: next box
      }
    }
  }
  // clauses the descriptors cannot express: the segment interpreter
  if (GPC_WAVE_ANY(ok & (gen != 0u))) {
    if (ok & (gen != 0u)) {
      const uint32_t roff = uint32_t(rec - blob);
      for (uint32_t k = 0; k < ncl; k++)
        if ((gen >> k) & 1u) ok = ok && clause_match(im, roff, rec + rec_off(w2, k), p);
    }
  }
  return ok;
}

// An inline hard pseudo-rule (TableHdr.hf) against the packet: descriptor kinds are uniform, so
// the only per-lane work is the compares (and the point-hash probe of an FK_HASH clause).
GPC_HD bool hard_fast_match(const Img& im, const HardFast& hf, const Pkt& p) {
  const uint32_t ncl = hf.pv >> 24;
  bool ok = true;
#pragma unroll
  for (uint32_t k = 0; k < uint32_t(kMaxClauses); k++) {
    if (k >= ncl) break;
    const uint32_t A = hf.d[3 * k], B = hf.d[3 * k + 1], C = hf.d[3 * k + 2], kind = A & 15u;
    const uint32_t v = p.ax[(A >> 4) & 15u];
    if (kind == FK_HASH) {
      ok = ok & hash_contains(im, set_key(B, v));
    } else {
      const bool r = kind == FK_IV1 ? (B <= v) & (v <= C)
                     : kind == FK_MK1 ? (v & C) == B
                     : kind == FK_MK2 ? ((v & hf.mk[1]) == hf.mk[0]) | ((v & hf.mk[3]) == hf.mk[2])
                                      : true;
      ok = ok & r;
    }
  }
  return ok;
}

// xv: the packet's value of the table's composite axis (exact-value entries; any value elsewhere).
// kSetProbes (base images): a probe entry's low 20 bits are its point set's id, not Bloom bits --
// the probe itself is the test (a set large enough for the point hash saturates 20 Bloom bits).
// cp: the packet's combination id (kBandCombo lists; 16 bits).
template <bool kSetProbes = true>
GPC_HD bool entry_pass(const Pkt& p, const Ent& e, uint32_t xv, uint32_t cp = 0u) {  // branch-free
  const uint32_t bax = e.x & 15u, iax = (e.x >> 4) & 15u;
  const bool exact = (e.x & kEntExactX) != 0u;
  const bool l4 = (e.y & p.l4m) != 0u;
  // Bloom axis < 8: IP / exact-axis bits; 8..14 (probe entry): set id (base) or the probed clause's
  // Bloom bits (journal); 15: none. Exact-value entries: 15, or kFiltCombo (a combination list)
  const bool bl = (bax == kFiltNoAxis) | (kSetProbes & (bax >= 8u)) | ((e.y & p.fm[bax & 7u]) != 0u);
  const bool cmb = exact & (bax == kFiltCombo);
  const uint32_t lo = cmb ? e.lo & 0xffffffu : e.lo, hi = cmb ? e.hi & 0xffffffu : e.hi;
  const bool cok = !cmb | (((e.lo >> 24) | ((e.hi >> 24) << 8)) == cp);
  const uint32_t v = p.ax[iax < AX_N ? iax : 0];
  const bool iv = (iax == kFiltNoAxis) | ((lo <= v) & (v <= hi));
  return (exact ? (e.y == xv) & cok : l4 & bl) & iv;
}

// Scan length of one table for the packet (the driver clause's candidate count, as eval_part picks
// it): the kernel can group lanes of similar length into the same wavefront (classify.hip).
GPC_HD uint32_t scan_estimate(const Img& im, uint32_t table, const Pkt& p) {
  const TableHdr& th = im.hdr->t[table - 1];
  if (th.n_cidx) {  // the composite driver is always taken (eval_part)
    const uint32_t xb = cx_bit(p.ax[th.cx]);
    if (!((im.blob[th.xmap_off + (xb >> 5)] >> (xb & 31u)) & 1u)) return 0;
    uint32_t c = th.always_n[th.cband];
    for (uint32_t i = 0; i < th.n_cidx && i < uint32_t(kIdxPerClause); i++) {
      const SubIdx& si = th.cidx[i];
      const uint32_t key = ckey_of(im.blob, si, p.ax[si.axis]);
      if (si.band == kBandCombo && key == 0u) continue;
      const uint32_t bk = cbucket_of(si.band, si.bits, key, p.ax[th.cx]);
      c += sub_bucket_len(im.blob, si, bk);
    }
    return c;
  }
  uint32_t cnt[2] = {th.always_n[0], th.always_n[1]};
#pragma unroll
  for (int k = 0; k < 2; k++)
#pragma unroll
    for (int i = 0; i < kIdxPerClause; i++) {
      if (uint32_t(i) >= th.n_idx[k]) break;
      const SubIdx& si = th.idx[k][i];
      const uint32_t* o = im.blob + si.off + bucket_of(si.axis, si.band, si.bits, p.ax[si.axis]);
      uint32_t ob, oe;
      load_pair(o, &ob, &oe);
      cnt[k] += oe - ob;
    }
  return cnt[0] < cnt[1] ? cnt[0] : cnt[1];
}

constexpr int kLists = kIdxPerClause + 1;  // always list + sub-indexes of the driver clause
#ifndef GPC_SCAN_UNROLL
#define GPC_SCAN_UNROLL 4
#endif
constexpr int kScanUnroll = GPC_SCAN_UNROLL;  // entry loads in flight per lane in the candidate scan

// One pass of the candidate scan over the first kL driver lists, flattened: entry j of the
// sequence is entry j + dl[l] of the image for the list l holding it (dl[l] = first entry of list l
// minus the entries of lists 0..l-1; upto[l] = cumulative end of list l). Every entry is loaded and
// prefiltered with a branch-free body; the two smallest passing record offsets above `after` and
// below `rH` (the two best-ranked candidates) are kept in c0 < c1; `more` = a third one passed.
// kL = 2 (tables whose clauses have one sub-index, e.g. AddressGroup / ofport rules) locates an
// entry with one compare instead of kLists - 1.
template <int kL>
GPC_HD void scan_lists(const Img& im, const Pkt& p, const uint32_t* dl, const uint32_t* upto, uint32_t total,
                       uint32_t after, uint32_t rH, uint32_t xv, uint32_t cp, uint32_t& c0, uint32_t& c1, bool& more) {
  const Ent* E = reinterpret_cast<const Ent*>(im.blob);
  c0 = c1 = 0xffffffffu;
  more = false;
  // wave-uniform trip count (the wave's longest candidate list); finished lanes read the zero
  // entry at index 0 (offset 0 is never a record), so the body has no divergent branches.
  // kScanUnroll entries are loaded before any is used: that many loads in flight per lane.
  for (uint32_t j0 = 0; GPC_WAVE_ANY(j0 < total); j0 += kScanUnroll) {
    GPC_STAT(10, 1);
    Ent ev[kScanUnroll];
#pragma unroll
    for (int u = 0; u < kScanUnroll; u++) {
      const uint32_t j = j0 + u;
      uint32_t d = dl[0];
#pragma unroll
      for (int l = 1; l < kL; l++) d = j >= upto[l - 1] ? dl[l] : d;
      const uint32_t idx = j < total ? j + d : 0u;
      GPC_TOUCH(&E[idx], 16);
      GPC_STAT(4, j < total ? 1 : 0);
      ev[u] = E[idx];
    }
    bool ps[kScanUnroll];
    bool probe = false;
#pragma unroll
    for (int u = 0; u < kScanUnroll; u++) {
      const uint32_t off = ent_off(ev[u].x);
      ps[u] = (off > after) & (off < rH) & entry_pass(p, ev[u], xv, cp);
      probe |= ps[u] & ((ev[u].x & 15u) - 8u < 7u) & !(ev[u].x & kEntExactX);
    }
    // Probe entries that passed: exact membership of the packet in the non-driver point-set
    // clause (point hash, both choices loaded before the compare), one entry slot at a time
    // and only when a lane of the wave needs it.
    if (GPC_WAVE_ANY(probe)) {
#pragma unroll
      for (int u = 0; u < kScanUnroll; u++) {
        const uint32_t pax = (ev[u].x & 15u) - 8u;
        const bool need = ps[u] & (pax < 7u) & !(ev[u].x & kEntExactX);
        if (GPC_WAVE_ANY(need)) {
          if (need) ps[u] = hash_contains(im, set_key(set_key_hi(ev[u].y & (kPointSetMax - 1u), pax), p.ax[pax]));
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kScanUnroll; u++) {
      const uint32_t off = ent_off(ev[u].x);
      const bool pass = ps[u];
      const uint32_t v = pass ? off : 0xffffffffu;
      const bool fresh = (v != 0xffffffffu) & (v != c0) & (v != c1);
      more |= fresh & (c1 != 0xffffffffu);  // a third distinct survivor: one of them is dropped
      const bool lt0 = fresh & (v < c0), lt1 = fresh & (v < c1);
      c1 = lt0 ? c0 : (lt1 ? v : c1);
      c0 = lt0 ? v : c0;
    }
  }
}

// One rule table (table = 1..6). All per-list merge state is indexed with compile-time indices
// only (unrolled), so it stays in VGPRs.
GPC_HD TablePart eval_part(const Img& im, uint32_t table, const Pkt& p) {
  GPC_MARK(ST_HARD);
  const TableHdr& th = im.hdr->t[table - 1];
  TablePart res;
  res.h = res.s = res.win = 0;
  uint32_t htie = 0, noact = 0;
  // --- hard pseudo-rules (few): best hard match H
  // (wave-uniform: the list, the records and their clause data are read with scalar loads)
  uint32_t rH = th.end_off;
  uint32_t hprio = 0, hverdict = RV_MISS;
  if (th.n_hfast) {
    // inline hard rules, rank order; branch-free per lane (a tie among hard flows of equal priority
    // and different verdicts; lower-priority ones after the first match do not count)
    bool stop = false;
    for (uint32_t h = 0; h < th.n_hfast; h++) {
      const HardFast& hf = th.hf[h];
      if (rule_dead(im, hf.rid)) continue;
      const uint32_t prio = hf.pv & 0xffffu, verdict = (hf.pv >> 16) & 0xffu;
      const bool m = hard_fast_match(im, hf, p);
      const bool found = rH != th.end_off;
      stop = stop | (found & (prio != hprio));
      htie = (!stop & found & (verdict != hverdict) & m) ? kHTie : htie;
      const bool take = !found & m;
      rH = take ? hf.roff : rH;
      hprio = take ? prio : hprio;
      hverdict = take ? verdict : hverdict;
    }
  } else {
    const cword* cblob = (const cword*)im.blob;
    const cword* hard = cblob + th.hard_off;
    for (uint32_t h = 0; h < th.n_hard; h++) {
      GPC_TOUCH(&hard[h], 4);
      const uint32_t off = hard[h];
      const cword* rec = cblob + off;
      GPC_TOUCH(rec, 4 * kRecLine);
      const uint32_t w1 = rec[1], w2 = rec[2], rid = rec[4] >> 8;
      if (rule_dead(im, rid)) continue;
      uint32_t dsc[3 * kMaxClauses];
#pragma unroll
      for (int j = 0; j < 3 * kMaxClauses; j++) dsc[j] = rec[kRecFcd + j];
      if (rH != th.end_off) {  // tie among hard flows of equal priority and different verdicts
        if ((w1 & 0xffffu) != hprio) break;
        if (rec_verdict(w2) != hverdict && rule_match(im, rec, w2, dsc, 0u, p)) htie = kHTie;
        continue;
      }
      if (rule_match(im, rec, w2, dsc, 0u, p)) {
        rH = off;
        hprio = w1 & 0xffffu;
        hverdict = rec_verdict(w2);
      }
    }
  }
  GPC_MARK(ST_DRV);
  // the hard match is packed now: of it only rH stays live (the scan's bound), and "found" is
  // res.h's kHFound bit (a separate flag was the base kernels' last spilled register)
  if (rH != th.end_off) res.h = hprio | (hverdict << 16) | kHFound | htie;
  if (th.bits_off && !im.dead) {  // bit-parallel table (tombstones: the scan below honours them)
    const BitTable& bt = *reinterpret_cast<const BitTable*>(im.blob + th.bits_off);
    uint32_t s0 = bt.absent[0], s1 = bt.absent[1], s2 = bt.absent[2];
    const uint32_t np = bt.n_probe;
    constexpr uint32_t kBatch = 3;  // probes whose slot loads are in flight together (register budget)
#pragma unroll
    for (uint32_t q0 = 0; q0 < kBitProbes; q0 += kBatch) {
      if (q0 >= np) break;
      BitSlot c1[kBatch], c2[kBatch];
      uint32_t key[kBatch];
#pragma unroll
      for (uint32_t j = 0; j < kBatch; j++) {  // every slot load of the batch issued before any is used
        const uint32_t q = q0 + j;
        key[j] = 0;
        c1[j] = c2[j] = BitSlot{1u, 0u};
        if (q < np) {
          const BitProbe pr = bt.probe[q];
          key[j] = p.ax[pr.ak & 15u] & pr.mask;
          const uint32_t h = bit_hash(q, key[j]), m = (1u << pr.lg) - 1u;
          const BitSlot* sl = reinterpret_cast<const BitSlot*>(im.blob + pr.off);
          GPC_TOUCH(sl + (h & m), 8);
          GPC_TOUCH(sl + ((h >> 16) & m), 8);
          c1[j] = sl[h & m];
          c2[j] = sl[(h >> 16) & m];
        }
      }
#pragma unroll
      for (uint32_t j = 0; j < kBatch; j++) {
        const uint32_t q = q0 + j;
        if (q < np) {
          const uint32_t k = bt.probe[q].ak >> 8;
          const uint32_t v = (c1[j].x == key[j] ? c1[j].y : 0u) | (c2[j].x == key[j] ? c2[j].y : 0u);
          s0 |= k == 0 ? v : 0u;
          s1 |= k == 1 ? v : 0u;
          s2 |= k == 2 ? v : 0u;
        }
      }
    }
    uint32_t done = s0 & s1 & s2;
    if (res.h & kHFound) {  // only rules ranked above the hard match
      const uint32_t np_ = rH == th.hf[0].roff ? bt.hard_prefix[0] : bt.hard_prefix[1];
      done &= np_ >= 32u ? 0xffffffffu : (1u << np_) - 1u;
    }
    if (done) {
      const uint32_t w = uint32_t(__builtin_ctz(done));
      GPC_TOUCH(&bt.info[2 * w], 8);
      uint32_t roff, pe;
      load_pair(&bt.info[2 * w], &roff, &pe);
      const uint32_t end = pe >> 16;  // rules w + 1 .. end - 1 share w's priority
      const uint32_t later = end >= 32u ? 0xffffffffu : (1u << end) - 1u;
      const bool tie = (done & later & ~((2u << w) - 1u)) != 0u;
      res.s = (pe & 0xffffu) | kSHave | (tie ? kSTie : 0u);
      res.win = roff;
    }
    return res;
  }
  const uint32_t n0 = th.n_idx[0], n1 = th.n_idx[1];
  if (th.n_cidx == 0 && n0 == 0 && th.always_n[0] == 0 && n1 == 0 && th.always_n[1] == 0) return res;  // no soft rules
  // --- driver clause: the composite driver when the table has one (a subset of either plain
  // driver's candidates, table-uniform branch), else the clause with fewer candidate records
  uint32_t lo0[kIdxPerClause], hi0[kIdxPerClause], lo1[kIdxPerClause], hi1[kIdxPerClause];
  const uint32_t nc = th.n_cidx;
  bool d1 = false;
  uint32_t d = 0;
  uint32_t always_n = 0;  // entries of the driver's always list to scan
  uint32_t cp = 0;        // the packet's combination id (kBandCombo sub-index)
  if (nc) {
    d = th.cband;
    const uint32_t xv = p.ax[th.cx];
    const uint32_t xb = cx_bit(xv);
    GPC_TOUCH(im.blob + th.xmap_off + (xb >> 5), 4);
    const bool xin = (im.blob[th.xmap_off + (xb >> 5)] >> (xb & 31u)) & 1u;  // else no soft rule can match
    always_n = xin ? th.always_n[d] : 0u;
    uint32_t cnt = always_n;
    // bucket keys: the band keys, or for a combination sub-index (table-uniform) the packet's
    // combination id, looked up in the value-map word's round; 0 (in no set): an empty list
    uint32_t key[kIdxPerClause];
#pragma unroll
    for (int i = 0; i < kIdxPerClause; i++) {
      key[i] = 0u;
      if (uint32_t(i) < nc) {
        const SubIdx& si = th.cidx[i];
        key[i] = si.band == kBandCombo ? combo_of(im.blob, si.pres, p.ax[si.axis]) : p.ax[si.axis];
        if (si.band == kBandCombo) cp = key[i];
      }
    }
    if (th.cidx[0].fmt) {
      // bucket directories: one 16-B block per sub-index (and a pointer entry where a bucket
      // overflowed), read in the value-map word's round (fmt 1) or, where the map filters most
      // packets, only for the packets in it (fmt 2). The branch is wave-uniform, so the fmt-1 loads
      // do not wait for the map word.
      bool ovf = false;
#pragma unroll
      for (int i = 0; i < kIdxPerClause; i++) lo0[i] = hi0[i] = lo1[i] = hi1[i] = 0;
      if (th.cidx[0].fmt == 1) {
#pragma unroll
        for (int i = 0; i < kIdxPerClause; i++)
          if ((uint32_t(i) < nc) && (th.cidx[i].band != kBandCombo || key[i] != 0u)) {
            const SubIdx& si = th.cidx[i];
            dir_list(im.blob, si, cbucket_of(si.band, si.bits, key[i], xv), &lo0[i], &hi0[i]);
          }
      } else {
#pragma unroll
        for (int i = 0; i < kIdxPerClause; i++)
          if ((uint32_t(i) < nc) & xin && (th.cidx[i].band != kBandCombo || key[i] != 0u)) {
            const SubIdx& si = th.cidx[i];
            dir_list(im.blob, si, cbucket_of(si.band, si.bits, key[i], xv), &lo0[i], &hi0[i]);
          }
      }
#pragma unroll
      for (int i = 0; i < kIdxPerClause; i++) {
        if (!xin) hi0[i] = lo0[i];
        ovf = ovf | (hi0[i] - lo0[i] == kDirCountMax);
      }
      if (GPC_WAVE_ANY(ovf)) {
        const Ent* E = reinterpret_cast<const Ent*>(im.blob);
#pragma unroll
        for (int i = 0; i < kIdxPerClause; i++) {
          if ((uint32_t(i) < nc) && hi0[i] - lo0[i] == kDirCountMax) {
            GPC_TOUCH(&E[lo0[i]], 16);
            const Ent pe = E[lo0[i]];
            lo0[i] = th.cidx[i].ent / 4u + pe.y;
            hi0[i] = lo0[i] + pe.lo;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < kIdxPerClause; i++) cnt += hi0[i] - lo0[i];
    } else {
    // presence words (L2-resident) are read in the value-map word's round; an offset pair only
    // for a present bucket of a packet whose value is in the map
    uint32_t bk[kIdxPerClause], pw[kIdxPerClause];
#pragma unroll
    for (int i = 0; i < kIdxPerClause; i++) {
      bk[i] = pw[i] = 0;
      if (uint32_t(i) < nc) {
        const SubIdx& si = th.cidx[i];
        bk[i] = cbucket_of(si.band, si.bits, key[i], xv);
        if (si.pres) {
          GPC_TOUCH(im.blob + si.pres + (bk[i] >> 5), 4);
          pw[i] = im.blob[si.pres + (bk[i] >> 5)];
        } else {
          pw[i] = ~0u;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kIdxPerClause; i++) {
      lo0[i] = hi0[i] = lo1[i] = hi1[i] = 0;
      if ((uint32_t(i) < nc) & xin & ((pw[i] >> (bk[i] & 31u)) & 1u)) {
        const SubIdx& si = th.cidx[i];
        const uint32_t* o = im.blob + si.off;
        GPC_TOUCH(o + bk[i], 8);
        uint32_t ob, oe;
        load_pair(o + bk[i], &ob, &oe);
        lo0[i] = si.ent / 4 + ob;
        hi0[i] = si.ent / 4 + oe;
        cnt += hi0[i] - lo0[i];
      }
    }
    }
    GPC_STAT(0, 1);
    GPC_STAT(1, cnt);
  } else {
    uint32_t cnt0 = th.always_n[0], cnt1 = th.always_n[1];
#pragma unroll
    for (int i = 0; i < kIdxPerClause; i++) {
      lo0[i] = hi0[i] = lo1[i] = hi1[i] = 0;
      if (uint32_t(i) < n0) {
        const SubIdx& si = th.idx[0][i];
        const uint32_t b = bucket_of(si.axis, si.band, si.bits, p.ax[si.axis]);
        const uint32_t* o = im.blob + si.off;
        GPC_TOUCH(o + b, 8);
        uint32_t ob, oe;
        load_pair(o + b, &ob, &oe);
        lo0[i] = si.ent / 4 + ob;
        hi0[i] = si.ent / 4 + oe;
        cnt0 += hi0[i] - lo0[i];
      }
      if (uint32_t(i) < n1) {
        const SubIdx& si = th.idx[1][i];
        const uint32_t b = bucket_of(si.axis, si.band, si.bits, p.ax[si.axis]);
        const uint32_t* o = im.blob + si.off;
        GPC_TOUCH(o + b, 8);
        uint32_t ob, oe;
        load_pair(o + b, &ob, &oe);
        lo1[i] = si.ent / 4 + ob;
        hi1[i] = si.ent / 4 + oe;
        cnt1 += hi1[i] - lo1[i];
      }
    }
    d1 = cnt1 < cnt0;
    d = d1 ? 1u : 0u;
    always_n = th.always_n[d];
    GPC_STAT(0, 1);
    GPC_STAT(1, d1 ? cnt1 : cnt0);
    GPC_STAT(2, d1 ? cnt0 : cnt1);
  }
  // Candidate scan. The driver lists (0 = always list, 1.. = sub-index buckets) are walked as one
  // flattened sequence (scan_lists), keeping the two best-ranked prefilter survivors. They are then
  // verified in rank order; if more candidates passed and no decision was reached, the lists are
  // rescanned above the last verified offset. Same result as a k-way merge in rank order.
  uint32_t dl[kLists], upto[kLists];  // entry index offset per list; cumulative end in the flattened scan
  dl[0] = th.always_off[d] / 4;
  upto[0] = always_n;
#pragma unroll
  for (int i = 0; i < kIdxPerClause; i++) {
    const uint32_t lo = d1 ? lo1[i] : lo0[i], hi = d1 ? hi1[i] : hi0[i];
    dl[i + 1] = lo - upto[i];
    upto[i + 1] = upto[i] + (hi - lo);
  }
  const uint32_t total = upto[kLists - 1];
  const bool one_idx = nc ? nc <= 1 : n0 <= 1 && n1 <= 1;  // table-uniform: every driver list set has <= 1 sub-index
  const uint32_t xv = nc ? p.ax[th.cx] : 0u;  // exact-value entries exist only in composite lists
  uint32_t after = 0;       // rescan bound (exclusive); record offsets are > 0
  int have = 0;             // result found
  uint32_t level = 0xffffffffu;
  uint32_t level_done = 0;  // completed conjunctions at the current level
  uint32_t win = 0;         // winner record offset (soft) when have == 1 and !noact
  bool done = total == 0;
  while (!done) {
    uint32_t c0, c1;
    bool more;
    GPC_MARK(ST_SCAN);
    GPC_STAT(8, 1);
    if (one_idx) scan_lists<2>(im, p, dl, upto, total, after, rH, xv, cp, c0, c1, more);
    else scan_lists<kLists>(im, p, dl, upto, total, after, rH, xv, cp, c0, c1, more);
    GPC_MARK(ST_VER);
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const uint32_t off = q ? c1 : c0;
      if (off == 0xffffffffu || done) break;
      after = off;
      const uint32_t* rec = im.blob + off;
      GPC_TOUCH(rec, 4 * kRecLine);
      const RecLine hd = load_rec_line(rec);
      const uint32_t w1 = hd.w[1], w2 = hd.w[2];
      const uint32_t prio = w1 & 0xffffu;
      if (prio != level) {
        if (have) {  // winning level finished
          done = true;
          break;
        }
        level = prio;
        level_done = 0;
      }
      GPC_STAT(3, 1);
      const uint32_t rid = hd.w[4] >> 8;
      if (rule_dead(im, rid) || !rule_match(im, rec, w2, &hd.w[kRecFcd], (hd.w[5] >> (3 * d)) & 7u, p)) {
        GPC_STAT(5, 1);
        continue;
      }
      level_done++;
      if (have) {  // a second completion at the winning level
        done = true;
        break;
      }
      if (rec_has_act(w2)) {
        have = 1;
        win = off;
      } else if (res.h & kHFound) {
        have = 1;
        noact = kSNoAct;
      }
    }
    if (!more) done = true;
  }
  GPC_MARK(ST_TAIL);
  if (have) {
    res.s = level | kSHave | noact | (level_done > 1 ? kSTie : 0u);
    res.win = win;
  }
  return res;
}

// Union of two images' rule sets for one table (base with tombstones + overlay). The best hard
// match is the higher one (equal priorities: lower verdict, tie if they differ); a soft decision
// survives only above the combined hard priority; equal levels tie and the lower conj id wins.
GPC_HD TablePart combine_parts(const View& v, const TablePart& a, TablePart b) {
  b.s |= b.s & kSHave ? kSImg : 0u;  // b is the overlay's part
  TablePart r;
  const uint32_t ah = a.h & 0xffffu, bh = b.h & 0xffffu;
  const bool af = (a.h & kHFound) != 0, bf = (b.h & kHFound) != 0;
  if (bf && (!af || bh > ah)) {
    r.h = b.h;
  } else if (bf && af && bh == ah) {
    const uint32_t av = (a.h >> 16) & 0xffu, bv = (b.h >> 16) & 0xffu;
    r.h = ah | ((av < bv ? av : bv) << 16) | kHFound | ((a.h | b.h) & kHTie) | (av != bv ? kHTie : 0u);
  } else {
    r.h = a.h;
  }
  const bool hf = (r.h & kHFound) != 0;
  const uint32_t hp = r.h & 0xffffu;
  const uint32_t al = a.s & 0xffffu, bl = b.s & 0xffffu;
  const bool va = (a.s & kSHave) && (!hf || al > hp);
  const bool vb = (b.s & kSHave) && (!hf || bl > hp);
  if (va && vb && al == bl) {  // both decided at one level: a tie; the lower conj id wins
    const uint32_t ca = (a.s & kSNoAct) ? 0xffffffffu : v.base.blob[a.win];
    const uint32_t cb = (b.s & kSNoAct) ? 0xffffffffu : v.ovl.blob[b.win];
    const bool pb = cb < ca;  // fields selected one by one: a reference select puts both parts on the stack
    r.s = (pb ? b.s : a.s) | kSTie;
    r.win = pb ? b.win : a.win;
  } else if (vb && (!va || bl > al)) {
    r.s = b.s;
    r.win = b.win;
  } else if (va) {
    r.s = a.s;
    r.win = a.win;
  } else {
    r.s = 0;
    r.win = 0;
  }
  return r;
}

GPC_HD TableResult finish_part(const uint32_t* base_blob, const uint32_t* ovl_blob, const TablePart& q) {
  GPC_MARK(ST_FIN);
  TableResult res;
  res.verdict = RV_MISS;
  res.tie = (q.h & kHTie) ? 1 : 0;
  res.tier = 0;
  res.counted = 0;
  res.conj = 0;
  res.slot = 0;
  res.pin = 0;
  res.prio = 0;
  const bool hf = (q.h & kHFound) != 0, have = (q.s & kSHave) != 0;
  if (have && !(q.s & kSNoAct)) {
    const RecHdr hd = load_rec_hdr(((q.s & kSImg) ? ovl_blob : base_blob) + q.win);
    const uint32_t w2 = hd.w[2];
    if (!(hf && (q.h & 0xffffu) > (hd.w[1] >> 16))) {  // the soft winner's action flow beats the hard match
      res.verdict = uint8_t(rec_verdict(w2));
      res.conj = hd.w[0];
      res.tier = uint8_t(hd.w[4] & 0xffu);
      res.counted = uint8_t(rec_counted(w2));
      res.slot = hd.w[3];
      res.pin = (hd.w[5] & kRecPacketIn) ? uint32_t(GPC_VFLAG_PACKETIN) : 0u;
      res.prio = hd.w[1] >> 16;
      if (q.s & kSTie) res.tie = 1;
      return res;
    }
  }
  if (hf) {
    res.verdict = uint8_t((q.h >> 16) & 0xffu);
    res.prio = q.h & 0xffffu;
    if (have && (q.s & kSTie)) res.tie = 1;
  }
  return res;
}

// The journal's decision for one table: hard pseudo-rules in rank order (as eval_part), then the
// chains of the driver clause with the shorter total chain length, every live entry whose key and
// prefilter pass verified; the best completion (priority desc, conj id asc) and whether another
// completed at its level. Unordered: the journal is small and its records are not in rank order.
GPC_HD TablePart eval_journal(const View& v, uint32_t table, const Pkt& p) {
  const uint32_t* pool = v.ovl.blob;
  const JournalHdr* jh = reinterpret_cast<const JournalHdr*>(pool + v.jhdr);
  TablePart res;
  res.h = res.s = res.win = 0;
  if (!((jh->live >> (table - 1)) & 1u)) return res;  // nothing of this table in the journal (uniform)
  const JournalTable& jt = jh->t[table - 1];
  const uint32_t* odead = jh->odead_off ? pool + jh->odead_off : nullptr;
  Img im{pool, nullptr, odead, pool};
  uint32_t hprio = 0, hverdict = RV_MISS, htie = 0;
  bool hfound = false;
  for (uint32_t h = 0; h < jt.n_hard; h++) {
    const uint32_t off = pool[jt.hard_off + h];
    const uint32_t* rec = pool + off;
    const RecLine hd = load_rec_line(rec);
    const uint32_t w1 = hd.w[1], w2 = hd.w[2], rid = hd.w[4] >> 8;
    if (rule_dead(im, rid)) continue;
    if (hfound) {
      if ((w1 & 0xffffu) != hprio) break;
      if (rec_verdict(w2) != hverdict && rule_match(im, rec, w2, &hd.w[kRecFcd], 0u, p)) htie = kHTie;
      continue;
    }
    if (rule_match(im, rec, w2, &hd.w[kRecFcd], 0u, p)) {
      hfound = true;
      hprio = w1 & 0xffffu;
      hverdict = rec_verdict(w2);
    }
  }
  if (hfound) res.h = hprio | (hverdict << 16) | kHFound | htie;
  // Driver clause of the journal walk. A table with a composite base index: its band clause (the
  // other one holds the AppliedTo values, whose chains list every changed rule of a Pod), chosen
  // without reading any head; else the clause with the shorter chains (saturating chain lengths).
  uint32_t d;
  const TableHdr& bt = v.base.hdr->t[table - 1];
#if defined(GPC_JOURNAL_COUNT_ALWAYS)  // experiments: the pre-composite choice
  if (false) {
#else
  if (bt.n_cidx) {  // (every soft rule has clauses 0 and 1: one-clause rules compile to plain flows)
#endif
    d = bt.cband;
  } else {
    uint32_t cnt[2] = {jt.always[0] >> 24, jt.always[1] >> 24};
#pragma unroll
    for (uint32_t k = 0; k < 2; k++)
      for (uint32_t i = 0; i < jt.n_kinds[k]; i++) {
        const uint32_t axis = jt.kinds[k][i] & 15u, band = jt.kinds[k][i] >> 4;
        const uint32_t meta = jmeta(table, k, axis, band);
        cnt[k] += jhead(pool, jh, jbucket(meta, jkey(axis, band, p.ax[axis]), jh->lg)) >> 24;
      }
    if (cnt[0] + cnt[1] == 0) return res;
    d = (jt.n_kinds[1] || jt.always[1]) && cnt[1] < cnt[0] ? 1u : 0u;
  }
  uint32_t best = 0, best_prio = 0, best_conj = 0, at_best = 0;
  for (uint32_t i = 0; i <= jt.n_kinds[d]; i++) {
    uint32_t meta = 0, key = 0, e;
    if (i == jt.n_kinds[d]) {
      e = jt.always[d];
    } else {
      const uint32_t axis = jt.kinds[d][i] & 15u, band = jt.kinds[d][i] >> 4;
      meta = jmeta(table, d, axis, band);
      key = jkey(axis, band, p.ax[axis]);
      if (bt.n_cidx) key = jxkey(key, p.ax[bt.cx]);
      e = jhead(pool, jh, jbucket(meta, key, jh->lg));
    }
    const bool always = i == jt.n_kinds[d];
    while (e & 0xffffffu) {
      const uint32_t* en = pool + size_t(e & 0xffffffu) * kJEntWords;
      GPC_TOUCH(en, 4 * kJEntWords);
      // the 32-B entry as two 16-B loads (entries are 32-B aligned)
      uint32_t ew[kJEntWords];
#if defined(__HIPCC__) && !defined(GPC_JOURNAL_WORD_LOADS)
      const uint4 ea = reinterpret_cast<const uint4*>(en)[0], eb = reinterpret_cast<const uint4*>(en)[1];
      ew[0] = ea.x, ew[1] = ea.y, ew[2] = ea.z, ew[3] = ea.w, ew[4] = eb.x, ew[5] = eb.y, ew[6] = eb.z, ew[7] = eb.w;
#else
      for (uint32_t w = 0; w < kJEntWords; w++) ew[w] = en[w];
#endif
      e = ew[0];
      if (!always && (ew[1] != key || (ew[2] & kJMetaMask) != meta)) continue;
      GPC_STAT(15, 1u);  // (emulation: journal entries of the packet's keys)
      if (rule_dead(im, ew[2] >> kJOridShift)) continue;
      Ent f;
      f.x = ew[4];
      f.y = ew[5];
      f.lo = ew[6];
      f.hi = ew[7];
      if (!entry_pass<false>(p, f, 0u)) continue;  // (journal entries are never exact-value entries)
      const uint32_t off = ew[3];
      const uint32_t* rec = pool + off;
      GPC_TOUCH(rec, 4 * kRecLine);
      const RecLine hd = load_rec_line(rec);
      const uint32_t w1 = hd.w[1], w2 = hd.w[2];
      const uint32_t prio = w1 & 0xffffu, conj = hd.w[0];
      if (best && prio < best_prio) continue;  // cannot change the decision
      if (!rule_match(im, rec, w2, &hd.w[kRecFcd], 0u, p)) continue;
      if (!best || prio > best_prio) {
        best = off;
        best_prio = prio;
        best_conj = conj;
        at_best = 1;
      } else if (conj != best_conj) {  // same level (the same rule may be listed under several keys)
        at_best++;
        if (conj < best_conj) {
          best = off;
          best_conj = conj;
        }
      }
    }
  }
  if (best) {
    res.s = best_prio | kSHave | (at_best > 1 ? kSTie : 0u);
    res.win = best;
  }
  return res;
}

// ------------------------------------------------------------------------------ point extensions
// A rule whose current version differs from its base record only by exact values added to ONE
// clause (AddPolicyRuleAddress of Pod IPs / ofports / single ports, network_policy.go:1661) keeps
// its base record live: no tombstone, no journal copy (image.cpp Journal::apply). Each added value
// is an entry (table, axis, value) -> (base record, clause). Why that is exact: a packet the new
// version matches either matches the base version -- the base driver lists and verifies it as
// before, and a base match implies a match of the superset -- or fails some base clause and then
// holds an added value on the extended clause's axis, where the probe finds the rule and verifies
// its other clauses from the base record (the extended clause is decided by the probe). The index
// is small (live added values) and emitted whole per epoch: a presence bitmap (one L2-resident
// load settles almost every packet), bucket offsets, 16-B entries {value, table | axis << 3 |
// clause << 7 | composite << 9, record offset, priority}.
// Composite keys: in a table with a composite base index (TableHdr n_cidx), a value added to the
// band clause cband is keyed by (value, x) for every exact value x of the rule's clause 1 - cband
// (on axis cx), like the base's composite driver. Without that, a Pod IP added to many rules (C5
// mixed: ~70 rules per local Pod IP) made every packet from that Pod verify all of them (the
// extension probe went from 0 to 13 ms per 64 M-packet launch as the adds accumulated). The
// probe's hash then includes the packet's cx value; the record check still verifies clause
// 1 - cband, so a hash collision costs a verification, never a wrong verdict.
// Two levels (image.cpp emit_ext): the bulk level B, appended when rebuilt and shared by the
// epochs after it, and the delta level D of the rules changed since, appended per epoch with a
// bitmap over B's entries that tombstones the changed rules' B entries. Both levels are probed.
struct ExtHdr {
  uint32_t n;                   // D entries
  uint32_t pres_off, pres_log2;  // presence bitmap of B and D entries: 2^pres_log2 bits
  uint32_t bkt_off, bkt_log2;    // D: 2^bkt_log2 + 1 bucket offsets (entry index)
  uint32_t ent_off;              // D: entries, kExtEntWords words each, bucket-sorted
  // per table: bit a = some plain entry of the table is on axis a; bit 16 + a = a composite one
  uint32_t axes[6];
  uint32_t b_n, b_bkt_off, b_bkt_log2, b_ent_off;  // B (b_n 0: none)
  uint32_t b_tomb_off;                              // bit i: B entry i is dead
};
// Entries (32 B): {value, meta, record offset, priority, x, lo, hi, conj id}. meta = table | axis
// << 3 | clause << 7 | composite << 9 | exact << 10 | interval axis << 11. A composite entry holds
// the cx value x it is listed under (hash collisions are rejected without the record); an exact one
// also decides the rule's remaining clause (one interval [lo, hi] on the interval axis, or none: one
// entry per interval, like the base's exact-value entries), so the probe completes the rule from the
// entry alone -- no record read, no rule_match: C5 mixed packets that hit an added (Pod IP, ofport)
// pair paid a dependent record line and a point-set probe per candidate.
constexpr uint32_t kExtEntWords = 8;
constexpr uint32_t kExtComposite = 1u << 9;  // entry meta: keyed by (value, cx value)
constexpr uint32_t kExtExact = 1u << 10;     // entry meta: decides every clause (no record read)
GPC_HD uint32_t ext_meta(uint32_t table, uint32_t axis, uint32_t clause) { return table | (axis << 3) | (clause << 7); }
GPC_HD uint32_t ext_hash(uint32_t table, uint32_t axis, uint32_t v) {
  return mix32(v ^ mix32(((table << 4) | axis) * 0x9e3779b1u + 0x632be5abu));
}
GPC_HD uint32_t ext_hash_x(uint32_t table, uint32_t axis, uint32_t v, uint32_t x) {
  return mix32(ext_hash(table, axis, v) ^ cx_hash(x));
}
// The probe hash of kind bit b (ExtHdr axes) for packet p.
GPC_HD uint32_t ext_kind_hash(const View& v, uint32_t table, uint32_t b, const Pkt& p) {
  const uint32_t a = b & 15u;
  return b < 16u ? ext_hash(table, a, p.ax[a]) : ext_hash_x(table, a, p.ax[a], p.ax[v.base.hdr->t[table - 1].cx]);
}

// The presence words of a table's extended axes (at most two; more: scanned unconditionally),
// loaded before the base walk so their latency hides behind it (ext_begin), tested after it
// (ext_hits). Three registers live across the walk: the two words and their bit positions.
struct ExtProbe {
  uint32_t w0, w1;  // presence words of the first two extended axes
  uint32_t bits;    // their bit positions: b0 | b1 << 8 (0xffff: no such axis)
};
GPC_HD ExtProbe ext_begin(const View& v, uint32_t table, const Pkt& p) {
  const uint32_t* pool = v.ovl.blob;
  const ExtHdr* eh = reinterpret_cast<const ExtHdr*>(pool + v.ext);
  uint32_t axes = eh->axes[table - 1];
  ExtProbe x;
  x.w0 = x.w1 = 0;
  x.bits = 0xffffu;
  const uint32_t sh = 32u - eh->pres_log2;
  for (uint32_t i = 0; i < 2 && axes; i++) {
    const uint32_t b = uint32_t(__builtin_ctz(axes));
    axes &= axes - 1u;
    const uint32_t pb = ext_kind_hash(v, table, b, p) >> sh;
    GPC_TOUCH(pool + eh->pres_off + (pb >> 5), 4);
    const uint32_t w = pool[eh->pres_off + (pb >> 5)];
    if (i == 0) {
      x.w0 = w;
      x.bits = (x.bits & 0xff00u) | (pb & 31u);
    } else {
      x.w1 = w;
      x.bits = (x.bits & 0x00ffu) | ((pb & 31u) << 8);
    }
  }
  return x;
}
// Which extended axes the packet must scan: bit i = the i-th extended axis of the table (the first
// two by their presence bits, the others always).
GPC_HD uint32_t ext_hits(const View& v, uint32_t table, const ExtProbe& x) {
  const ExtHdr* eh = reinterpret_cast<const ExtHdr*>(v.ovl.blob + v.ext);
  const uint32_t axes = eh->axes[table - 1];
  const uint32_t n = uint32_t(__builtin_popcount(axes));
  const uint32_t b0 = (x.bits & 0xffu) != 0xffu ? (x.w0 >> (x.bits & 31u)) & 1u : 0u;
  const uint32_t b1 = ((x.bits >> 8) & 0xffu) != 0xffu ? (x.w1 >> ((x.bits >> 8) & 31u)) & 1u : 0u;
  return b0 | (b1 << 1) | (n > 2 ? ((1u << n) - 1u) & ~3u : 0u);
}

// Best completion among the extended rules the packet's values reach in this table (hard rules are
// never extended): priority desc, conj id asc, and whether two rules completed at that level.
// hits: ext_hits.
GPC_HD TablePart eval_ext(const View& v, uint32_t table, const Pkt& p, uint32_t hits) {
  TablePart res;
  res.h = res.s = res.win = 0;
  const uint32_t* pool = v.ovl.blob;
  const ExtHdr* eh = reinterpret_cast<const ExtHdr*>(pool + v.ext);
  uint32_t axes = eh->axes[table - 1];
  uint32_t best = 0, best_prio = 0, best_conj = 0, at_best = 0;
  const uint32_t xv = p.ax[v.base.hdr->t[table - 1].cx];  // (composite entries)
  for (uint32_t i = 0; axes; i++) {
    const uint32_t b = uint32_t(__builtin_ctz(axes)), a = b & 15u;
    axes &= axes - 1u;
    if (!((hits >> i) & 1u)) continue;
    const uint32_t val = p.ax[a], h = ext_kind_hash(v, table, b, p);
    const uint32_t meta = table | (a << 3) | (b < 16u ? 0u : kExtComposite);
    // both levels' bucket ranges are loaded before either is walked (two loads in flight, not two
    // dependent rounds); an empty level reads the range [0, 0)
    uint32_t rng[2][2] = {{0u, 0u}, {0u, 0u}};
#pragma unroll
    for (uint32_t lv = 0; lv < 2; lv++)
      if (lv ? eh->b_n : eh->n) {
        const uint32_t* bk = pool + (lv ? eh->b_bkt_off : eh->bkt_off) + (h & ((1u << (lv ? eh->b_bkt_log2 : eh->bkt_log2)) - 1u));
        GPC_TOUCH(bk, 8);
        load_pair(bk, &rng[lv][0], &rng[lv][1]);
      }
    for (uint32_t lv = 0; lv < 2; lv++) {  // D, then B
    const uint32_t eo = lv ? eh->b_ent_off : eh->ent_off;
    for (uint32_t e = rng[lv][0], end = rng[lv][1]; e < end; e++) {
      const uint32_t* en = pool + eo + e * kExtEntWords;
      GPC_TOUCH(en, 32);
#if defined(__HIPCC__)
      const uint4 q = reinterpret_cast<const uint4*>(en)[0], r = reinterpret_cast<const uint4*>(en)[1];
#else
      const struct { uint32_t x, y, z, w; } q = {en[0], en[1], en[2], en[3]}, r = {en[4], en[5], en[6], en[7]};
#endif
      if (q.x != val || (q.y & (0x7fu | kExtComposite)) != meta) continue;
      if ((q.y & kExtComposite) && r.x != xv) continue;  // another x (a bucket collision)
      if (lv && ((pool[eh->b_tomb_off + (e >> 5)] >> (e & 31u)) & 1u)) continue;  // a changed rule's B entry
      const uint32_t prio = q.w;
      if (best && prio < best_prio) continue;  // cannot change the decision
      const uint32_t conj = r.w;
      if (q.y & kExtExact) {
        const uint32_t iax = (q.y >> 11) & 15u, sv = p.ax[iax < AX_N ? iax : 0];
        if (iax != kFiltNoAxis && (sv < r.y || sv > r.z)) continue;
      } else {
        const uint32_t* rec = v.base.blob + q.z;
        GPC_TOUCH(rec, 4 * kRecLine);
        // the extended clause is decided by the value; a composite entry's clause 1 - clause by x
        const uint32_t k = (q.y >> 7) & 3u, skip = (1u << k) | ((q.y & kExtComposite) ? 1u << (1u - k) : 0u);
        if (!rule_match(v.base, rec, rec[2], rec + kRecFcd, skip, p)) continue;
      }
      if (!best || prio > best_prio) {
        best = q.z;
        best_prio = prio;
        best_conj = conj;
        at_best = 1;
      } else if (conj != best_conj) {
        at_best++;
        if (conj < best_conj) {
          best = q.z;
          best_conj = conj;
        }
      }
    }
    }
  }
  if (best) {
    res.s = best_prio | kSHave | (at_best > 1 ? kSTie : 0u);
    res.win = best;
  }
  return res;
}

// a (base, or base + journal) and e (extended rules; records in the base) for one table. The hard
// match is a's; e counts only above it. One rule reached both ways is one completion, not a tie.
GPC_HD TablePart merge_ext(const View& v, const TablePart& a, const TablePart& e) {
  if (!(e.s & kSHave)) return a;
  const bool hf = (a.h & kHFound) != 0;
  const uint32_t hp = a.h & 0xffffu, al = a.s & 0xffffu, el = e.s & 0xffffu;
  const bool va = (a.s & kSHave) != 0;
  if (hf && el <= hp) return a;
  TablePart r;
  r.h = a.h;
  if (va && al == el) {
    if (!(a.s & (kSImg | kSNoAct)) && a.win == e.win) {
      r.s = a.s | (e.s & kSTie);
      r.win = a.win;
      return r;
    }
    // (the blobs are read into values first: selecting between two fields of the View by address
    // keeps the whole View in scratch memory)
    const uint32_t* const ob = v.ovl.blob;
    const uint32_t* const bb = v.base.blob;
    const uint32_t ca = (a.s & kSNoAct) ? 0xffffffffu : (a.s & kSImg) ? ob[a.win] : bb[a.win];
    const uint32_t ce = v.base.blob[e.win];
    const bool pe = ce < ca;
    r.s = (pe ? e.s : a.s) | kSTie;
    r.win = pe ? e.win : a.win;
    return r;
  }
  if (!va || el > al) {
    r.s = e.s;
    r.win = e.win;
    return r;
  }
  return a;
}

// kMode (kModeBase / kModeExt / kModeJournal): what of the epoch the table walk reads; the base
// instantiation compiles neither the journal nor the extension code.
template <int kMode>
GPC_HD TableResult eval_table(const View& v, uint32_t table, const Pkt& p) {
  // point extensions: presence words in flight during the base walk. (Waiting for them first and
  // parking the result in LDS (Pkt::park) cut the extension kernels' spills from 9-10 to 8 VGPRs
  // but made C5 1 ms slower per step: the wait costs more than the scratch traffic.)
  ExtProbe xp;
  const bool ext = kMode >= kModeExt && v.ext;
  if (ext) xp = ext_begin(v, table, p);
  TablePart acc = eval_part(v.base, table, p);
  if (kMode >= kModeJournal && v.n_img > 1) acc = combine_parts(v, acc, eval_journal(v, table, p));
  if (ext) {
    const uint32_t hits = ext_hits(v, table, xp);
    if (GPC_WAVE_ANY(hits != 0u)) acc = merge_ext(v, acc, eval_ext(v, table, p, hits));
  }
  return finish_part(v.base.blob, kMode >= kModeJournal ? v.ovl.blob : nullptr, acc);
}

// ------------------------------------------------------------------------------ Service image
// AntreaProxy stage in front of the policy tables, resolved at build time from the
// realized ServiceLB flows, select groups, EndpointDNAT flows and the Pod map (service.cpp):
//   SvcHdr at word 0; a key -> service hash (2-choice, 8-way buckets: 16 words of uint64 keys
//   (1 << 63 | proto << 48 | port << 32 | ip), 8 words of values = service index, 8 pad);
//   service records {first endpoint, n_ep | slot_log2 << 24, group id, flags};
//   endpoint records {ip, port | flags << 16, out_port (reg1), destination class}.
struct SvcHdr {
  uint32_t hash_off, hash_log2, svc_off, n_svc, ep_off, n_ep;
  uint32_t map_off, map_log2;  // 2^map_log2-bit map of the keys (svc_map_bit): most packets that
                               // address no Service are settled by one load
  // NodePort addresses (the NodePortMark flows' nw_dst, pipeline.go:2282-2314; 0 when no NodePort
  // Service exists): a packet to one of them that misses the (protocol, address, port) key takes
  // the NodePort key (protocol, 0, port) -- ServiceLB's ToNodePortAddressRegMark flows
  uint32_t np_off, n_np;
};
constexpr uint32_t kSvcMaxNodePortAddrs = 64;
// Service hash: 2-choice cuckoo, buckets of two 16-B slots {key low, key high, service index, 0}:
// a lookup is one 128-bit load per slot (four per packet), not a 96-B scan of an 8-way bucket.
constexpr uint32_t kSvcBucketWords = 8, kSvcSlots = 2, kSvcSlotWords = 4;
constexpr uint32_t kSvcLoadReg7 = 1u;  // service flag: the ServiceLB flow loads reg7 = group id
// endpoint flags (port word >> 16): GPC_LB_DNAT / GPC_LB_REMOTE values
GPC_HD uint64_t svc_key(uint32_t proto, uint32_t ip, uint32_t port) {
  return (1ull << 63) | (uint64_t(proto & 0xffu) << 48) | (uint64_t(port & 0xffffu) << 32) | ip;
}
GPC_HD uint32_t svc_map_bit(uint64_t key, uint32_t log2) { return uint32_t(mix64(key ^ 0xa0761d6478bd642full) >> (64 - log2)); }
// Endpoint selection of the select group. OVS picks a bucket by dp_hash over a symmetric L4 hash
// with a 64-slot table for equal weights (OVS-internal, not in the reference: parity unpinned);
// restated: symmetric hash of (src ^ dst, sport ^ dport, proto), slot table of 2^slot_log2 >= 64
// entries, slot s -> bucket s mod n (Antrea gives every bucket weight 100).
GPC_HD uint32_t lb_hash(uint32_t src, uint32_t dst, uint32_t sport, uint32_t dport, uint32_t proto) {
  return mix32((src ^ dst) ^ (mix32(((sport ^ dport) << 8) | (proto & 0xffu)) * 0x9e3779b1u));
}
// Index into the service records, or 0xffffffff.
GPC_HD uint32_t svc_lookup(const uint32_t* sv, uint32_t proto, uint32_t ip, uint32_t port) {
  const SvcHdr* h = reinterpret_cast<const SvcHdr*>(sv);
  const uint64_t key = svc_key(proto, ip, port);
  const uint32_t mb = svc_map_bit(key, h->map_log2);
  GPC_TOUCH(sv + h->map_off + (mb >> 5), 4);
  if (!((sv[h->map_off + (mb >> 5)] >> (mb & 31u)) & 1u)) return 0xffffffffu;
  const uint32_t mask = (1u << h->hash_log2) - 1u;
  const uint32_t bs[2] = {hash_b1(key, mask), hash_b2(key, mask)};
  const uint32_t klo = uint32_t(key), khi = uint32_t(key >> 32);
  uint32_t r = 0xffffffffu;
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const uint32_t* b = sv + h->hash_off + size_t(bs[c]) * kSvcBucketWords;
    GPC_TOUCH(b, 4 * kSvcBucketWords);
#pragma unroll
    for (uint32_t i = 0; i < kSvcSlots; i++) {
#if defined(__HIPCC__)
      const uint4 v = reinterpret_cast<const uint4*>(b)[i];
      const uint32_t w0 = v.x, w1 = v.y, w2 = v.z;
#else
      const uint32_t w0 = b[kSvcSlotWords * i], w1 = b[kSvcSlotWords * i + 1], w2 = b[kSvcSlotWords * i + 2];
#endif
      r = (w0 == klo && w1 == khi) ? w2 : r;
    }
  }
  return r;
}

// The Service stage of one packet (ServiceLB -> group bucket -> EndpointDNAT -> L3Forwarding):
// rewrites dst / dport (DNAT), reg7, reg1 and the destination class; o[0..3] = gpc_lb_result
// words {endpoint ip, port | flags << 16, group id, out_port}. Returns the GPC_LB_* flags (0: the
// packet is not addressed to a Service). ct_nw_dst keeps the pre-NAT destination: the caller
// takes it before this call.
GPC_HD uint32_t lb_stage(const uint32_t* sv, uint32_t src, uint32_t& dst, uint32_t sport, uint32_t& dport, uint32_t proto,
                         uint32_t& svc_group, uint32_t& out_port, uint32_t& dest, uint32_t* o) {
  o[0] = o[1] = o[2] = o[3] = 0;
  if (proto != 6 && proto != 17 && proto != 132) return 0;
  const SvcHdr* h = reinterpret_cast<const SvcHdr*>(sv);
  uint32_t si = svc_lookup(sv, proto, dst, dport);
  if (si == 0xffffffffu && h->n_np) {  // NodePortMark, then the NodePort ServiceLB flows
    bool np = false;
    for (uint32_t i = 0; i < h->n_np; i++) np |= sv[h->np_off + i] == dst;
    if (np) si = svc_lookup(sv, proto, 0u, dport);
  }
  if (si == 0xffffffffu) return 0;
  const uint32_t* s = sv + h->svc_off + 4 * si;
  GPC_TOUCH(s, 16);
  const uint32_t n = s[1] & 0xffffffu, lg = s[1] >> 24;
  uint32_t flags = GPC_LB_HIT;
  o[2] = s[2];
  if (s[3] & kSvcLoadReg7) svc_group = s[2];
  if (n == 0) {
    flags |= GPC_LB_NO_ENDPOINT;
    o[1] = flags << 16;
    return flags;
  }
  const uint32_t slot = lb_hash(src, dst, sport, dport, proto) & ((1u << lg) - 1u);
  const uint32_t* e = sv + h->ep_off + 4 * (s[0] + slot % n);
  GPC_TOUCH(e, 16);
  flags |= e[1] >> 16;
  o[0] = e[0];
  o[1] = (e[1] & 0xffffu) | (flags << 16);
  o[3] = e[2];
  if (flags & GPC_LB_DNAT) {
    dst = e[0];
    dport = e[1] & 0xffffu;
  }
  out_port = e[2];
  dest = e[3];
  return flags;
}

// Verdict word layout (gpc_verdict): conj_id | action | table | tier | flags.
struct VerdictOut {
  uint32_t conj;
  uint32_t packed;  // action | table << 8 | tier << 16 | flags << 24
};

GPC_HD uint32_t pack_verdict(uint32_t action, uint32_t table, uint32_t tier, uint32_t flags) {
  return action | (table << 8) | (tier << 16) | (flags << 24);
}

// Both stages of one packet (the kernel body): one loop over the six rule tables so the table
// evaluation is instantiated once. Egress = tables 1-3, ingress = 4-6; per stage the walk is
// AntreaPolicy*Rule -> *Rule -> *DefaultRule with miss = next and Pass = goto *Rule
// (pipeline.go:1861-1886); reg5/reg6 after a Pass keep the Pass rule's conj id and tier.
struct PacketOut {
  VerdictOut e, g;
  uint32_t eslot, gslot;
  int ecounted, gcounted;
};

// gpc_trace (Traceflow readback, traceflow/packetin.go:211-270): one record per rule table the
// packet's walk evaluated, in walk order.
struct TraceStep {
  uint32_t table;       // 1..6
  uint32_t verdict;     // RVerdict of the table (RV_MISS: table-miss -> next table)
  uint32_t flags;       // GPC_VFLAG_TIE / GPC_VFLAG_PACKETIN of this table's decision
  uint32_t conj;        // deciding conjunction (0: hard flow or miss)
  uint32_t priority;    // priority of the deciding flow (0: miss)
  uint32_t candidates;  // driver-list entries the table's scan had to consider (scan_estimate)
};
constexpr uint32_t kMaxTraceSteps = 8;

// One policy stage: its three rule tables from t0 (1 = egress, 4 = ingress). Every exit returns from
// inside the loop, so the only state carried from one table to the next is the Pass rule's conj id
// and the packed flags | tier word (register pressure: the walk is the kernel's hot region).
struct StageOut {
  VerdictOut v;
  uint32_t slot;
  int counted;
};
template <int kMode, bool kTrace>
GPC_HD StageOut walk_stage(const View& im, const Pkt& p, uint32_t t0, TraceStep* trace, uint32_t* n_trace) {
  uint32_t conj = 0, ft = 0;  // ft = flags | tier << 8 (reg5/reg6 after a Pass keep its conj id and tier)
  for (uint32_t i = 0;; i++) {
    const uint32_t t = t0 + i;
    // a table without rules (base, or journal: neither the base nor the journal has any; extended
    // rules are base rules): a miss, without reading its header
    const uint32_t live = kMode < kModeJournal || im.n_img < 2
                              ? im.base.hdr->live
                              : im.base.hdr->live | reinterpret_cast<const JournalHdr*>(im.ovl.blob + im.jhdr)->live;
    if (!kTrace && !((live >> (t - 1)) & 1u)) {
      if (i < 2) continue;
      StageOut o;
      o.slot = 0;
      o.counted = 0;
      o.v.conj = conj;
      o.v.packed = pack_verdict(1 /*NO_MATCH*/, 0, ft >> 8, ft & 0xffu);
      return o;
    }
    const TableResult r = eval_table<kMode>(im, t, p);
    GPC_MARK(ST_WALK);
    if (kTrace && *n_trace < kMaxTraceSteps) {
      TraceStep& st = trace[(*n_trace)++];
      st.table = t;
      st.verdict = r.verdict;
      st.flags = (r.tie ? 2u : 0u) | r.pin;
      st.conj = r.conj;  // the soft winner's conjunction (0 for hard flows and misses)
      st.priority = r.prio;
      st.candidates = scan_estimate(im.base, t, p);
    }
    ft |= (r.tie ? 2u : 0u) | r.pin;
    if (r.verdict == RV_PASS) {
      conj = r.conj;
      ft = (ft & 0xffu) | 1u | (uint32_t(r.tier) << 8);
    }
    StageOut o;
    o.slot = 0;
    o.counted = 0;
    if (r.verdict == RV_MISS || r.verdict == RV_PASS) {
      if (i < 2) continue;
      o.v.conj = conj;
      o.v.packed = pack_verdict(1 /*NO_MATCH*/, 0, ft >> 8, ft & 0xffu);
      return o;
    }
    const uint32_t act = r.verdict;  // RV_* values 2..6 equal GPC_ACT_*
    if (act != RV_ISO_DROP && act != RV_BYPASS) {
      conj = r.conj;
      ft = (ft & 0xffu) | (uint32_t(r.tier) << 8);
    }
    o.v.conj = conj;
    o.v.packed = pack_verdict(act, i + 1, ft >> 8, ft & 0xffu);
    o.slot = r.slot;
    o.counted = r.counted && (act == RV_ALLOW || act == RV_DROP || act == RV_REJECT);
    return o;
  }
}

// kStage: 0 = both stages; 1 = egress only; 2 = ingress only (the caller has checked that the
// egress verdict lets the packet reach the ingress tables). kStage 0 runs walk_stage in a loop over
// the two stages so the table evaluation is instantiated once.
template <int kMode = kModeJournal, int kStage = 0, bool kTrace = false>
GPC_HD PacketOut classify_packet(const View& im, const Pkt& p, uint32_t dest, uint32_t ct_mark,
                                 TraceStep* trace = nullptr, uint32_t* n_trace = nullptr) {
  PacketOut o;
  o.e.conj = o.g.conj = 0;
  o.e.packed = o.g.packed = 0;
  o.eslot = o.gslot = 0;
  o.ecounted = o.gcounted = 0;
  if (kStage == 1 || kStage == 2) {
    const StageOut s = walk_stage<kMode, kTrace>(im, p, kStage == 1 ? 1u : 4u, trace, n_trace);
    if (kStage == 1) {
      o.e = s.v;
      o.eslot = s.slot;
      o.ecounted = s.counted;
    } else {
      o.g = s.v;
      o.gslot = s.slot;
      o.gcounted = s.counted;
    }
    return o;
  }
#pragma nounroll
  for (uint32_t stage = 0; stage < 2; stage++) {
    const StageOut s = walk_stage<kMode, kTrace>(im, p, stage ? 4u : 1u, trace, n_trace);
    if (stage) {
      o.g = s.v;
      o.gslot = s.slot;
      o.gcounted = s.counted;
      break;
    }
    o.e = s.v;
    o.eslot = s.slot;
    o.ecounted = s.counted;
    const uint32_t act = s.v.packed & 0xffu;
    if (act == RV_DROP || act == RV_REJECT || act == RV_ISO_DROP) break;  // ingress never reached (NONE)
    if (const uint32_t b = ingress_bypass(im.base.hdr->isc, dest, ct_mark)) {  // IngressSecurityClassifier
      o.g.packed = b & 0xffu ? pack_verdict(b & 0xffu, 0, 0, (b >> 8) ? 2u : 0u) : 0u;
      break;
    }
  }
  return o;
}

// Per-rule counters: kCounterWords uint64 per slot. Sessions follow the Metric flows
// (pipeline.go:1604-1670, parseMetricFlow network_policy.go:1917-1980): allow rules count
// ct_state=+new packets, deny rules count every packet. The kernels accumulate {packets, bytes,
// packets that are not sessions} (api.cpp fold_counters publishes {packets, bytes, sessions}):
// every add is a scattered device-scope atomic executed at the memory side (~40 B of fabric
// traffic each; C3 with counters 4.70 ms vs 4.26 without), and in the common case -- new
// connections, no len column -- a counted packet then costs one add instead of three.
constexpr uint32_t kCounterWords = 3;
constexpr uint32_t kCounterBytes = kCounterWords * 8;

GPC_HD uint32_t count_session(const VerdictOut& v, uint32_t ct_state) {
  return ((v.packed & 0xffu) != RV_ALLOW || (ct_state & GPC_CT_NEW)) ? 1u : 0u;
}

template <typename Add>
GPC_HD void count_stage(const VerdictOut& v, uint32_t slot, uint32_t len, uint32_t ct_state, Add add) {
  const uint32_t base = kCounterWords * slot;
  add(base, 1ull);
  if (len) add(base + 1, (unsigned long long)len);
  if (!count_session(v, ct_state)) add(base + 2, 1ull);
}

template <typename Add>
GPC_HD void count_packet(const PacketOut& o, uint32_t len, uint32_t ct_state, Add add) {
  if (o.ecounted) count_stage(o.e, o.eslot, len, ct_state, add);
  if (o.gcounted) count_stage(o.g, o.gslot, len, ct_state, add);
}

// Column loads -> axes (kernel and emulation share the defaults of gpc_pkt_soa).
GPC_HD void make_axes(Pkt& p, uint32_t src, uint32_t dst, uint32_t sport, uint32_t dport, uint32_t proto, uint32_t out_port,
                      uint32_t in_port, uint32_t svc_group, uint32_t tun_id, uint32_t ct_src, uint32_t ct_dst, uint32_t ct_state) {
  p.ax[AX_SRC] = src;
  p.ax[AX_DST] = dst;
  p.ax[AX_CTSRC] = ct_src;
  p.ax[AX_CTDST] = ct_dst;
  p.ax[AX_INPORT] = in_port;
  p.ax[AX_REG1] = out_port;
  p.ax[AX_REG7] = svc_group;
  p.ax[AX_TUN] = tun_id;
  const bool ported = proto == 6 || proto == 17 || proto == 132 || proto == 1 || proto == 58;
  p.ax[AX_L4D] = (proto << 16) | (ported ? dport : 0u);
  p.ax[AX_L4S] = (proto << 16) | (ported ? sport : 0u);
  p.ax[AX_CTST] = ct_state;
}
// Axes whose Bloom bits the entries of an epoch test (base image and journal): make_pkt hashes only
// those (wave-uniform), the others are never read.
GPC_HD uint32_t view_bloom_axes(const View& v) {
  uint32_t m = v.base.hdr->bloom_axes;
  if (v.n_img > 1) m |= reinterpret_cast<const JournalHdr*>(v.ovl.blob + v.jhdr)->bloom_axes;
  return m;
}
// bloom_axes: bit a = compute the filter bits of axis a (view_bloom_axes; ~0u = all).
GPC_HD void make_pkt(Pkt& p, uint32_t src, uint32_t dst, uint32_t sport, uint32_t dport, uint32_t proto, uint32_t out_port,
                     uint32_t in_port, uint32_t svc_group, uint32_t tun_id, uint32_t ct_src, uint32_t ct_dst, uint32_t ct_state,
                     uint32_t bloom_axes) {
  make_axes(p, src, dst, sport, dport, proto, out_port, in_port, svc_group, tun_id, ct_src, ct_dst, ct_state);
#pragma unroll
  for (uint32_t a = 0; a < 8; a++) p.fm[a] = (bloom_axes >> a) & 1u ? filt_pkt_axis(a, p.ax[a]) : 0u;
  p.l4m = (bloom_axes & kBloomL4) ? filt_l4_bit(proto_class(proto), (p.ax[AX_L4D] & 0xffffu) >> 12) |
                                        filt_l4x_bit(proto_class(proto), p.ax[AX_L4D] & 0xffffu)
                                  : 0u;
}

}  // namespace gpc
