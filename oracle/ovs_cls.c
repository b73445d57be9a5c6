/*
 * ovs_cls.c -- TEST INFRASTRUCTURE ONLY (checker + timed CPU baseline of bench.py).
 *
 * Plain-C restatement of the OVS 2.17.7 userspace classifier (lib/classifier.c; third-party, not
 * vendored in the reference) as Antrea's policy tables exercise it, plus the Antrea policy-stage
 * walk. Same verdicts as oracle/ovs_cls.py, organised the way OVS organises the lookup:
 *
 *   - tuple-space search: one subtable per distinct match mask, each a hash table keyed by the
 *     masked field vector; a bucket holds the flows with identical match, highest priority first;
 *   - subtables visited in descending max-priority order, stopping below the best hard match found
 *     so far (classifier_lookup__: PVECTOR_FOR_EACH_PRIORITY(subtable, hard_pri + 1, ...); this
 *     restatement scans down to hard_pri itself so that equal-priority hard flows with different
 *     actions are reported as a TIE, as the Python oracle and the device do);
 *   - prefix tries on nw_src / nw_dst (OVS's default classifier prefix fields): a subtable whose
 *     mask on the field is a /L prefix is skipped when no flow of the table has a /L prefix on that
 *     field containing the packet's address (the trie lookup of find_match_wc);
 *   - soft (conjunction-only) matches collected per subtable head; the `again` loop: drop soft
 *     entries at or below the hard match, take the highest soft priority and the number of soft
 *     matches at it (n_soft_pri), accumulate clause bitmaps per conjunction id in a hash map
 *     (find_conjunctive_match: skipped when n_soft_pri < the set's min_n_clauses, and for
 *     conjunctions with more clauses than n_soft_pri), try the completed ids' conj_id lookups, and
 *     otherwise step every entry at that priority to the next lower flow with identical match
 *     (next_visible_rule_in_list; a hard flow there becomes a hard candidate and ends the chain);
 *   - tie (several conjunctions completing at one priority; the order is implementation-defined in
 *     OVS, docs/antrea-network-policy.md:1966-1980): the lowest conj id whose conj_id lookup
 *     succeeds wins and TIE is reported.
 *
 * Every buffer grows on demand; nothing is truncated. An allocation failure aborts the process (a
 * checker must not silently drop work).
 *
 * The Antrea walk (docs/design/ovs-pipeline.md:1159-1330, 1633-1812): {AntreaPolicy,,Default}Rule
 * tables with miss = next table, Pass -> {Egress,Ingress}Rule, allow / deny -> Metric, drop flows,
 * IngressSecurityClassifier bypass for packets not destined to a local Pod.
 *
 * Build: oracle/cbuild.py (gcc -O2 -shared -fPIC -pthread).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum {
  F_DL_TYPE, F_NW_PROTO, F_NW_SRC, F_NW_DST, F_CT_NW_SRC, F_CT_NW_DST, F_IN_PORT, F_REG0, F_REG1, F_REG3, F_REG7,
  F_TUN_ID, F_TP_SRC, F_TP_DST, F_CT_STATE, F_CONJ_ID, F_LABEL_LO, F_LABEL_HI, F_CT_MARK, F_REG4, NF
};
/* tables: 1..6 rule tables, 7 EgressMetric, 8 IngressMetric, 12 IngressSecurityClassifier,
 * 13 ServiceLB, 14 EndpointDNAT (the AntreaProxy stage in front of the policy tables) */
#define T_ISC 12
#define T_SVCLB 13
#define T_EPDNAT 14
#define N_TABLES 15
static const int kTables[] = {1, 2, 3, 4, 5, 6, 7, 8, T_ISC, T_SVCLB, T_EPDNAT};
#define N_USED_TABLES (int)(sizeof kTables / sizeof kTables[0])

/* flow action kinds (decoded by oracle/cls_c.py from the flow text) */
enum { A_CONJ = 1, A_SET_REG = 2, A_CT_COMMIT = 3, A_GOTO = 4, A_GROUP = 5, A_CONTROLLER = 6 };

typedef struct {
  uint8_t kind, reg;
  uint32_t a, b, c;          /* CONJ id,clause,n | SET_REG value,mask | CT table, nat ip, nat port | 1 << 16
                                (c == 0: no nat) | GOTO table | GROUP id */
  uint64_t lv, lm;           /* CT label */
} ocls_action;

typedef struct {
  int32_t table;             /* 1..6 rule tables, 7 EgressMetric, 8 IngressMetric, others ignored */
  uint32_t priority;
  uint32_t val[NF], mask[NF];
  int32_t act_off, n_act;
  int32_t soft;              /* conjunction-only */
  uint32_t sig;              /* verdict signature of a hard flow (equal-priority overlap = TIE) */
} ocls_flow;

typedef struct {
  const uint32_t *src, *dst;
  const uint16_t *sport, *dport;
  const uint8_t* proto;
  const uint32_t* out_port;
  const uint32_t *in_port, *svc_group, *tun_id, *ct_src, *ct_dst;
  const uint8_t *ct_state, *dest;
  const uint16_t* len;
  const uint8_t* ct_mark;    /* HairpinCTMark = 0x40 (NULL: 0) */
} ocls_pkts;

static void* xmalloc(size_t n) {
  void* p = malloc(n ? n : 1);
  if (!p) {
    fprintf(stderr, "ovs_cls: out of memory (%zu bytes)\n", n);
    abort();
  }
  return p;
}
static void* xcalloc(size_t n, size_t sz) {
  void* p = calloc(n ? n : 1, sz ? sz : 1);
  if (!p) {
    fprintf(stderr, "ovs_cls: out of memory (%zu x %zu bytes)\n", n, sz);
    abort();
  }
  return p;
}
static void* xrealloc(void* q, size_t n) {
  void* p = realloc(q, n ? n : 1);
  if (!p) {
    fprintf(stderr, "ovs_cls: out of memory (%zu bytes)\n", n);
    abort();
  }
  return p;
}

/* ------------------------------------------------------------------------------------ model */
typedef struct {
  uint32_t mask[NF];
  uint32_t max_pri;
  int8_t plen_src, plen_dst; /* prefix length of the mask on nw_src / nw_dst (-1: not a prefix / 0) */
  uint32_t nb;               /* buckets (power of two) */
  int32_t* head;             /* bucket -> first entry index (-1) */
  int32_t* next;             /* entry -> next entry in bucket chain */
  int32_t* list_off;         /* entry -> offset into lists */
  int32_t* list_n;
  uint32_t* key;             /* entry -> masked key [NF] */
  int32_t n_entries;
  int32_t* lists;            /* flow indices, priority desc */
  uint32_t* lpri;            /* per list slot: priority << 1 | soft (the soft loop reads only this) */
} subtable;

typedef struct {             /* binary prefix trie of one field of one table */
  int32_t (*child)[2];
  uint8_t* ends;             /* a prefix of the table ends at this node */
  int32_t n, cap;
} trie;

typedef struct {
  subtable* st;
  int n_st;
  trie tr[2];                /* nw_src, nw_dst */
} table_t;

typedef struct ocls {
  ocls_flow* flows;
  int n_flows;
  ocls_action* acts;
  uint8_t* min_ncl;          /* per flow: min n_clauses of its conjunction actions (OVS min_n_clauses) */
  table_t tables[N_TABLES];
  uint32_t* tier_conj;       /* sorted conj ids */
  uint8_t* tier_val;
  int n_tier;
  uint64_t* cnt;             /* per flow: packets, bytes (metric flows) */
  uint64_t stats[8];         /* summed over classify calls: see ocls_stats */
  /* AntreaProxy stage (ocls_set_services): select groups and the Pod map of L3Forwarding */
  uint32_t* gw;              /* group words: gid, n_buckets, per bucket n_sets, (reg, value, mask) x n_sets */
  uint32_t* g_id;            /* sorted group ids and the word offset of each group in gw */
  size_t* g_off;
  int n_groups;
  uint32_t* pod_ip;          /* sorted Pod IPs and their ofports */
  uint32_t* pod_port;
  int n_pods;
} ocls;

/* per-thread lookup workspace */
typedef struct {
  const int32_t* list;
  const uint32_t* pri;       /* lpri of the same list */
  int n, pos;
} soft_ent;

typedef struct {
  soft_ent* soft;
  int soft_cap;
  uint32_t* hkey;            /* conjunction id hash map (open addressing; gen-stamped) */
  uint64_t* hbits;
  uint32_t* hgen;
  uint32_t hcap, gen;
  uint32_t* done;
  int done_cap;
  uint64_t stats[8];         /* 0 lookups, 1 subtables probed, 2 subtables skipped by tries,
                                3 soft matches collected, 4 soft-loop levels, 5 conj actions hashed */
} ws_t;

static uint64_t mixk(const uint32_t* k) {
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < NF; i++) {
    h ^= k[i];
    h *= 1099511628211ull;
    h ^= h >> 29;
  }
  return h;
}

static const ocls_flow* g_sort_flows;
static int cmp_pri_desc_g(const void* a, const void* b) {
  const ocls_flow* f = g_sort_flows;
  int x = *(const int*)a, y = *(const int*)b;
  if (f[x].priority != f[y].priority) return f[x].priority < f[y].priority ? 1 : -1;
  return x < y ? -1 : x > y;
}

static int same_mask(const uint32_t* a, const uint32_t* b) { return memcmp(a, b, sizeof(uint32_t) * NF) == 0; }

static int prefix_len(uint32_t m) { /* 1..32 for a CIDR mask, 0 for none, -1 otherwise */
  if (m == 0) return 0;
  int l = 0;
  while (l < 32 && (m >> (31 - l)) & 1u) l++;
  uint32_t want = l == 32 ? 0xffffffffu : ~(0xffffffffu >> l);
  return m == want ? l : -1;
}

static int trie_node(trie* t) {
  if (t->n == t->cap) {
    t->cap = t->cap ? 2 * t->cap : 64;
    t->child = (int32_t(*)[2])xrealloc(t->child, sizeof(int32_t[2]) * (size_t)t->cap);
    t->ends = (uint8_t*)xrealloc(t->ends, (size_t)t->cap);
  }
  t->child[t->n][0] = t->child[t->n][1] = -1;
  t->ends[t->n] = 0;
  return t->n++;
}
static void trie_insert(trie* t, uint32_t v, int len) {
  if (!t->n) trie_node(t);
  int x = 0;
  for (int d = 0; d < len; d++) {
    int b = (v >> (31 - d)) & 1u;
    if (t->child[x][b] < 0) {
      int y = trie_node(t);
      t->child[x][b] = y;
    }
    x = t->child[x][b];
  }
  t->ends[x] = 1;
}
/* bit L (1..32) set: a /L prefix of the table contains `v` */
static uint64_t trie_lookup(const trie* t, uint32_t v) {
  uint64_t m = 0;
  if (!t->n) return 0;
  int x = 0;
  for (int d = 0; d < 32; d++) {
    x = t->child[x][(v >> (31 - d)) & 1u];
    if (x < 0) break;
    if (t->ends[x]) m |= 1ull << (d + 1);
  }
  return m;
}

ocls* ocls_create(const ocls_flow* flows, int n_flows, const ocls_action* acts, int n_acts, const uint32_t* tier_conj,
                  const uint8_t* tier_val, int n_tier) {
  ocls* c = (ocls*)xcalloc(1, sizeof(ocls));
  c->flows = (ocls_flow*)xmalloc(sizeof(ocls_flow) * (size_t)n_flows);
  memcpy(c->flows, flows, sizeof(ocls_flow) * (size_t)n_flows);
  c->n_flows = n_flows;
  c->acts = (ocls_action*)xmalloc(sizeof(ocls_action) * (size_t)n_acts);
  memcpy(c->acts, acts, sizeof(ocls_action) * (size_t)n_acts);
  c->min_ncl = (uint8_t*)xcalloc((size_t)n_flows, 1);
  for (int i = 0; i < n_flows; i++) {
    uint32_t mn = 255;
    for (int a = 0; a < flows[i].n_act; a++) {
      const ocls_action* ac = &acts[flows[i].act_off + a];
      if (ac->kind == A_CONJ && ac->c < mn) mn = ac->c;
      if (ac->kind == A_CONJ && (ac->c < 1 || ac->c > 64 || ac->b < 1 || ac->b > ac->c)) {
        fprintf(stderr, "ovs_cls: malformed conjunction(%u,%u/%u)\n", ac->a, ac->b, ac->c);
        abort();
      }
    }
    c->min_ncl[i] = (uint8_t)mn;
  }
  c->tier_conj = (uint32_t*)xmalloc(4 * (size_t)n_tier);
  c->tier_val = (uint8_t*)xmalloc((size_t)n_tier);
  memcpy(c->tier_conj, tier_conj, 4 * (size_t)n_tier);
  memcpy(c->tier_val, tier_val, (size_t)n_tier);
  c->n_tier = n_tier;
  c->cnt = (uint64_t*)xcalloc(2 * (size_t)n_flows, 8);
  int* idx = (int*)xmalloc(sizeof(int) * (size_t)n_flows);
  int* owner = (int*)xmalloc(sizeof(int) * (size_t)n_flows);
  for (int ti = 0; ti < N_USED_TABLES; ti++) {
    const int t = kTables[ti];
    int n = 0;
    for (int i = 0; i < n_flows; i++)
      if (c->flows[i].table == t) idx[n++] = i;
    /* group flows by mask: hash of the mask -> subtable */
    subtable* sts = NULL;
    int nst = 0, stcap = 0;
    uint32_t mnb = 1;
    while (mnb < 2u * (uint32_t)n + 2u) mnb <<= 1;
    int32_t* mhead = (int32_t*)xmalloc(sizeof(int32_t) * mnb);
    int32_t* mnext = NULL;
    for (uint32_t b = 0; b < mnb; b++) mhead[b] = -1;
    for (int j = 0; j < n; j++) {
      const ocls_flow* f = &c->flows[idx[j]];
      uint32_t b = (uint32_t)mixk(f->mask) & (mnb - 1);
      int s;
      for (s = mhead[b]; s >= 0; s = mnext[s])
        if (same_mask(sts[s].mask, f->mask)) break;
      if (s < 0) {
        if (nst == stcap) {
          stcap = stcap ? 2 * stcap : 16;
          sts = (subtable*)xrealloc(sts, sizeof(subtable) * (size_t)stcap);
          mnext = (int32_t*)xrealloc(mnext, sizeof(int32_t) * (size_t)stcap);
        }
        s = nst++;
        memset(&sts[s], 0, sizeof(subtable));
        memcpy(sts[s].mask, f->mask, sizeof(uint32_t) * NF);
        sts[s].plen_src = (int8_t)prefix_len(f->mask[F_NW_SRC]);
        sts[s].plen_dst = (int8_t)prefix_len(f->mask[F_NW_DST]);
        mnext[s] = mhead[b];
        mhead[b] = s;
      }
      owner[j] = s;
      if (f->priority > sts[s].max_pri) sts[s].max_pri = f->priority;
      if (sts[s].plen_src > 0) trie_insert(&c->tables[t].tr[0], f->val[F_NW_SRC], sts[s].plen_src);
      if (sts[s].plen_dst > 0) trie_insert(&c->tables[t].tr[1], f->val[F_NW_DST], sts[s].plen_dst);
    }
    free(mhead);
    free(mnext);
    /* per subtable: flow count, then entries */
    int* cnt = (int*)xcalloc((size_t)nst, sizeof(int));
    for (int j = 0; j < n; j++) cnt[owner[j]]++;
    int** members = (int**)xmalloc(sizeof(int*) * (size_t)nst);
    int* fill = (int*)xcalloc((size_t)nst, sizeof(int));
    for (int s = 0; s < nst; s++) members[s] = (int*)xmalloc(sizeof(int) * (size_t)cnt[s]);
    for (int j = 0; j < n; j++) members[owner[j]][fill[owner[j]]++] = idx[j];
    for (int s = 0; s < nst; s++) {
      subtable* st = &sts[s];
      const int m = cnt[s];
      uint32_t nb = 1;
      while (nb < (uint32_t)m * 2) nb <<= 1;
      st->nb = nb;
      st->head = (int32_t*)xmalloc(sizeof(int32_t) * nb);
      for (uint32_t b = 0; b < nb; b++) st->head[b] = -1;
      st->next = (int32_t*)xmalloc(sizeof(int32_t) * (size_t)m);
      st->list_off = (int32_t*)xmalloc(sizeof(int32_t) * (size_t)m);
      st->list_n = (int32_t*)xcalloc((size_t)m, sizeof(int32_t));
      st->key = (uint32_t*)xmalloc(sizeof(uint32_t) * NF * (size_t)m);
      st->lists = (int32_t*)xmalloc(sizeof(int32_t) * (size_t)m);
      int* fent = (int*)xmalloc(sizeof(int) * (size_t)m);
      for (int k = 0; k < m; k++) {
        const ocls_flow* f = &c->flows[members[s][k]];
        uint32_t key[NF];
        for (int q = 0; q < NF; q++) key[q] = f->val[q] & f->mask[q];
        uint32_t b = (uint32_t)mixk(key) & (nb - 1);
        int e;
        for (e = st->head[b]; e >= 0; e = st->next[e])
          if (memcmp(st->key + (size_t)e * NF, key, sizeof key) == 0) break;
        if (e < 0) {
          e = st->n_entries++;
          memcpy(st->key + (size_t)e * NF, key, sizeof key);
          st->next[e] = st->head[b];
          st->head[b] = e;
        }
        st->list_n[e]++;
        fent[k] = e;
      }
      int off = 0;
      for (int e = 0; e < st->n_entries; e++) {
        st->list_off[e] = off;
        off += st->list_n[e];
        st->list_n[e] = 0;
      }
      for (int k = 0; k < m; k++) {
        int e = fent[k];
        st->lists[st->list_off[e] + st->list_n[e]++] = members[s][k];
      }
      g_sort_flows = c->flows;
      for (int e = 0; e < st->n_entries; e++) qsort(st->lists + st->list_off[e], (size_t)st->list_n[e], sizeof(int32_t), cmp_pri_desc_g);
      st->lpri = (uint32_t*)xmalloc(sizeof(uint32_t) * (size_t)m);
      for (int k = 0; k < m; k++) st->lpri[k] = (c->flows[st->lists[k]].priority << 1) | (c->flows[st->lists[k]].soft ? 1u : 0u);
      free(fent);
      free(members[s]);
    }
    free(members);
    free(fill);
    free(cnt);
    /* subtables by max priority, descending (pvector order) */
    for (int a = 1; a < nst; a++)
      for (int b = a; b > 0 && sts[b].max_pri > sts[b - 1].max_pri; b--) {
        subtable tmp = sts[b];
        sts[b] = sts[b - 1];
        sts[b - 1] = tmp;
      }
    c->tables[t].st = sts;
    c->tables[t].n_st = nst;
  }
  free(idx);
  free(owner);
  return c;
}

void ocls_destroy(ocls* c) {
  if (!c) return;
  for (int ti = 0; ti < N_USED_TABLES; ti++) {
    const int t = kTables[ti];
    for (int s = 0; s < c->tables[t].n_st; s++) {
      subtable* st = &c->tables[t].st[s];
      free(st->head);
      free(st->next);
      free(st->list_off);
      free(st->list_n);
      free(st->key);
      free(st->lists);
      free(st->lpri);
    }
    free(c->tables[t].st);
    for (int k = 0; k < 2; k++) {
      free(c->tables[t].tr[k].child);
      free(c->tables[t].tr[k].ends);
    }
  }
  free(c->flows);
  free(c->acts);
  free(c->min_ncl);
  free(c->tier_conj);
  free(c->tier_val);
  free(c->cnt);
  free(c->gw);
  free(c->g_id);
  free(c->g_off);
  free(c->pod_ip);
  free(c->pod_port);
  free(c);
}

/* find_match: the bucket list of `st` matching packet vector `pv`, or NULL */
static const int32_t* find_match(const subtable* st, const uint32_t* pv, int* n, const uint32_t** pri) {
  uint32_t key[NF];
  for (int q = 0; q < NF; q++) key[q] = pv[q] & st->mask[q];
  uint32_t b = (uint32_t)mixk(key) & (st->nb - 1);
  for (int e = st->head[b]; e >= 0; e = st->next[e])
    if (memcmp(st->key + (size_t)e * NF, key, sizeof key) == 0) {
      *n = st->list_n[e];
      *pri = st->lpri + st->list_off[e];
      return st->lists + st->list_off[e];
    }
  return NULL;
}

static void ws_soft_push(ws_t* w, int* n_soft, const int32_t* list, const uint32_t* pri, int n, int pos) {
  if (*n_soft == w->soft_cap) {
    w->soft_cap = w->soft_cap ? 2 * w->soft_cap : 256;
    w->soft = (soft_ent*)xrealloc(w->soft, sizeof(soft_ent) * (size_t)w->soft_cap);
  }
  w->soft[*n_soft].list = list;
  w->soft[*n_soft].pri = pri;
  w->soft[*n_soft].n = n;
  w->soft[*n_soft].pos = pos;
  (*n_soft)++;
}

/* conjunction-id map: clause bitmap of id (initialised as OVS does, UINT64_MAX << n_clauses) */
static uint64_t* ws_conj(ws_t* w, uint32_t id, uint32_t n_clauses) {
  uint32_t m = w->hcap - 1, h = (id * 0x9e3779b1u) & m;
  while (w->hgen[h] == w->gen && w->hkey[h] != id) h = (h + 1) & m;
  if (w->hgen[h] != w->gen) {
    w->hgen[h] = w->gen;
    w->hkey[h] = id;
    w->hbits[h] = n_clauses >= 64 ? 0 : (~0ull << n_clauses);
  }
  return &w->hbits[h];
}
static void ws_conj_reset(ws_t* w, size_t need) {
  if (w->hcap < 2 * need + 16) {
    uint32_t cap = 64;
    while (cap < 2 * need + 16) cap <<= 1;
    free(w->hkey);
    free(w->hbits);
    free(w->hgen);
    w->hkey = (uint32_t*)xmalloc(4 * (size_t)cap);
    w->hbits = (uint64_t*)xmalloc(8 * (size_t)cap);
    w->hgen = (uint32_t*)xcalloc(cap, 4);
    w->hcap = cap;
    w->gen = 0;
  }
  if (++w->gen == 0) { /* stamp wrap: clear */
    memset(w->hgen, 0, 4 * (size_t)w->hcap);
    w->gen = 1;
  }
}
static void ws_done_push(ws_t* w, int* nd, uint32_t id) {
  if (*nd == w->done_cap) {
    w->done_cap = w->done_cap ? 2 * w->done_cap : 64;
    w->done = (uint32_t*)xrealloc(w->done, 4 * (size_t)w->done_cap);
  }
  w->done[(*nd)++] = id;
}
static int cmp_u32(const void* a, const void* b) {
  uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  return x < y ? -1 : x > y;
}

/* classifier_lookup__ restated. Returns flow index or -1; *tie set on conj ties (and on
 * equal-priority hard flows with different actions when no conjunction decides). */
static int lookup(const ocls* c, ws_t* w, int table, uint32_t* pv, int allow_conj, int* tie) {
  const table_t* T = &c->tables[table];
  const ocls_flow* F = c->flows;
  int hard = -1, htie = 0;
  int64_t hard_pri = -1, soft_pri = -1;
  int n_soft = 0;
  w->stats[0]++;
  const uint64_t tsrc = trie_lookup(&T->tr[0], pv[F_NW_SRC]);
  const uint64_t tdst = trie_lookup(&T->tr[1], pv[F_NW_DST]);
  for (int s = 0; s < T->n_st; s++) {
    const subtable* st = &T->st[s];
    if ((int64_t)st->max_pri < hard_pri) break;
    if ((st->plen_src > 0 && !((tsrc >> st->plen_src) & 1)) || (st->plen_dst > 0 && !((tdst >> st->plen_dst) & 1))) {
      w->stats[2]++;
      continue;
    }
    w->stats[1]++;
    int n;
    const uint32_t* lp;
    const int32_t* l = find_match(st, pv, &n, &lp);
    if (!l) continue;
    const ocls_flow* f = &F[l[0]];
    if (f->soft) {
      if (!allow_conj || (int64_t)f->priority <= hard_pri) continue; /* OVS: ignored, not stepped past */
      ws_soft_push(w, &n_soft, l, lp, n, 0);
      if ((int64_t)f->priority > soft_pri) soft_pri = f->priority;
      continue;
    }
    if ((int64_t)f->priority > hard_pri) {
      hard = l[0];
      hard_pri = f->priority;
      htie = 0;
    } else if ((int64_t)f->priority == hard_pri && f->sig != F[hard].sig) {
      htie = 1;
    }
  }
  w->stats[3] += (uint64_t)n_soft;
  if (!allow_conj || hard_pri >= soft_pri) {
    if (hard >= 0 && htie) *tie = 1;
    return hard;
  }
  soft_ent* soft = w->soft;
  for (;;) {
    soft = w->soft;
    /* delete chain ends and soft matches at or below the hard match */
    for (int i = 0; i < n_soft;) {
      if (soft[i].pos >= soft[i].n || (int64_t)(soft[i].pri[soft[i].pos] >> 1) <= hard_pri) soft[i] = soft[--n_soft];
      else i++;
    }
    if (!n_soft) break;
    w->stats[4]++;
    /* highest soft priority and the number of soft matches at it */
    uint32_t top = 0;
    int n_top = 0;
    for (int i = 0; i < n_soft; i++) {
      uint32_t p = soft[i].pri[soft[i].pos] >> 1;
      if (p > top) {
        top = p;
        n_top = 1;
      } else if (p == top) {
        n_top++;
      }
    }
    /* find_conjunctive_match over the soft matches at `top` */
    size_t n_acts = 0;
    for (int i = 0; i < n_soft; i++) {
      if ((soft[i].pri[soft[i].pos] >> 1) != top) continue;
      const int fi = soft[i].list[soft[i].pos];
      if ((uint32_t)n_top >= c->min_ncl[fi]) n_acts += (size_t)F[fi].n_act;
    }
    int nd = 0;
    if (n_acts) {
      ws_conj_reset(w, n_acts);
      w->stats[5] += n_acts;
      for (int i = 0; i < n_soft; i++) {
        if ((soft[i].pri[soft[i].pos] >> 1) != top) continue;
        const int fi = soft[i].list[soft[i].pos];
        const ocls_flow* f = &F[fi];
        if ((uint32_t)n_top < c->min_ncl[fi]) continue;
        for (int a = 0; a < f->n_act; a++) {
          const ocls_action* ac = &c->acts[f->act_off + a];
          if (ac->kind != A_CONJ || ac->c > (uint32_t)n_top) continue;
          uint64_t* cm = ws_conj(w, ac->a, ac->c);
          const uint64_t before = *cm;
          *cm |= 1ull << (ac->b - 1);
          if (*cm == ~0ull && before != ~0ull) ws_done_push(w, &nd, ac->a);
        }
      }
    }
    if (nd) {
      qsort(w->done, (size_t)nd, 4, cmp_u32);
      for (int d = 0; d < nd; d++) {
        uint32_t saved = pv[F_CONJ_ID];
        pv[F_CONJ_ID] = w->done[d];
        int dummy = 0;
        int r = lookup(c, w, table, pv, 0, &dummy);
        pv[F_CONJ_ID] = saved;
        if (r >= 0) {
          if (nd > 1) *tie = 1;
          return r;
        }
      }
    }
    /* next_visible_rule_in_list for every entry at `top` */
    soft = w->soft;
    for (int i = 0; i < n_soft; i++) {
      if ((soft[i].pri[soft[i].pos] >> 1) != top) continue;
      soft[i].pos++;
      if (soft[i].pos < soft[i].n && !(soft[i].pri[soft[i].pos] & 1u)) {
        const int fi = soft[i].list[soft[i].pos];
        {
          if ((int64_t)F[fi].priority > hard_pri) {
            hard = fi;
            hard_pri = F[fi].priority;
            htie = 0;
          } else if ((int64_t)F[fi].priority == hard_pri && hard >= 0 && F[fi].sig != F[hard].sig) {
            htie = 1;
          }
          soft[i].pos = soft[i].n; /* a hard flow ends the chain */
        }
      }
    }
  }
  if (hard >= 0 && htie) *tie = 1;
  return hard;
}

static uint8_t tier_of(const ocls* c, uint32_t conj) {
  int lo = 0, hi = c->n_tier;
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (c->tier_conj[mid] < conj) lo = mid + 1;
    else hi = mid;
  }
  return (lo < c->n_tier && c->tier_conj[lo] == conj) ? c->tier_val[lo] : 0;
}

enum { ACT_NONE, ACT_NO_MATCH, ACT_ALLOW, ACT_DROP, ACT_REJECT, ACT_ISO_DROP, ACT_BYPASS };

/* one policy stage; tables t1,t2,t3 then metric (7 egress / 8 ingress). Returns packed verdict. */
static void stage(const ocls* c, ws_t* w, int base, uint32_t* pv, uint32_t len, uint64_t* cnt, uint32_t* out_conj,
                  uint32_t* out_packed) {
  int metric = base == 0 ? 7 : 8;
  int t = base + 1;
  uint32_t flags = 0, conj = 0, tindex = 0, action = ACT_NO_MATCH;
  int t2 = base + 2;
  while (t != metric) {
    int tie = 0;
    int fi = lookup(c, w, t, pv, 1, &tie);
    if (fi < 0) {
      t = t == base + 3 ? metric : t + 1;
      continue;
    }
    const ocls_flow* f = &c->flows[fi];
    int go = -1, deny = 0, reject = 0, group = 0, commit = 0;
    for (int a = 0; a < f->n_act; a++) {
      const ocls_action* ac = &c->acts[f->act_off + a];
      if (ac->kind == A_SET_REG) {
        uint32_t m = ac->b, v = ac->a;
        int fld = ac->reg == 0 ? F_REG0 : ac->reg == 3 ? F_REG3 : -1;
        if (fld >= 0) pv[fld] = (pv[fld] & ~m) | (v & m);
        if (ac->reg == 0 && (v & m & 0x400)) deny = 1;
        if (ac->reg == 0 && m == 0xfe000000u && ((v >> 25) & 4)) reject = 1;
      } else if (ac->kind == A_CONTROLLER) {
        flags |= 4; /* packet-in (paused for the DNS interception flow) */
      } else if (ac->kind == A_CT_COMMIT) {
        commit = 1;
        pv[F_LABEL_LO] = (pv[F_LABEL_LO] & ~(uint32_t)ac->lm) | ((uint32_t)ac->lv & (uint32_t)ac->lm);
        pv[F_LABEL_HI] = (pv[F_LABEL_HI] & ~(uint32_t)(ac->lm >> 32)) | ((uint32_t)(ac->lv >> 32) & (uint32_t)(ac->lm >> 32));
        go = (int)ac->a;
      } else if (ac->kind == A_GOTO) {
        go = (int)ac->a;
      } else if (ac->kind == A_GROUP) {
        group = 1;
      }
    }
    if (tie) flags |= 2;
    tindex = (uint32_t)(t - base);
    uint32_t cid = f->mask[F_CONJ_ID] ? f->val[F_CONJ_ID] : 0;
    if (cid) {
      if (deny) {
        conj = cid;
        action = reject ? ACT_REJECT : ACT_DROP;
        go = metric;
      } else if (go == t2 || (group && ((pv[F_REG0] >> 11) & 3) == 3)) {
        conj = cid;
        flags |= 1;
        t = t2;
        continue;
      } else if (commit) {
        conj = cid;
        action = ACT_ALLOW;
        go = metric;
      } else { /* conj_id flow straight to the Metric table, no commit (DNS interception) */
        action = ACT_BYPASS;
        go = metric;
      }
    } else {
      if ((go < 0 && !group) || go == 11 /* Output: logging drop, packet-in */) {
        *out_conj = conj;
        *out_packed = ACT_ISO_DROP | (tindex << 8) | ((conj ? tier_of(c, conj) : 0u) << 16) | (flags << 24);
        return;
      }
      action = ACT_BYPASS;
      go = metric;
    }
    t = go;
  }
  int tie = 0;
  int mf = lookup(c, w, metric, pv, 0, &tie);
  if (mf >= 0 && cnt) {
    cnt[2 * mf] += 1;
    cnt[2 * mf + 1] += len;
  }
  if (action == ACT_NO_MATCH) tindex = 0;
  *out_conj = conj;
  *out_packed = action | (tindex << 8) | ((conj ? tier_of(c, conj) : 0u) << 16) | (flags << 24);
}

/* ------------------------------------------------------------------ AntreaProxy stage (C4)
 * ServiceLB -> select group bucket -> EndpointDNAT -> L3Forwarding, restated as oracle/ovs_cls.py
 * Pipeline.service_stage does over the realized flows (pipeline.go:2374-2431 ServiceLB, 2502-2528
 * EndpointDNAT, 2553-2592 select groups). The bucket choice of an OVS select group is OVS-internal
 * (dp_hash; not in the reference): restated with the symmetric hash of core.hpp lb_hash over a
 * 2^k >= 64 slot table, slot s -> bucket s mod n (parity of the bucket choice is unpinned). */
enum { LB_HIT = 1, LB_NO_ENDPOINT = 2, LB_DNAT = 4, LB_REMOTE = 8 };
#define EP_TO_SELECT 0x10000u     /* fields.go EpToSelectRegMark (reg4[16..18] = 1) */
#define SVC_NO_EP (1u << 14)      /* reg0 SvcNoEpRegMark */
#define REMOTE_EP (1u << 26)      /* reg4 RemoteEndpointRegMark */

/* Pod map and select groups (words: gid, n_buckets, then per bucket n_sets and n_sets x (reg,
 * value, mask) of its set_field actions); copied. */
int ocls_set_services(ocls* c, const uint32_t* gw, size_t n_gw, const uint32_t* pod_ip, const uint32_t* pod_port, int n_pods) {
  free(c->gw);
  free(c->g_id);
  free(c->g_off);
  free(c->pod_ip);
  free(c->pod_port);
  c->gw = (uint32_t*)xmalloc(4 * (n_gw + 1));
  memcpy(c->gw, gw, 4 * n_gw);
  int ng = 0;
  for (size_t o = 0; o + 1 < n_gw; ng++) {  /* count, validating the encoding */
    uint32_t nb = gw[o + 1];
    o += 2;
    for (uint32_t b = 0; b < nb; b++) {
      if (o >= n_gw) return -1;
      o += 1 + 3 * (size_t)gw[o];
    }
    if (o > n_gw) return -1;
  }
  c->g_id = (uint32_t*)xmalloc(4 * (size_t)(ng + 1));
  c->g_off = (size_t*)xmalloc(sizeof(size_t) * (size_t)(ng + 1));
  size_t o = 0;
  for (int g = 0; g < ng; g++) {
    c->g_id[g] = gw[o];
    c->g_off[g] = o;
    uint32_t nb = gw[o + 1];
    o += 2;
    for (uint32_t b = 0; b < nb; b++) o += 1 + 3 * (size_t)gw[o];
  }
  for (int i = 1; i < ng; i++)  /* sort by id (insertion: groups arrive nearly sorted) */
    for (int j = i; j > 0 && c->g_id[j - 1] > c->g_id[j]; j--) {
      uint32_t t = c->g_id[j];
      c->g_id[j] = c->g_id[j - 1];
      c->g_id[j - 1] = t;
      size_t u = c->g_off[j];
      c->g_off[j] = c->g_off[j - 1];
      c->g_off[j - 1] = u;
    }
  c->n_groups = ng;
  c->pod_ip = (uint32_t*)xmalloc(4 * (size_t)(n_pods + 1));
  c->pod_port = (uint32_t*)xmalloc(4 * (size_t)(n_pods + 1));
  memcpy(c->pod_ip, pod_ip, 4 * (size_t)n_pods);
  memcpy(c->pod_port, pod_port, 4 * (size_t)n_pods);
  for (int i = 1; i < n_pods; i++)
    for (int j = i; j > 0 && c->pod_ip[j - 1] > c->pod_ip[j]; j--) {
      uint32_t t = c->pod_ip[j];
      c->pod_ip[j] = c->pod_ip[j - 1];
      c->pod_ip[j - 1] = t;
      t = c->pod_port[j];
      c->pod_port[j] = c->pod_port[j - 1];
      c->pod_port[j - 1] = t;
    }
  c->n_pods = n_pods;
  return 0;
}

static uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}
static uint32_t lb_hash(uint32_t src, uint32_t dst, uint32_t sport, uint32_t dport, uint32_t proto) {
  return mix32((src ^ dst) ^ (mix32(((sport ^ dport) << 8) | (proto & 0xffu)) * 0x9e3779b1u));
}

static void apply_set_reg(uint32_t reg, uint32_t v, uint32_t m, uint32_t* r0, uint32_t* r3, uint32_t* r4, uint32_t* r7,
                          int* set7) {
  uint32_t* r = reg == 0 ? r0 : reg == 3 ? r3 : reg == 4 ? r4 : reg == 7 ? r7 : NULL;
  if (!r) return;
  *r = (*r & ~m) | (v & m);
  if (reg == 7) *set7 = 1;
}

/* The Service stage of one packet: rewrites pv (nw_dst / tp_dst after DNAT, reg1 = the Endpoint's
 * ofport, reg7 when the ServiceLB flow loads it) and *dest; lb = gpc_lb_result words {endpoint
 * ip, port | flags << 16, group id, out_port}. Returns the LB flags (0: not a Service packet).
 * pv[F_CT_NW_DST] keeps the pre-NAT destination. */
static uint32_t service_stage(const ocls* c, ws_t* w, uint32_t* pv, uint32_t* dest, uint32_t* lb) {
  lb[0] = lb[1] = lb[2] = lb[3] = 0;
  const uint32_t proto = pv[F_NW_PROTO];
  if ((proto != 6 && proto != 17 && proto != 132) || !c->tables[T_SVCLB].n_st) return 0;
  uint32_t sv[NF];
  memcpy(sv, pv, sizeof sv);
  uint32_t r0 = 0, r3 = 0, r4 = EP_TO_SELECT, r7 = 0;
  int set7 = 0, tie = 0;
  sv[F_REG0] = r0;
  sv[F_REG3] = r3;
  sv[F_REG4] = r4;
  const int fi = lookup(c, w, T_SVCLB, sv, 0, &tie);
  if (fi < 0) return 0;
  uint32_t flags = LB_HIT, gid = 0;
  int has_group = 0;
  const ocls_flow* f = &c->flows[fi];
  for (int a = 0; a < f->n_act; a++) {
    const ocls_action* ac = &c->acts[f->act_off + a];
    if (ac->kind == A_SET_REG) apply_set_reg(ac->reg, ac->a, ac->b, &r0, &r3, &r4, &r7, &set7);
    else if (ac->kind == A_GROUP) gid = ac->a, has_group = 1;
  }
  if (set7) pv[F_REG7] = r7;
  lb[2] = gid;
  int lo = 0, hi = c->n_groups;
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (c->g_id[mid] < gid) lo = mid + 1;
    else hi = mid;
  }
  const uint32_t* g = (has_group && lo < c->n_groups && c->g_id[lo] == gid) ? c->gw + c->g_off[lo] : NULL;
  if (!g || g[1] == 0) {
    flags |= LB_NO_ENDPOINT;
    lb[1] = flags << 16;
    return flags;
  }
  const uint32_t nb = g[1];
  uint32_t lg = 6;
  while ((1u << lg) < nb) lg++;
  const uint32_t slot = lb_hash(pv[F_NW_SRC], pv[F_NW_DST], pv[F_TP_SRC], pv[F_TP_DST], proto) & ((1u << lg) - 1u);
  const uint32_t* b = g + 2;
  for (uint32_t k = 0; k < slot % nb; k++) b += 1 + 3 * b[0];
  for (uint32_t k = 0; k < b[0]; k++) apply_set_reg(b[1 + 3 * k], b[2 + 3 * k], b[3 + 3 * k], &r0, &r3, &r4, &r7, &set7);
  if (r0 & SVC_NO_EP) {  /* serviceNoEndpointFlow: packet-in, rejected */
    flags |= LB_NO_ENDPOINT;
    lb[1] = flags << 16;
    return flags;
  }
  if (r4 & REMOTE_EP) flags |= LB_REMOTE;
  const uint32_t ep_ip = r3, ep_port = r4 & 0xffffu;
  sv[F_REG0] = r0;
  sv[F_REG3] = r3;
  sv[F_REG4] = r4;
  const int di = lookup(c, w, T_EPDNAT, sv, 0, &tie);
  if (di >= 0) {
    const ocls_flow* d = &c->flows[di];
    for (int a = 0; a < d->n_act; a++) {
      const ocls_action* ac = &c->acts[d->act_off + a];
      if (ac->kind == A_CT_COMMIT && (ac->c >> 16)) {
        pv[F_NW_DST] = ac->b;
        pv[F_TP_DST] = ac->c & 0xffffu;
        flags |= LB_DNAT;
      }
    }
  }
  lo = 0, hi = c->n_pods;
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (c->pod_ip[mid] < ep_ip) lo = mid + 1;
    else hi = mid;
  }
  if (lo < c->n_pods && c->pod_ip[lo] == ep_ip) {
    pv[F_REG1] = c->pod_port[lo];
    *dest = 0; /* Pod */
  } else {
    pv[F_REG1] = 0;
    *dest = (flags & LB_REMOTE) ? 2u /* tunnel */ : 1u /* gateway */;
  }
  lb[0] = ep_ip;
  lb[1] = ep_port | (flags << 16);
  lb[3] = pv[F_REG1];
  return flags;
}

/* IngressSecurityClassifier as installed (pipeline.go:2144-2182): the destination class as its
 * PktDestinationField mark in reg0[4..7] (fields.go:54-57: tunnel 1, gateway 2, uplink 4) and the
 * packet's ct_mark; a flow out of the policy tables (IngressMetric / ConntrackCommit) makes the
 * ingress verdict BYPASS (+TIE on an equal-priority overlap). Returns the packed verdict or 0. */
static uint32_t ingress_classifier(const ocls* c, ws_t* w, uint32_t* pv, uint32_t dest, uint32_t ct_mark) {
  static const uint32_t marks[4] = {0, 0x20, 0x10, 0x40}; /* gpc_dest: pod, gateway, tunnel, uplink */
  if (!c->tables[T_ISC].n_st) return 0;
  const uint32_t r0 = pv[F_REG0], cm = pv[F_CT_MARK];
  pv[F_REG0] = dest < 4 ? marks[dest] : 0;
  pv[F_CT_MARK] = ct_mark;
  int tie = 0;
  const int fi = lookup(c, w, T_ISC, pv, 0, &tie);
  pv[F_REG0] = r0;
  pv[F_CT_MARK] = cm;
  if (fi < 0) return 0;
  const ocls_flow* f = &c->flows[fi];
  for (int a = 0; a < f->n_act; a++) {
    const ocls_action* ac = &c->acts[f->act_off + a];
    if (ac->kind == A_GOTO && (ac->a == 8 || ac->a == 10)) return ACT_BYPASS | ((tie ? 2u : 0u) << 24);
  }
  return 0;
}

static void classify_range(const ocls* c, ws_t* w, const ocls_pkts* p, size_t lo, size_t hi, uint32_t* out, uint32_t* lb_out,
                           uint64_t* cnt) {
  for (size_t i = lo; i < hi; i++) {
    uint32_t pv[NF];
    memset(pv, 0, sizeof pv);
    uint32_t proto = p->proto[i];
    int ported = proto == 6 || proto == 17 || proto == 132 || proto == 1 || proto == 58;
    pv[F_DL_TYPE] = 0x0800;
    pv[F_NW_PROTO] = proto;
    pv[F_NW_SRC] = p->src[i];
    pv[F_NW_DST] = p->dst[i];
    pv[F_CT_NW_SRC] = p->ct_src ? p->ct_src[i] : p->src[i];
    pv[F_CT_NW_DST] = p->ct_dst ? p->ct_dst[i] : p->dst[i];
    pv[F_IN_PORT] = p->in_port ? p->in_port[i] : 0;
    pv[F_REG1] = p->out_port[i];
    pv[F_REG7] = p->svc_group ? p->svc_group[i] : 0;
    pv[F_TUN_ID] = p->tun_id ? p->tun_id[i] : 0;
    pv[F_TP_SRC] = ported ? p->sport[i] : 0;
    pv[F_TP_DST] = ported ? p->dport[i] : 0;
    pv[F_CT_STATE] = p->ct_state ? p->ct_state[i] : 0x21;
    uint32_t len = p->len ? p->len[i] : 0;
    uint32_t dest = p->dest ? p->dest[i] : 0, lb[4];
    const uint32_t lbf = service_stage(c, w, pv, &dest, lb);
    if (lb_out) memcpy(lb_out + 4 * i, lb, sizeof lb);
    if (lbf & LB_NO_ENDPOINT) { /* EndpointDNAT serviceNoEndpointFlow: rejected before the policy stages */
      out[4 * i + 0] = 0;
      out[4 * i + 1] = ACT_REJECT | (4u << 8); /* table code GPC_VTABLE_ENDPOINT_DNAT */
      out[4 * i + 2] = 0;
      out[4 * i + 3] = ACT_NONE;
      continue;
    }
    uint32_t ec, ep, gc, gp, isc;
    stage(c, w, 0, pv, len, cnt, &ec, &ep);
    uint32_t ea = ep & 0xff;
    if (ea == ACT_DROP || ea == ACT_REJECT || ea == ACT_ISO_DROP) {
      gc = 0;
      gp = ACT_NONE;
    } else if ((isc = ingress_classifier(c, w, pv, dest, p->ct_mark ? p->ct_mark[i] : 0)) != 0) {
      gc = 0;
      gp = isc;
    } else {
      pv[F_REG0] = 0;
      pv[F_REG3] = 0;
      pv[F_CONJ_ID] = 0;
      stage(c, w, 3, pv, len, cnt, &gc, &gp);
    }
    out[4 * i + 0] = ec;
    out[4 * i + 1] = ep;
    out[4 * i + 2] = gc;
    out[4 * i + 3] = gp;
  }
}

typedef struct {
  const ocls* c;
  const ocls_pkts* p;
  size_t lo, hi;
  uint32_t* out;
  uint32_t* lb;
  uint64_t* cnt;
  ws_t ws;
} job;

static void* worker(void* arg) {
  job* j = (job*)arg;
  classify_range(j->c, &j->ws, j->p, j->lo, j->hi, j->out, j->lb, j->cnt);
  return NULL;
}

/* out: 4 uint32 per packet (egress conj, egress packed, ingress conj, ingress packed); lb_out (or
 * NULL): 4 uint32 per packet, the Service stage's gpc_lb_result words. */
int ocls_classify_lb(ocls* c, const ocls_pkts* p, size_t n, uint32_t* out, uint32_t* lb_out, int threads, int count) {
  if (threads < 1) threads = 1;
  if ((size_t)threads > n && n) threads = (int)n;
  pthread_t* th = (pthread_t*)xmalloc(sizeof(pthread_t) * (size_t)threads);
  job* jobs = (job*)xcalloc((size_t)threads, sizeof(job));
  for (int t = 0; t < threads; t++) {
    jobs[t].cnt = count ? (uint64_t*)xcalloc(2 * (size_t)c->n_flows, 8) : NULL;
    jobs[t].c = c;
    jobs[t].p = p;
    jobs[t].lo = n * (size_t)t / (size_t)threads;
    jobs[t].hi = n * (size_t)(t + 1) / (size_t)threads;
    jobs[t].out = out;
    jobs[t].lb = lb_out;
    if (threads == 1) {
      worker(&jobs[t]);
    } else if (pthread_create(&th[t], NULL, worker, &jobs[t]) != 0) {
      fprintf(stderr, "ovs_cls: pthread_create failed\n");
      abort();
    }
  }
  for (int t = 0; t < threads; t++) {
    if (threads > 1) pthread_join(th[t], NULL);
    if (count) {
      for (int f = 0; f < 2 * c->n_flows; f++) c->cnt[f] += jobs[t].cnt[f];
      free(jobs[t].cnt);
    }
    for (int k = 0; k < 8; k++) c->stats[k] += jobs[t].ws.stats[k];
    free(jobs[t].ws.soft);
    free(jobs[t].ws.hkey);
    free(jobs[t].ws.hbits);
    free(jobs[t].ws.hgen);
    free(jobs[t].ws.done);
  }
  free(th);
  free(jobs);
  return 0;
}

int ocls_classify(ocls* c, const ocls_pkts* p, size_t n, uint32_t* out, int threads, int count) {
  return ocls_classify_lb(c, p, n, out, NULL, threads, count);
}

const uint64_t* ocls_counters(const ocls* c) { return c->cnt; }

/* Lookup statistics summed over every classify call (profiling the baseline): 0 table lookups,
 * 1 subtables probed, 2 subtables skipped by the prefix tries, 3 soft matches collected, 4 soft-loop
 * levels, 5 conjunction actions hashed. */
void ocls_stats(const ocls* c, uint64_t* out) { memcpy(out, c->stats, sizeof c->stats); }
int ocls_n_subtables(const ocls* c, int table) { return (table >= 1 && table < N_TABLES) ? c->tables[table].n_st : 0; }
