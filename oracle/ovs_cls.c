/*
 * ovs_cls.c -- TEST INFRASTRUCTURE ONLY (checker + timed CPU baseline of bench.py).
 *
 * Plain-C restatement of the OVS 2.17.7 userspace classifier (lib/classifier.c; third-party, not
 * vendored in the reference) as Antrea's policy tables exercise it, plus the Antrea policy-stage
 * walk. Same semantics as oracle/ovs_cls.py, organised the way OVS organises it:
 *
 *   - tuple-space search: one subtable per distinct match mask, each a hash table keyed by the
 *     masked field vector; a bucket holds the flows with identical match, highest priority first;
 *   - subtables visited in descending max-priority order, skipping those that cannot beat the best
 *     hard match found so far (PVECTOR_FOR_EACH_PRIORITY(subtable, hard_pri + 1, ...));
 *   - soft (conjunction-only) matches collected per subtable head; the highest soft level above the
 *     hard match is resolved by clause bitmaps; if nothing completes, each soft entry at that level
 *     steps to the next lower flow with identical match (next_visible_rule_in_list) and the loop
 *     repeats; a completed conjunction triggers a lookup with conj_id set that ignores soft flows.
 *   - tie (several conjunctions completing at one priority; order is implementation-defined in
 *     OVS): the lowest conj id whose conj_id lookup succeeds wins and TIE is reported.
 *
 * The Antrea walk (docs/design/ovs-pipeline.md:1159-1330, 1633-1812): {AntreaPolicy,,Default}Rule
 * tables with miss = next table, Pass -> {Egress,Ingress}Rule, allow / deny -> Metric, drop flows,
 * IngressSecurityClassifier bypass for packets not destined to a local Pod.
 *
 * Build: oracle/cbuild.py (gcc -O2 -shared -fPIC -pthread).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum {
  F_DL_TYPE, F_NW_PROTO, F_NW_SRC, F_NW_DST, F_CT_NW_SRC, F_CT_NW_DST, F_IN_PORT, F_REG0, F_REG1, F_REG3, F_REG7,
  F_TUN_ID, F_TP_SRC, F_TP_DST, F_CT_STATE, F_CONJ_ID, F_LABEL_LO, F_LABEL_HI, NF
};

/* flow action kinds (decoded by oracle/cls_c.py from the flow text) */
enum { A_CONJ = 1, A_SET_REG = 2, A_CT_COMMIT = 3, A_GOTO = 4, A_GROUP = 5 };

typedef struct {
  uint8_t kind, reg;
  uint32_t a, b, c;          /* CONJ id,clause,n | SET_REG value,mask | CT table | GOTO table | GROUP id */
  uint64_t lv, lm;           /* CT label */
} ocls_action;

typedef struct {
  int32_t table;             /* 1..6 rule tables, 7 EgressMetric, 8 IngressMetric, others ignored */
  uint32_t priority;
  uint32_t val[NF], mask[NF];
  int32_t act_off, n_act;
  int32_t soft;              /* conjunction-only */
} ocls_flow;

typedef struct {
  const uint32_t *src, *dst;
  const uint16_t *sport, *dport;
  const uint8_t* proto;
  const uint32_t* out_port;
  const uint32_t *in_port, *svc_group, *tun_id, *ct_src, *ct_dst;
  const uint8_t *ct_state, *dest;
  const uint16_t* len;
} ocls_pkts;

/* ------------------------------------------------------------------------------------ model */
typedef struct {
  uint32_t mask[NF];
  uint32_t max_pri;
  uint32_t nb;               /* buckets (power of two) */
  int32_t* head;             /* bucket -> first entry index (-1) */
  int32_t* next;             /* entry -> next entry in bucket chain */
  int32_t* list_off;         /* entry -> offset into lists */
  int32_t* list_n;
  uint32_t* key;             /* entry -> masked key [NF] */
  int32_t n_entries;
  int32_t* lists;            /* flow indices, priority desc */
} subtable;

typedef struct {
  subtable* st;
  int n_st;
} table_t;

typedef struct ocls {
  ocls_flow* flows;
  int n_flows;
  ocls_action* acts;
  table_t tables[9];
  uint32_t* tier_conj;       /* sorted conj ids */
  uint8_t* tier_val;
  int n_tier;
  uint64_t* cnt;             /* per flow: packets, bytes (metric flows) */
} ocls;

static uint64_t mixk(const uint32_t* k) {
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < NF; i++) {
    h ^= k[i];
    h *= 1099511628211ull;
    h ^= h >> 29;
  }
  return h;
}

static int cmp_pri_desc(const void* a, const void* b, void* ctx) {
  const ocls_flow* f = (const ocls_flow*)ctx;
  int x = *(const int*)a, y = *(const int*)b;
  if (f[x].priority != f[y].priority) return f[x].priority < f[y].priority ? 1 : -1;
  return x < y ? -1 : x > y;
}

static const ocls_flow* g_sort_flows;
static int cmp_pri_desc_g(const void* a, const void* b) { return cmp_pri_desc(a, b, (void*)g_sort_flows); }

static int same_mask(const uint32_t* a, const uint32_t* b) { return memcmp(a, b, sizeof(uint32_t) * NF) == 0; }

ocls* ocls_create(const ocls_flow* flows, int n_flows, const ocls_action* acts, int n_acts, const uint32_t* tier_conj,
                  const uint8_t* tier_val, int n_tier) {
  ocls* c = (ocls*)calloc(1, sizeof(ocls));
  c->flows = (ocls_flow*)malloc(sizeof(ocls_flow) * (n_flows ? n_flows : 1));
  memcpy(c->flows, flows, sizeof(ocls_flow) * n_flows);
  c->n_flows = n_flows;
  c->acts = (ocls_action*)malloc(sizeof(ocls_action) * (n_acts ? n_acts : 1));
  memcpy(c->acts, acts, sizeof(ocls_action) * n_acts);
  c->tier_conj = (uint32_t*)malloc(4 * (n_tier ? n_tier : 1));
  c->tier_val = (uint8_t*)malloc(n_tier ? n_tier : 1);
  memcpy(c->tier_conj, tier_conj, 4 * n_tier);
  memcpy(c->tier_val, tier_val, n_tier);
  c->n_tier = n_tier;
  c->cnt = (uint64_t*)calloc(2 * (size_t)(n_flows ? n_flows : 1), 8);
  for (int t = 1; t <= 8; t++) {
    /* group flows by mask */
    int* idx = (int*)malloc(sizeof(int) * (n_flows ? n_flows : 1));
    int n = 0;
    for (int i = 0; i < n_flows; i++)
      if (c->flows[i].table == t) idx[n++] = i;
    subtable* sts = NULL;
    int nst = 0;
    int* owner = (int*)malloc(sizeof(int) * (n ? n : 1));
    for (int j = 0; j < n; j++) {
      const ocls_flow* f = &c->flows[idx[j]];
      int s;
      for (s = 0; s < nst; s++)
        if (same_mask(sts[s].mask, f->mask)) break;
      if (s == nst) {
        sts = (subtable*)realloc(sts, sizeof(subtable) * (nst + 1));
        memset(&sts[nst], 0, sizeof(subtable));
        memcpy(sts[nst].mask, f->mask, sizeof(uint32_t) * NF);
        nst++;
      }
      owner[j] = s;
      if (f->priority > sts[s].max_pri) sts[s].max_pri = f->priority;
    }
    for (int s = 0; s < nst; s++) {
      subtable* st = &sts[s];
      int m = 0;
      for (int j = 0; j < n; j++) m += owner[j] == s;
      uint32_t nb = 1;
      while (nb < (uint32_t)m * 2) nb <<= 1;
      st->nb = nb;
      st->head = (int32_t*)malloc(sizeof(int32_t) * nb);
      for (uint32_t b = 0; b < nb; b++) st->head[b] = -1;
      st->next = (int32_t*)malloc(sizeof(int32_t) * (m ? m : 1));
      st->list_off = (int32_t*)malloc(sizeof(int32_t) * (m ? m : 1));
      st->list_n = (int32_t*)calloc(m ? m : 1, sizeof(int32_t));
      st->key = (uint32_t*)malloc(sizeof(uint32_t) * NF * (m ? m : 1));
      st->lists = (int32_t*)malloc(sizeof(int32_t) * (m ? m : 1));
      /* entries: distinct masked values; first pass count */
      int* fent = (int*)malloc(sizeof(int) * (m ? m : 1));
      int* fidx = (int*)malloc(sizeof(int) * (m ? m : 1));
      int k = 0;
      for (int j = 0; j < n; j++) {
        if (owner[j] != s) continue;
        const ocls_flow* f = &c->flows[idx[j]];
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
        fidx[k] = idx[j];
        k++;
      }
      int off = 0;
      for (int e = 0; e < st->n_entries; e++) {
        st->list_off[e] = off;
        off += st->list_n[e];
        st->list_n[e] = 0;
      }
      for (int q = 0; q < k; q++) {
        int e = fent[q];
        st->lists[st->list_off[e] + st->list_n[e]++] = fidx[q];
      }
      g_sort_flows = c->flows;
      for (int e = 0; e < st->n_entries; e++) qsort(st->lists + st->list_off[e], st->list_n[e], sizeof(int32_t), cmp_pri_desc_g);
      free(fent);
      free(fidx);
    }
    /* subtables by max priority, descending (pvector order) */
    for (int a = 1; a < nst; a++)
      for (int b = a; b > 0 && sts[b].max_pri > sts[b - 1].max_pri; b--) {
        subtable tmp = sts[b];
        sts[b] = sts[b - 1];
        sts[b - 1] = tmp;
      }
    c->tables[t].st = sts;
    c->tables[t].n_st = nst;
    free(idx);
    free(owner);
  }
  return c;
}

void ocls_destroy(ocls* c) {
  if (!c) return;
  for (int t = 1; t <= 8; t++) {
    for (int s = 0; s < c->tables[t].n_st; s++) {
      subtable* st = &c->tables[t].st[s];
      free(st->head);
      free(st->next);
      free(st->list_off);
      free(st->list_n);
      free(st->key);
      free(st->lists);
    }
    free(c->tables[t].st);
  }
  free(c->flows);
  free(c->acts);
  free(c->tier_conj);
  free(c->tier_val);
  free(c->cnt);
  free(c);
}

/* find_match: the bucket list of `st` matching packet vector `pv`, or NULL */
static const int32_t* find_match(const subtable* st, const uint32_t* pv, int* n) {
  uint32_t key[NF];
  for (int q = 0; q < NF; q++) key[q] = pv[q] & st->mask[q];
  uint32_t b = (uint32_t)mixk(key) & (st->nb - 1);
  for (int e = st->head[b]; e >= 0; e = st->next[e])
    if (memcmp(st->key + (size_t)e * NF, key, sizeof key) == 0) {
      *n = st->list_n[e];
      return st->lists + st->list_off[e];
    }
  return NULL;
}

typedef struct {
  const int32_t* list;
  int n, pos;
} soft_ent;

#define MAX_SOFT 256

/* classifier_lookup__ restated. Returns flow index or -1; *tie set on conj ties. */
static int lookup(const ocls* c, int table, uint32_t* pv, int allow_conj, int* tie) {
  const table_t* T = &c->tables[table];
  int hard = -1;
  int64_t hard_pri = -1;
  soft_ent soft[MAX_SOFT];
  int n_soft = 0;
  for (int s = 0; s < T->n_st; s++) {
    const subtable* st = &T->st[s];
    if ((int64_t)st->max_pri < hard_pri + 1) break;
    int n;
    const int32_t* l = find_match(st, pv, &n);
    if (!l) continue;
    int pos = 0;
    const ocls_flow* f = &c->flows[l[pos]];
    if (!allow_conj && f->soft) continue; /* soft heads are ignored, not stepped past (OVS) */
    if ((int64_t)f->priority <= hard_pri) continue;
    if (!f->soft) {
      hard = l[pos];
      hard_pri = f->priority;
    } else if (n_soft < MAX_SOFT) {
      soft[n_soft].list = l;
      soft[n_soft].n = n;
      soft[n_soft].pos = pos;
      n_soft++;
    }
  }
  if (!allow_conj || n_soft == 0) return hard;
  for (;;) {
    /* drop soft entries at or below the hard match */
    int m = 0;
    for (int i = 0; i < n_soft; i++)
      if (soft[i].pos < soft[i].n && (int64_t)c->flows[soft[i].list[soft[i].pos]].priority > hard_pri) soft[m++] = soft[i];
    n_soft = m;
    if (!n_soft) return hard;
    uint32_t top = 0;
    for (int i = 0; i < n_soft; i++) {
      uint32_t p = c->flows[soft[i].list[soft[i].pos]].priority;
      if (p > top) top = p;
    }
    /* conjunction completion at `top` (find_conjunctive_match): clause bitmaps per conj id */
    uint32_t ids[MAX_SOFT * 8];
    uint64_t bits[MAX_SOFT * 8];
    uint32_t ncl[MAX_SOFT * 8];
    int nid = 0;
    for (int i = 0; i < n_soft; i++) {
      const ocls_flow* f = &c->flows[soft[i].list[soft[i].pos]];
      if (f->priority != top) continue;
      for (int a = 0; a < f->n_act; a++) {
        const ocls_action* ac = &c->acts[f->act_off + a];
        if (ac->kind != A_CONJ) continue;
        int j;
        for (j = 0; j < nid; j++)
          if (ids[j] == ac->a) break;
        if (j == nid) {
          if (nid >= MAX_SOFT * 8) continue;
          ids[nid] = ac->a;
          bits[nid] = 0;
          ncl[nid] = ac->c;
          nid++;
        }
        bits[j] |= 1ull << (ac->b - 1);
      }
    }
    /* completed ids, ascending */
    int ndone = 0;
    uint32_t done[MAX_SOFT * 8];
    for (int j = 0; j < nid; j++) {
      uint64_t full = ncl[j] >= 64 ? ~0ull : ((1ull << ncl[j]) - 1);
      if ((bits[j] & full) == full) done[ndone++] = ids[j];
    }
    for (int a = 1; a < ndone; a++)
      for (int b = a; b > 0 && done[b] < done[b - 1]; b--) {
        uint32_t t = done[b];
        done[b] = done[b - 1];
        done[b - 1] = t;
      }
    for (int d = 0; d < ndone; d++) {
      uint32_t saved = pv[F_CONJ_ID];
      pv[F_CONJ_ID] = done[d];
      int dummy = 0;
      int r = lookup(c, table, pv, 0, &dummy);
      pv[F_CONJ_ID] = saved;
      if (r >= 0) {
        if (ndone > 1) *tie = 1;
        return r;
      }
    }
    /* next_visible_rule_in_list for every entry at `top` */
    for (int i = 0; i < n_soft; i++) {
      if (c->flows[soft[i].list[soft[i].pos]].priority != top) continue;
      soft[i].pos++;
      if (soft[i].pos < soft[i].n) {
        int fi = soft[i].list[soft[i].pos];
        if (!c->flows[fi].soft) {
          if ((int64_t)c->flows[fi].priority > hard_pri) {
            hard = fi;
            hard_pri = c->flows[fi].priority;
          }
          soft[i].pos = soft[i].n; /* a hard flow ends the chain */
        }
      }
    }
  }
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
static void stage(const ocls* c, int base, uint32_t* pv, uint32_t len, uint64_t* cnt, uint32_t* out_conj, uint32_t* out_packed) {
  int metric = base == 0 ? 7 : 8;
  int t = base + 1;
  uint32_t flags = 0, conj = 0, tindex = 0, action = ACT_NO_MATCH;
  int t2 = base + 2;
  while (t != metric) {
    int tie = 0;
    int fi = lookup(c, t, pv, 1, &tie);
    if (fi < 0) {
      t = t == base + 3 ? metric : t + 1;
      continue;
    }
    const ocls_flow* f = &c->flows[fi];
    int go = -1, deny = 0, reject = 0, group = 0;
    for (int a = 0; a < f->n_act; a++) {
      const ocls_action* ac = &c->acts[f->act_off + a];
      if (ac->kind == A_SET_REG) {
        uint32_t m = ac->b, v = ac->a;
        int fld = ac->reg == 0 ? F_REG0 : ac->reg == 3 ? F_REG3 : -1;
        if (fld >= 0) pv[fld] = (pv[fld] & ~m) | (v & m);
        if (ac->reg == 0 && (v & m & 0x400)) deny = 1;
        if (ac->reg == 0 && m == 0xfe000000u && ((v >> 25) & 4)) reject = 1;
      } else if (ac->kind == A_CT_COMMIT) {
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
      conj = cid;
      if (deny) {
        action = reject ? ACT_REJECT : ACT_DROP;
        go = metric;
      } else if (go == t2 || (group && ((pv[F_REG0] >> 11) & 3) == 3)) {
        flags |= 1;
        t = t2;
        continue;
      } else {
        action = ACT_ALLOW;
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
  int mf = lookup(c, metric, pv, 0, &tie);
  if (mf >= 0 && cnt) {
    cnt[2 * mf] += 1;
    cnt[2 * mf + 1] += len;
  }
  if (action == ACT_NO_MATCH) tindex = 0;
  *out_conj = conj;
  *out_packed = action | (tindex << 8) | ((conj ? tier_of(c, conj) : 0u) << 16) | (flags << 24);
}

static void classify_range(const ocls* c, const ocls_pkts* p, size_t lo, size_t hi, uint32_t* out, uint64_t* cnt) {
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
    uint32_t ec, ep, gc, gp;
    stage(c, 0, pv, len, cnt, &ec, &ep);
    uint32_t ea = ep & 0xff;
    if (ea == ACT_DROP || ea == ACT_REJECT || ea == ACT_ISO_DROP) {
      gc = 0;
      gp = ACT_NONE;
    } else if (p->dest && p->dest[i] != 0) {
      gc = 0;
      gp = ACT_BYPASS;
    } else {
      pv[F_REG0] = 0;
      pv[F_REG3] = 0;
      pv[F_CONJ_ID] = 0;
      stage(c, 3, pv, len, cnt, &gc, &gp);
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
  uint64_t* cnt;
} job;

static void* worker(void* arg) {
  job* j = (job*)arg;
  classify_range(j->c, j->p, j->lo, j->hi, j->out, j->cnt);
  return NULL;
}

/* out: 4 uint32 per packet (egress conj, egress packed, ingress conj, ingress packed). */
int ocls_classify(ocls* c, const ocls_pkts* p, size_t n, uint32_t* out, int threads, int count) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  job jobs[256];
  uint64_t* cnts[256];
  for (int t = 0; t < threads; t++) {
    cnts[t] = count ? (uint64_t*)calloc(2 * (size_t)(c->n_flows ? c->n_flows : 1), 8) : NULL;
    jobs[t].c = c;
    jobs[t].p = p;
    jobs[t].lo = n * t / threads;
    jobs[t].hi = n * (t + 1) / threads;
    jobs[t].out = out;
    jobs[t].cnt = cnts[t];
    if (threads == 1) worker(&jobs[t]);
    else pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) {
    if (threads > 1) pthread_join(th[t], NULL);
    if (count) {
      for (int f = 0; f < 2 * c->n_flows; f++) c->cnt[f] += cnts[t][f];
      free(cnts[t]);
    }
  }
  return 0;
}

const uint64_t* ocls_counters(const ocls* c) { return c->cnt; }
