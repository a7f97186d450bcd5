/*
 * ORACLE (test infrastructure only) -- C restatement of the kube-scheduler hot path on the
 * compiled SoA inputs of include/kgpu.h.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library;
 * the product never does.  It follows the reference's control flow, not the GPU kernels':
 *
 *   genericScheduler.Schedule        pkg/scheduler/core/generic_scheduler.go:146-209
 *   findNodesThatPassFilters         generic_scheduler.go:424-495 (parallelize.Until over nodes,
 *                                    internal/parallelize/parallelism.go:26-43: 16 workers,
 *                                    chunk = min(sqrt(n), n/16+1))
 *   RunFilterPlugins                 framework/v1alpha1/framework.go:477-502 (early exit)
 *   prioritizeNodes/RunScorePlugins  generic_scheduler.go:622-716, framework.go:579-656
 *   selectHost                       generic_scheduler.go:217-238 (deterministic tie-break key,
 *                                    oracle/refsched/tiebreak.py)
 *   assume                           framework/v1alpha1/types.go:456-480
 *   plugins                          as cited per function below.
 *
 * Feasible nodes are collected in Snapshot.List() order (the reference appends through an
 * atomic counter; DESIGN.md "Determinism contract").  Build: oracle/c/Makefile.
 */
#include <math.h>
#include <stdio.h>
#include <time.h>
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/kgpu.h"

#define MAXN_SCORE 100

typedef struct pool_s pool_t;
static void pool_free(pool_t* p);

typedef struct {
  kgpu_config cfg;
  int N, base, total, S, K, TW, PS, nzones;
  int64_t *alloc_cpu, *alloc_mem, *alloc_eph, *req_cpu, *req_mem, *req_eph, *nz_cpu, *nz_mem;
  int32_t *alloc_pods, *num_pods;
  int64_t *alloc_scalar, *req_scalar;
  uint8_t* unsched;
  int32_t* label_val;
  int32_t* value_off;
  int64_t* value_int;
  uint8_t* value_int_ok;
  uint64_t *taint_nosched, *taint_prefer;
  int32_t* port_count;
  kgpu_port* ports;
  int32_t *image_off, *image_id;
  int64_t* image_score;
  int32_t *avoid_off, *avoid_id, *zone_id;
  int32_t *key_n_values, *key_empty_value;
  int threads;
  void* pool;
  int to_find, next_start; /* numFeasibleNodesToFind(total), nextStartNodeIndex */
  /* existing pods (snapshot pods, then pods assumed by kgpu_ref_schedule) and their terms */
  int PK;
  struct rpod_s* pods;
  int npods, cap_pods;
  int** node_pods; /* [N] pod indices per node (NodeInfo.Pods order) */
  int *node_npods, *node_cap;
} ref_state;

static void* dup_bytes(const void* src, size_t bytes) {
  void* p = malloc(bytes ? bytes : 1);
  if (src && bytes) memcpy(p, src, bytes);
  else memset(p, 0, bytes ? bytes : 1);
  return p;
}

/* ------------------------------------------------------------------ existing pods
 * framework.NodeInfo.Pods / PodInfo (framework/v1alpha1/types.go:79-160, 171-209): every pod
 * keeps its namespace, labels and (anti-)affinity terms.  Terms are deep-copied so that pods
 * assumed from one kgpu_ref_schedule call outlive that call's pools. */
typedef struct {
  int key, op, nvals;
  int32_t* vals;
} oreq;
typedef struct {
  int kind; /* KGPU_SEL_* */
  int nreq;
  oreq* reqs;
} osel;
typedef struct {
  int kind, weight, topo_key, nns;
  int32_t* ns;
  osel sel;
} oterm;
typedef struct rpod_s {
  int node, ns;
  uint32_t flags;
  int nlab;
  int32_t* lab; /* (key id, value id) pairs */
  int nterms;
  oterm* terms;
} rpod;

static osel osel_from(const kgpu_selector* s, const kgpu_pools* p) {
  osel o;
  o.kind = s->kind;
  o.nreq = s->kind == KGPU_SEL_AND ? s->reqs.count : 0;
  o.reqs = (oreq*)calloc(o.nreq ? o.nreq : 1, sizeof(oreq));
  for (int i = 0; i < o.nreq; ++i) {
    const kgpu_req* q = &p->reqs[s->reqs.begin + i];
    o.reqs[i].key = q->key;
    o.reqs[i].op = q->op;
    o.reqs[i].nvals = q->vals.count;
    o.reqs[i].vals = (int32_t*)dup_bytes(p->ints + q->vals.begin, sizeof(int32_t) * q->vals.count);
  }
  return o;
}

static void osel_free(osel* o) {
  for (int i = 0; i < o->nreq; ++i) free(o->reqs[i].vals);
  free(o->reqs);
}

static oterm oterm_from(int kind, const kgpu_pod_term* t, const kgpu_pools* p) {
  oterm o;
  o.kind = kind;
  o.weight = t->weight;
  o.topo_key = t->topo_key;
  o.nns = t->ns.count;
  o.ns = (int32_t*)dup_bytes(p->ints + t->ns.begin, sizeof(int32_t) * t->ns.count);
  o.sel = osel_from(&t->sel, p);
  return o;
}

static void oterm_free(oterm* o) {
  free(o->ns);
  osel_free(&o->sel);
}

static int pod_label(const rpod* pd, int key) {
  if (key < 0) return -1;
  for (int i = 0; i < pd->nlab; ++i)
    if (pd->lab[2 * i] == key) return pd->lab[2 * i + 1];
  return -1;
}

/* labels.Selector.Matches on pod labels (selector.go:198-242, 346-353); Nothing() matches nothing */
static int sel_matches_pod(const osel* s, const rpod* pd) {
  if (s->kind != KGPU_SEL_AND) return 0;
  for (int i = 0; i < s->nreq; ++i) {
    const oreq* q = &s->reqs[i];
    int v = pod_label(pd, q->key), in = 0;
    for (int j = 0; j < q->nvals; ++j) in |= (q->vals[j] == v);
    switch (q->op) {
      case KGPU_OP_IN: if (!(v >= 0 && in)) return 0; break;
      case KGPU_OP_NOTIN: if (v >= 0 && in) return 0; break;
      case KGPU_OP_EXISTS: if (v < 0) return 0; break;
      case KGPU_OP_DNE: if (v >= 0) return 0; break;
      default: return 0;
    }
  }
  return 1;
}

/* schedutil.PodMatchesTermsNamespaceAndSelector (util/topologies.go:40-49) */
static int term_matches_pod(const oterm* t, const rpod* pd) {
  int ok = 0;
  for (int i = 0; i < t->nns; ++i) ok |= (t->ns[i] == pd->ns);
  return ok && sel_matches_pod(&t->sel, pd);
}

static void node_add_pod(ref_state* r, int n, int idx) {
  if (r->node_npods[n] == r->node_cap[n]) {
    r->node_cap[n] = r->node_cap[n] ? 2 * r->node_cap[n] : 4;
    r->node_pods[n] = (int*)realloc(r->node_pods[n], sizeof(int) * r->node_cap[n]);
  }
  r->node_pods[n][r->node_npods[n]++] = idx;
}

static rpod* new_pod(ref_state* r) {
  if (r->npods == r->cap_pods) {
    r->cap_pods = r->cap_pods ? 2 * r->cap_pods : 64;
    r->pods = (rpod*)realloc(r->pods, sizeof(rpod) * r->cap_pods);
  }
  rpod* pd = &r->pods[r->npods++];
  memset(pd, 0, sizeof(*pd));
  return pd;
}

static void load_pods(ref_state* r, const kgpu_snapshot* s) {
  r->PK = s->n_pod_label_keys;
  r->node_pods = (int**)calloc(r->N ? r->N : 1, sizeof(int*));
  r->node_npods = (int*)calloc(r->N ? r->N : 1, sizeof(int));
  r->node_cap = (int*)calloc(r->N ? r->N : 1, sizeof(int));
  for (int i = 0; i < s->n_pods; ++i) {
    rpod* pd = new_pod(r);
    pd->node = s->pod_node[i];
    pd->ns = s->pod_ns[i];
    pd->flags = s->pod_flags[i];
    pd->lab = (int32_t*)calloc(2 * (r->PK ? r->PK : 1), sizeof(int32_t));
    for (int k = 0; k < r->PK; ++k) {
      int v = s->pod_label_val[(size_t)k * s->n_pods + i];
      if (v >= 0) { pd->lab[2 * pd->nlab] = k; pd->lab[2 * pd->nlab + 1] = v; pd->nlab++; }
    }
  }
  for (int t = 0; t < s->n_terms; ++t) {
    const kgpu_term* tm = &s->terms[t];
    rpod* pd = &r->pods[tm->pod];
    pd->terms = (oterm*)realloc(pd->terms, sizeof(oterm) * (pd->nterms + 1));
    pd->terms[pd->nterms++] = oterm_from(tm->kind, &tm->t, &s->pools);
  }
  for (int i = 0; i < r->npods; ++i) {
    int n = r->pods[i].node - r->base;
    if (n >= 0 && n < r->N) node_add_pod(r, n, i);
  }
}

static void free_pods(ref_state* r) {
  for (int i = 0; i < r->npods; ++i) {
    for (int t = 0; t < r->pods[i].nterms; ++t) oterm_free(&r->pods[i].terms[t]);
    free(r->pods[i].terms);
    free(r->pods[i].lab);
  }
  free(r->pods);
  for (int n = 0; n < r->N; ++n) free(r->node_pods[n]);
  free(r->node_pods);
  free(r->node_npods);
  free(r->node_cap);
}

/* The incoming pod as a PodInfo: its labels from the query's (key, value) pairs, its terms. */
static void incoming_pod(rpod* pd, const kgpu_pod_query* q, const kgpu_pools* p) {
  memset(pd, 0, sizeof(*pd));
  pd->node = -1;
  pd->ns = q->ns;
  pd->flags = KGPU_PF_ACTIVE | ((q->flags & KGPU_Q_TERMINATING) ? KGPU_PF_TERMINATING : 0) |
              ((q->flags & (KGPU_Q_HAS_POD_AFFINITY | KGPU_Q_HAS_POD_ANTI)) ? KGPU_PF_WITH_AFFINITY : 0);
  pd->nlab = q->labels.count / 2;
  pd->lab = (int32_t*)dup_bytes(p->ints + q->labels.begin, sizeof(int32_t) * 2 * pd->nlab);
  const kgpu_range rs[4] = {q->ipa_req_aff, q->ipa_req_anti, q->ipa_pref_aff, q->ipa_pref_anti};
  const int kinds[4] = {KGPU_TERM_REQ_AFF, KGPU_TERM_REQ_ANTI, KGPU_TERM_PREF_AFF, KGPU_TERM_PREF_ANTI};
  int nt = 0;
  for (int k = 0; k < 4; ++k) nt += rs[k].count;
  pd->terms = (oterm*)calloc(nt ? nt : 1, sizeof(oterm));
  for (int k = 0; k < 4; ++k)
    for (int i = 0; i < rs[k].count; ++i) pd->terms[pd->nterms++] = oterm_from(kinds[k], &p->pod_terms[rs[k].begin + i], p);
}

static void free_pod(rpod* pd) {
  for (int t = 0; t < pd->nterms; ++t) oterm_free(&pd->terms[t]);
  free(pd->terms);
  free(pd->lab);
}

/* numFeasibleNodesToFind (generic_scheduler.go:379-399): minFeasibleNodesToFind 100,
 * minFeasibleNodesPercentageToFind 5, adaptive 50 - N/125 for percentage 0 (types.go:251). */
static int num_feasible_nodes_to_find(int n, int pct) {
  if (n < 100 || pct >= 100) return n;
  int adaptive = pct;
  if (adaptive <= 0) {
    adaptive = 50 - n / 125;
    if (adaptive < 5) adaptive = 5;
  }
  int k = (int)((int64_t)n * adaptive / 100);
  return k < 100 ? 100 : k;
}

int kgpu_ref_create(const kgpu_config* cfg, const kgpu_snapshot* s, int threads, ref_state** out) {
  ref_state* r = (ref_state*)calloc(1, sizeof(ref_state));
  size_t N = (size_t)s->n_nodes;
  r->cfg = *cfg;
  r->N = s->n_nodes;
  r->base = s->node_base;
  r->total = s->n_total_nodes > 0 ? s->n_total_nodes : s->n_nodes;
  r->S = s->n_scalar;
  r->K = s->n_label_keys;
  r->TW = s->taint_words > 0 ? s->taint_words : 1;
  r->PS = s->port_slots > 8 ? s->port_slots : 8;
  r->nzones = s->n_zones;
  r->threads = threads > 0 ? threads : 1;
  r->pool = NULL;
  r->to_find = num_feasible_nodes_to_find(r->total, cfg->percentage_of_nodes_to_score);
  r->next_start = 0;
#define D(f, src, n, T) r->f = (T*)dup_bytes(src, (n) * sizeof(T))
  D(alloc_cpu, s->alloc_cpu, N, int64_t);
  D(alloc_mem, s->alloc_mem, N, int64_t);
  D(alloc_eph, s->alloc_eph, N, int64_t);
  D(alloc_pods, s->alloc_pods, N, int32_t);
  D(req_cpu, s->req_cpu, N, int64_t);
  D(req_mem, s->req_mem, N, int64_t);
  D(req_eph, s->req_eph, N, int64_t);
  D(nz_cpu, s->nz_cpu, N, int64_t);
  D(nz_mem, s->nz_mem, N, int64_t);
  D(num_pods, s->num_pods, N, int32_t);
  D(alloc_scalar, s->alloc_scalar, (size_t)r->S * N, int64_t);
  D(req_scalar, s->req_scalar, (size_t)r->S * N, int64_t);
  D(unsched, s->unschedulable, N, uint8_t);
  D(label_val, s->label_val, (size_t)r->K * N, int32_t);
  D(value_off, s->value_off, (size_t)r->K + 1, int32_t);
  {
    size_t nv = (r->K > 0 && s->value_off) ? (size_t)s->value_off[r->K] : 0;
    D(value_int, s->value_int, nv, int64_t);
    D(value_int_ok, s->value_int_ok, nv, uint8_t);
  }
  D(taint_nosched, s->taint_words > 0 ? s->taint_nosched : NULL, (size_t)r->TW * N, uint64_t);
  D(taint_prefer, s->taint_words > 0 ? s->taint_prefer : NULL, (size_t)r->TW * N, uint64_t);
  D(port_count, s->port_count, N, int32_t);
  r->ports = (kgpu_port*)calloc((size_t)r->PS * N + 1, sizeof(kgpu_port));
  for (int sl = 0; sl < s->port_slots; ++sl)
    memcpy(r->ports + (size_t)sl * N, s->ports + (size_t)sl * N, N * sizeof(kgpu_port));
  D(image_off, s->image_off, N + 1, int32_t);
  D(image_id, s->image_id, (size_t)s->image_off[N], int32_t);
  D(image_score, s->image_score, (size_t)s->image_off[N], int64_t);
  D(avoid_off, s->avoid_off, N + 1, int32_t);
  D(avoid_id, s->avoid_id, (size_t)s->avoid_off[N], int32_t);
  D(zone_id, s->zone_id, N, int32_t);
  D(key_n_values, s->key_n_values, (size_t)r->K, int32_t);
  D(key_empty_value, s->key_empty_value, (size_t)r->K, int32_t);
#undef D
  load_pods(r, s);
  *out = r;
  return 0;
}

void kgpu_ref_destroy(ref_state* r) {
  if (!r) return;
  void* ptrs[] = {r->alloc_cpu, r->alloc_mem, r->alloc_eph, r->req_cpu, r->req_mem, r->req_eph, r->nz_cpu,
                  r->nz_mem, r->alloc_pods, r->num_pods, r->alloc_scalar, r->req_scalar, r->unsched,
                  r->label_val, r->value_off, r->value_int, r->value_int_ok, r->taint_nosched, r->taint_prefer,
                  r->port_count, r->ports, r->image_off, r->image_id, r->image_score, r->avoid_off, r->avoid_id,
                  r->zone_id, r->key_n_values, r->key_empty_value};
  for (size_t i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); ++i) free(ptrs[i]);
  free_pods(r);
  pool_free((pool_t*)r->pool);
  free(r);
}

/* ------------------------------------------------------------------ labels (selector.go:198-242) */
static int has_val(const kgpu_pools* p, kgpu_range r, int v) {
  for (int i = 0; i < r.count; ++i)
    if (p->ints[r.begin + i] == v) return 1;
  return 0;
}

static int req_matches_node(const ref_state* r, const kgpu_pools* p, const kgpu_req* q, int n) {
  int v = q->key >= 0 ? r->label_val[(size_t)q->key * r->N + n] : -1; /* -1: label key absent */
  switch (q->op) {
    case KGPU_OP_IN: return v >= 0 && has_val(p, q->vals, v);
    case KGPU_OP_NOTIN: return v < 0 || !has_val(p, q->vals, v);
    case KGPU_OP_EXISTS: return v >= 0;
    case KGPU_OP_DNE: return v < 0;
    case KGPU_OP_GT:
    case KGPU_OP_LT: {
      if (v < 0) return 0;
      int idx = r->value_off[q->key] + v;
      if (!r->value_int_ok[idx]) return 0; /* strconv.ParseInt failed */
      return q->op == KGPU_OP_GT ? r->value_int[idx] > q->imm : r->value_int[idx] < q->imm;
    }
  }
  return 0;
}

static int selector_matches_node(const ref_state* r, const kgpu_pools* p, kgpu_range reqs, int n) {
  for (int i = 0; i < reqs.count; ++i)
    if (!req_matches_node(r, p, &p->reqs[reqs.begin + i], n)) return 0;
  return 1;
}

/* plugins/helper/node_affinity.go:28-78 + core/v1/helper/helpers.go:317-346 */
static int pod_matches_node_selector_and_affinity(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q,
                                                  int n) {
  if (q->node_selector.count > 0 && !selector_matches_node(r, p, q->node_selector, n)) return 0;
  if (!(q->flags & KGPU_Q_REQ_NODE_AFFINITY)) return 1;
  for (int t = 0; t < q->req_terms.count; ++t) {
    const kgpu_node_term* term = &p->node_terms[q->req_terms.begin + t];
    if (term->never_match) continue; /* nil/empty term or invalid requirement selects nothing */
    if (term->reqs.count && !selector_matches_node(r, p, term->reqs, n)) continue;
    if (term->field_op == KGPU_OP_IN && r->base + n != term->field_node) continue;
    if (term->field_op == KGPU_OP_NOTIN && r->base + n == term->field_node) continue;
    return 1;
  }
  return 0;
}

/* ------------------------------------------------------------------ math.Log (Go stdlib)
 * Go's math.Log is the FreeBSD e_log.c algorithm (src/math/log.go, go1.13.9); restated here.
 * Used by PodTopologySpread topologyNormalizingWeight (podtopologyspread/scoring.go:286-288). */
static double go_log(double x) {
  const double ln2hi = 6.93147180369123816490e-01, ln2lo = 1.90821492927058770002e-10;
  const double l1 = 6.666666666666735130e-01, l2 = 3.999999999940941908e-01, l3 = 2.857142874366239149e-01,
               l4 = 2.222219843214978396e-01, l5 = 1.818357216161805012e-01, l6 = 1.531383769920937332e-01,
               l7 = 1.479819860511658591e-01;
  if (x != x || x == INFINITY) return x;
  if (x < 0) return NAN;
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = frexp(x, &ki);
  if (f1 < 0.70710678118654752440 /* Sqrt2/2 */) {
    f1 *= 2;
    ki--;
  }
  double f = f1 - 1;
  double k = (double)ki;
  double s = f / (2 + f);
  double s2 = s * s;
  double s4 = s2 * s2;
  double t1 = s2 * (l1 + s4 * (l3 + s4 * (l5 + s4 * l7)));
  double t2 = s4 * (l2 + s4 * (l4 + s4 * l6));
  double R = t1 + t2;
  double hfsq = 0.5 * f * f;
  return k * ln2hi - ((hfsq - (s * (hfsq + R) + k * ln2lo)) - f);
}

/* ------------------------------------------------------------------ per-cycle plugin state
 * CycleState of PodTopologySpread (preFilterState filtering.go:47-60, preScoreState
 * scoring.go:39-48), InterPodAffinity (filtering.go:47-60, scoring.go:38-43) and
 * DefaultPodTopologySpread (the selector, default_pod_topology_spread.go:191-205). Maps keyed by
 * topologyPair{key, value} are per-key arrays indexed by the value id. */
typedef struct {
  rpod self;
  int64_t** arr[8]; /* per-key arrays, lazily allocated: see A_* */
  /* PodTopologySpread filter */
  int pn;
  const kgpu_spread* hard;
  osel* hsel;
  int pany;
  int64_t* pmin; /* [pn] critical-path minimum of the constraint's key */
  /* PodTopologySpread score */
  int sn;
  const kgpu_spread* soft;
  osel* ssel;
  double* sw;
  uint8_t* ignored; /* [N] */
  /* InterPodAffinity */
  int ex_any, aff_any, topo_any;
  /* DefaultPodTopologySpread */
  osel dsel;
} qstate;

enum { A_PREG, A_PCNT, A_SREG, A_SCNT, A_EXANTI, A_AFF, A_ANTI, A_TOPO };

static int64_t* karr(qstate* s, const ref_state* r, int which, int k) {
  if (!s->arr[which]) s->arr[which] = (int64_t**)calloc(r->K ? r->K : 1, sizeof(int64_t*));
  if (!s->arr[which][k]) s->arr[which][k] = (int64_t*)calloc(r->key_n_values[k] ? r->key_n_values[k] : 1, sizeof(int64_t));
  return s->arr[which][k];
}

/* read-only lookup (filter / score run on the worker threads) */
static int64_t kget(const qstate* s, int which, int k, int v) {
  if (k < 0 || v < 0 || !s->arr[which] || !s->arr[which][k]) return 0;
  return s->arr[which][k][v];
}

static int nval(const ref_state* r, int k, int n) { return k >= 0 ? r->label_val[(size_t)k * r->N + n] : -1; }

static int node_has_labels(const ref_state* r, int n) {
  for (int k = 0; k < r->K; ++k)
    if (r->label_val[(size_t)k * r->N + n] >= 0) return 1;
  return 0;
}

/* countPodsMatchSelector (podtopologyspread/common.go:85-99): same namespace, not terminating */
static int64_t count_match(const ref_state* r, int n, const osel* sel, int ns) {
  int64_t c = 0;
  for (int i = 0; i < r->node_npods[n]; ++i) {
    const rpod* pd = &r->pods[r->node_pods[n][i]];
    if ((pd->flags & KGPU_PF_TERMINATING) || pd->ns != ns) continue;
    if (sel_matches_pod(sel, pd)) c++;
  }
  return c;
}

static int all_keys(const ref_state* r, const kgpu_spread* c, int nc, int n) {
  for (int i = 0; i < nc; ++i)
    if (nval(r, c[i].key, n) < 0) return 0;
  return 1;
}

/* PodTopologySpread PreFilter (filtering.go:198-273) */
static void pts_prefilter(qstate* s, const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q) {
  s->pn = q->pts_hard.count;
  if (!s->pn) return;
  s->hard = &p->spreads[q->pts_hard.begin];
  s->hsel = (osel*)calloc(s->pn, sizeof(osel));
  s->pmin = (int64_t*)calloc(s->pn, sizeof(int64_t));
  for (int i = 0; i < s->pn; ++i) s->hsel[i] = osel_from(&s->hard[i].sel, p);
  for (int n = 0; n < r->N; ++n) {
    if (!pod_matches_node_selector_and_affinity(r, p, q, n) || !all_keys(r, s->hard, s->pn, n)) continue;
    for (int i = 0; i < s->pn; ++i) karr(s, r, A_PREG, s->hard[i].key)[nval(r, s->hard[i].key, n)] = 1;
    s->pany = 1;
  }
  for (int n = 0; n < r->N; ++n) {
    for (int i = 0; i < s->pn; ++i) {
      int k = s->hard[i].key;
      if (k < 0) continue;
      int v = nval(r, k, n);
      if (v < 0) v = r->key_empty_value[k]; /* node.Labels[key] of a missing key is "" */
      if (v < 0 || !karr(s, r, A_PREG, k)[v]) continue;
      karr(s, r, A_PCNT, k)[v] += count_match(r, n, &s->hsel[i], q->ns);
    }
  }
  /* criticalPaths.update (filtering.go:93-121) keeps the minimum over the key's pairs in [0] */
  for (int i = 0; i < s->pn; ++i) {
    int k = s->hard[i].key;
    int64_t mn = 2147483647;
    if (k >= 0) {
      const int64_t* reg = karr(s, r, A_PREG, k);
      const int64_t* cnt = karr(s, r, A_PCNT, k);
      for (int v = 0; v < r->key_n_values[k]; ++v)
        if (reg[v] && cnt[v] < mn) mn = cnt[v];
    }
    s->pmin[i] = mn;
  }
}

/* PodTopologySpread Filter (filtering.go:276-328) */
static int pts_filter_ok(const qstate* s, const ref_state* r, int n) {
  if (!s->pn || !s->pany) return 1;
  for (int i = 0; i < s->pn; ++i) {
    int k = s->hard[i].key;
    int v = nval(r, k, n);
    if (v < 0) return 0;
    int64_t match = kget(s, A_PREG, k, v) ? kget(s, A_PCNT, k, v) : 0;
    if (match + s->hard[i].self_match - s->pmin[i] > s->hard[i].max_skew) return 0;
  }
  return 1;
}

/* PodTopologySpread PreScore (scoring.go:59-169) over the feasible nodes F */
static void pts_prescore(qstate* s, const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, const int* F,
                         int nf) {
  s->sn = q->pts_soft.count;
  s->ignored = (uint8_t*)calloc(r->N ? r->N : 1, 1);
  if (!s->sn || nf == 0) {
    s->sn = 0;
    return;
  }
  s->soft = &p->spreads[q->pts_soft.begin];
  s->ssel = (osel*)calloc(s->sn, sizeof(osel));
  s->sw = (double*)calloc(s->sn, sizeof(double));
  int64_t* size = (int64_t*)calloc(s->sn, sizeof(int64_t));
  for (int i = 0; i < s->sn; ++i) s->ssel[i] = osel_from(&s->soft[i].sel, p);
  int nign = 0;
  for (int j = 0; j < nf; ++j) {
    int n = F[j];
    if (!all_keys(r, s->soft, s->sn, n)) {
      s->ignored[n] = 1;
      nign++;
      continue;
    }
    for (int i = 0; i < s->sn; ++i) {
      if (s->soft[i].is_hostname) continue;
      int64_t* reg = karr(s, r, A_SREG, s->soft[i].key);
      int v = nval(r, s->soft[i].key, n);
      if (!reg[v]) {
        reg[v] = 1;
        size[i]++;
      }
    }
  }
  for (int i = 0; i < s->sn; ++i) {
    int64_t sz = s->soft[i].is_hostname ? (int64_t)(nf - nign) : size[i];
    s->sw[i] = go_log((double)(sz + 2)); /* topologyNormalizingWeight */
  }
  free(size);
  for (int n = 0; n < r->N; ++n) {
    if (!pod_matches_node_selector_and_affinity(r, p, q, n) || !all_keys(r, s->soft, s->sn, n)) continue;
    for (int i = 0; i < s->sn; ++i) {
      int k = s->soft[i].key, v = nval(r, k, n);
      if (s->soft[i].is_hostname || !karr(s, r, A_SREG, k)[v]) continue;
      karr(s, r, A_SCNT, k)[v] += count_match(r, n, &s->ssel[i], q->ns);
    }
  }
}

/* PodTopologySpread Score (scoring.go:174-208) */
static int64_t pts_score(const qstate* s, const ref_state* r, const kgpu_pod_query* q, int n) {
  if (s->ignored[n]) return 0;
  double score = 0;
  for (int i = 0; i < s->sn; ++i) {
    int k = s->soft[i].key, v = nval(r, k, n);
    if (v < 0) continue;
    int64_t cnt = s->soft[i].is_hostname ? count_match(r, n, &s->ssel[i], q->ns) : kget(s, A_SCNT, k, v);
    if (cnt < s->soft[i].max_skew) cnt = s->soft[i].max_skew - 1; /* adjustForMaxSkew */
    score += (double)cnt * s->sw[i];
  }
  return (int64_t)score;
}

/* PodTopologySpread NormalizeScore (scoring.go:211-257) */
static void pts_normalize(qstate* s, int64_t* sc, const int* F, int nf) {
  int64_t mn = INT64_MAX, mx = 0;
  for (int j = 0; j < nf; ++j) {
    if (s->ignored[F[j]]) continue;
    if (sc[j] < mn) mn = sc[j];
    if (sc[j] > mx) mx = sc[j];
  }
  for (int j = 0; j < nf; ++j) {
    if (s->ignored[F[j]]) sc[j] = 0;
    else if (mx == 0) sc[j] = MAXN_SCORE;
    else sc[j] = MAXN_SCORE * (mx + mn - sc[j]) / mx;
  }
}

/* DefaultPodTopologySpread Score (default_pod_topology_spread.go:75-106) */
static int64_t dpts_score(const qstate* s, const ref_state* r, const kgpu_pod_query* q, int n) {
  if (q->flags & KGPU_Q_HAS_TSC) return 0;
  if (r->node_npods[n] == 0 || s->dsel.kind == KGPU_SEL_EMPTY) return 0;
  return count_match(r, n, &s->dsel, q->ns);
}

/* DefaultPodTopologySpread NormalizeScore (default_pod_topology_spread.go:109-163) */
static void dpts_normalize(const ref_state* r, const kgpu_pod_query* q, int64_t* sc, const int* F, int nf) {
  if (q->flags & KGPU_Q_HAS_TSC) return;
  const double zw = 2.0 / 3.0;
  int Z = r->nzones > 0 ? r->nzones : 1;
  int64_t* zc = (int64_t*)calloc(Z, sizeof(int64_t));
  uint8_t* zh = (uint8_t*)calloc(Z, 1);
  int64_t max_node = 0, max_zone = 0;
  int have_zones = 0;
  for (int j = 0; j < nf; ++j) {
    if (sc[j] > max_node) max_node = sc[j];
    int z = r->zone_id[F[j]];
    if (z < 0) continue;
    zc[z] += sc[j];
    zh[z] = 1;
    have_zones = 1;
  }
  for (int z = 0; z < Z; ++z)
    if (zh[z] && zc[z] > max_zone) max_zone = zc[z];
  for (int j = 0; j < nf; ++j) {
    double f = (double)MAXN_SCORE;
    if (max_node > 0) f = (double)MAXN_SCORE * ((double)(max_node - sc[j]) / (double)max_node);
    int z = r->zone_id[F[j]];
    if (have_zones && z >= 0) {
      double zs = (double)MAXN_SCORE;
      if (max_zone > 0) zs = (double)MAXN_SCORE * ((double)(max_zone - zc[z]) / (double)max_zone);
      f = (f * (1.0 - zw)) + (zw * zs);
    }
    sc[j] = (int64_t)f;
  }
  free(zc);
  free(zh);
}

/* podMatchesAllAffinityTerms (interpodaffinity/filtering.go:151-161) */
static int pod_matches_all(const rpod* self, const rpod* pd) {
  int any = 0;
  for (int t = 0; t < self->nterms; ++t) {
    if (self->terms[t].kind != KGPU_TERM_REQ_AFF) continue;
    any = 1;
    if (!term_matches_pod(&self->terms[t], pd)) return 0;
  }
  return any;
}

/* InterPodAffinity PreFilter (filtering.go:166-271) */
static void ipa_prefilter(qstate* s, const ref_state* r) {
  const rpod* self = &s->self;
  for (int i = 0; i < r->npods; ++i) {
    const rpod* ep = &r->pods[i];
    int n = ep->node - r->base;
    if (!(ep->flags & KGPU_PF_WITH_AFFINITY) || n < 0 || n >= r->N) continue;
    for (int t = 0; t < ep->nterms; ++t) {
      const oterm* tm = &ep->terms[t];
      if (tm->kind != KGPU_TERM_REQ_ANTI || !term_matches_pod(tm, self)) continue;
      int v = nval(r, tm->topo_key, n);
      if (v < 0) continue;
      karr(s, r, A_EXANTI, tm->topo_key)[v] += 1;
      s->ex_any = 1;
    }
  }
  int has_req = 0;
  for (int t = 0; t < self->nterms; ++t) has_req |= (self->terms[t].kind <= KGPU_TERM_REQ_ANTI);
  if (!has_req) return;
  for (int n = 0; n < r->N; ++n) {
    for (int j = 0; j < r->node_npods[n]; ++j) {
      const rpod* ep = &r->pods[r->node_pods[n][j]];
      if (pod_matches_all(self, ep)) {
        for (int t = 0; t < self->nterms; ++t) {
          const oterm* tm = &self->terms[t];
          if (tm->kind != KGPU_TERM_REQ_AFF) continue;
          int v = nval(r, tm->topo_key, n);
          if (v < 0) continue;
          karr(s, r, A_AFF, tm->topo_key)[v] += 1;
          s->aff_any = 1;
        }
      }
      for (int t = 0; t < self->nterms; ++t) {
        const oterm* tm = &self->terms[t];
        if (tm->kind != KGPU_TERM_REQ_ANTI || !term_matches_pod(tm, ep)) continue;
        int v = nval(r, tm->topo_key, n);
        if (v < 0) continue;
        karr(s, r, A_ANTI, tm->topo_key)[v] += 1;
      }
    }
  }
}

/* InterPodAffinity Filter (filtering.go:314-396); returns 0 or the rule that failed (1..3) */
static int ipa_filter(const qstate* s, const ref_state* r, const kgpu_pod_query* q, int n) {
  const rpod* self = &s->self;
  int exist = 1;
  for (int t = 0; t < self->nterms; ++t) {
    const oterm* tm = &self->terms[t];
    if (tm->kind != KGPU_TERM_REQ_AFF) continue;
    int v = nval(r, tm->topo_key, n);
    if (v < 0) return 1;
    if (kget(s, A_AFF, tm->topo_key, v) <= 0) exist = 0;
  }
  if (!exist && !(!s->aff_any && (q->flags & KGPU_Q_SELF_MATCH_ALL_AFF))) return 1;
  for (int t = 0; t < self->nterms; ++t) {
    const oterm* tm = &self->terms[t];
    if (tm->kind != KGPU_TERM_REQ_ANTI) continue;
    int v = nval(r, tm->topo_key, n);
    if (v >= 0 && kget(s, A_ANTI, tm->topo_key, v) > 0) return 2;
  }
  if (s->ex_any) {
    for (int k = 0; k < r->K; ++k) {
      int v = nval(r, k, n);
      if (v >= 0 && kget(s, A_EXANTI, k, v) > 0) return 3;
    }
  }
  return 0;
}

/* InterPodAffinity PreScore (scoring.go:47-199): topologyScore[key][value] */
static void ipa_prescore(qstate* s, const ref_state* r, int hard_weight) {
  const rpod* self = &s->self;
  const int self_aff = (self->flags & KGPU_PF_WITH_AFFINITY) != 0;
  for (int n = 0; n < r->N; ++n) {
    if (!node_has_labels(r, n)) continue; /* processTerm: len(fixedNode.Labels) == 0 */
    for (int j = 0; j < r->node_npods[n]; ++j) {
      const rpod* ep = &r->pods[r->node_pods[n][j]];
      if (!self_aff && !(ep->flags & KGPU_PF_WITH_AFFINITY)) continue; /* PodsWithAffinity only */
      for (int t = 0; t < self->nterms; ++t) {
        const oterm* tm = &self->terms[t];
        if (tm->kind < KGPU_TERM_PREF_AFF) continue;
        int v = nval(r, tm->topo_key, n);
        if (v < 0 || !term_matches_pod(tm, ep)) continue;
        karr(s, r, A_TOPO, tm->topo_key)[v] += (int64_t)tm->weight * (tm->kind == KGPU_TERM_PREF_AFF ? 1 : -1);
        s->topo_any = 1;
      }
      for (int t = 0; t < ep->nterms; ++t) {
        const oterm* tm = &ep->terms[t];
        int64_t w;
        if (tm->kind == KGPU_TERM_REQ_AFF) {
          if (hard_weight <= 0) continue;
          w = hard_weight;
        } else if (tm->kind == KGPU_TERM_PREF_AFF) {
          w = tm->weight;
        } else if (tm->kind == KGPU_TERM_PREF_ANTI) {
          w = -(int64_t)tm->weight;
        } else {
          continue;
        }
        int v = nval(r, tm->topo_key, n);
        if (v < 0 || !term_matches_pod(tm, self)) continue;
        karr(s, r, A_TOPO, tm->topo_key)[v] += w;
        s->topo_any = 1;
      }
    }
  }
}

/* InterPodAffinity Score (scoring.go:217-236) */
static int64_t ipa_score(const qstate* s, const ref_state* r, int n) {
  if (!s->topo_any) return 0;
  int64_t sc = 0;
  for (int k = 0; k < r->K; ++k) {
    if (!s->arr[A_TOPO] || !s->arr[A_TOPO][k]) continue;
    int v = nval(r, k, n);
    if (v >= 0) sc += s->arr[A_TOPO][k][v];
  }
  return sc;
}

/* InterPodAffinity NormalizeScore (scoring.go:241-272) */
static void ipa_normalize(qstate* s, int64_t* sc, int nf) {
  if (!s->topo_any) return;
  int64_t mx = 0, mn = 0;
  for (int j = 0; j < nf; ++j) {
    if (sc[j] > mx) mx = sc[j];
    if (sc[j] < mn) mn = sc[j];
  }
  int64_t diff = mx - mn;
  for (int j = 0; j < nf; ++j) {
    double f = 0;
    if (diff > 0) f = (double)MAXN_SCORE * ((double)(sc[j] - mn) / (double)diff);
    sc[j] = (int64_t)f;
  }
}

static void qstate_free(qstate* s, const ref_state* r) {
  for (int a = 0; a < 8; ++a) {
    if (!s->arr[a]) continue;
    for (int k = 0; k < r->K; ++k) free(s->arr[a][k]);
    free(s->arr[a]);
  }
  for (int i = 0; i < s->pn; ++i) osel_free(&s->hsel[i]);
  for (int i = 0; i < s->sn; ++i) osel_free(&s->ssel[i]);
  free(s->hsel);
  free(s->ssel);
  free(s->pmin);
  free(s->sw);
  free(s->ignored);
  osel_free(&s->dsel);
  free_pod(&s->self);
}

/* NodeInfo.AddPod's pod-list side (types.go:456-480): the assumed pod becomes an existing pod */
static void add_pod_record(ref_state* r, const kgpu_pod_query* q, const kgpu_pools* p, int n) {
  rpod tmp;
  incoming_pod(&tmp, q, p);
  tmp.node = r->base + n;
  rpod* pd = new_pod(r);
  *pd = tmp;
  node_add_pod(r, n, r->npods - 1);
}

/* ------------------------------------------------------------------ filters */
static uint32_t filter_fit(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, int n) {
  /* noderesources/fit.go:194-267 fitsRequest */
  uint32_t ins = 0;
  if (r->num_pods[n] + 1 > r->alloc_pods[n]) ins |= 1;
  if (q->flags & KGPU_Q_FIT_ALL_ZERO) return ins;
  if (r->alloc_cpu[n] < q->req[0] + r->req_cpu[n]) ins |= 2;
  if (r->alloc_mem[n] < q->req[1] + r->req_mem[n]) ins |= 4;
  if (r->alloc_eph[n] < q->req[2] + r->req_eph[n]) ins |= 8;
  for (int i = 0; i < q->scalars.count; ++i) {
    const kgpu_scalar_req* s = &p->scalars[q->scalars.begin + i];
    if (!s->check) continue;
    int64_t alloc = s->col >= 0 ? r->alloc_scalar[(size_t)s->col * r->N + n] : 0;
    int64_t used = s->col >= 0 ? r->req_scalar[(size_t)s->col * r->N + n] : 0;
    if (alloc < s->value + used) ins |= 16u << (i < 11 ? i : 11);
  }
  return ins;
}

static int filter_ports_ok(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, int n) {
  /* nodeports/node_ports.go:115-123 + HostPortInfo.CheckConflict types.go:726-756 */
  for (int i = 0; i < q->ports.count; ++i) {
    const kgpu_port* w = &p->ports[q->ports.begin + i];
    for (int s = 0; s < r->port_count[n]; ++s) {
      const kgpu_port* u = &r->ports[(size_t)s * r->N + n];
      if (u->proto != w->proto || u->port != w->port) continue;
      if (w->ip == 0 /* 0.0.0.0: any ip */ || u->ip == 0 || u->ip == w->ip) return 0;
    }
  }
  return 1;
}

static int filter_taints_ok(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, int n) {
  /* tainttoleration/taint_toleration.go:54-72: any untolerated NoSchedule/NoExecute taint */
  for (int w = 0; w < r->TW; ++w) {
    uint64_t tol = w < q->tol_nosched.count ? p->words[q->tol_nosched.begin + w] : 0;
    if (r->taint_nosched[(size_t)w * r->N + n] & ~tol) return 0;
  }
  return 1;
}

static int has_filter(const ref_state* r, int f) {
  for (int i = 0; i < r->cfg.n_filters; ++i)
    if (r->cfg.filters[i] == f) return 1;
  return 0;
}

static int has_score(const ref_state* r, int sc) {
  for (int i = 0; i < r->cfg.n_scores; ++i)
    if (r->cfg.scores[i] == sc) return 1;
  return 0;
}

/* RunFilterPlugins with early exit; returns the status word of include/kgpu.h */
static uint32_t run_filter_plugins(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, qstate* qs,
                                   int n) {
  for (int i = 0; i < r->cfg.n_filters; ++i) {
    uint32_t pos = (uint32_t)(i + 1);
    switch (r->cfg.filters[i]) {
      case KGPU_F_NODE_UNSCHEDULABLE:
        if (r->unsched[n] && !(q->flags & KGPU_Q_TOLERATES_UNSCHEDULABLE)) return pos | (KGPU_CODE_UNRESOLVABLE << 8);
        break;
      case KGPU_F_NODE_RESOURCES_FIT: {
        uint32_t ins = filter_fit(r, p, q, n);
        if (ins) return pos | (KGPU_CODE_UNSCHEDULABLE << 8) | (ins << 16);
        break;
      }
      case KGPU_F_NODE_NAME:
        if (q->node_name != -1 && q->node_name != r->base + n) return pos | (KGPU_CODE_UNRESOLVABLE << 8);
        break;
      case KGPU_F_NODE_PORTS:
        if (!filter_ports_ok(r, p, q, n)) return pos | (KGPU_CODE_UNSCHEDULABLE << 8);
        break;
      case KGPU_F_NODE_AFFINITY:
        if (!pod_matches_node_selector_and_affinity(r, p, q, n)) return pos | (KGPU_CODE_UNRESOLVABLE << 8);
        break;
      case KGPU_F_TAINT_TOLERATION:
        if (!filter_taints_ok(r, p, q, n)) return pos | (KGPU_CODE_UNRESOLVABLE << 8);
        break;
      case KGPU_F_POD_TOPOLOGY_SPREAD:
        if (!pts_filter_ok(qs, r, n)) return pos | (KGPU_CODE_UNSCHEDULABLE << 8);
        break;
      case KGPU_F_INTER_POD_AFFINITY: {
        int rule = ipa_filter(qs, r, q, n);
        if (rule) return pos | ((rule == 1 ? KGPU_CODE_UNRESOLVABLE : KGPU_CODE_UNSCHEDULABLE) << 8) | ((uint32_t)rule << 16);
        break;
      }
      default:
        break;
    }
  }
  return 0;
}

/* ------------------------------------------------------------------ scores */
static int64_t pod_score_scalar(const kgpu_pools* p, const kgpu_pod_query* q, int col) {
  for (int i = 0; i < q->scalars.count; ++i)
    if (p->scalars[q->scalars.begin + i].col == col) return p->scalars[q->scalars.begin + i].score_value;
  return 0;
}

/* resource_allocation.go:92-113 */
static void allocatable_requested(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, int res, int n,
                                  int64_t* alloc, int64_t* req) {
  if (res == 0) { *alloc = r->alloc_cpu[n]; *req = r->nz_cpu[n] + q->score_req[0]; }
  else if (res == 1) { *alloc = r->alloc_mem[n]; *req = r->nz_mem[n] + q->score_req[1]; }
  else if (res == 2) { *alloc = r->alloc_eph[n]; *req = r->req_eph[n] + q->score_req[2]; }
  else if (res >= 3) {
    *alloc = r->alloc_scalar[(size_t)(res - 3) * r->N + n];
    *req = r->req_scalar[(size_t)(res - 3) * r->N + n] + pod_score_scalar(p, q, res - 3);
  } else { *alloc = 0; *req = 0; }
}

static int64_t least_requested_score(int64_t requested, int64_t capacity) { /* least_allocated.go:105-117 */
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  return ((capacity - requested) * MAXN_SCORE) / capacity;
}

static int64_t most_requested_score(int64_t requested, int64_t capacity) { /* most_allocated.go:105-117 */
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  return (requested * MAXN_SCORE) / capacity;
}

static int64_t resource_scorer(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, int n, int most) {
  int64_t node_score = 0, weight_sum = 0;
  int cnt = most ? r->cfg.n_most : r->cfg.n_least;
  const kgpu_resource_weight* rw = most ? r->cfg.most : r->cfg.least;
  for (int i = 0; i < cnt; ++i) {
    int64_t a, rq;
    allocatable_requested(r, p, q, rw[i].resource, n, &a, &rq);
    int64_t s = most ? most_requested_score(rq, a) : least_requested_score(rq, a);
    node_score += s * rw[i].weight;
    weight_sum += rw[i].weight;
  }
  return weight_sum ? node_score / weight_sum : 0;
}

/* requested_to_capacity_ratio.go:150-170 buildBrokenLinearFunction */
static int64_t broken_linear(const kgpu_config* c, int64_t p) {
  for (int i = 0; i < c->n_shape; ++i) {
    if (p <= c->shape[i].utilization) {
      if (i == 0) return c->shape[0].score;
      return c->shape[i - 1].score + (c->shape[i].score - c->shape[i - 1].score) * (p - c->shape[i - 1].utilization) /
                                         (c->shape[i].utilization - c->shape[i - 1].utilization);
    }
  }
  return c->shape[c->n_shape - 1].score;
}

/* requested_to_capacity_ratio.go:124-148 buildRequestedToCapacityRatioScorerFunction */
static int64_t rtcr_score(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, int n) {
  int64_t node_score = 0, weight_sum = 0;
  for (int i = 0; i < r->cfg.n_rtcr; ++i) {
    int64_t cap, req, s;
    int64_t w = r->cfg.rtcr[i].weight ? r->cfg.rtcr[i].weight : 1;
    allocatable_requested(r, p, q, r->cfg.rtcr[i].resource, n, &cap, &req);
    if (cap == 0 || req > cap) s = broken_linear(&r->cfg, 100);
    else s = broken_linear(&r->cfg, 100 - (cap - req) * 100 / cap);
    if (s > 0) {
      node_score += s * w;
      weight_sum += w;
    }
  }
  if (weight_sum == 0) return 0;
  return (int64_t)round((double)node_score / (double)weight_sum); /* math.Round: half away from zero */
}

/* resource_limits.go:118-160 */
static int64_t limits_score(const ref_state* r, const kgpu_pod_query* q, int n) {
  int cpu = q->limits[0] != 0 && r->alloc_cpu[n] != 0 && q->limits[0] <= r->alloc_cpu[n];
  int mem = q->limits[1] != 0 && r->alloc_mem[n] != 0 && q->limits[1] <= r->alloc_mem[n];
  return (cpu || mem) ? 1 : 0;
}

static double fraction_of_capacity(int64_t req, int64_t cap) { return cap == 0 ? 1.0 : (double)req / (double)cap; }

static int64_t balanced_score(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, int n) {
  /* balanced_allocation.go:83-120 */
  int64_t ca, cr, ma, mr;
  allocatable_requested(r, p, q, 0, n, &ca, &cr);
  allocatable_requested(r, p, q, 1, n, &ma, &mr);
  double cpu = fraction_of_capacity(cr, ca), mem = fraction_of_capacity(mr, ma);
  if (cpu >= 1 || mem >= 1) return 0;
  double diff = fabs(cpu - mem);
  return (int64_t)((1 - diff) * (double)MAXN_SCORE);
}

static int64_t taint_raw(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, int n) {
  /* taint_toleration.go:123-136 countIntolerableTaintsPreferNoSchedule */
  int64_t c = 0;
  for (int w = 0; w < r->TW; ++w) {
    uint64_t tol = w < q->tol_prefer.count ? p->words[q->tol_prefer.begin + w] : 0;
    c += __builtin_popcountll(r->taint_prefer[(size_t)w * r->N + n] & ~tol);
  }
  return c;
}

static int64_t node_affinity_raw(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, int n) {
  /* node_affinity.go:80-99 */
  int64_t count = 0;
  for (int t = 0; t < q->pref_terms.count; ++t) {
    const kgpu_pref_term* pt = &p->pref_terms[q->pref_terms.begin + t];
    if (pt->weight == 0 || pt->sel.kind == KGPU_SEL_NOTHING) continue;
    if (selector_matches_node(r, p, pt->sel.reqs, n)) count += pt->weight;
  }
  return count;
}

static int64_t image_locality(const ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, int n) {
  /* image_locality.go:53-101 */
  const int64_t mb = 1024 * 1024, min_t = 23 * mb, max_c = 1000 * mb;
  int64_t sum = 0;
  for (int i = 0; i < q->images.count; ++i) {
    int id = p->ints[q->images.begin + i];
    if (id < 0) continue;
    for (int k = r->image_off[n]; k < r->image_off[n + 1]; ++k)
      if (r->image_id[k] == id) { sum += r->image_score[k]; break; }
  }
  int64_t max_t = max_c * (int64_t)q->n_containers;
  if (sum < min_t) sum = min_t;
  else if (sum > max_t) sum = max_t;
  return (int64_t)MAXN_SCORE * (sum - min_t) / (max_t - min_t);
}

static int64_t prefer_avoid(const ref_state* r, const kgpu_pod_query* q, int n) {
  if (q->avoid_id < 0) return MAXN_SCORE;
  for (int k = r->avoid_off[n]; k < r->avoid_off[n + 1]; ++k)
    if (r->avoid_id[k] == q->avoid_id) return 0;
  return MAXN_SCORE;
}

/* plugins/helper/normalize_score.go:26-54 */
static void default_normalize(int64_t* s, int n, int reverse) {
  int64_t mx = 0;
  for (int i = 0; i < n; ++i) if (s[i] > mx) mx = s[i];
  if (mx == 0) {
    if (reverse) for (int i = 0; i < n; ++i) s[i] = MAXN_SCORE;
    return;
  }
  for (int i = 0; i < n; ++i) {
    int64_t v = MAXN_SCORE * s[i] / mx;
    s[i] = reverse ? MAXN_SCORE - v : v;
  }
}

/* ------------------------------------------------------------------ tie-break (tiebreak.py) */
static uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static uint64_t tie_key(const kgpu_config* cfg, int64_t seq, int64_t score, uint64_t idx) {
  const uint64_t M = (1ull << 40) - 1;
  uint64_t rank;
  if (cfg->tie_break_mode == 1) {
    rank = M - idx;
  } else {
    uint64_t k = splitmix64(cfg->seed ^ ((uint64_t)seq * 0x9E3779B97F4A7C15ull));
    uint64_t x = idx & M;
    x ^= k & M;
    x = (x * 0xD6E8FEB865ull) & M;
    x ^= x >> 19;
    x = (x * 0x94D049BB13ull) & M;
    x ^= x >> 23;
    x ^= (k >> 24) & M;
    rank = x;
  }
  return ((uint64_t)score << 40) | rank;
}

/* ------------------------------------------------------------------ parallelize.Until */
typedef struct {
  const ref_state* r;
  const kgpu_pools* p;
  const kgpu_pod_query* q;
  int phase; /* 0 filter, 1 score */
  int n, chunk;
  _Alignas(64) _Atomic int next;
  _Alignas(64) _Atomic int done;  /* items processed (parallel_until's join), on a line of its own */
  _Alignas(64) char pad_;
  uint32_t* status;
  const int* feasible;
  int nf;
  int64_t* scores; /* [n_scores][nf] */
  qstate* qs;
} work_t;

static void process(work_t* w, int i) {
  const ref_state* r = w->r;
  if (w->phase == 0) {
    w->status[i] = run_filter_plugins(r, w->p, w->q, w->qs, i);
    return;
  }
  int n = w->feasible[i];
  for (int k = 0; k < r->cfg.n_scores; ++k) {
    int64_t v = 0;
    switch (r->cfg.scores[k]) {
      case KGPU_S_BALANCED_ALLOCATION: v = balanced_score(r, w->p, w->q, n); break;
      case KGPU_S_LEAST_ALLOCATED: v = resource_scorer(r, w->p, w->q, n, 0); break;
      case KGPU_S_MOST_ALLOCATED: v = resource_scorer(r, w->p, w->q, n, 1); break;
      case KGPU_S_IMAGE_LOCALITY: v = image_locality(r, w->p, w->q, n); break;
      case KGPU_S_NODE_PREFER_AVOID_PODS: v = prefer_avoid(r, w->q, n); break;
      case KGPU_S_TAINT_TOLERATION: v = taint_raw(r, w->p, w->q, n); break;
      case KGPU_S_NODE_AFFINITY: v = node_affinity_raw(r, w->p, w->q, n); break;
      case KGPU_S_POD_TOPOLOGY_SPREAD: v = pts_score(w->qs, r, w->q, n); break;
      case KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD: v = dpts_score(w->qs, r, w->q, n); break;
      case KGPU_S_INTER_POD_AFFINITY: v = ipa_score(w->qs, r, n); break;
      case KGPU_S_REQUESTED_TO_CAPACITY_RATIO: v = rtcr_score(r, w->p, w->q, n); break;
      case KGPU_S_RESOURCE_LIMITS: v = limits_score(r, w->q, n); break;
      default: v = 0; break;
    }
    w->scores[(size_t)k * w->nf + i] = v;
  }
}

/* A persistent pool of (threads - 1) workers plus the calling thread.  Go's ParallelizeUntil
 * starts 16 goroutines per call and hands out chunks through a channel; goroutine start and
 * channel receive cost well under a microsecond, so a faithful (and strong) baseline must not pay
 * an OS sleep/wake per parallel section.  Workers therefore spin on a sequence word (yielding
 * after a bounded spin) and take chunks with an atomic fetch-add.  A condition-variable pool
 * measured 2.7x SLOWER at 16 threads than 1 thread on 5k nodes (two futex wake-ups of 15 threads
 * per pod dominate a 70 us cycle).
 *
 * The join waits for the ITEMS, not for the workers: until round 4 the caller waited for every
 * worker to check in, so one worker the OS had descheduled (16 spinning threads on a 16-CPU share
 * beside the interpreter's and the runtime's threads) held the whole section for a scheduler quantum
 * even when it took no chunk -- the reason 16 workers were slower than one at 5k nodes
 * (KGPU_REF_PHASES: the filter section 63 us at 1 thread, 1.3 ms at 8).  Now:
 *   seq is odd while a job is open (2k+1) and even after it (2k+2);
 *   a worker that sees an open job registers in `active`, then re-checks seq: only if the job is
 *   still open does it touch the job, else it unregisters;
 *   the caller, once every item is done, closes the job (seq + 1) and waits for `active` to drain --
 *   only workers already inside run_chunks, each of which finds no chunk left. */
struct pool_s {
  _Atomic long seq;
  _Atomic int active, quit;
  work_t* _Atomic job;
  int nthreads;
  pthread_t tid[256];
};

static void run_chunks(work_t* w) {
  for (;;) {
    int start = atomic_fetch_add_explicit(&w->next, w->chunk, memory_order_relaxed);
    if (start >= w->n) return;
    int end = start + w->chunk < w->n ? start + w->chunk : w->n;
    for (int i = start; i < end; ++i) process(w, i);
    atomic_fetch_add_explicit(&w->done, end - start, memory_order_release);
  }
}

static void* pool_worker(void* arg) {
  pool_t* p = (pool_t*)arg;
  long seen = 0;
  for (;;) {
    int spins = 0;
    long s;
    while ((s = atomic_load_explicit(&p->seq, memory_order_acquire)) == seen || !(s & 1)) {
      if (atomic_load_explicit(&p->quit, memory_order_relaxed)) return NULL;
      if (++spins > 4096) { sched_yield(); spins = 0; }
    }
    seen = s;
    atomic_fetch_add_explicit(&p->active, 1, memory_order_seq_cst);
    if (atomic_load_explicit(&p->seq, memory_order_seq_cst) == s)
      run_chunks(atomic_load_explicit(&p->job, memory_order_acquire));
    atomic_fetch_sub_explicit(&p->active, 1, memory_order_release);
  }
}

static pool_t* pool_new(int threads) {
  pool_t* p = (pool_t*)calloc(1, sizeof(pool_t));
  p->nthreads = threads > 256 ? 256 : threads;
  for (int i = 0; i < p->nthreads - 1; ++i) pthread_create(&p->tid[i], NULL, pool_worker, p);
  return p;
}

static void pool_free(pool_t* p) {
  if (!p) return;
  atomic_store(&p->quit, 1);
  for (int i = 0; i < p->nthreads - 1; ++i) pthread_join(p->tid[i], NULL);
  free(p);
}

static void parallel_until(pool_t* pool, work_t* w, int n) {
  /* parallelism.go:26-43: 16 workers, chunk = min(floor(sqrt(n)), n/16 + 1) */
  int chunk = (int)sqrt((double)n);
  if (n / 16 + 1 < chunk) chunk = n / 16 + 1;
  if (chunk < 1) chunk = 1;
  w->n = n;
  w->chunk = chunk;
  atomic_store_explicit(&w->next, 0, memory_order_relaxed);
  atomic_store_explicit(&w->done, 0, memory_order_relaxed);
  if (!pool || pool->nthreads <= 1 || n < 2) {
    for (int i = 0; i < n; ++i) process(w, i);
    return;
  }
  atomic_store_explicit(&pool->job, w, memory_order_relaxed);
  const long open = atomic_load_explicit(&pool->seq, memory_order_relaxed) + 1;  /* odd: job open */
  atomic_store_explicit(&pool->seq, open, memory_order_seq_cst);
  run_chunks(w);
  while (atomic_load_explicit(&w->done, memory_order_acquire) < n) {
  }
  atomic_store_explicit(&pool->seq, open + 1, memory_order_seq_cst);  /* closed: late workers stay out */
  while (atomic_load_explicit(&pool->active, memory_order_acquire) > 0) {
  }
}

/* ------------------------------------------------------------------ assume (types.go:456-480) */
static void add_pod(ref_state* r, const kgpu_pools* p, const kgpu_pod_query* q, int n) {
  r->req_cpu[n] += q->req[0];
  r->req_mem[n] += q->req[1];
  r->req_eph[n] += q->req[2];
  for (int i = 0; i < q->scalars.count; ++i) {
    const kgpu_scalar_req* s = &p->scalars[q->scalars.begin + i];
    if (s->col >= 0) r->req_scalar[(size_t)s->col * r->N + n] += s->value;
  }
  r->nz_cpu[n] += q->nz[0];
  r->nz_mem[n] += q->nz[1];
  r->num_pods[n] += 1;
  for (int i = 0; i < q->ports.count; ++i) {
    const kgpu_port* w = &p->ports[q->ports.begin + i];
    int dup = 0;
    for (int s = 0; s < r->port_count[n]; ++s) {
      const kgpu_port* u = &r->ports[(size_t)s * r->N + n];
      if (u->ip == w->ip && u->proto == w->proto && u->port == w->port) dup = 1;
    }
    if (!dup && r->port_count[n] < r->PS) r->ports[(size_t)(r->port_count[n]++) * r->N + n] = *w;
  }
}

/* One scheduling cycle per query, in order; placements are assumed before the next pod.
 * status/raw/norm (optional, for the last pod only) receive the per-node diagnostics. */
int kgpu_ref_schedule(ref_state* r, const kgpu_pod_query* qs, int nq, const kgpu_pools* p, int64_t first_seq,
                      kgpu_result* out, uint32_t* status_out, int64_t* raw_out, int64_t* norm_out) {
  int N = r->N;
  if (!r->pool && r->threads > 1) r->pool = pool_new(r->threads);
  uint32_t* status = (uint32_t*)malloc(sizeof(uint32_t) * (N ? N : 1));
  int* feasible = (int*)malloc(sizeof(int) * (N ? N : 1));
  int64_t* scores = (int64_t*)malloc(sizeof(int64_t) * (size_t)(N ? N : 1) * (r->cfg.n_scores ? r->cfg.n_scores : 1));
  int64_t* totals = (int64_t*)malloc(sizeof(int64_t) * (N ? N : 1));
  /* KGPU_REF_PHASES=1: wall time per pod of each phase to stderr (where a parallel baseline's time goes) */
  const int phases = getenv("KGPU_REF_PHASES") != NULL;
  double ph[5] = {0, 0, 0, 0, 0};
  struct timespec t0, t1;
#define PHASE(k)                                                                                       \
  do {                                                                                                 \
    if (phases) {                                                                                      \
      clock_gettime(CLOCK_MONOTONIC, &t1);                                                             \
      ph[k] += (double)(t1.tv_sec - t0.tv_sec) * 1e6 + (double)(t1.tv_nsec - t0.tv_nsec) / 1e3;       \
      t0 = t1;                                                                                         \
    }                                                                                                  \
  } while (0)
  for (int qi = 0; qi < nq; ++qi) {
    if (phases) clock_gettime(CLOCK_MONOTONIC, &t0);
    const kgpu_pod_query* q = &qs[qi];
    work_t w;
    memset(&w, 0, sizeof(w));
    w.r = r; w.p = p; w.q = q; w.status = status;
    w.phase = 0;
    /* PreFilter (framework.go:369-389) */
    qstate qst;
    memset(&qst, 0, sizeof(qst));
    incoming_pod(&qst.self, q, p);
    qst.dsel = osel_from(&q->dpts, p);
    if (has_filter(r, KGPU_F_POD_TOPOLOGY_SPREAD)) pts_prefilter(&qst, r, p, q);
    if (has_filter(r, KGPU_F_INTER_POD_AFFINITY)) ipa_prefilter(&qst, r);
    w.qs = &qst;
    PHASE(0);
    parallel_until((pool_t*)r->pool, &w, N);
    PHASE(1);
    int nf = 0;
    int evaluated = r->total;
    if (r->to_find < N && r->total == N) {
      /* findNodesThatPassFilters (generic_scheduler.go:424-495) run by one worker: nodes are checked
       * from nextStartNodeIndex on; after to_find nodes fit, the next node that fits cancels the
       * search (it is in neither `filtered` nor the statuses).  Verdicts do not depend on the order
       * (PreFilter state is fixed for the cycle), so they were computed above for every node. */
      int p = N, seen = 0;
      if (r->cfg.n_filters == 0) { /* no filter plugins: the first to_find nodes, unrotated (:438-444) */
        for (int i = 0; i < N; ++i) {
          if (i < r->to_find) feasible[nf++] = i;
          else status[i] = 0xFFu;
        }
        p = r->to_find;
      } else {
        int start = r->next_start % N;
        for (int j = 0; j < N; ++j) {
          int i = (start + j) % N;
          if (p < N) { status[i] = 0xFFu; continue; }
          if (status[i] == 0) {
            if (seen++ < r->to_find) feasible[nf++] = i;
            else { p = j; status[i] = 0xFFu; }
          }
        }
        /* `filtered` stays in rotated order: normalize, PreScore and the packed-key selectHost are
         * order independent */
      }
      r->next_start = (r->next_start % N + p) % N;
      evaluated = p;
    } else {
      for (int i = 0; i < N; ++i) if (status[i] == 0) feasible[nf++] = i;
    }
    kgpu_result res;
    memset(&res, 0, sizeof(res));
    res.feasible = nf;
    res.evaluated = evaluated;
    res.node = -1;
    int last = (qi == nq - 1);
    if (last && status_out) memcpy(status_out, status, sizeof(uint32_t) * N);
    if (last && raw_out) memset(raw_out, 0, sizeof(int64_t) * KGPU_NUM_SCORES * N);
    if (last && norm_out) memset(norm_out, 0, sizeof(int64_t) * KGPU_NUM_SCORES * N);
    if (nf == 1) {
      res.node = r->base + feasible[0];
      add_pod(r, p, q, feasible[0]);
      add_pod_record(r, q, p, feasible[0]);
    } else if (nf > 1) {
      if (q->flags & KGPU_Q_SCORE_ERROR) {
        res.node = -2;
      } else {
        /* PreScore (framework.go:543-563) */
        if (has_score(r, KGPU_S_POD_TOPOLOGY_SPREAD)) pts_prescore(&qst, r, p, q, feasible, nf);
        if (has_score(r, KGPU_S_INTER_POD_AFFINITY)) ipa_prescore(&qst, r, r->cfg.hard_pod_affinity_weight);
        w.phase = 1;
        w.feasible = feasible;
        w.nf = nf;
        w.scores = scores;
        PHASE(2);
        parallel_until((pool_t*)r->pool, &w, nf);
        PHASE(3);
        for (int i = 0; i < nf; ++i) totals[i] = 0;
        for (int k = 0; k < r->cfg.n_scores; ++k) {
          int64_t* s = scores + (size_t)k * nf;
          int plugin = r->cfg.scores[k];
          if (last && raw_out) for (int i = 0; i < nf; ++i) raw_out[(size_t)plugin * N + feasible[i]] = s[i];
          if (plugin == KGPU_S_TAINT_TOLERATION) default_normalize(s, nf, 1);
          else if (plugin == KGPU_S_NODE_AFFINITY) default_normalize(s, nf, 0);
          else if (plugin == KGPU_S_POD_TOPOLOGY_SPREAD) pts_normalize(&qst, s, feasible, nf);
          else if (plugin == KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD) dpts_normalize(r, q, s, feasible, nf);
          else if (plugin == KGPU_S_INTER_POD_AFFINITY) ipa_normalize(&qst, s, nf);
          if (last && norm_out) for (int i = 0; i < nf; ++i) norm_out[(size_t)plugin * N + feasible[i]] = s[i];
          int64_t wgt = r->cfg.score_weights[k] > 0 ? r->cfg.score_weights[k] : 1;
          for (int i = 0; i < nf; ++i) totals[i] += s[i] * wgt;
        }
        if (r->cfg.n_scores == 0) for (int i = 0; i < nf; ++i) totals[i] = 1;
        /* selectHost (generic_scheduler.go:217-238): a max scan, then the tie-break key only over
         * the nodes that share the maximum (the reference draws random numbers only on ties) */
        int64_t top = totals[0];
        for (int i = 1; i < nf; ++i) if (totals[i] > top) top = totals[i];
        uint64_t best = 0;
        int bi = -1;
        for (int i = 0; i < nf; ++i) {
          if (totals[i] != top) continue;
          uint64_t k = tie_key(&r->cfg, first_seq + qi, totals[i], (uint64_t)(r->base + feasible[i]));
          if (bi < 0 || k > best) { best = k; bi = i; }
        }
        res.node = r->base + feasible[bi];
        res.scored = 1;
        res.score = totals[bi];
        add_pod(r, p, q, feasible[bi]);
        add_pod_record(r, q, p, feasible[bi]);
        PHASE(4);
      }
    }
    qstate_free(&qst, r);
    out[qi] = res;
  }
  free(status);
  free(feasible);
  free(scores);
  free(totals);
  if (phases && nq > 0)
    fprintf(stderr, "kgpu_ref %d thread(s), us/pod: prefilter %.1f, filter (parallel) %.1f, feasible list %.1f, "
            "score (parallel) %.1f, normalize+totals+selectHost+assume %.1f\n", r->threads, ph[0] / nq, ph[1] / nq,
            ph[2] / nq, ph[3] / nq, ph[4] / nq);
#undef PHASE
  return 0;
}

int kgpu_ref_read_nodes(const ref_state* r, int64_t* req_cpu, int64_t* req_mem, int64_t* req_eph, int64_t* nz_cpu,
                        int64_t* nz_mem, int32_t* num_pods) {
  size_t N = (size_t)r->N;
  if (req_cpu) memcpy(req_cpu, r->req_cpu, 8 * N);
  if (req_mem) memcpy(req_mem, r->req_mem, 8 * N);
  if (req_eph) memcpy(req_eph, r->req_eph, 8 * N);
  if (nz_cpu) memcpy(nz_cpu, r->nz_cpu, 8 * N);
  if (nz_mem) memcpy(nz_mem, r->nz_mem, 8 * N);
  if (num_pods) memcpy(num_pods, r->num_pods, 4 * N);
  return 0;
}

/* The broken-linear function alone over a config's shape points (requested_to_capacity_ratio_test.go:119
 * checks buildBrokenLinearFunction directly, with unscaled points). */
int kgpu_ref_broken_linear(const kgpu_config* cfg, const int64_t* p, int n, int64_t* out) {
  if (!cfg || cfg->n_shape <= 0) return -1;
  for (int i = 0; i < n; ++i) out[i] = broken_linear(cfg, p[i]);
  return 0;
}
