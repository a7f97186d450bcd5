// CDNA4 (gfx950) kernels for kube-scheduler's per-pod node evaluation.
//
// One thread per node over Snapshot.List()-ordered SoA rows (coalesced 8-byte loads), every
// filter and score plugin of the profile fused into one pass, workgroup argmax through wave64
// shuffles + LDS, and the previous pod's selectHost + assume folded into the head of the next
// pod's launch (each workgroup reduces the <= kMaxBlocks partials of the previous launch
// redundantly; only the workgroup that owns the winning node row writes it).  No dense
// contraction exists anywhere on this path: the bound is memory, not MFMA.
//
// Reference semantics (file:line in /root/reference):
//   filters  framework/v1alpha1/framework.go:477-502 (profile order, first failure wins)
//   Fit      noderesources/fit.go:194-267            NodeUnschedulable node_unschedulable.go:51-65
//   NodeName nodename/node_name.go:46-59              NodePorts nodeports/node_ports.go:100-129,
//                                                     framework/v1alpha1/types.go:726-756
//   NodeAffinity plugins/helper/node_affinity.go:28-78, core/v1/helper/helpers.go:237-346,
//            labels/selector.go:198-242; Score nodeaffinity/node_affinity.go:65-108
//   TaintToleration tainttoleration/taint_toleration.go:54-157
//   Least/Most/Balanced noderesources/{least,most,balanced}_allocated.go, resource_allocation.go
//   ImageLocality imagelocality/image_locality.go:53-125
//   NodePreferAvoidPods nodepreferavoidpods/node_prefer_avoid_pods.go:47-82
//   DefaultNormalizeScore plugins/helper/normalize_score.go:26-54
//   weights + sum framework.go:633-648, core/generic_scheduler.go:660-668
//   selectHost core/generic_scheduler.go:217-238 (deterministic tie-break)
//   assume   framework/v1alpha1/types.go:456-480 (NodeInfo.AddPod)
#include <hip/hip_runtime.h>

#include "kgpu_internal.h"

namespace kgpu {

// ---------------------------------------------------------------- tie-break
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t pod_tie_key(uint64_t seed, int64_t seq) {
  return splitmix64(seed ^ ((uint64_t)seq * 0x9E3779B97F4A7C15ull));
}
__device__ __forceinline__ uint64_t rank40(uint64_t k, uint64_t idx, int mode) {
  if (mode == 1) return kMask40 - idx;
  uint64_t x = idx & kMask40;
  x ^= k & kMask40;
  x = (x * 0xD6E8FEB865ull) & kMask40;
  x ^= x >> 19;
  x = (x * 0x94D049BB13ull) & kMask40;
  x ^= x >> 23;
  x ^= (k >> 24) & kMask40;
  return x;
}

// ---------------------------------------------------------------- selectors
__device__ __forceinline__ bool list_has(const int32_t* v, int n, int x) {
  for (int i = 0; i < n; ++i)
    if (v[i] == x) return true;
  return false;
}

// labels.Requirement.Matches on node labels (selector.go:198-242); v < 0 = key absent.
__device__ bool node_req(const DevState& st, const kgpu_req& r, int n) {
  const int v = r.key >= 0 ? st.label_val[(size_t)r.key * st.N + n] : -1;
  switch (r.op) {
    case KGPU_OP_IN:
      return v >= 0 && list_has(st.qp.ints + r.vals.begin, r.vals.count, v);
    case KGPU_OP_NOTIN:
      return v < 0 || !list_has(st.qp.ints + r.vals.begin, r.vals.count, v);
    case KGPU_OP_EXISTS:
      return v >= 0;
    case KGPU_OP_DNE:
      return v < 0;
    default: {
      if (v < 0) return false;
      const int idx = st.value_off[r.key] + v;
      if (!st.value_int_ok[idx]) return false;
      const int64_t lv = st.value_int[idx];
      return r.op == KGPU_OP_GT ? lv > r.imm : lv < r.imm;
    }
  }
}

__device__ bool node_reqs_all(const DevState& st, kgpu_range rr, int n) {
  for (int i = 0; i < rr.count; ++i)
    if (!node_req(st, st.qp.reqs[rr.begin + i], n)) return false;
  return true;
}

// PodMatchesNodeSelectorAndAffinityTerms (plugins/helper/node_affinity.go:28-78).
__device__ bool node_affinity_ok(const DevState& st, const kgpu_pod_query& q, int n) {
  if (!node_reqs_all(st, q.node_selector, n)) return false;
  if (!(q.flags & KGPU_Q_REQ_NODE_AFFINITY)) return true;
  const int g = st.node_base + n;
  for (int t = 0; t < q.req_terms.count; ++t) {
    const kgpu_node_term term = st.qp.node_terms[q.req_terms.begin + t];
    if (term.never_match) continue;
    if (!node_reqs_all(st, term.reqs, n)) continue;
    if (term.field_op == KGPU_OP_IN && g != term.field_node) continue;
    if (term.field_op == KGPU_OP_NOTIN && g == term.field_node) continue;
    return true;
  }
  return false;
}

// ---------------------------------------------------------------- node resource row
// The 72 bytes of NodeInfo.{Allocatable,Requested,NonZeroRequested,len(Pods)} every resource
// plugin reads, loaded once per node into registers (8-byte coalesced loads per column).
struct NodeRes {
  int64_t ac, am, ae;   // Allocatable milliCPU / memory / ephemeral-storage
  int64_t rc, rm, re;   // Requested
  int64_t zc, zm;       // NonZeroRequested
  int32_t ap, np;       // AllowedPodNumber, len(Pods)
};

__device__ __forceinline__ NodeRes load_res(const DevState& st, int n) {
  NodeRes r;
  r.ac = st.alloc_cpu[n]; r.am = st.alloc_mem[n]; r.ae = st.alloc_eph[n];
  r.rc = st.req_cpu[n]; r.rm = st.req_mem[n]; r.re = st.req_eph[n];
  r.zc = st.nz_cpu[n]; r.zm = st.nz_mem[n];
  r.ap = st.alloc_pods[n]; r.np = st.num_pods[n];
  return r;
}

// ---------------------------------------------------------------- plugins
__device__ __forceinline__ uint32_t fit_detail(const DevState& st, const kgpu_pod_query& q, const NodeRes& r, int n) {
  uint32_t d = 0;
  if (r.np + 1 > r.ap) d |= 1u;
  if (q.flags & KGPU_Q_FIT_ALL_ZERO) return d;
  if (r.ac < q.req[0] + r.rc) d |= 2u;
  if (r.am < q.req[1] + r.rm) d |= 4u;
  if (r.ae < q.req[2] + r.re) d |= 8u;
  for (int i = 0; i < q.scalars.count; ++i) {
    const kgpu_scalar_req s = st.qp.scalars[q.scalars.begin + i];
    if (!s.check) continue;
    const int64_t alloc = s.col >= 0 ? st.alloc_scalar[(size_t)s.col * st.N + n] : 0;
    const int64_t used = s.col >= 0 ? st.req_scalar[(size_t)s.col * st.N + n] : 0;
    if (alloc < s.value + used) d |= 16u << (i < 11 ? i : 11);
  }
  return d;
}

__device__ __forceinline__ bool ports_conflict(const DevState& st, const kgpu_pod_query& q, int n) {
  const int have = st.port_count[n];
  for (int i = 0; i < q.ports.count; ++i) {
    const kgpu_port w = st.qp.ports[q.ports.begin + i];
    for (int s = 0; s < have; ++s) {
      const kgpu_port p = st.ports[(size_t)s * st.N + n];
      if (p.port == w.port && p.proto == w.proto && (w.ip == 0 || p.ip == 0 || p.ip == w.ip)) return true;
    }
  }
  return false;
}

__device__ __forceinline__ bool taints_ok(const DevState& st, const kgpu_pod_query& q, int n) {
  for (int w = 0; w < st.TW; ++w) {
    const uint64_t t = st.taint_nosched[(size_t)w * st.N + n];
    const uint64_t tol = w < q.tol_nosched.count ? st.qp.words[q.tol_nosched.begin + w] : 0ull;
    if (t & ~tol) return false;
  }
  return true;
}

__device__ __forceinline__ int taint_raw(const DevState& st, const kgpu_pod_query& q, int n) {
  int c = 0;
  for (int w = 0; w < st.TW; ++w) {
    const uint64_t t = st.taint_prefer[(size_t)w * st.N + n];
    const uint64_t tol = w < q.tol_prefer.count ? st.qp.words[q.tol_prefer.begin + w] : 0ull;
    c += __popcll(t & ~tol);
  }
  return c;
}

__device__ __forceinline__ int na_raw(const DevState& st, const kgpu_pod_query& q, int n) {
  int s = 0;
  for (int t = 0; t < q.pref_terms.count; ++t) {
    const kgpu_pref_term pt = st.qp.pref_terms[q.pref_terms.begin + t];
    if (pt.sel.kind == KGPU_SEL_NOTHING) continue;
    if (node_reqs_all(st, pt.sel.reqs, n)) s += pt.weight;
  }
  return s;
}

__device__ __forceinline__ int64_t pod_scalar_score(const DevState& st, const kgpu_pod_query& q, int col) {
  for (int i = 0; i < q.scalars.count; ++i) {
    const kgpu_scalar_req s = st.qp.scalars[q.scalars.begin + i];
    if (s.col == col) return s.score_value;
  }
  return 0;
}

// Exact int64 floor division for 0 <= a, 0 < b: one IEEE double division (correctly rounded,
// error < 1/4 for operands < 2^52) plus a one-step remainder correction; the 64-bit integer
// division sequence is the fallback for larger operands.
__device__ __forceinline__ int64_t div_nonneg(int64_t a, int64_t b) {
  if (a < (1ll << 52) && b < (1ll << 52)) {
    int64_t q = (int64_t)((double)a / (double)b);
    const int64_t r = a - q * b;
    if (r < 0) q -= 1;
    else if (r >= b) q += 1;
    return q;
  }
  return a / b;
}

// calculateResourceAllocatableRequest (resource_allocation.go:92-113).
__device__ __forceinline__ void alloc_req(const DevState& st, const kgpu_pod_query& q, const NodeRes& nr, int res,
                                          int n, int64_t& cap, int64_t& req) {
  switch (res) {
    case 0: cap = nr.ac; req = nr.zc + q.score_req[0]; break;
    case 1: cap = nr.am; req = nr.zm + q.score_req[1]; break;
    case 2: cap = nr.ae; req = nr.re + q.score_req[2]; break;
    default:
      if (res >= 3) {
        const int col = res - 3;
        cap = st.alloc_scalar[(size_t)col * st.N + n];
        req = st.req_scalar[(size_t)col * st.N + n] + pod_scalar_score(st, q, col);
      } else {
        cap = 0;
        req = 0;
      }
  }
}

__device__ __forceinline__ int64_t least_score(const DevState& st, const kgpu_pod_query& q, const NodeRes& nr,
                                               int n) {
  int64_t s = 0;
  for (int i = 0; i < st.n_least; ++i) {
    int64_t cap, req;
    alloc_req(st, q, nr, st.least[i].resource, n, cap, req);
    const int64_t r = (cap == 0 || req > cap) ? 0 : (cap > 0 ? div_nonneg((cap - req) * 100, cap) : ((cap - req) * 100) / cap);
    s += r * st.least[i].weight;
  }
  return s >= 0 ? div_nonneg(s, st.least_wsum) : s / st.least_wsum;
}

__device__ __forceinline__ int64_t most_score(const DevState& st, const kgpu_pod_query& q, const NodeRes& nr,
                                              int n) {
  int64_t s = 0;
  for (int i = 0; i < st.n_most; ++i) {
    int64_t cap, req;
    alloc_req(st, q, nr, st.most[i].resource, n, cap, req);
    const int64_t r = (cap == 0 || req > cap) ? 0 : (req >= 0 && cap > 0 ? div_nonneg(req * 100, cap) : (req * 100) / cap);
    s += r * st.most[i].weight;
  }
  return s >= 0 ? div_nonneg(s, st.most_wsum) : s / st.most_wsum;
}

// balancedResourceScorer (balanced_allocation.go:83-120): IEEE double, no contraction.
__device__ __forceinline__ int64_t balanced_score(const kgpu_pod_query& q, const NodeRes& nr) {
  const int64_t cc = nr.ac, cr = nr.zc + q.score_req[0];
  const int64_t mc = nr.am, mr = nr.zm + q.score_req[1];
  const double cf = cc == 0 ? 1.0 : (double)cr / (double)cc;
  const double mf = mc == 0 ? 1.0 : (double)mr / (double)mc;
  if (cf >= 1.0 || mf >= 1.0) return 0;
  const double diff = fabs(cf - mf);
  return (int64_t)((1.0 - diff) * 100.0);
}

__device__ __forceinline__ int64_t image_score(const DevState& st, const kgpu_pod_query& q, int n) {
  constexpr int64_t MB = 1024 * 1024, kMin = 23 * MB, kMaxC = 1000 * MB;
  int64_t sum = 0;
  const int lo0 = st.image_off[n], hi0 = st.image_off[n + 1];
  for (int i = 0; i < q.images.count; ++i) {
    const int id = st.qp.ints[q.images.begin + i];
    if (id < 0) continue;
    int lo = lo0, hi = hi0;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (st.image_id[mid] < id) lo = mid + 1; else hi = mid;
    }
    if (lo < hi0 && st.image_id[lo] == id) sum += st.image_score[lo];
  }
  const int64_t maxT = kMaxC * (int64_t)q.n_containers;
  if (sum < kMin) sum = kMin;
  else if (sum > maxT) sum = maxT;
  return (100 * (sum - kMin)) / (maxT - kMin);
}

__device__ __forceinline__ int64_t npap_score(const DevState& st, const kgpu_pod_query& q, int n) {
  if (q.avoid_id < 0) return 100;
  for (int i = st.avoid_off[n]; i < st.avoid_off[n + 1]; ++i)
    if (st.avoid_id[i] == q.avoid_id) return 0;
  return 100;
}

// DefaultPodTopologySpread with an empty selector (every count is 0): 100 off-zone; zoned
// nodes get fScore*(1-zoneWeighting) + zoneWeighting*100 (default_pod_topology_spread.go:136-162).
__device__ __forceinline__ int64_t dpts_empty_score(const DevState& st, int n) {
  if (st.zone_id[n] < 0) return 100;
  const double zw = 2.0 / 3.0;
  const double f = (100.0 * (1.0 - zw)) + (zw * 100.0);
  return (int64_t)f;
}

// ---------------------------------------------------------------- one node
struct NodeEval {
  uint32_t status;  // filter status word, 0 = feasible
  int64_t partial;  // weighted sum of scores that need no normalize pass
  int32_t taint;    // raw TaintToleration score
  int32_t na;       // raw NodeAffinity score
};

__device__ __forceinline__ uint32_t run_filters(const DevState& st, const kgpu_pod_query& q, const NodeRes& r,
                                                int n) {
  for (int i = 0; i < st.n_filters; ++i) {
    const int f = st.filters[i];
    const uint32_t pos = (uint32_t)(i + 1);
    switch (f) {
      case KGPU_F_NODE_UNSCHEDULABLE:
        if (st.unsched[n] && !(q.flags & KGPU_Q_TOLERATES_UNSCHEDULABLE))
          return pos | (KGPU_CODE_UNRESOLVABLE << 8);
        break;
      case KGPU_F_NODE_RESOURCES_FIT: {
        const uint32_t d = fit_detail(st, q, r, n);
        if (d) return pos | (KGPU_CODE_UNSCHEDULABLE << 8) | (d << 16);
        break;
      }
      case KGPU_F_NODE_NAME:
        if (q.node_name != -1 && q.node_name != st.node_base + n) return pos | (KGPU_CODE_UNRESOLVABLE << 8);
        break;
      case KGPU_F_NODE_PORTS:
        if (q.ports.count && ports_conflict(st, q, n)) return pos | (KGPU_CODE_UNSCHEDULABLE << 8);
        break;
      case KGPU_F_NODE_AFFINITY:
        if (!node_affinity_ok(st, q, n)) return pos | (KGPU_CODE_UNRESOLVABLE << 8);
        break;
      case KGPU_F_TAINT_TOLERATION:
        if (!taints_ok(st, q, n)) return pos | (KGPU_CODE_UNRESOLVABLE << 8);
        break;
      default:  // PodTopologySpread / InterPodAffinity: pass for pods without constraints
        break;
    }
  }
  return 0;
}

__device__ __forceinline__ void run_scores(const DevState& st, const kgpu_pod_query& q, const NodeRes& r, int n,
                                           NodeEval& e, bool diag) {
  int64_t part = 0;
  for (int i = 0; i < st.n_scores; ++i) {
    const int s = st.scores[i];
    int64_t v = 0;
    switch (s) {
      case KGPU_S_BALANCED_ALLOCATION: v = balanced_score(q, r); break;
      case KGPU_S_LEAST_ALLOCATED: v = least_score(st, q, r, n); break;
      case KGPU_S_MOST_ALLOCATED: v = most_score(st, q, r, n); break;
      case KGPU_S_IMAGE_LOCALITY: v = image_score(st, q, n); break;
      case KGPU_S_NODE_PREFER_AVOID_PODS: v = npap_score(st, q, n); break;
      case KGPU_S_POD_TOPOLOGY_SPREAD: v = 100; break;           // no soft constraints: max == 0
      case KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD:
        v = (q.flags & KGPU_Q_HAS_TSC) ? 0 : dpts_empty_score(st, n);
        break;
      case KGPU_S_INTER_POD_AFFINITY: v = 0; break;              // empty topologyScore
      case KGPU_S_TAINT_TOLERATION:
        e.taint = taint_raw(st, q, n);
        if (diag) st.diag_raw[(size_t)s * st.N + n] = e.taint;
        continue;
      case KGPU_S_NODE_AFFINITY:
        e.na = na_raw(st, q, n);
        if (diag) st.diag_raw[(size_t)s * st.N + n] = e.na;
        continue;
      default: break;
    }
    if (diag) st.diag_raw[(size_t)s * st.N + n] = v;
    part += v * st.weights[i];
  }
  e.partial = part;
}

__device__ __forceinline__ int64_t norm_total(const DevState& st, int64_t partial, int taint, int na, int maxT,
                                              int maxNA) {
  int64_t t = partial;
  for (int i = 0; i < st.n_scores; ++i) {
    if (st.scores[i] == KGPU_S_TAINT_TOLERATION) {
      const int64_t v = maxT == 0 ? 100 : 100 - (100 * (int64_t)taint) / maxT;
      t += v * st.weights[i];
    } else if (st.scores[i] == KGPU_S_NODE_AFFINITY) {
      const int64_t v = maxNA == 0 ? (int64_t)na : (100 * (int64_t)na) / maxNA;
      t += v * st.weights[i];
    }
  }
  return t;
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ void key_max(uint64_t& k, int& i, uint64_t k2, int i2) {
  if (k2 > k) { k = k2; i = i2; }
}

__device__ __forceinline__ void wave_reduce_key(uint64_t& k, int& i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t k2 = __shfl_xor(k, off);
    const int i2 = __shfl_xor(i, off);
    key_max(k, i, k2, i2);
  }
}

__device__ __forceinline__ int wave_reduce_sum(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

__device__ __forceinline__ int wave_reduce_max(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off));
  return v;
}

struct Winner {
  uint64_t key;
  int idx;
  int feasible;
};

// selectHost over the partials of a finished launch, computed by every wave on its own (lanes
// stride over the <= kMaxBlocks partials, then a 64-lane shuffle reduction): no LDS, no barrier.
__device__ __forceinline__ Winner wave_winner(const BlkKey* kb, int nb) {
  uint64_t k = 0;
  int idx = -1, f = 0;
  for (int b = threadIdx.x & 63; b < nb; b += 64) {
    const BlkKey p = kb[b];
    key_max(k, idx, p.key, p.idx);
    f += p.feasible;
  }
  wave_reduce_key(k, idx);
  f = wave_reduce_sum(f);
  return Winner{k, idx, f};
}

// NodeInfo.AddPod on the chosen row (types.go:456-480): applied by the thread that owns the row,
// on its register copy (written back) plus the rarely used scalar and host-port columns.
__device__ void assume_row(const DevState& st, const kgpu_pod_query& q, NodeRes& r, int n) {
  r.rc += q.req[0];
  r.rm += q.req[1];
  r.re += q.req[2];
  r.zc += q.nz[0];
  r.zm += q.nz[1];
  r.np += 1;
  st.req_cpu[n] = r.rc;
  st.req_mem[n] = r.rm;
  st.req_eph[n] = r.re;
  st.nz_cpu[n] = r.zc;
  st.nz_mem[n] = r.zm;
  st.num_pods[n] = r.np;
  for (int i = 0; i < q.scalars.count; ++i) {
    const kgpu_scalar_req s = st.qp.scalars[q.scalars.begin + i];
    if (s.col >= 0) st.req_scalar[(size_t)s.col * st.N + n] += s.value;
  }
  if (q.ports.count) {
    int pc = st.port_count[n];
    for (int i = 0; i < q.ports.count && pc < st.PS; ++i) {
      const kgpu_port w = st.qp.ports[q.ports.begin + i];
      bool dup = false;
      for (int s = 0; s < pc; ++s) {
        const kgpu_port p = st.ports[(size_t)s * st.N + n];
        if (p.ip == w.ip && p.proto == w.proto && p.port == w.port) dup = true;
      }
      if (!dup) st.ports[(size_t)(pc++) * st.N + n] = w;
    }
    st.port_count[n] = pc;
  }
}

// The pending pod's outcome (generic_scheduler.go:171-208): FitError, the len==1 shortcut, or
// the scored winner.  placed_idx = local row to assume (-1 none).
__device__ __forceinline__ int settle_prev(const DevState& st, const PodArgs& a, const Winner& w) {
  const kgpu_pod_query& q = st.queries[a.prev];
  const bool error = (q.flags & KGPU_Q_SCORE_ERROR) && w.feasible >= 2;
  const bool placed = w.feasible > 0 && !error;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    kgpu_result r;
    r.node = placed ? st.node_base + w.idx : (error ? -2 : -1);
    r.feasible = w.feasible;
    r.evaluated = st.n_total;
    r.scored = (placed && w.feasible >= 2) ? 1 : 0;
    r.score = r.scored ? (int64_t)(w.key >> 40) : 0;
    st.results[a.prev] = r;
  }
  return (placed && a.assume) ? w.idx : -1;
}

__device__ __forceinline__ void chunk_of(int N, int& lo, int& hi) {
  const int per = (N + gridDim.x - 1) / gridDim.x;
  lo = blockIdx.x * per;
  hi = min(N, lo + per);
}

// ---------------------------------------------------------------- kernels
// One workgroup = one wave64: the workgroup argmax is a pure shuffle reduction (no LDS, no
// barrier), and every wave resolves the previous pod's winner on its own.
__global__ __launch_bounds__(kBlock) void k_eval(const DevState* __restrict__ stp, PodArgs a) {
  const DevState& st = *stp;
  int lo, hi;
  chunk_of(st.N, lo, hi);
  const int n0 = lo + threadIdx.x;
  // Independent loads first -- this lane's first node row, the pod query and the pending pod's
  // partials -- so that their latencies overlap instead of chaining.
  NodeRes r0{};
  if (n0 < hi) r0 = load_res(st, n0);
  const kgpu_pod_query q = st.queries[a.pod];
  int assume_idx = -1;
  if (a.prev >= 0) {
    const Winner w = wave_winner(st.kbuf + (size_t)a.prev_parity * kMaxBlocks, a.prev_blocks);
    assume_idx = settle_prev(st, a, w);
  }
  const uint64_t tk = pod_tie_key(st.seed, a.seq);
  const bool write_nodes = a.norm || a.diag;

  uint64_t best = 0;
  int best_i = -1, feas = 0, maxT = 0, maxNA = 0;
  for (int n = n0; n < hi; n += kBlock) {
    NodeRes r = (n == n0) ? r0 : load_res(st, n);
    if (n == assume_idx) assume_row(st, st.queries[a.prev], r, n);
    NodeEval e{0, 0, 0, 0};
    e.status = run_filters(st, q, r, n);
    if (e.status == 0) {
      run_scores(st, q, r, n, e, a.diag);
      ++feas;
      maxT = max(maxT, e.taint);
      maxNA = max(maxNA, e.na);
      if (!a.norm) {
        // constant DefaultNormalizeScore maxima: every raw TaintToleration / NodeAffinity score is 0
        const int64_t total = st.n_scores ? norm_total(st, e.partial, e.taint, e.na, 0, 0) : 1;
        const uint64_t key = ((uint64_t)total << 40) | rank40(tk, (uint64_t)(st.node_base + n), st.tie_mode);
        key_max(best, best_i, key, n);
      }
    }
    if (write_nodes) {
      st.status[n] = e.status;
      st.partial[n] = e.partial;
      st.raw_taint[n] = e.taint;
      st.raw_na[n] = e.na;
    }
  }
  wave_reduce_key(best, best_i);
  feas = wave_reduce_sum(feas);
  maxT = wave_reduce_max(maxT);
  maxNA = wave_reduce_max(maxNA);
  if (threadIdx.x == 0) {
    st.sbuf[(size_t)a.parity * kMaxBlocks + blockIdx.x] = BlkStat{feas, maxT, maxNA, 0};
    if (!a.norm) st.kbuf[(size_t)a.parity * kMaxBlocks + blockIdx.x] = BlkKey{best, best_i, feas};
  }
}

// Normalize pass: DefaultNormalizeScore maxima over the feasible set are known only after the
// evaluation launch; combine them with the stored raw values and take the argmax.
__global__ __launch_bounds__(kBlock) void k_final(const DevState* __restrict__ stp, PodArgs a, int stat_blocks) {
  const DevState& st = *stp;
  int maxT = 0, maxNA = 0;
  const BlkStat* sb = st.sbuf + (size_t)a.parity * kMaxBlocks;
  for (int b = threadIdx.x; b < stat_blocks; b += kBlock) {
    const BlkStat p = sb[b];
    maxT = max(maxT, p.max_taint);
    maxNA = max(maxNA, p.max_na);
  }
  maxT = wave_reduce_max(maxT);
  maxNA = wave_reduce_max(maxNA);
  int lo, hi;
  chunk_of(st.N, lo, hi);
  const uint64_t tk = pod_tie_key(st.seed, a.seq);
  uint64_t best = 0;
  int best_i = -1, bf = 0;
  for (int n = lo + threadIdx.x; n < hi; n += kBlock) {
    if (st.status[n] != 0) continue;
    ++bf;
    const int64_t total = st.n_scores ? norm_total(st, st.partial[n], st.raw_taint[n], st.raw_na[n], maxT, maxNA) : 1;
    const uint64_t key = ((uint64_t)total << 40) | rank40(tk, (uint64_t)(st.node_base + n), st.tie_mode);
    key_max(best, best_i, key, n);
    if (a.diag) {
      for (int i = 0; i < st.n_scores; ++i) {
        const int s = st.scores[i];
        int64_t v = st.diag_raw[(size_t)s * st.N + n];
        if (s == KGPU_S_TAINT_TOLERATION) v = maxT == 0 ? 100 : 100 - (100 * v) / maxT;
        if (s == KGPU_S_NODE_AFFINITY) v = maxNA == 0 ? v : (100 * v) / maxNA;
        st.diag_norm[(size_t)s * st.N + n] = v;
      }
    }
  }
  wave_reduce_key(best, best_i);
  bf = wave_reduce_sum(bf);
  if (threadIdx.x == 0) st.kbuf[(size_t)a.parity * kMaxBlocks + blockIdx.x] = BlkKey{best, best_i, bf};
}

// Resolve-only launch (end of a batch / single cycle), with the evaluation grid's chunk mapping
// so that the lane owning the winning row applies the assume.
__global__ __launch_bounds__(kBlock) void k_resolve(const DevState* __restrict__ stp, PodArgs a) {
  const DevState& st = *stp;
  int lo, hi;
  chunk_of(st.N, lo, hi);
  const Winner w = wave_winner(st.kbuf + (size_t)a.prev_parity * kMaxBlocks, a.prev_blocks);
  const int idx = settle_prev(st, a, w);
  if (idx >= lo && idx < hi && ((idx - lo) % kBlock) == (int)threadIdx.x) {
    NodeRes r = load_res(st, idx);
    assume_row(st, st.queries[a.prev], r, idx);
  }
}

int eval_blocks(int N) {
  int b = (N + kBlock - 1) / kBlock;
  if (b > kMaxBlocks) b = kMaxBlocks;
  if (b < 1) b = 1;
  return b;
}

int launch_eval(const DevState* st, const PodArgs& a, int blocks, void* stream) {
  hipLaunchKernelGGL(k_eval, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_final(const DevState* st, const PodArgs& a, int blocks, int stat_blocks, void* stream) {
  hipLaunchKernelGGL(k_final, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, st, a, stat_blocks);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_resolve(const DevState* st, int N, const PodArgs& a, void* stream) {
  // same grid as the evaluation so that chunk ownership matches
  hipLaunchKernelGGL(k_resolve, dim3(eval_blocks(N)), dim3(kBlock), 0, (hipStream_t)stream, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace kgpu
