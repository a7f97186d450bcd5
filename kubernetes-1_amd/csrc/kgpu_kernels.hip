// CDNA4 (gfx950) kernels for kube-scheduler's per-pod node evaluation.
//
// One thread per node over Snapshot.List()-ordered SoA rows (coalesced 8-byte loads), every
// filter and score plugin of the profile fused into one pass, workgroup argmax through wave64
// shuffles, and the previous pod's selectHost + assume folded into the head of the next pod's
// launch (each wave reduces the <= kMaxBlocks partials of the previous launch redundantly; only
// the lane that owns the winning node row writes it).  No dense contraction exists anywhere on
// this path: the bound is memory latency/bandwidth, not MFMA.
//
// The evaluation kernel is a template over the profile: FM = enabled filters (profile order =
// ascending plugin id, the default order), SM = enabled score plugins.  Common profiles get a
// straight-line instantiation (no per-node plugin dispatch, no dependent loads of the plugin
// list); any other profile runs the kRuntime instantiation that walks the lists from DevState.
// Uniform data (DevState, queries, pools) is read through the constant address space (scalar
// loads); node columns through the global address space (no flat instructions).
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

#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>

#include "kgpu_internal.h"

// Address spaces exist only in the device pass; the host pass parses the same code unqualified.
#if defined(__HIP_DEVICE_COMPILE__)
#define GAS __attribute__((address_space(1)))
#define CAS __attribute__((address_space(4)))
#else
#define GAS
#define CAS
#endif

namespace kgpu {

template <class T>
__device__ __forceinline__ GAS T* gp(T* p) {
  return (GAS T*)p;
}
template <class T>
__device__ __forceinline__ const CAS T* cp(const T* p) {
  return (const CAS T*)p;
}


constexpr uint32_t kRuntime = 0xFFFFFFFFu;  // FM/SM of the list-walking instantiation
constexpr uint32_t kDefRes = 1u << 31;      // SM flag: Least/Most over {cpu: 1, memory: 1}
constexpr uint32_t kSMask = (1u << KGPU_NUM_SCORES) - 1;

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

__device__ __forceinline__ uint64_t rank40_inv(uint64_t k, uint64_t x, int mode) {
  // inverse of rank40 (every step is a bijection on 40 bits)
  if (mode == 1) return kMask40 - x;
  x ^= (k >> 24) & kMask40;
  x ^= x >> 23;                                      // 2 * 23 > 40
  x = (x * 0x38E12D471Bull) & kMask40;               // 0x94D049BB13^-1 mod 2^40
  x ^= (x >> 19) ^ (x >> 38);
  x = (x * 0xB38E39396Dull) & kMask40;               // 0xD6E8FEB865^-1 mod 2^40
  x ^= k & kMask40;
  return x;
}

// ---------------------------------------------------------------- selectors
__device__ __forceinline__ bool list_has(const int32_t* v, int n, int x) {
  for (int i = 0; i < n; ++i)
    if (cp(v)[i] == x) return true;
  return false;
}

// labels.Requirement.Matches on node labels (selector.go:198-242); v < 0 = key absent.
__device__ bool node_req(const DevState& st, const kgpu_req& r, int n) {
  const int v = r.key >= 0 ? gp(st.label_val)[(size_t)r.key * st.N + n] : -1;
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
      const int idx = gp(st.value_off)[r.key] + v;
      if (!gp(st.value_int_ok)[idx]) return false;
      const int64_t lv = gp(st.value_int)[idx];
      return r.op == KGPU_OP_GT ? lv > r.imm : lv < r.imm;
    }
  }
}

__device__ bool node_reqs_all(const DevState& st, kgpu_range rr, int n) {
  for (int i = 0; i < rr.count; ++i)
    if (!node_req(st, cp(st.qp.reqs)[rr.begin + i], n)) return false;
  return true;
}

// PodMatchesNodeSelectorAndAffinityTerms (plugins/helper/node_affinity.go:28-78).
__device__ bool node_affinity_ok(const DevState& st, const kgpu_pod_query& q, int n) {
  if (!node_reqs_all(st, q.node_selector, n)) return false;
  if (!(q.flags & KGPU_Q_REQ_NODE_AFFINITY)) return true;
  const int g = st.node_base + n;
  for (int t = 0; t < q.req_terms.count; ++t) {
    const kgpu_node_term term = cp(st.qp.node_terms)[q.req_terms.begin + t];
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
  double ic, im;        // 1/ac, 1/am where > 0 (persistent rows: Allocatable never changes), else 0
};

__device__ __forceinline__ NodeRes load_res(const DevState& st, int n) {
  NodeRes r;
  r.ac = gp(st.alloc_cpu)[n]; r.am = gp(st.alloc_mem)[n]; r.ae = gp(st.alloc_eph)[n];
  r.rc = gp(st.req_cpu)[n]; r.rm = gp(st.req_mem)[n]; r.re = gp(st.req_eph)[n];
  r.zc = gp(st.nz_cpu)[n]; r.zm = gp(st.nz_mem)[n];
  r.ap = gp(st.alloc_pods)[n]; r.np = gp(st.num_pods)[n];
  r.ic = 0.0;
  r.im = 0.0;
  return r;
}

// Reciprocals for register-resident rows, computed once per launch.
__device__ __forceinline__ void set_recips(NodeRes& r) {
  r.ic = (r.ac > 0 && r.ac < (1ll << 52)) ? 1.0 / (double)r.ac : 0.0;
  r.im = (r.am > 0 && r.am < (1ll << 52)) ? 1.0 / (double)r.am : 0.0;
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
    const kgpu_scalar_req s = cp(st.qp.scalars)[q.scalars.begin + i];
    if (!s.check) continue;
    const int64_t alloc = s.col >= 0 ? gp(st.alloc_scalar)[(size_t)s.col * st.N + n] : 0;
    const int64_t used = s.col >= 0 ? gp(st.req_scalar)[(size_t)s.col * st.N + n] : 0;
    if (alloc < s.value + used) d |= 16u << (i < 11 ? i : 11);
  }
  return d;
}

__device__ __forceinline__ bool ports_conflict(const DevState& st, const kgpu_pod_query& q, int n) {
  const int have = gp(st.port_count)[n];
  for (int i = 0; i < q.ports.count; ++i) {
    const kgpu_port w = cp(st.qp.ports)[q.ports.begin + i];
    for (int s = 0; s < have; ++s) {
      const kgpu_port p = gp(st.ports)[(size_t)s * st.N + n];
      if (p.port == w.port && p.proto == w.proto && (w.ip == 0 || p.ip == 0 || p.ip == w.ip)) return true;
    }
  }
  return false;
}

__device__ __forceinline__ bool taints_ok(const DevState& st, const kgpu_pod_query& q, int n) {
  for (int w = 0; w < st.TW; ++w) {
    const uint64_t t = gp(st.taint_nosched)[(size_t)w * st.N + n];
    const uint64_t tol = w < q.tol_nosched.count ? cp(st.qp.words)[q.tol_nosched.begin + w] : 0ull;
    if (t & ~tol) return false;
  }
  return true;
}

__device__ __forceinline__ int taint_raw(const DevState& st, const kgpu_pod_query& q, int n) {
  if (!st.any_prefer_taint) return 0;
  int c = 0;
  for (int w = 0; w < st.TW; ++w) {
    const uint64_t t = gp(st.taint_prefer)[(size_t)w * st.N + n];
    const uint64_t tol = w < q.tol_prefer.count ? cp(st.qp.words)[q.tol_prefer.begin + w] : 0ull;
    c += __popcll(t & ~tol);
  }
  return c;
}

__device__ __forceinline__ int na_raw(const DevState& st, const kgpu_pod_query& q, int n) {
  int s = 0;
  for (int t = 0; t < q.pref_terms.count; ++t) {
    const kgpu_pref_term pt = cp(st.qp.pref_terms)[q.pref_terms.begin + t];
    if (pt.sel.kind == KGPU_SEL_NOTHING) continue;
    if (node_reqs_all(st, pt.sel.reqs, n)) s += pt.weight;
  }
  return s;
}

__device__ __forceinline__ int64_t pod_scalar_score(const DevState& st, const kgpu_pod_query& q, int col) {
  for (int i = 0; i < q.scalars.count; ++i) {
    const kgpu_scalar_req s = cp(st.qp.scalars)[q.scalars.begin + i];
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
        cap = gp(st.alloc_scalar)[(size_t)col * st.N + n];
        req = gp(st.req_scalar)[(size_t)col * st.N + n] + pod_scalar_score(st, q, col);
      } else {
        cap = 0;
        req = 0;
      }
  }
}

// leastResourceScorer / mostResourceScorer per resource (least_allocated.go:93-101,
// most_allocated.go:93-107), Go's truncating int64 arithmetic.
__device__ __forceinline__ int64_t least_one(int64_t cap, int64_t req) {
  if (cap == 0 || req > cap) return 0;
  return cap > 0 ? div_nonneg((cap - req) * 100, cap) : ((cap - req) * 100) / cap;
}
__device__ __forceinline__ int64_t most_one(int64_t cap, int64_t req) {
  if (cap == 0 || req > cap) return 0;
  return (req >= 0 && cap > 0) ? div_nonneg(req * 100, cap) : (req * 100) / cap;
}
// floor(x / cap) for 0 <= x <= 100 * cap, 0 < cap < 2^52 (inv ~ 1/cap != 0 only then), without a
// branch: the quotient is 0..100, so one int32 conversion of the product suffices, and the remainder
// test makes it exact.  A lane outside that range sets `slow` (the caller re-runs it through the
// integer division): per-lane branches around the fallback cost more exec-mask updates and taken
// branches than the arithmetic they skip.
__device__ __forceinline__ int64_t ratio100(int64_t x, int64_t cap, double inv, bool& slow) {
  const bool ok = inv != 0.0 && x >= 0 && x <= 100 * cap && x < (1ll << 52);
  slow = !ok;
  const int64_t xs = ok ? x : 0;
  int32_t q = (int32_t)((double)xs * inv);
  const int64_t r = xs - (int64_t)q * cap;
  q += r < 0 ? -1 : (r >= cap ? 1 : 0);
  return q;
}
// floor(x / cap) for 0 <= x <= 100 * cap < 2^31 (cap > 0, inv ~ 1/cap): 32-bit operands, one
// conversion each way and the remainder correction
__device__ __forceinline__ int32_t ratio100_32(int32_t x, int32_t cap, double inv) {
  int32_t q = (int32_t)((double)x * inv);
  const int32_t r = x - q * cap;
  q += r < 0 ? -1 : (r >= cap ? 1 : 0);
  return q;
}
__device__ __forceinline__ int64_t least_one(int64_t cap, int64_t req, double inv, bool& slow) {
  const bool zero = cap == 0 || req > cap;
  bool s;
  const int64_t q = ratio100((cap - req) * 100, cap, inv, s);
  slow |= s && !zero;
  return zero ? 0 : q;
}
__device__ __forceinline__ int64_t most_one(int64_t cap, int64_t req, double inv, bool& slow) {
  const bool zero = cap == 0 || req > cap;
  bool s;
  const int64_t q = ratio100(req * 100, cap, inv, s);
  slow |= s && !zero;
  return zero ? 0 : q;
}
__device__ __forceinline__ int64_t wdiv(int64_t s, int64_t w) { return s >= 0 ? div_nonneg(s, w) : s / w; }
__device__ __forceinline__ int64_t half(int64_t s) { return s >= 0 ? (s >> 1) : s / 2; }

template <bool kDef>
__device__ __forceinline__ int64_t least_score(const DevState& st, const kgpu_pod_query& q, const NodeRes& nr,
                                               int n) {
  if constexpr (kDef) {
    const int64_t rc = nr.zc + q.score_req[0], rm = nr.zm + q.score_req[1];
    bool slow = false;
    int64_t a = least_one(nr.ac, rc, nr.ic, slow), b = least_one(nr.am, rm, nr.im, slow);
    if (slow) {
      a = least_one(nr.ac, rc);
      b = least_one(nr.am, rm);
    }
    return half(a + b);
  } else {
    int64_t s = 0;
    for (int i = 0; i < st.n_least; ++i) {
      int64_t cap, req;
      alloc_req(st, q, nr, st.least[i].resource, n, cap, req);
      s += least_one(cap, req) * st.least[i].weight;
    }
    return wdiv(s, st.least_wsum);
  }
}

template <bool kDef>
__device__ __forceinline__ int64_t most_score(const DevState& st, const kgpu_pod_query& q, const NodeRes& nr,
                                              int n) {
  if constexpr (kDef) {
    const int64_t rc = nr.zc + q.score_req[0], rm = nr.zm + q.score_req[1];
    bool slow = false;
    int64_t a = most_one(nr.ac, rc, nr.ic, slow), b = most_one(nr.am, rm, nr.im, slow);
    if (slow) {
      a = most_one(nr.ac, rc);
      b = most_one(nr.am, rm);
    }
    return half(a + b);
  } else {
    int64_t s = 0;
    for (int i = 0; i < st.n_most; ++i) {
      int64_t cap, req;
      alloc_req(st, q, nr, st.most[i].resource, n, cap, req);
      s += most_one(cap, req) * st.most[i].weight;
    }
    return wdiv(s, st.most_wsum);
  }
}

// RequestedToCapacityRatio (requested_to_capacity_ratio.go:124-170): the broken-linear shape over
// utilization per resource, weighted mean over resources with a positive score, math.Round.
// buildBrokenLinearFunction (requested_to_capacity_ratio.go:150-170) over `n` ascending points
__device__ __forceinline__ int64_t broken_linear(const kgpu_shape_point* sh, int n, int64_t p) {
  for (int i = 0; i < n; ++i)
    if (p <= sh[i].utilization) {
      if (i == 0) return sh[0].score;
      // Go int64 arithmetic: the product may be negative, division truncates toward zero
      return sh[i - 1].score + (sh[i].score - sh[i - 1].score) * (p - sh[i - 1].utilization) /
                                   (sh[i].utilization - sh[i - 1].utilization);
    }
  return sh[n - 1].score;
}
__device__ __forceinline__ int64_t rtcr_shape(const DevState& st, int64_t p) { return broken_linear(st.shape, st.n_shape, p); }

// kgpu_debug_broken_linear: the device's broken-linear function at given utilizations (the reference's
// requested_to_capacity_ratio_test.go:119 table, unscaled points)
struct ShapeProbe {
  kgpu_shape_point pts[16];
  int32_t n;
};
__global__ void k_dbg_broken_linear(ShapeProbe s, const int64_t* __restrict__ p, int64_t* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = broken_linear(s.pts, s.n, p[i]);
}
__device__ __forceinline__ int64_t rtcr_score(const DevState& st, const kgpu_pod_query& q, const NodeRes& nr, int n) {
  int64_t node_score = 0, wsum = 0;
  for (int i = 0; i < st.n_rtcr; ++i) {
    int64_t cap, req;
    alloc_req(st, q, nr, st.rtcr[i].resource, n, cap, req);
    const int64_t util = (cap == 0 || req > cap) ? 100 : 100 - ((cap - req) * 100) / cap;
    const int64_t rs = rtcr_shape(st, util);
    if (rs > 0) {
      node_score += rs * st.rtcr[i].weight;
      wsum += st.rtcr[i].weight;
    }
  }
  if (wsum == 0) return 0;
  // math.Round(float64(a) / float64(b)) for 0 <= a, 0 < b: a / b is never within an ulp of a .5
  // that it does not equal, so the exact half-away-from-zero integer rounding is the same value
  return (2 * node_score + wsum) / (2 * wsum);
}

// NodeResourceLimits (resource_limits.go:104-160): 1 when the pod's cpu or memory limit fits the
// node's allocatable.
__device__ __forceinline__ int64_t limits_score(const kgpu_pod_query& q, const NodeRes& nr) {
  const bool c = q.limits[0] != 0 && nr.ac != 0 && q.limits[0] <= nr.ac;
  const bool m = q.limits[1] != 0 && nr.am != 0 && q.limits[1] <= nr.am;
  return (c || m) ? 1 : 0;
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
  if (q.flags & KGPU_Q_NO_KNOWN_IMAGE) return 0;  // sum stays below minThreshold on every node
  int64_t sum = 0;
  if (q.images.count) {
    const int lo0 = gp(st.image_off)[n], hi0 = gp(st.image_off)[n + 1];
    for (int i = 0; i < q.images.count; ++i) {
      const int id = cp(st.qp.ints)[q.images.begin + i];
      if (id < 0) continue;
      int lo = lo0, hi = hi0;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (gp(st.image_id)[mid] < id) lo = mid + 1; else hi = mid;
      }
      if (lo < hi0 && gp(st.image_id)[lo] == id) sum += gp(st.image_score)[lo];
    }
  }
  const int64_t maxT = kMaxC * (int64_t)q.n_containers;
  if (sum < kMin) sum = kMin;
  else if (sum > maxT) sum = maxT;
  const int64_t den = maxT - kMin;  // > 0 unless the pod has no containers
  return den > 0 ? div_nonneg(100 * (sum - kMin), den) : (100 * (sum - kMin)) / den;
}

__device__ __forceinline__ int64_t npap_score(const DevState& st, const kgpu_pod_query& q, int n) {
  if (q.avoid_id < 0) return 100;
  for (int i = gp(st.avoid_off)[n]; i < gp(st.avoid_off)[n + 1]; ++i)
    if (gp(st.avoid_id)[i] == q.avoid_id) return 0;
  return 100;
}

// DefaultPodTopologySpread with an empty selector (every count is 0): 100 off-zone; zoned
// nodes get fScore*(1-zoneWeighting) + zoneWeighting*100 (default_pod_topology_spread.go:136-162).
__device__ __forceinline__ int64_t dpts_empty_score(const DevState& st, int n) {
  if (gp(st.zone_id)[n] < 0) return 100;
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

__device__ uint32_t topo_filter(int f, const DevState& st, const QPlan& pl, int n);

// One Filter plugin: 0 = Success, else (code << 8) | (detail << 16) of the status word.
__device__ __forceinline__ uint32_t filter_one(int f, const DevState& st, const kgpu_pod_query& q, const NodeRes& r,
                                               int n, const QPlan* pl = nullptr) {
  switch (f) {
    case KGPU_F_NODE_UNSCHEDULABLE:
      if (gp(st.unsched)[n] && !(q.flags & KGPU_Q_TOLERATES_UNSCHEDULABLE)) return KGPU_CODE_UNRESOLVABLE << 8;
      return 0;
    case KGPU_F_NODE_RESOURCES_FIT: {
      const uint32_t d = fit_detail(st, q, r, n);
      return d ? (KGPU_CODE_UNSCHEDULABLE << 8) | (d << 16) : 0;
    }
    case KGPU_F_NODE_NAME:
      return (q.node_name != -1 && q.node_name != st.node_base + n) ? KGPU_CODE_UNRESOLVABLE << 8 : 0;
    case KGPU_F_NODE_PORTS:
      return (q.ports.count && ports_conflict(st, q, n)) ? KGPU_CODE_UNSCHEDULABLE << 8 : 0;
    case KGPU_F_NODE_AFFINITY:
      return node_affinity_ok(st, q, n) ? 0 : KGPU_CODE_UNRESOLVABLE << 8;
    case KGPU_F_TAINT_TOLERATION:
      return taints_ok(st, q, n) ? 0 : KGPU_CODE_UNRESOLVABLE << 8;
    default:  // PodTopologySpread / InterPodAffinity: pass for pods outside the topology pipeline
      return pl ? topo_filter(f, st, *pl, n) : 0;
  }
}

// PluginToStatus.Merge (interface.go:162-191) of the words so far and the next failing plugin's word:
// UnschedulableAndUnresolvable wins over Unschedulable (the device's filters return no Error); the
// first failing plugin keeps the position and detail bits (its reasons come first).
__device__ __forceinline__ uint32_t merge_status(uint32_t acc, uint32_t w) {
  if (!acc) return w;
  const uint32_t ca = (acc >> 8) & 3u, cw = (w >> 8) & 3u;
  return cw > ca ? (acc & ~(3u << 8)) | (cw << 8) : acc;
}

// runAllFilters (framework.go:484-499 without the early exit): every plugin of the profile, each word
// in status_all, the merged word returned.
__device__ __forceinline__ uint32_t run_filters_all(const DevState& st, const kgpu_pod_query& q, const NodeRes& r, int n,
                                                 const QPlan* pl) {
  uint32_t acc = 0;
  for (int i = 0; i < st.n_filters; ++i) {
    const uint32_t c = filter_one(cp(st.filters)[i], st, q, r, n, pl);
    const uint32_t w = c ? c | (uint32_t)(i + 1) : 0u;
    gp(st.status_all)[(size_t)i * st.N + n] = w;
    acc = w ? merge_status(acc, w) : acc;
  }
  return acc;
}

// Filters in profile order; the first failure's 1-based position goes in the low byte.
template <uint32_t FM, int F = 0>
__device__ __forceinline__ uint32_t run_filters(const DevState& st, const kgpu_pod_query& q, const NodeRes& r, int n,
                                                const QPlan* pl = nullptr) {
  if constexpr (FM == kRuntime) {
    if (st.run_all) return run_filters_all(st, q, r, n, pl);
    for (int i = 0; i < st.n_filters; ++i) {
      const uint32_t c = filter_one(cp(st.filters)[i], st, q, r, n, pl);
      if (c) return c | (uint32_t)(i + 1);
    }
    return 0;
  } else if constexpr (F >= KGPU_NUM_FILTERS) {
    return 0;
  } else {
    if constexpr ((FM >> F) & 1u) {
      constexpr uint32_t pos = __builtin_popcount(FM & ((2u << F) - 1));
      const uint32_t c = filter_one(F, st, q, r, n);
      if (c) return c | pos;
    }
    return run_filters<FM, F + 1>(st, q, r, n);
  }
}

// One Score plugin's raw value (TaintToleration / NodeAffinity go to e.taint / e.na: they are
// normalized over the feasible set before weighting).
template <bool kDef>
__device__ __forceinline__ int64_t score_one(int s, const DevState& st, const kgpu_pod_query& q, const NodeRes& r,
                                             int n, NodeEval& e) {
  switch (s) {
    case KGPU_S_BALANCED_ALLOCATION: return balanced_score(q, r);
    case KGPU_S_LEAST_ALLOCATED: return least_score<kDef>(st, q, r, n);
    case KGPU_S_MOST_ALLOCATED: return most_score<kDef>(st, q, r, n);
    case KGPU_S_IMAGE_LOCALITY: return image_score(st, q, n);
    case KGPU_S_NODE_PREFER_AVOID_PODS: return npap_score(st, q, n);
    case KGPU_S_POD_TOPOLOGY_SPREAD: return 100;  // no soft constraints: max == 0
    case KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD: return (q.flags & KGPU_Q_HAS_TSC) ? 0 : dpts_empty_score(st, n);
    case KGPU_S_INTER_POD_AFFINITY: return 0;     // empty topologyScore
    case KGPU_S_TAINT_TOLERATION: e.taint = taint_raw(st, q, n); return e.taint;
    case KGPU_S_NODE_AFFINITY: e.na = na_raw(st, q, n); return e.na;
    case KGPU_S_REQUESTED_TO_CAPACITY_RATIO: return rtcr_score(st, q, r, n);
    case KGPU_S_RESOURCE_LIMITS: return limits_score(q, r);
    default: return 0;
  }
}

__device__ __forceinline__ bool normalized(int s) {
  return s == KGPU_S_TAINT_TOLERATION || s == KGPU_S_NODE_AFFINITY;
}

// dv (compile-time profiles only): a diagnostic evaluation collects each plugin's raw score in dv[S]
// (registers) instead of storing its rows; the caller stores them later.
template <uint32_t SM, int S = 0>
__device__ __forceinline__ void run_scores(const DevState& st, const kgpu_pod_query& q, const NodeRes& r, int n,
                                           NodeEval& e, bool diag, int64_t* dv = nullptr) {
  if constexpr (SM == kRuntime) {
    int64_t part = 0;
    for (int i = 0; i < st.n_scores; ++i) {
      const int s = cp(st.scores)[i];
      const int64_t v = score_one<false>(s, st, q, r, n, e);
      if (diag) {
        gp(st.diag_raw)[(size_t)s * st.N + n] = v;
        // a plugin without NormalizeScore: its normalized score is the raw one (the normalize
        // passes write only the normalized plugins, with no read-back of these rows)
        if (!normalized(s)) gp(st.diag_norm)[(size_t)s * st.N + n] = v;
      }
      if (!normalized(s)) part += v * cp(st.w_of)[s];
    }
    e.partial = part;
  } else if constexpr (S >= KGPU_NUM_SCORES) {
    return;
  } else {
    if constexpr ((SM >> S) & 1u) {
      const int64_t v = score_one<(SM & kDefRes) != 0>(S, st, q, r, n, e);
      if (diag && dv) {
        dv[S] = v;
      } else if (diag) {
        gp(st.diag_raw)[(size_t)S * st.N + n] = v;
        if constexpr (!(S == KGPU_S_TAINT_TOLERATION || S == KGPU_S_NODE_AFFINITY)) gp(st.diag_norm)[(size_t)S * st.N + n] = v;
      }
      if constexpr (!(S == KGPU_S_TAINT_TOLERATION || S == KGPU_S_NODE_AFFINITY)) e.partial += v * st.w_of[S];
    }
    run_scores<SM, S + 1>(st, q, r, n, e, diag, dv);
  }
}

// DefaultNormalizeScore of the two normalized plugins (reverse for TaintToleration), weighted.
// Plugins not in the profile have weight 0 in w_of.
__device__ __forceinline__ int64_t norm_total(const DevState& st, int64_t partial, int taint, int na, int maxT,
                                              int maxNA) {
  const int64_t vt = maxT == 0 ? 100 : 100 - (100 * (int64_t)taint) / maxT;
  const int64_t vn = maxNA == 0 ? (int64_t)na : (100 * (int64_t)na) / maxNA;
  return partial + vt * st.w_of[KGPU_S_TAINT_TOLERATION] + vn * st.w_of[KGPU_S_NODE_AFFINITY];
}

template <uint32_t SM>
__device__ __forceinline__ int64_t key_total(const DevState& st, int64_t partial, int taint, int na) {
  if constexpr (SM == kRuntime) {
    return st.n_scores ? norm_total(st, partial, taint, na, 0, 0) : 1;
  } else if constexpr ((SM & kSMask) == 0) {
    return 1;
  } else {
    int64_t t = partial;
    if constexpr ((SM >> KGPU_S_TAINT_TOLERATION) & 1u) t += 100 * st.w_of[KGPU_S_TAINT_TOLERATION];
    if constexpr ((SM >> KGPU_S_NODE_AFFINITY) & 1u) t += (int64_t)na * st.w_of[KGPU_S_NODE_AFFINITY];
    return t;
  }
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ void key_max(uint64_t& k, int& i, uint64_t k2, int i2) {
  if (k2 > k) { k = k2; i = i2; }
}

// Wave64 reductions on the VALU through DPP (no LDS round trip per step, unlike __shfl_xor's
// ds_bpermute): quad_perm xor 1 and xor 2, row_half_mirror, row_mirror (every lane of a 16-lane row
// then holds the row's result), row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3;
// lane 63 ends with the wave's result and readlane broadcasts it.  Masked-off or out-of-row lanes
// read 0, the identity of max (unsigned) and sum.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, true);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp64(uint64_t x) {
  return (uint64_t)dpp32<CTRL, ROWS>((uint32_t)x) | ((uint64_t)dpp32<CTRL, ROWS>((uint32_t)(x >> 32)) << 32);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t x, int lane) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, lane) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), lane) << 32);
}
struct OpMaxU64 {
  __device__ __forceinline__ uint64_t operator()(uint64_t a, uint64_t b) const { return a > b ? a : b; }
};
struct OpSumU64 {
  __device__ __forceinline__ uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; }
};
template <class Op>
__device__ __forceinline__ uint64_t wave_red64(uint64_t x, Op op) {
  x = op(x, dpp64<0xB1, 0xF>(x));
  x = op(x, dpp64<0x4E, 0xF>(x));
  x = op(x, dpp64<0x141, 0xF>(x));
  x = op(x, dpp64<0x140, 0xF>(x));
  x = op(x, dpp64<0x142, 0xA>(x));
  x = op(x, dpp64<0x143, 0xC>(x));
  return readlane64(x, 63);
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t x) {
  x += dpp32<0xB1, 0xF>(x);
  x += dpp32<0x4E, 0xF>(x);
  x += dpp32<0x141, 0xF>(x);
  x += dpp32<0x140, 0xF>(x);
  x += dpp32<0x142, 0xA>(x);
  x += dpp32<0x143, 0xC>(x);
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
__device__ __forceinline__ uint32_t wave_max32u(uint32_t x) {
  x = max(x, dpp32<0xB1, 0xF>(x));
  x = max(x, dpp32<0x4E, 0xF>(x));
  x = max(x, dpp32<0x141, 0xF>(x));
  x = max(x, dpp32<0x140, 0xF>(x));
  x = max(x, dpp32<0x142, 0xA>(x));
  x = max(x, dpp32<0x143, 0xC>(x));
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
// Unsigned 64-bit wave max in two 32-bit passes: the high words' max, then the low words' max over
// the lanes holding it.  A 32-bit DPP step is one max with a DPP operand; a 64-bit one is two DPP
// moves, a 64-bit compare and two selects.
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
  const uint32_t mh = wave_max32u((uint32_t)(x >> 32));
  const uint32_t ml = wave_max32u((uint32_t)(x >> 32) == mh ? (uint32_t)x : 0u);
  return ((uint64_t)mh << 32) | ml;
}
// signed 64-bit max / min through the order-preserving unsigned map
__device__ __forceinline__ int64_t wave_max_i64(int64_t x) {
  return (int64_t)(wave_max_u64((uint64_t)x ^ (1ull << 63)) ^ (1ull << 63));
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t x) {
  return (int64_t)(~wave_max_u64(~((uint64_t)x ^ (1ull << 63))) ^ (1ull << 63));
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t x) { return (int64_t)wave_red64((uint64_t)x, OpSumU64{}); }
struct OpOrU64 {
  __device__ __forceinline__ uint64_t operator()(uint64_t a, uint64_t b) const { return a | b; }
};
// two independent unsigned max reductions (the compiler interleaves the two pass chains)
__device__ __forceinline__ void wave_red64x2(uint64_t& x, uint64_t& y) {
  x = wave_max_u64(x);
  y = wave_max_u64(y);
}

// argmax of unique keys: the maximum, then the one lane holding it
__device__ __forceinline__ void wave_argmax(uint64_t& k, int& i) {
  const uint64_t m = wave_max_u64(k);
  const uint64_t b = __ballot(k == m && m != 0);
  i = b ? __builtin_amdgcn_readlane(i, (int)__builtin_ctzll(b)) : -1;
  k = m;
}

// keys are unique per node (rank40 is a bijection), so a max + ballot finds the argmax
__device__ __forceinline__ void wave_reduce_key(uint64_t& k, int& i) { wave_argmax(k, i); }

__device__ __forceinline__ int wave_reduce_sum(int v) { return (int)wave_sum32((uint32_t)v); }

// non-negative values only (raw TaintToleration / NodeAffinity scores, counts)
__device__ __forceinline__ int wave_reduce_max(int v) { return (int)wave_max32u((uint32_t)max(v, 0)); }

struct Winner {
  uint64_t key;
  int idx;
  int feasible;
};

// selectHost over the partials of a finished launch, computed by every wave on its own (lanes
// stride over the <= kMaxBlocks partials, four loads in flight per lane, then a 64-lane shuffle
// reduction): no LDS, no barrier.
__device__ __forceinline__ Winner wave_winner(const BlkKey* kb, int nb) {
  uint64_t k = 0;
  int idx = -1, f = 0;
  const GAS BlkKey* g = gp(kb);
  for (int b = threadIdx.x & 63; b < nb; b += 256) {
    BlkKey p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] = BlkKey{0, -1, 0};
      if (b + 64 * j < nb) {
        p[j].key = g[b + 64 * j].key;
        p[j].idx = g[b + 64 * j].idx;
        p[j].feasible = g[b + 64 * j].feasible;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      key_max(k, idx, p[j].key, p[j].idx);
      f += p[j].feasible;
    }
  }
  wave_reduce_key(k, idx);
  f = wave_reduce_sum(f);
  return Winner{k, idx, f};
}

// NodeInfo.AddPod on the chosen row (types.go:456-480): applied by the thread that owns the row,
// on its register copy (written back) plus the rarely used scalar and host-port columns.
__device__ __forceinline__ void assume_row(const DevState& st, const kgpu_pod_query& q, NodeRes& r, int n) {
  r.rc += q.req[0];
  r.rm += q.req[1];
  r.re += q.req[2];
  r.zc += q.nz[0];
  r.zm += q.nz[1];
  r.np += 1;
  gp(st.req_cpu)[n] = r.rc;
  gp(st.req_mem)[n] = r.rm;
  gp(st.req_eph)[n] = r.re;
  gp(st.nz_cpu)[n] = r.zc;
  gp(st.nz_mem)[n] = r.zm;
  gp(st.num_pods)[n] = r.np;
  for (int i = 0; i < q.scalars.count; ++i) {
    const kgpu_scalar_req s = cp(st.qp.scalars)[q.scalars.begin + i];
    if (s.col >= 0) gp(st.req_scalar)[(size_t)s.col * st.N + n] += s.value;
  }
  if (q.ports.count) {
    int pc = gp(st.port_count)[n];
    for (int i = 0; i < q.ports.count; ++i) {
      const kgpu_port w = cp(st.qp.ports)[q.ports.begin + i];
      bool dup = false;
      for (int s = 0; s < pc; ++s) {
        const kgpu_port p = gp(st.ports)[(size_t)s * st.N + n];
        if (p.ip == w.ip && p.proto == w.proto && p.port == w.port) dup = true;
      }
      if (dup) continue;
      // the host sizes PS for the batch's ports (kgpu_api.cpp reserve_ports); running out means a
      // lost UsedPorts entry, which the host turns into an error
      if (pc >= st.PS) {
        gp(st.port_overflow)[0] = 1;
        continue;
      }
      gp(st.ports)[(size_t)(pc++) * st.N + n] = w;
    }
    gp(st.port_count)[n] = pc;
  }
}

// The assumed pod's side of the topology state: the match-count columns of the pod classes it
// matches and of the term classes it carries (NodeInfo.AddPod -> Pods / PodsWithAffinity).
__device__ __forceinline__ void assume_counts(const DevState& st, int pod, int n) {
  if (!st.plans) return;
  const QPlan* pl = st.plans + pod;
  const kgpu_range ac = pl->assume_cls, ot = pl->own_tcls;
  for (int i = 0; i < ac.count; ++i) gp(st.mcnt)[(size_t)st.aux[ac.begin + i] * st.N + n] += 1;
  for (int i = 0; i < ot.count; ++i) gp(st.tcnt)[(size_t)st.aux[ot.begin + i] * st.N + n] += 1;
}

// The pending pod's winner: over the partials of this shard's previous launch or -- when nodes
// are sharded across GPUs -- over every rank's packed shard winner (all-gathered by RCCL, global
// node index).  w.idx comes back LOCAL (-1: the row lives on another rank); *gidx is global.
__device__ __forceinline__ Winner prev_winner(const DevState& st, const PodArgs& a, int* gidx) {
  if (st.shard_keys) {
    Winner w = wave_winner(st.shard_keys + (size_t)a.prev_parity * kMaxRanks, st.nranks);
    *gidx = w.idx;
    const int l = w.idx - st.node_base;
    w.idx = (w.idx >= 0 && l >= 0 && l < st.N) ? l : -1;
    return w;
  }
  const Winner w = wave_winner(st.kbuf + (size_t)a.prev_parity * kMaxBlocks, a.prev_blocks);
  *gidx = w.idx >= 0 ? st.node_base + w.idx : -1;
  return w;
}

// The pending pod's outcome (generic_scheduler.go:171-208): FitError, the len==1 shortcut, or
// the scored winner.  Returns the local row to assume (-1 none).
__device__ __forceinline__ int settle_prev(const DevState& st, const PodArgs& a, const kgpu_pod_query& pq,
                                           const Winner& w, int gidx, bool writer) {
  const bool error = (pq.flags & KGPU_Q_SCORE_ERROR) && w.feasible >= 2;
  const bool placed = w.feasible > 0 && !error;
  if (writer) {
    kgpu_result r;
    r.node = placed ? gidx : (error ? -2 : -1);
    r.feasible = w.feasible;
    r.evaluated = (a.cut && st.cut_state) ? gp(st.cut_state)[1] : st.n_total;
    r.scored = (placed && w.feasible >= 2) ? 1 : 0;
    r.score = r.scored ? (int64_t)(w.key >> 40) : 0;
    gp(st.results)[a.prev] = r;
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
// The last workgroup of a one-pod launch to finish resolves the pod -- selectHost, the result record and
// the assume -- in place of a k_resolve launch (PodArgs.resolve_self: the end of a short cycle, after
// k_final, or after k_eval when the pod needs no normalize pass).  Release / acquire fences around the
// ticket make every workgroup's partial visible to it across XCDs.
constexpr int kTicketSplit = 128;  // grids this large count their tickets in 8 groups (resolve_tail)
constexpr int kTicketLine = 16;    // int32 words between ticket counters (64-byte lines; 9 counters)
__device__ __forceinline__ void resolve_tail(const DevState& st, const PodArgs& a) {
  __shared__ int last;
  // a cycle the host completes on done_out: every wave's stores (the diagnostic rows included) reach L2
  // before thread 0's release writes the L2 back (one write-back per workgroup: a fence in every wave
  // cost a 100k-node cycle 5 us, profiles/r05_host_trace.txt)
  if (a.done_out) __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    // release: this workgroup's partial (and rows) written back before its ticket -- no invalidate here
    // (a full __threadfence() adds a buffer_inv whose wait every workgroup paid before its ticket)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const int G = (int)gridDim.x;
    if (G < kTicketSplit) {
      last = atomicAdd(st.ticket, 1) == G - 1;
    } else {
      // many workgroups finish together: arrivals on one device-scope counter serialize (~12 ns each,
      // MI355X_MICROARCH.md fanin), so they count on 8 group counters (blockIdx mod 8, one line each) and
      // each group's last arriver carries the group on to the top counter -- acquire its members' partials,
      // release them with its own ticket
      const int grp = (int)blockIdx.x & 7;
      int32_t* sub = st.ticket + kTicketLine * (grp + 1);
      last = 0;
      if (atomicAdd(sub, 1) == ((G - grp + 7) >> 3) - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __hip_atomic_store(sub, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next cycle
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        last = atomicAdd(st.ticket, 1) == 7;
      }
    }
  }
  __syncthreads();
  if (last) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every other workgroup's partial
    PodArgs r{};
    r.prev = a.pod;
    r.prev_blocks = (int32_t)gridDim.x;
    r.prev_parity = a.parity;
    r.assume = a.assume;
    r.cut = a.cut;
    int gidx;
    const Winner w = prev_winner(st, r, &gidx);
    const kgpu_pod_query pq = a.q_inline ? a.q : (kgpu_pod_query)*cp(st.queries + a.pod);
    const int idx = settle_prev(st, r, pq, w, gidx, threadIdx.x == 0);
    if (threadIdx.x == 0) {
      if (idx >= 0) {
        NodeRes row = load_res(st, idx);
        assume_row(st, pq, row, idx);
        assume_counts(st, a.pod, idx);
      }
      __hip_atomic_store(st.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next cycle
    }
    if (a.done_out) {
      __builtin_amdgcn_s_waitcnt(0);  // the record, the assume and the last workgroup's rows in L2 ...
      __syncthreads();
      if (threadIdx.x == 0)  // ... written back by the store's own system-scope release, then the word
        __hip_atomic_store(a.done_out, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <uint32_t FM, uint32_t SM>
__global__ __launch_bounds__(kBlock) void k_eval(const DevState* __restrict__ stp, PodArgs a) {
  const DevState& st = *stp;
  int lo, hi;
  chunk_of(st.N, lo, hi);
  const int n0 = lo + threadIdx.x;
  // Independent loads first -- this lane's first node row, the pod query and the pending pod's
  // partials -- so that their latencies overlap instead of chaining.
  NodeRes r0{};
  if (n0 < hi) r0 = load_res(st, n0);
  const kgpu_pod_query q = a.q_inline ? a.q : (kgpu_pod_query)*cp(st.queries + a.pod);
  int assume_idx = -1;
  const kgpu_pod_query* pq = st.queries + (a.prev >= 0 ? a.prev : 0);
  if (a.prev >= 0) {
    int gidx;
    const Winner w = prev_winner(st, a, &gidx);
    assume_idx = settle_prev(st, a, *cp(pq), w, gidx, blockIdx.x == 0 && threadIdx.x == 0);
  }
  const uint64_t tk = pod_tie_key(st.seed, a.seq);
  const bool write_nodes = a.norm || a.diag;

  uint64_t best = 0;
  int best_i = -1, feas = 0, maxT = 0, maxNA = 0;
  for (int n = n0; n < hi; n += kBlock) {
    NodeRes r = (n == n0) ? r0 : load_res(st, n);
    if (n == assume_idx) {
      assume_row(st, *cp(pq), r, n);
      assume_counts(st, a.prev, n);
    }
    if (a.zero_diag) {
      // a diagnostic cycle without memsets: this node's rows of the profile's plugins start at 0 (a node
      // that fails a filter reads 0 as after hipMemset); a plugin outside the profile has rows no kernel
      // writes, zeroed once when they were allocated
      for (int si = 0; si < st.n_scores; ++si) {
        const int s = st.scores[si];
        gp(st.diag_raw)[(size_t)s * st.N + n] = 0;
        gp(st.diag_norm)[(size_t)s * st.N + n] = 0;
      }
    }
    NodeEval e{0, 0, 0, 0};
    // nominated pods: a failed first pass (k_victims, nominated mode) is the node's verdict
    // (podPassesFiltersOnNode, generic_scheduler.go:578-612)
    const uint32_t s1 = st.nom_status ? gp(st.nom_status)[n] : 0u;
    e.status = s1 ? s1 : run_filters<FM>(st, q, r, n);
    if (e.status == 0) {
      run_scores<SM>(st, q, r, n, e, a.diag);
      if (a.diag && !a.norm) {
        // the normalized rows k_final would write: without a normalize pass every raw TaintToleration /
        // NodeAffinity score is 0 (needs_norm), so DefaultNormalizeScore gives 100 / 0
        for (int si = 0; si < st.n_scores; ++si) {
          const int s = st.scores[si];
          if (s == KGPU_S_TAINT_TOLERATION) gp(st.diag_norm)[(size_t)s * st.N + n] = 100;
          else if (s == KGPU_S_NODE_AFFINITY) gp(st.diag_norm)[(size_t)s * st.N + n] = e.na;
        }
      }
      ++feas;
      maxT = max(maxT, e.taint);
      maxNA = max(maxNA, e.na);
      if (!a.norm) {
        // constant DefaultNormalizeScore maxima: every raw TaintToleration / NodeAffinity score is 0
        const int64_t total = key_total<SM>(st, e.partial, e.taint, e.na);
        const uint64_t key = ((uint64_t)total << 40) | rank40(tk, (uint64_t)(st.node_base + n), st.tie_mode);
        key_max(best, best_i, key, n);
      }
    }
    if (write_nodes) {
      gp(st.status)[n] = e.status;
      gp(st.partial)[n] = e.partial;
      gp(st.raw_taint)[n] = e.taint;
      gp(st.raw_na)[n] = e.na;
    }
  }
  wave_reduce_key(best, best_i);
  feas = wave_reduce_sum(feas);
  maxT = wave_reduce_max(maxT);
  maxNA = wave_reduce_max(maxNA);
  if (threadIdx.x == 0) {
    gp(st.sbuf)[(size_t)a.parity * kMaxBlocks + blockIdx.x] = BlkStat{feas, maxT, maxNA, 0};
    if (!a.norm) gp(st.kbuf)[(size_t)a.parity * kMaxBlocks + blockIdx.x] = BlkKey{best, best_i, feas};
  }
  // a one-pod diagnostic cycle without a normalize pass resolves here: no k_final / k_resolve launch
  if (a.resolve_self && !a.norm) resolve_tail(st, a);
}

// Normalize pass: DefaultNormalizeScore maxima over the feasible set are known only after the
// evaluation launch; combine them with the stored raw values and take the argmax.
__global__ __launch_bounds__(kBlock) void k_final(const DevState* __restrict__ stp, PodArgs a, int stat_blocks) {
  const DevState& st = *stp;
  int maxT = 0, maxNA = 0;
  // sharded: the maxima over the whole cluster's feasible set, one all-gathered record per rank
  const GAS BlkStat* sb = st.shard_stats ? gp(st.shard_stats) + (size_t)a.parity * kMaxRanks
                                         : gp(st.sbuf) + (size_t)a.parity * kMaxBlocks;
  if (st.shard_stats) stat_blocks = st.nranks;
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
    if (gp(st.status)[n] != 0) continue;
    ++bf;
    const int64_t total =
        st.n_scores ? norm_total(st, gp(st.partial)[n], gp(st.raw_taint)[n], gp(st.raw_na)[n], maxT, maxNA) : 1;
    const uint64_t key = ((uint64_t)total << 40) | rank40(tk, (uint64_t)(st.node_base + n), st.tie_mode);
    key_max(best, best_i, key, n);
    if (a.diag) {
      // the normalized plugins only (run_scores wrote the others' normalized rows)
      for (int i = 0; i < st.n_scores; ++i) {
        const int s = st.scores[i];
        if (s == KGPU_S_TAINT_TOLERATION) {
          const int64_t v = gp(st.raw_taint)[n];
          gp(st.diag_norm)[(size_t)s * st.N + n] = maxT == 0 ? 100 : 100 - (100 * v) / maxT;
        } else if (s == KGPU_S_NODE_AFFINITY) {
          const int64_t v = gp(st.raw_na)[n];
          gp(st.diag_norm)[(size_t)s * st.N + n] = maxNA == 0 ? v : (100 * v) / maxNA;
        }
      }
    }
  }
  wave_reduce_key(best, best_i);
  bf = wave_reduce_sum(bf);
  if (threadIdx.x == 0) gp(st.kbuf)[(size_t)a.parity * kMaxBlocks + blockIdx.x] = BlkKey{best, best_i, bf};
  if (a.resolve_self) resolve_tail(st, a);
}

// Resolve-only launch (end of a batch / single cycle), with the evaluation grid's chunk mapping
// so that the lane owning the winning row applies the assume.
__global__ __launch_bounds__(kBlock) void k_resolve(const DevState* __restrict__ stp, PodArgs a) {
  const DevState& st = *stp;
  int lo, hi;
  chunk_of(st.N, lo, hi);
  int gidx;
  const Winner w = prev_winner(st, a, &gidx);
  const kgpu_pod_query pq = *cp(st.queries + a.prev);
  const int idx = settle_prev(st, a, pq, w, gidx, blockIdx.x == 0 && threadIdx.x == 0);
  if (idx >= lo && idx < hi && ((idx - lo) % kBlock) == (int)threadIdx.x) {
    NodeRes r = load_res(st, idx);
    assume_row(st, pq, r, idx);
    assume_counts(st, a.prev, idx);
  }
}

// percentageOfNodesToScore < 100 (generic_scheduler.go:379-399 numFeasibleNodesToFind, :424-495
// findNodesThatPassFilters): the reference checks nodes from nextStartNodeIndex on, in rotated
// Snapshot.List() order, and cancels the search when one more node fits after `to_find` already
// did.  Under the determinism contract (a one-worker run of parallelize.Until) that is:
//   kept    = the first to_find feasible nodes in rotated order;
//   p       = rotated position of feasible node to_find + 1 (N if there is none);
//   statuses = the failing nodes at positions < p; nodes at positions >= p were never examined;
//   EvaluatedNodes = len(filtered) + len(statuses) = p; nextStartNodeIndex += p (mod N).
// A profile without filter plugins keeps the first to_find nodes in NON-rotated order and advances
// by to_find (generic_scheduler.go:438-444).  One 1024-thread workgroup: each thread owns a
// contiguous run of rotated positions; a block scan of the feasible counts locates the cut.
constexpr int kCutThreads = 1024;
__global__ __launch_bounds__(kCutThreads) void k_cut(const DevState* __restrict__ stp, PodArgs a, int blocks,
                                                     int n_filters) {
  const DevState& st = *stp;
  const int N = st.N, K = st.to_find, tid = threadIdx.x;
  __shared__ int scan[kCutThreads];
  __shared__ int red[3][kCutThreads / 64];
  const int start = N > 0 ? gp(st.cut_state)[0] % N : 0;
  const int per = (N + kCutThreads - 1) / kCutThreads;
  const int r0 = min(N, tid * per), r1 = min(N, r0 + per);
  auto node_at = [&](int r) { return n_filters ? (start + r) % N : r; };
  int cnt = 0;
  for (int r = r0; r < r1; ++r) cnt += gp(st.status)[node_at(r)] == 0;
  // inclusive block scan of the per-thread feasible counts
  scan[tid] = cnt;
  __syncthreads();
  for (int off = 1; off < kCutThreads; off <<= 1) {
    const int v = tid >= off ? scan[tid - off] : 0;
    __syncthreads();
    scan[tid] += v;
    __syncthreads();
  }
  const int before = scan[tid] - cnt;  // feasible nodes at positions < r0
  const int total = scan[kCutThreads - 1];
  // p: position of feasible node K + 1 (the one that cancels the search), N if none
  __shared__ int p_sh;
  if (tid == 0) p_sh = N;
  __syncthreads();
  if (n_filters && total > K && before <= K && before + cnt > K) {
    int seen = before;
    for (int r = r0; r < r1; ++r)
      if (gp(st.status)[node_at(r)] == 0 && ++seen == K + 1) {
        p_sh = r;
        break;
      }
  }
  __syncthreads();
  const int p = n_filters ? p_sh : K;
  int feas = 0, maxT = 0, maxNA = 0;
  int seen = before;
  for (int r = r0; r < r1; ++r) {
    const int n = node_at(r);
    const uint32_t w = gp(st.status)[n];
    if (w == 0) {
      if (++seen <= K) {
        ++feas;
        maxT = max(maxT, gp(st.raw_taint)[n]);
        maxNA = max(maxNA, gp(st.raw_na)[n]);
        continue;
      }
      gp(st.status)[n] = kStatusNotEvaluated;  // feasible but beyond the cut
    } else if (r >= p) {
      gp(st.status)[n] = kStatusNotEvaluated;  // never examined
    }
  }
  feas = wave_reduce_sum(feas);
  maxT = wave_reduce_max(maxT);
  maxNA = wave_reduce_max(maxNA);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = feas;
    red[1][tid >> 6] = maxT;
    red[2][tid >> 6] = maxNA;
  }
  __syncthreads();
  for (int b = tid; b < blocks; b += kCutThreads) {
    BlkStat o{0, 0, 0, 0};
    if (b == 0) {
      for (int w = 0; w < kCutThreads / 64; ++w) {
        o.feasible += red[0][w];
        o.max_taint = max(o.max_taint, red[1][w]);
        o.max_na = max(o.max_na, red[2][w]);
      }
    }
    gp(st.sbuf)[(size_t)a.parity * kMaxBlocks + b] = o;
  }
  if (tid == 0) {
    gp(st.cut_state)[0] = N > 0 ? (start + p) % N : 0;
    gp(st.cut_state)[1] = p;
  }
}

// Node sharding: this shard's contribution to the pod's cluster-wide selectHost (what = 0: the
// best packed key with its GLOBAL node index and the shard's feasible count) or to the
// DefaultNormalizeScore maxima (what = 1).  One wave; the RCCL all-gather that follows on the same
// stream makes every rank's record visible to the next launch (prev_winner / k_final).
__global__ __launch_bounds__(kBlock) void k_shard_pack(const DevState* __restrict__ stp, int parity, int blocks,
                                                       int what) {
  const DevState& st = *stp;
  if (what == 0) {
    const Winner w = wave_winner(st.kbuf + (size_t)parity * kMaxBlocks, blocks);
    if (threadIdx.x == 0)
      *gp(st.shard_send_key) = BlkKey{w.key, (w.key && w.idx >= 0) ? st.node_base + w.idx : -1, w.feasible};
    return;
  }
  int f = 0, mt = 0, mn = 0;
  const GAS BlkStat* sb = gp(st.sbuf) + (size_t)parity * kMaxBlocks;
  for (int b = threadIdx.x; b < blocks; b += kBlock) {
    const BlkStat p = sb[b];
    f += p.feasible;
    mt = max(mt, p.max_taint);
    mn = max(mn, p.max_na);
  }
  f = wave_reduce_sum(f);
  mt = wave_reduce_max(mt);
  mn = wave_reduce_max(mn);
  if (threadIdx.x == 0) *gp(st.shard_send_stat) = BlkStat{f, mt, mn, 0};
}

// ---------------------------------------------------------------- persistent batch kernel
// A run of pods in queue order inside ONE launch.  Workgroup g owns nodes [g*per, (g+1)*per) and
// keeps their resource rows in registers for the whole run: K slots per row lane, per = K*B - 1
// (the last slot of the last lane is the spare below).  Per pod every workgroup publishes one
// 8-byte granule -- valid bit | ((score+1) << 40 | rank40), 0 key = no feasible node -- with a
// write-through (sc1) store into the pod's row of slots, and every workgroup derives the same
// winner from the complete row.  Slots are written once per launch (zeroed by the host), so a
// granule is its own flag.
//
// Roles inside a workgroup (B row threads, then one communication wave):
//  * the row waves evaluate pod i in two variants in one pass: variant A on the rows as they are,
//    variant B on the spare slot, which holds this workgroup's candidate row for pod i-1 with pod
//    i-1 assumed on it (staged in LDS when pod i-1 was published).  If this workgroup wins pod
//    i-1, variant B (candidate slot replaced by the spare) is pod i's view of the changed row;
//    otherwise variant A is.  The spare is just one more lane, so B costs no extra latency.
//  * the communication wave polls pod i-1's row of granules while the row waves evaluate pod i
//    and hands the winner over through LDS: the granule hop overlaps the evaluation.
// Two barriers per pod: (c) pod i evaluated and pod i-1 resolved; (e) pod i published, pod i-1
// assumed on the winning row, pod i's candidate row staged.  When pod i-1 carries extended
// resources or host ports (columns that live in memory) no variant B applies: a workgroup that
// wins such a pod re-evaluates its winning row after the assume, and that row's wave publishes.
//
// The chosen variant's feasible count goes to a side array; k_batch_fixup fills in
// FeasibleNodes and the scored flag after the launch.  A poll that waits longer than
// kSpinTimeout (lost co-residency) raises the abort word and every workgroup leaves the loop.
constexpr uint64_t kGValid = 1ull << 63;
constexpr uint64_t kSpinTimeout = 50000000ull;  // s_memrealtime ticks (100 MHz): 0.5 s

__device__ __forceinline__ void store_sc1(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t load_sc1(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int load_sc1(const int32_t* p) {
  return __hip_atomic_load(const_cast<int32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Lane `src`'s row (wave-uniform src), in every lane.
__device__ __forceinline__ int64_t lane64(int64_t x, int src) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, src);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)x >> 32), src);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ NodeRes lane_row(const NodeRes& r, int src) {
  NodeRes t;
  t.ac = lane64(r.ac, src); t.am = lane64(r.am, src); t.ae = lane64(r.ae, src);
  t.rc = lane64(r.rc, src); t.rm = lane64(r.rm, src); t.re = lane64(r.re, src);
  t.zc = lane64(r.zc, src); t.zm = lane64(r.zm, src);
  t.ap = __builtin_amdgcn_readlane(r.ap, src);
  t.np = __builtin_amdgcn_readlane(r.np, src);
  t.ic = __builtin_bit_cast(double, lane64(__builtin_bit_cast(int64_t, r.ic), src));
  t.im = __builtin_bit_cast(double, lane64(__builtin_bit_cast(int64_t, r.im), src));
  return t;
}

// NodeInfo.AddPod on a register copy only (the variant-B row): resource columns and pod count.
__device__ __forceinline__ void assume_regs(const kgpu_pod_query& q, NodeRes& r) {
  r.rc += q.req[0];
  r.rm += q.req[1];
  r.re += q.req[2];
  r.zc += q.nz[0];
  r.zm += q.nz[1];
  r.np += 1;
}

// Wait for this lane's outstanding vector loads.  Used at the end of paths that load only for
// some pods (extended resources, host ports): the join after them then carries no pending load,
// so no later register write in the pod loop waits on vmcnt -- which counts stores too, and would
// hold the evaluation behind the previous pod's write-through granule and assume stores.
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0) only

// Key of one node for one pod: 0 = infeasible, else ((score+1) << 40) | rank40.
template <uint32_t FM, uint32_t SM>
__device__ __forceinline__ uint64_t node_key(const DevState& st, const kgpu_pod_query& q, const NodeRes& r, int n,
                                             uint64_t tk) {
  // Scores run on every lane whose wave has a feasible node and are discarded for the infeasible
  // ones (read-only, in-bounds): a per-lane branch around them costs exec-mask updates on every
  // evaluation and saves nothing when the wave diverges.
  const uint32_t fs = run_filters<FM>(st, q, r, n);
  if (__ballot(fs == 0) == 0) {
    if (q.scalars.count | q.ports.count) vm_drain();
    return 0;
  }
  NodeEval e{0, 0, 0, 0};
  run_scores<SM>(st, q, r, n, e, false);
  if (q.scalars.count | q.ports.count) vm_drain();
  const int64_t total = key_total<SM>(st, e.partial, e.taint, e.na);
  const uint64_t key = ((uint64_t)(total + 1) << 40) | rank40(tk, (uint64_t)(st.node_base + n), st.tie_mode);
  return fs ? 0 : key;
}

struct Cand {
  uint64_t key;
  int idx;    // local node index within the workgroup's range
  int feas;
};

__device__ __forceinline__ void wave_reduce_cand(Cand& c) {
  c.feas = wave_reduce_sum(c.feas);
  wave_argmax(c.key, c.idx);
}

// Slots indexed [p] alternate by pod parity: a wave may write pod i+1's entry while a slower
// wave still reads pod i's.
template <int B>
struct BatchShared {
  static constexpr int W = B / 64;  // row waves
  uint64_t ka[2][W], kb[2][W];      // per-wave partials of variants A and B
  int ia[2][W], ib[2][W], fa[2][W], fb[2][W];
  int rwg[2];                       // communication wave: winning granule of pod p in slot p & 1
                                    // (-1: no feasible node)
  int rabort[2];                    // the poll gave up (abort word or timeout)
  NodeRes brow[2];                  // pod p's candidate row (pod p-1 assumed) for pod p+1's variant B
  int bready;                       // p + 1 once brow[p & 1] is written
  int cslow[2];                     // slow path: candidate of pod p
  int cready;                       // p + 1 once cslow[p & 1] is written
};

__device__ __forceinline__ void lds_release(int* f, int v) {
  __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// LDS hand-offs between the waves of a workgroup.  A wait that outlives 2 x kSpinTimeout (a protocol
// fault, never expected) raises the run's abort word instead of hanging the workgroup: the
// communication wave's next sweep sees it, every wave leaves the pod loop, and the host reports
// KGPU_E_DEVICE and invalidates the mirror.
template <bool GE>
__device__ __forceinline__ void lds_wait_t(int* f, int v, int32_t* abort_word) {
  // the clock is read only once the first check failed, and then every 64 spins: an s_memrealtime
  // in flight would hold every LDS read behind it (both count in lgkmcnt)
  uint64_t t0 = 0;
  for (int it = 0;; ++it) {
    const int x = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (GE ? x >= v : x == v) return;
    __builtin_amdgcn_s_sleep(1);
    if ((it & 63) == 0) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (it == 0) {
        t0 = now;
      } else if (now - t0 > 2 * kSpinTimeout) {
        // twice the global polls' limit: when a workgroup never started, the communication wave's poll
        // gives up first and reports the clean abort this wave would otherwise hide
        __hip_atomic_fetch_or(abort_word, kAbortDirty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
    }
  }
}
__device__ __forceinline__ void lds_wait(int* f, int v, int32_t* abort_word) { lds_wait_t<false>(f, v, abort_word); }
__device__ __forceinline__ void lds_wait_ge(int* f, int v, int32_t* abort_word) { lds_wait_t<true>(f, v, abort_word); }

__device__ __forceinline__ constexpr bool spare_slot(int j, int K, int tid, int B) {
  return j == K - 1 && tid == B - 1;
}

// Per-lane best over its K slots, then per-wave partials of variant A (rows as they are, spare
// excluded) and, when `vb`, variant B (slot jb of lane ob -- the candidate for the previous pod --
// replaced by the spare, reported under the candidate's index).  Feasible counts through ballots.
template <int K, int B>
__device__ __forceinline__ void wg_partials(BatchShared<B>& sh, int p, const uint64_t (&keys)[K], bool vb, int ob,
                                            int jb, int cand, Cand& ra, Cand& rb) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  Cand a{0, -1, 0}, b{0, -1, 0};
  if (!vb) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint64_t k = spare_slot(j, K, tid, B) ? 0 : keys[j];
      a.feas += __popcll(__ballot(k != 0));
      if (k > a.key) { a.key = k; a.idx = j * B + tid; }
    }
    wave_argmax(a.key, a.idx);
  } else {
    // Variant A (the rows as they are) and variant B (the candidate's slot replaced by the spare) share
    // every row but those two slots: one max chain over the shared rows, then each variant's own slot
    // from its lane -- one 64-bit DPP reduction per pod instead of two (the row wave is issue-bound).
    uint64_t m = 0, kc = 0, ks = 0;
    int mi = -1, f0 = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const bool spare = spare_slot(j, K, tid, B), isc = tid == ob && j == jb;
      const uint64_t k = (spare || isc) ? 0 : keys[j];
      f0 += __popcll(__ballot(k != 0));
      if (k > m) { m = k; mi = j * B + tid; }
      if (isc) kc = keys[j];
      if (spare) ks = keys[j];
    }
    wave_argmax(m, mi);
    const uint64_t kcu = (ob >> 6) == wave ? (uint64_t)lane64((int64_t)kc, ob & 63) : 0;        // A's own slot
    const uint64_t ksu = ((B - 1) >> 6) == wave ? (uint64_t)lane64((int64_t)ks, (B - 1) & 63) : 0;  // B's
    a = Cand{m, mi, f0 + (kcu != 0 ? 1 : 0)};
    if (kcu > m) { a.key = kcu; a.idx = jb * B + ob; }
    b = Cand{m, mi, f0 + (ksu != 0 ? 1 : 0)};
    if (ksu > m) { b.key = ksu; b.idx = cand; }
  }
  if (lane == 0) {
    sh.ka[p][wave] = a.key; sh.ia[p][wave] = a.idx; sh.fa[p][wave] = a.feas;
    sh.kb[p][wave] = b.key; sh.ib[p][wave] = b.idx; sh.fb[p][wave] = b.feas;
  }
  ra = a;
  rb = b;
}

template <int B>
__device__ __forceinline__ Cand wg_combine(const BatchShared<B>& sh, int p, bool variant_b) {
  Cand c{0, -1, 0};
#pragma unroll
  for (int w = 0; w < B / 64; ++w) {
    const uint64_t k = variant_b ? sh.kb[p][w] : sh.ka[p][w];
    const int i = variant_b ? sh.ib[p][w] : sh.ia[p][w];
    c.feas += variant_b ? sh.fb[p][w] : sh.fa[p][w];
    if (k > c.key) { c.key = k; c.idx = i; }
  }
  return c;
}

// Slow path: the wave holding the winning row recomputes its variant-A partial from its current
// keys (the winning row re-evaluated) and combines it with the other waves' partials in LDS.
template <int K, int B>
__device__ __forceinline__ Cand wave_recombine(const BatchShared<B>& sh, int p, const uint64_t (&keys)[K]) {
  const int tid = threadIdx.x, wave = tid >> 6;
  Cand a{0, -1, 0};
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint64_t k = spare_slot(j, K, tid, B) ? 0 : keys[j];
    a.feas += __popcll(__ballot(k != 0));
    if (k > a.key) { a.key = k; a.idx = j * B + tid; }
  }
  wave_argmax(a.key, a.idx);
  Cand c{0, -1, 0};
#pragma unroll
  for (int w = 0; w < B / 64; ++w) {
    const bool me = w == wave;
    const uint64_t k = me ? a.key : sh.ka[p][w];
    const int i = me ? a.idx : sh.ia[p][w];
    c.feas += me ? a.feas : sh.fa[p][w];
    if (k > c.key) { c.key = k; c.idx = i; }
  }
  return c;
}

// The communication wave: poll pod `row`'s GT granules (<= 64 * NJ) and return the winning key and
// granule index to every lane; the abort word rides along with every sweep.  A granule counts once
// its top four bits equal `expect` (valid bit + ring lap); the key is the rest (`kmask`).
// System-scope loads for a mailbox other ranks write over xGMI.  Returns false on timeout / abort.
template <int NJ>
struct Sweep {
  uint64_t v[NJ];
  int abort;
};
template <int NJ, bool SYS>
__device__ __forceinline__ Sweep<NJ> sweep(const uint64_t* row, int G, const int32_t* abort_word, uint64_t fill) {
  const int lane = threadIdx.x & 63;
  Sweep<NJ> s;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    uint64_t* p = const_cast<uint64_t*>(row + lane + 64 * j);
    s.v[j] = (lane + 64 * j < G) ? (SYS ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : load_sc1(p))
                                 : fill;  // a valid granule with key 0
  }
  s.abort = load_sc1(abort_word);
  return s;
}

// Two sweeps in flight: the older one is examined while the newer one travels, so a row that
// completes is seen about one round trip after its last granule lands rather than up to two.
template <int NJ>
__device__ __forceinline__ bool row_done(const Sweep<NJ>& cur, uint64_t tmask, uint64_t expect, uint64_t& wkey,
                                         int& wg) {
  const int lane = threadIdx.x & 63;
  bool all = true;
  uint64_t k = 0;
  int gsel = -1;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const uint64_t v = cur.v[j];
    if ((v & tmask) != expect) {
      all = false;
    } else if ((v & ~tmask) > k) {
      k = v & ~tmask;
      gsel = lane + 64 * j;
    }
  }
  if (!__all(all)) return false;
  wave_argmax(k, gsel);
  wkey = k;
  wg = k ? gsel : -1;
  return true;
}
template <int NJ, bool SYS>
__device__ __forceinline__ bool poll_row(const uint64_t* row, int G, const int32_t* abort_word, uint64_t tmask,
                                         uint64_t expect, uint64_t& wkey, int& wg) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  Sweep<NJ> a = sweep<NJ, SYS>(row, G, abort_word, expect);
  for (;;) {
    const Sweep<NJ> b = sweep<NJ, SYS>(row, G, abort_word, expect);
    if (a.abort != 0) return false;
    if (row_done<NJ>(a, tmask, expect, wkey, wg)) return true;
    a = sweep<NJ, SYS>(row, G, abort_word, expect);
    if (b.abort != 0) return false;
    if (row_done<NJ>(b, tmask, expect, wkey, wg)) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTimeout) return false;
  }
}

// HB (config (b)'s profile, one row wave): two helper waves beside the row wave evaluate the rows'
// NodeResourcesLeastAllocated (helper 1) and BalancedAllocation (helper 2) weighted scores of each pod
// while the row wave evaluates NodeResourcesFit and the tie-break ranks -- three instruction streams on
// three SIMDs instead of one (the evaluation is issue-bound: DESIGN.md 4.3) -- and hand them over
// through LDS; the row wave forms ((least + balanced + 1) << 40) | rank40.
struct HRow {
  int64_t ac, am, zc, zm;
  double ic, im;
};

// XG: the node-sharded instantiation (xGMI mailbox rings); the unsharded one carries none of its code.
template <uint32_t FM, uint32_t SM, int K, int B, bool XG, bool HB = false>
__global__ __launch_bounds__(B + 64 + (HB ? 2 * B : 0)) void k_batch(const DevState* __restrict__ stp, BatchArgs pa) {
  static_assert(!HB || (B == 64 && !XG &&
                       SM == ((1u << KGPU_S_BALANCED_ALLOCATION) | (1u << KGPU_S_LEAST_ALLOCATED) | kDefRes)),
                "the helper wave splits config (b)'s profile on the one-row-wave geometry");
  const DevState& st = *stp;
  constexpr int W = B / 64;  // row waves; wave W communicates; HB: waves W + 1, W + 2 help row wave 0
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int G = gridDim.x, g = blockIdx.x;
  if (g == pa.hold) return;  // KGPU_OPT_HOLD_GROUP: a workgroup that never became resident
  const int lo = g * pa.per;
  const int GT = pa.GT, gme = pa.rank * G + g;  // this workgroup's granule in every row
  constexpr bool xg = XG;                       // xGMI mailbox ring (node-sharded run)
  const uint64_t tmask = xg ? (0xFull << 60) : kGValid;
  __shared__ BatchShared<B> sh;
  __shared__ int64_t sh_hk[HB ? 2 * 2 * K * B : 1];  // HB: [helper][pod parity][slot][lane] weighted score
  __shared__ int sh_hready[2];                       // HB: i + 1 once pod i's parts of helper h are in sh_hk
  __shared__ uint64_t* sh_peer_g[XG ? kMaxRanks : 1];
  __shared__ int32_t* sh_peer_f[XG ? kMaxRanks : 1];
  if constexpr (XG) {
    if (wave == W && lane < pa.nranks) {
      sh_peer_g[lane] = pa.pgran[lane];
      sh_peer_f[lane] = pa.pfeas[lane];
    }
  }
  if (tid == 0) {
    sh.bready = 0;
    sh.cready = 0;
    sh_hready[0] = 0;
    sh_hready[1] = 0;
  }
  __syncthreads();
  auto ring_row = [&](int k) -> size_t { return xg ? (size_t)((pa.xseq0 + k) % pa.R) : (size_t)k; };
  auto ring_tag = [&](int k) -> uint64_t {
    return xg ? (kGValid | ((uint64_t)(((pa.xseq0 + k) / pa.R) & 7) << 60)) : kGValid;
  };
  // publish pod i's granule (and feasible count): into this launch's rows, or into every rank's
  // mailbox ring (peer bases staged in LDS at kernel start: no pointer load on this path)
  auto publish = [&](int i, uint64_t key, int feas) {
    const size_t roff = ring_row(i) * GT + gme;
    const uint64_t gtag = ring_tag(i);
    if constexpr (!XG) {
      store_sc1(pa.gran + roff, gtag | key);
      pa.feas[roff] = feas;
    } else {
      for (int rk = 0; rk < pa.nranks; ++rk) {
        __hip_atomic_store(sh_peer_g[rk] + roff, gtag | key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(sh_peer_f[rk] + roff, feas, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  };
  // phase stamps (diagnostics): per iteration i, 8 per traced workgroup (0 and last).  Row wave 0:
  // 0 start, 5 evaluated, 1 partials written, 2 past barrier (c), 4 iteration end.  The
  // communication wave: 7 pod i-1 resolved, 6 pod i's partials complete, 3 pod i published.
  const bool tr = pa.trace && (g == 0 || g == G - 1);
  int64_t* trow = pa.trace ? pa.trace + (g == 0 ? 0 : 8) : nullptr;
#define KGPU_STAMP(i, k) \
  if (tr && (tid == 0 || tid == B)) trow[(size_t)(i) * 16 + (k)] = (int64_t)__builtin_amdgcn_s_memrealtime()

  if constexpr (HB) {
    if (wave == W + 1 || wave == W + 2) {
      // ---- helper waves: Least (helper 0) or Balanced (helper 1) of every row of the row wave (same
      // lanes, same nodes) and of its spare lane's variant-B row; each follows the candidate and the
      // winner as the communication wave does, so its copies of the rows take the same assumes
      const int hw = wave - W - 1;
      HRow h[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const int n = lo + j * B + lane;
        h[j] = HRow{0, 0, 0, 0, 0.0, 0.0};
        if (!spare_slot(j, K, lane, B) && n < st.N) {
          h[j].ac = gp(st.alloc_cpu)[n];
          h[j].am = gp(st.alloc_mem)[n];
          h[j].zc = gp(st.nz_cpu)[n];
          h[j].zm = gp(st.nz_mem)[n];
          h[j].ic = (h[j].ac > 0 && h[j].ac < (1ll << 52)) ? 1.0 / (double)h[j].ac : 0.0;
          h[j].im = (h[j].am > 0 && h[j].am < (1ll << 52)) ? 1.0 / (double)h[j].am : 0.0;
        }
      }
      __builtin_amdgcn_s_waitcnt(0);
      const int64_t wl = st.w_of[KGPU_S_LEAST_ALLOCATED], wbal = st.w_of[KGPU_S_BALANCED_ALLOCATION];
      int cand = -1;
      bool staged = false;
      for (int i = 0; i <= pa.count; ++i) {
        const bool have_prev = i > 0, have_cur = i < pa.count;
        const int p = i & 1;
        const kgpu_pod_query* qc = st.queries + pa.first + i;       // pod i (have_cur)
        const kgpu_pod_query* qpp = st.queries + pa.first + i - 1;  // pod i-1 (have_prev)
        const bool qmem = have_prev && (cp(qpp)->scalars.count | cp(qpp)->ports.count) != 0;
        const bool fast_b = have_prev && cand >= 0 && staged && pa.assume && !qmem;
        const int ob = cand >= 0 ? cand % B : -1, jb = cand >= 0 ? cand / B : -1;
        if (have_cur) {
          if (fast_b) {
            // the candidate row for pod i-1 with pod i-1 applied (assume_regs), in the spare lane
            HRow t{};
#pragma unroll
            for (int j = 0; j < K; ++j)
              if (j == jb) {
                t.ac = lane64(h[j].ac, ob);
                t.am = lane64(h[j].am, ob);
                t.zc = lane64(h[j].zc, ob) + cp(qpp)->nz[0];
                t.zm = lane64(h[j].zm, ob) + cp(qpp)->nz[1];
                t.ic = __builtin_bit_cast(double, lane64(__builtin_bit_cast(int64_t, h[j].ic), ob));
                t.im = __builtin_bit_cast(double, lane64(__builtin_bit_cast(int64_t, h[j].im), ob));
              }
            if (lane == B - 1) h[K - 1] = t;
          }
          kgpu_pod_query qh;
          qh.score_req[0] = cp(qc)->score_req[0];
          qh.score_req[1] = cp(qc)->score_req[1];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const bool spare = spare_slot(j, K, lane, B);
            const int n = spare ? lo + cand : lo + j * B + lane;
            NodeRes nr{};
            nr.ac = h[j].ac; nr.am = h[j].am; nr.zc = h[j].zc; nr.zm = h[j].zm; nr.ic = h[j].ic; nr.im = h[j].im;
            sh_hk[((hw * 2 + p) * K + j) * B + lane] =
                hw == 0 ? least_score<true>(st, qh, nr, n) * wl : balanced_score(qh, nr) * wbal;
          }
          if (lane == 0) lds_release(&sh_hready[hw], i + 1);
        }
        __syncthreads();  // (c)
        int wg = -1;
        if (have_prev) {
          if (sh.rabort[(i - 1) & 1]) break;
          wg = sh.rwg[(i - 1) & 1];
        }
        const bool won = have_prev && wg == gme;
        if (won && pa.assume && lane == ob) {
#pragma unroll
          for (int j = 0; j < K; ++j)
            if (j == jb) {
              h[j].zc += cp(qpp)->nz[0];
              h[j].zm += cp(qpp)->nz[1];
            }
        }
        const bool slow = have_cur && won && pa.assume && !fast_b;
        int cn = -1;
        if (have_cur && !slow) {
          const Cand c = wg_combine<B>(sh, p, won && fast_b);
          cn = c.key ? c.idx : -1;
        }
        if (slow) {
          lds_wait(&sh.cready, i + 1, pa.abort);
          cand = sh.cslow[p];
        } else {
          cand = cn;
        }
        staged = have_cur && !slow && cand >= 0;
      }
      return;
    }
  }
  if (wave == W) {
    // ---- communication wave: resolve pod i-1 while the row waves evaluate pod i, then combine
    //      their partials and publish pod i (variant B when this workgroup won pod i-1), and write
    //      pod i-1's result record
    constexpr int kQWords = (int)(sizeof(kgpu_pod_query) / 8);
    static_assert(kQWords <= 64, "one query row per prefetch instruction");
    int cand = -1;        // this workgroup's candidate for pod i-1 (what it published)
    bool staged = false;  // its row is staged for variant B
    for (int i = 0; i <= pa.count; ++i) {
      const bool have_prev = i > 0, have_cur = i < pa.count;
      const int p = i & 1;
      if (i == pa.abort_at && g == 0 && lane == 0) __hip_atomic_store(pa.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // pod i+2's query into L2 (the row waves' scalar load of it, an iteration later, then hits)
      if (i + 2 < pa.count) {
        const uint64_t v = lane < kQWords ? reinterpret_cast<const uint64_t*>(st.queries + pa.first + i + 2)[lane] : 0;
        asm volatile("" ::"v"(v));
      }
      bool qmem = false;  // pod i-1 carries extended resources or host ports: no variant B
      if (have_prev) {
        const kgpu_pod_query* qq = st.queries + pa.first + i - 1;
        qmem = (cp(qq)->scalars.count | cp(qq)->ports.count) != 0;
      }
      const bool fast_b = have_prev && cand >= 0 && staged && pa.assume && !qmem;
      uint64_t wkey = 0;
      int wg = -1;
      bool ok = true;
      if (have_prev) {
        const uint64_t* prow = pa.gran + ring_row(i - 1) * GT;
        const uint64_t expect = ring_tag(i - 1);
        if constexpr (!XG)
          ok = poll_row<4, false>(prow, GT, pa.abort, tmask, expect, wkey, wg);
        else if (GT <= 256)
          ok = poll_row<4, true>(prow, GT, pa.abort, tmask, expect, wkey, wg);
        else
          ok = poll_row<16, true>(prow, GT, pa.abort, tmask, expect, wkey, wg);
        KGPU_STAMP(i, 7);
      }
      const bool won = have_prev && wg == gme;
      const bool slow = have_cur && won && pa.assume && !fast_b;
      if (ok) {
        // pod i-1's record (unsharded: by the winning workgroup; xGMI-sharded: by workgroup 0 of
        // every rank, which decodes the winner's global node index from its key)
        if (have_prev && lane == 0 && (xg ? g == 0 : (won || (wg < 0 && g == 0)))) {
          kgpu_result res;
          res.node = wg < 0 ? -1
                   : xg ? (int32_t)rank40_inv(pod_tie_key(st.seed, pa.seq0 + i - 1), wkey & kMask40, st.tie_mode)
                        : st.node_base + lo + cand;
          res.feasible = 0;   // k_batch_fixup
          res.evaluated = st.n_total;
          res.scored = 0;     // k_batch_fixup
          res.score = wg >= 0 ? (int64_t)(wkey >> 40) - 1 : 0;
          gp(st.results)[pa.first + i - 1] = res;
        }
      } else if (lane == 0) {
        // pod 0's granules never came (i == 1): no workgroup resolved a pod of this run
        __hip_atomic_fetch_or(pa.abort, (i <= 1 && !XG) ? kAbortClean : kAbortDirty, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lane == 0 && have_prev) {
        sh.rwg[(i - 1) & 1] = wg;
        sh.rabort[(i - 1) & 1] = ok ? 0 : 1;
      }
      // (c): pod i-1 resolved here, pod i's partials written by the row waves.  The row waves take
      // their candidate for pod i from the partials themselves and go on (assume, staging) while this
      // wave combines and publishes -- nobody waits for the publish.
      __syncthreads();  // (c)
      if (!ok) break;
      int cn = -1;
      if (have_cur && !slow) {
        KGPU_STAMP(i, 6);
        const Cand c = wg_combine<B>(sh, p, won && fast_b);
        if (lane == 0) publish(i, c.key, c.feas);
        KGPU_STAMP(i, 3);
        cn = c.key ? c.idx : -1;
      }
      if (slow) {
        lds_wait(&sh.cready, i + 1, pa.abort);
        cand = sh.cslow[p];
      } else {
        cand = cn;
      }
      staged = have_cur && !slow && cand >= 0;
    }
    return;
  }

  // ---- row waves.  Rows stay in registers; assume_row writes every change through to the node
  // columns as well.  The spare slot holds no node of its own.
  NodeRes r[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int n = lo + j * B + tid;
    r[j] = NodeRes{};
    if (!spare_slot(j, K, tid, B) && n < st.N) {
      r[j] = load_res(st, n);
      // Allocatable never changes inside the run: LeastAllocated / MostAllocated divide through
      // exact reciprocal-plus-remainder-correction division (ratio100)
      if constexpr ((SM & kDefRes) != 0 && SM != kRuntime) set_recips(r[j]);
    }
  }
  // The row loads complete here.  Left to the first use inside the pod loop, their wait would sit
  // in the loop body as a vmcnt(0) -- and vmcnt counts stores too, so every iteration would wait
  // there for the previous iteration's write-through granule and assume stores to be acknowledged.
  __builtin_amdgcn_s_waitcnt(0);

  kgpu_pod_query qp{};                      // pod i-1 (published, not yet resolved)
  kgpu_pod_query q = *cp(st.queries + pa.first);
  int cand = -1;                            // this workgroup's candidate for pod i-1 (uniform)
  bool staged = false;                      // its row is (being) staged in sh.brow[(i-1) & 1]
  for (int i = 0; i <= pa.count; ++i) {
    KGPU_STAMP(i, 0);
    const bool have_prev = i > 0;
    const bool have_cur = i < pa.count;
    const int p = i & 1;
    // variant B applies when pod i-1's assume is a register-only change of the candidate row
    const bool fast_b = have_prev && cand >= 0 && staged && pa.assume && qp.scalars.count == 0 && qp.ports.count == 0;
    const int ob = cand >= 0 ? cand % B : -1, jb = cand >= 0 ? cand / B : -1;
    uint64_t keys[K];
    Cand own_a{0, -1, 0}, own_b{0, -1, 0};  // this wave's variant-A / B reduction of pod i
    if (have_cur) {
      const uint64_t tk = pod_tie_key(st.seed, pa.seq0 + i);
      if (fast_b && wave == W - 1) {
        NodeRes t;
        if constexpr (W == 1) {
          // one row wave: the candidate row is read from its lane directly (it is unchanged since
          // barrier (c) of pod i-1, where the multi-wave geometries stage it in LDS)
#pragma unroll
          for (int j = 0; j < K; ++j)
            if (j == jb) t = lane_row(r[j], ob);
        } else {
          lds_wait(&sh.bready, i, pa.abort);  // the candidate lane staged it right after barrier (c) of pod i-1
          t = sh.brow[(i - 1) & 1];
        }
        assume_regs(qp, t);
        if (tid == B - 1) r[K - 1] = t;
      }
      if constexpr (HB) {
        // Fit and the tie-break rank here; Least and Balanced from the helper waves
        uint32_t fs[K];
        uint64_t rkj[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const bool spare = spare_slot(j, K, tid, B);
          const int n = spare ? lo + cand : lo + j * B + tid;
          fs[j] = (spare ? fast_b : n < st.N) ? run_filters<FM>(st, q, r[j], n) : 1u;
          rkj[j] = rank40(tk, (uint64_t)(st.node_base + n), st.tie_mode);
        }
        if (q.scalars.count | q.ports.count) vm_drain();
        lds_wait_ge(&sh_hready[0], i + 1, pa.abort);
        lds_wait_ge(&sh_hready[1], i + 1, pa.abort);
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const int64_t tot = sh_hk[((0 * 2 + p) * K + j) * B + tid] + sh_hk[((1 * 2 + p) * K + j) * B + tid];
          keys[j] = fs[j] ? 0 : (((uint64_t)(tot + 1) << 40) | rkj[j]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const bool spare = spare_slot(j, K, tid, B);
          const int n = spare ? lo + cand : lo + j * B + tid;
          keys[j] = (spare ? fast_b : n < st.N) ? node_key<FM, SM>(st, q, r[j], n, tk) : 0;
        }
      }
      KGPU_STAMP(i, 5);
      wg_partials<K, B>(sh, p, keys, fast_b, ob, jb, cand, own_a, own_b);
    }
    KGPU_STAMP(i, 1);
    // the next pod's query: issued now, consumed after the barrier.  (Issued before the evaluation
    // instead, it costs config (a)'s default-profile kernel 2.77 -> 2.93 us per pod -- the query's
    // fields then stay live through the evaluation -- and gains config (b) nothing once the
    // variant-B row is read across lanes: profiles/r03_qn_bench.jsonl.)
    kgpu_pod_query qn{};
    if (i + 1 < pa.count) qn = *cp(st.queries + pa.first + i + 1);
    __syncthreads();  // (c): pod i-1 resolved and pod i published (communication wave)
    KGPU_STAMP(i, 2);
    int wg = -1;
    if (have_prev) {
      const int s = (i - 1) & 1;
      if (sh.rabort[s]) break;
      wg = sh.rwg[s];
    }
    const bool won = have_prev && wg == gme;
    // pod i's candidate: what the communication wave publishes (the same combine of the partials),
    // or -2 when pod i-1's win makes this workgroup's winning row a slow-path re-evaluation
    int cn = -1;
    if (have_cur) {
      if (won && pa.assume && !fast_b) {
        cn = -2;
      } else {
        // one row wave: its own reduction is the workgroup's (no LDS read back)
        const Cand c = W == 1 ? ((won && fast_b) ? own_b : own_a) : wg_combine<B>(sh, p, won && fast_b);
        cn = c.key ? c.idx : -1;
      }
    }
    if (won && pa.assume && tid == ob) {
#pragma unroll
      for (int j = 0; j < K; ++j)
        if (j == jb) {
          assume_row(st, qp, r[j], lo + (j * B + tid));
          assume_counts(st, pa.first + i - 1, lo + (j * B + tid));
        }
    }
    const bool slow = cn == -2;
    if (slow) {
      // pod i-1 changed memory-resident columns of this workgroup's winning row: that row's wave
      // evaluates it again and publishes from its own partial and the other waves' partials;
      // the others wait for the candidate it found
      if (wave == ob / 64) {
        if (tid == ob) {
          const uint64_t tk = pod_tie_key(st.seed, pa.seq0 + i);
#pragma unroll
          for (int j = 0; j < K; ++j)
            if (j == jb) keys[j] = node_key<FM, SM>(st, q, r[j], lo + (j * B + tid), tk);
        }
        const Cand c = wave_recombine<K, B>(sh, p, keys);
        if (lane == 0) {
          publish(i, c.key, c.feas);
          sh.cslow[p] = c.key ? c.idx : -1;
          lds_release(&sh.cready, i + 1);
        }
      }
      lds_wait(&sh.cready, i + 1, pa.abort);
      cand = sh.cslow[p];
    } else {
      cand = cn;
      if (W > 1 && cand >= 0 && tid == cand % B) {
        // stage pod i's candidate row (pod i-1 already assumed on it) for pod i+1's variant B
#pragma unroll
        for (int j = 0; j < K; ++j)
          if (j == cand / B) sh.brow[p] = r[j];
        if (i != pa.skip_release_at) lds_release(&sh.bready, i + 1);
      }
    }
    staged = have_cur && !slow && cand >= 0;
    qp = q;
    q = qn;
    KGPU_STAMP(i, 4);
  }
#undef KGPU_STAMP
}

// FeasibleNodes and the scored flag of every pod of a persistent run (generic_scheduler.go:184-191:
// a single feasible node is returned without scoring).
__global__ __launch_bounds__(256) void k_batch_fixup(const DevState* __restrict__ stp, BatchArgs pa, int G) {
  // one wave per pod: its lanes sum the pod's per-workgroup feasible counts (coalesced), where one thread
  // per pod looping over G counts took 12.7 us per 1000-pod launch at 5k nodes (profiles/r05_*)
  const DevState& st = *stp;
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  // pipelined batches: the other slot's granules, zeroed for the batch after next (its last reader, that
  // slot's previous fixup, finished before this run's k_batch started)
  for (int64_t z = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; z < pa.zero_n16; z += (int64_t)gridDim.x * blockDim.x) {
    uint4* zp = reinterpret_cast<uint4*>(pa.zero_buf) + z;
    *zp = uint4{0, 0, 0, 0};
  }
  if (pa.abort_out && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(pa.abort_out, load_sc1(pa.abort), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (i >= pa.count) return;
  const size_t row = pa.R > 0 ? (size_t)((pa.xseq0 + i) % pa.R) : (size_t)i;
  int f = 0;
  for (int g = lane; g < pa.GT; g += 64) f += pa.feas[row * pa.GT + g];
  f = (int)wave_sum32((uint32_t)f);
  (void)G;
  if (lane == 0) {
    kgpu_result& r = gp(st.results)[pa.first + i];
    r.feasible = f;
    if (r.node >= 0 && f >= 2) {
      r.scored = 1;
    } else {
      r.scored = 0;
      r.score = 0;
    }
    if (pa.res_out) pa.res_out[pa.first + i] = r;
  }
}

// ---------------------------------------------------------------- topology pipeline
// PodTopologySpread (podtopologyspread/{filtering,scoring}.go), InterPodAffinity
// (interpodaffinity/{filtering,scoring}.go) and DefaultPodTopologySpread
// (default_pod_topology_spread.go) for one pod, as a chain of launches over the eval grid:
//   k_topo_pre      one pass over the nodes: topologyPair -> count histograms built from the
//                   match-count columns (the PreFilter maps and the PreScore counts), global
//                   atomics into the pod's scratch
//   k_topo_min      criticalPaths minimum per DoNotSchedule constraint (filtering.go:93-121)
//   k_topo_filter   every Filter plugin in profile order (PTS / IPA read the histograms), the
//                   non-topology scores, ScheduleAnyway pair registration (scoring.go:83-102)
//   k_topo_score    PTS / IPA / DPTS raw scores of the feasible nodes, their min / max / zone sums
//   k_topo_final    NormalizeScore of every plugin, weights, packed-key argmax per workgroup
//   k_topo_resolve  selectHost over the partials, assume (node row + match counts), zero the next
//                   pod's scratch
__device__ __forceinline__ int nval(const DevState& st, int k, int n) {
  return k >= 0 ? gp(st.label_val)[(size_t)k * st.N + n] : -1;
}
__device__ __forceinline__ int64_t* slot_ptr(const DevState& st, const QPlan& pl, int slot) {
  return st.scratch + pl.slot_off[slot];
}
__device__ __forceinline__ TopoHdr* hdr(const DevState& st) { return reinterpret_cast<TopoHdr*>(st.scratch); }
__device__ __forceinline__ int64_t* zone_sums(const DevState& st) { return st.scratch + kHdrWords; }
__device__ __forceinline__ void add64(int64_t* p, int64_t v) {
  atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v);
}
// order-preserving encodings for atomicMax on zero-initialized words
__device__ __forceinline__ unsigned long long enc_max(int64_t x) { return (unsigned long long)x ^ (1ull << 63); }
__device__ __forceinline__ void amax64(int64_t* p, int64_t x) {
  atomicMax(reinterpret_cast<unsigned long long*>(p), enc_max(x));
}
__device__ __forceinline__ void amin64(int64_t* p, int64_t x) {
  atomicMax(reinterpret_cast<unsigned long long*>(p), ~enc_max(x));
}
__device__ __forceinline__ int64_t read_max(const int64_t* p) {  // INT64_MIN when never set
  const unsigned long long u = *reinterpret_cast<const unsigned long long*>(p);
  return u ? (int64_t)(u ^ (1ull << 63)) : INT64_MIN;
}
__device__ __forceinline__ int64_t read_min(const int64_t* p) {  // INT64_MAX when never set
  const unsigned long long u = *reinterpret_cast<const unsigned long long*>(p);
  return u ? (int64_t)(~u ^ (1ull << 63)) : INT64_MAX;
}

__device__ __forceinline__ bool all_keys(const DevState& st, const TSpread* c, int nc, int n) {
  for (int i = 0; i < nc; ++i)
    if (nval(st, c[i].key, n) < 0) return false;
  return true;
}

// PodTopologySpread / InterPodAffinity Filter on the histograms of k_topo_pre / k_topo_min.
__device__ uint32_t topo_filter(int f, const DevState& st, const QPlan& pl, int n) {
  const TopoHdr* h = hdr(st);
  if (f == KGPU_F_POD_TOPOLOGY_SPREAD) {  // filtering.go:276-328
    if (pl.n_hard == 0 || !h->pany) return 0;
    for (int i = 0; i < pl.n_hard; ++i) {
      const TSpread& c = pl.hard[i];
      const int v = nval(st, c.key, n);
      if (v < 0) return KGPU_CODE_UNSCHEDULABLE << 8;
      const int64_t match = slot_ptr(st, pl, c.rslot)[v] ? slot_ptr(st, pl, c.cslot)[v] : 0;
      int64_t mn = read_min(&h->pmin[i]);
      if (mn == INT64_MAX) mn = 2147483647;  // criticalPaths initial MatchNum (math.MaxInt32)
      if (match + c.self_match - mn > c.max_skew) return KGPU_CODE_UNSCHEDULABLE << 8;
    }
    return 0;
  }
  if (f == KGPU_F_INTER_POD_AFFINITY) {  // filtering.go:314-396
    bool exist = true;
    for (int i = 0; i < pl.n_aff; ++i) {  // satisfyPodAffinity
      const int v = nval(st, pl.aff[i].key, n);
      if (v < 0) return (KGPU_CODE_UNRESOLVABLE << 8) | (1u << 16);
      if (slot_ptr(st, pl, pl.aff[i].slot)[v] <= 0) exist = false;
    }
    if (!exist && !(!h->aff_any && pl.self_all)) return (KGPU_CODE_UNRESOLVABLE << 8) | (1u << 16);
    for (int i = 0; i < pl.n_anti; ++i) {  // satisfyPodAntiAffinity
      const int v = nval(st, pl.anti[i].key, n);
      if (v >= 0 && slot_ptr(st, pl, pl.anti[i].slot)[v] > 0) return (KGPU_CODE_UNSCHEDULABLE << 8) | (2u << 16);
    }
    if (h->ex_any) {  // satisfyExistingPodsAntiAffinity: every node label pair
      for (int s = 0; s < pl.n_slots; ++s) {
        if (pl.slot_kind[s] != kSlotExA) continue;
        const int v = nval(st, pl.slot_key[s], n);
        if (v >= 0 && slot_ptr(st, pl, s)[v] > 0) return (KGPU_CODE_UNSCHEDULABLE << 8) | (3u << 16);
      }
    }
    return 0;
  }
  return 0;
}

__device__ __forceinline__ void topo_pre(const DevState* __restrict__ stp, PodArgs a) {
  const DevState& st = *stp;
  const QPlan& pl = st.plans[a.pod];
  const kgpu_pod_query q = *cp(st.queries + a.pod);
  TopoHdr* h = hdr(st);
  int lo, hi;
  chunk_of(st.N, lo, hi);
  bool pany = false, ex_any = false, aff_any = false;
  for (int n = lo + threadIdx.x; n < hi; n += kBlock) {
    const bool aff_ok = (pl.n_hard || pl.n_soft) ? node_affinity_ok(st, q, n) : false;
    // PreFilter TpPairToMatchNum (filtering.go:198-273): eligible pairs, then counts over all nodes
    if (pl.n_hard) {
      if (aff_ok && all_keys(st, pl.hard, pl.n_hard, n)) {
        for (int i = 0; i < pl.n_hard; ++i) slot_ptr(st, pl, pl.hard[i].rslot)[nval(st, pl.hard[i].key, n)] = 1;
        pany = true;
      }
      for (int i = 0; i < pl.n_hard; ++i) {
        const TSpread& c = pl.hard[i];
        if (c.key < 0) continue;
        int v = nval(st, c.key, n);
        if (v < 0) v = gp(st.key_empty)[c.key];  // node.Labels[key] of a missing key is ""
        const int cnt = gp(st.mcnt)[(size_t)c.cls * st.N + n];
        if (v >= 0 && cnt) add64(slot_ptr(st, pl, c.cslot) + v, cnt);
      }
    }
    // PreScore counts (scoring.go:145-167): nodes matching affinity and carrying every key
    if (pl.n_soft && aff_ok && all_keys(st, pl.soft, pl.n_soft, n)) {
      for (int i = 0; i < pl.n_soft; ++i) {
        const TSpread& c = pl.soft[i];
        if (c.is_hostname) continue;
        const int cnt = gp(st.mcnt)[(size_t)c.cls * st.N + n];
        if (cnt) add64(slot_ptr(st, pl, c.cslot) + nval(st, c.key, n), cnt);
      }
    }
    // InterPodAffinity PreFilter maps (filtering.go:166-271) and PreScore topologyScore (scoring.go:47-199)
    for (int j = 0; j < pl.ex.count; ++j) {
      const TTerm t = st.aux_terms[pl.ex.begin + j];
      const int v = nval(st, t.key, n);
      if (v < 0) continue;
      const int cnt = gp(st.tcnt)[(size_t)t.cls * st.N + n];
      if (!cnt) continue;
      if (j < pl.n_ex_anti) {
        add64(slot_ptr(st, pl, t.slot) + v, cnt);
        ex_any = true;
      } else {
        add64(slot_ptr(st, pl, t.slot) + v, (int64_t)t.weight * cnt);
      }
    }
    if (pl.n_aff) {
      const int cnt = gp(st.mcnt)[(size_t)pl.conj_cls * st.N + n];
      if (cnt) {
        for (int i = 0; i < pl.n_aff; ++i) {
          const int v = nval(st, pl.aff[i].key, n);
          if (v < 0) continue;
          add64(slot_ptr(st, pl, pl.aff[i].slot) + v, cnt);
          aff_any = true;
        }
      }
    }
    for (int i = 0; i < pl.n_anti; ++i) {
      const int v = nval(st, pl.anti[i].key, n);
      const int cnt = gp(st.mcnt)[(size_t)pl.anti[i].cls * st.N + n];
      if (v >= 0 && cnt) add64(slot_ptr(st, pl, pl.anti[i].slot) + v, cnt);
    }
    for (int i = 0; i < pl.n_pref; ++i) {
      const int v = nval(st, pl.pref[i].key, n);
      const int cnt = gp(st.mcnt)[(size_t)pl.pref[i].cls * st.N + n];
      if (v >= 0 && cnt) add64(slot_ptr(st, pl, pl.pref[i].slot) + v, (int64_t)pl.pref[i].weight * cnt);
    }
  }
  if (__any(pany) && threadIdx.x == 0) h->pany = 1;
  if (__any(ex_any) && threadIdx.x == 0) h->ex_any = 1;
  if (__any(aff_any) && threadIdx.x == 0) h->aff_any = 1;
}

// criticalPaths[0].MatchNum per DoNotSchedule constraint: minimum count over the registered pairs
// of its key (MaxInt32 when none), grid-stride over the key's values.
__device__ __forceinline__ void topo_min(const DevState* __restrict__ stp, PodArgs a) {
  const DevState& st = *stp;
  const QPlan& pl = st.plans[a.pod];
  TopoHdr* h = hdr(st);
  for (int i = 0; i < pl.n_hard; ++i) {
    const TSpread& c = pl.hard[i];
    const int nv = c.key >= 0 ? gp(st.key_n_values)[c.key] : 0;
    int64_t mn = INT64_MAX;
    const int64_t* reg = slot_ptr(st, pl, c.rslot);
    const int64_t* cnt = slot_ptr(st, pl, c.cslot);
    for (int v = blockIdx.x * kBlock + threadIdx.x; v < nv; v += gridDim.x * kBlock)
      if (reg[v] && cnt[v] < mn) mn = cnt[v];
    mn = wave_min_i64(mn);
    if (threadIdx.x == 0 && mn != INT64_MAX) amin64(&h->pmin[i], mn);
  }
}

// initPreScoreState for one filtered node (scoring.go:83-102): ignored when a soft key is missing,
// else register its ScheduleAnyway pairs (topoSize counts first registrations).  Returns 1 if the
// node is not ignored.
__device__ __forceinline__ int soft_register(const DevState& st, const QPlan& pl, int n) {
  if (!pl.n_soft || !all_keys(st, pl.soft, pl.n_soft, n)) return 0;
  TopoHdr* h = hdr(st);
  for (int i = 0; i < pl.n_soft; ++i) {
    const TSpread& c = pl.soft[i];
    if (c.is_hostname) continue;
    int64_t* reg = slot_ptr(st, pl, c.rslot) + nval(st, c.key, n);
    const unsigned long long old = atomicExch(reinterpret_cast<unsigned long long*>(reg), 1ull);
    // node-sharded: a pair may first register on several ranks; k_topo_ssize counts the summed bins
    if (old == 0 && c.first_of_key && !st.shard_keys) add64(&h->ssize[i], 1);
  }
  return 1;
}

// ScheduleAnyway registration over the feasible set kept by k_cut.
__device__ __forceinline__ void topo_reg(const DevState* __restrict__ stp, PodArgs a) {
  const DevState& st = *stp;
  const QPlan& pl = st.plans[a.pod];
  int lo, hi;
  chunk_of(st.N, lo, hi);
  int nonign = 0;
  for (int n = lo + threadIdx.x; n < hi; n += kBlock)
    if (gp(st.status)[n] == 0) nonign += soft_register(st, pl, n);
  nonign = wave_reduce_sum(nonign);
  if (threadIdx.x == 0 && nonign) atomicAdd(&hdr(st)->feas_nonign, nonign);
}

// Filters + the non-topology scores; the feasible set's ScheduleAnyway pairs and sizes.
__device__ __forceinline__ void topo_filter(const DevState* __restrict__ stp, PodArgs a) {
  const DevState& st = *stp;
  const QPlan& pl = st.plans[a.pod];
  const kgpu_pod_query q = *cp(st.queries + a.pod);
  TopoHdr* h = hdr(st);
  QPlan const* plp = &pl;
  int lo, hi;
  chunk_of(st.N, lo, hi);
  int feas = 0, maxT = 0, maxNA = 0, nonign = 0;
  for (int n = lo + threadIdx.x; n < hi; n += kBlock) {
    NodeRes r = load_res(st, n);
    NodeEval e{0, 0, 0, 0};
    const uint32_t s1 = st.nom_status ? gp(st.nom_status)[n] : 0u;
    e.status = s1 ? s1 : run_filters<kRuntime>(st, q, r, n, plp);
    if (e.status == 0) {
      int64_t part = 0;
      for (int i = 0; i < st.n_scores; ++i) {
        const int s = cp(st.scores)[i];
        if (s == KGPU_S_POD_TOPOLOGY_SPREAD || s == KGPU_S_INTER_POD_AFFINITY ||
            s == KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD)
          continue;  // k_topo_score / k_topo_final
        const int64_t v = score_one<false>(s, st, q, r, n, e);
        if (a.diag) {
          gp(st.diag_raw)[(size_t)s * st.N + n] = v;
          if (!normalized(s)) gp(st.diag_norm)[(size_t)s * st.N + n] = v;  // topo_final writes the others
        }
        if (!normalized(s)) part += v * cp(st.w_of)[s];
      }
      e.partial = part;
      ++feas;
      maxT = max(maxT, e.taint);
      maxNA = max(maxNA, e.na);
      // PTS PreScore over the filtered nodes (scoring.go:83-102): pairs, sizes, ignored nodes
      // (after k_cut when the feasible set is trimmed: k_topo_reg)
      if (!a.cut) nonign += soft_register(st, pl, n);
    }
    gp(st.status)[n] = e.status;
    gp(st.partial)[n] = e.partial;
    gp(st.raw_taint)[n] = e.taint;
    gp(st.raw_na)[n] = e.na;
  }
  feas = wave_reduce_sum(feas);
  maxT = wave_reduce_max(maxT);
  maxNA = wave_reduce_max(maxNA);
  nonign = wave_reduce_sum(nonign);
  if (threadIdx.x == 0) {
    gp(st.sbuf)[(size_t)a.parity * kMaxBlocks + blockIdx.x] = BlkStat{feas, maxT, maxNA, 0};
    if (nonign) atomicAdd(&h->feas_nonign, nonign);
  }
}

// Raw PodTopologySpread (scoring.go:174-208), InterPodAffinity (scoring.go:217-236) and
// DefaultPodTopologySpread (default_pod_topology_spread.go:75-106) scores of the feasible nodes.
__device__ __forceinline__ void topo_score(const DevState* __restrict__ stp, PodArgs a) {
  const DevState& st = *stp;
  const QPlan& pl = st.plans[a.pod];
  TopoHdr* h = hdr(st);
  int lo, hi;
  chunk_of(st.N, lo, hi);
  double w[kMaxSpread];
  for (int i = 0; i < pl.n_soft; ++i) {  // topologyNormalizingWeight (scoring.go:286-288)
    const int64_t sz = pl.soft[i].is_hostname ? (int64_t)h->feas_nonign : (pl.soft[i].first_of_key ? h->ssize[i] : 0);
    w[i] = st.log_table[sz + 2];
  }
  int64_t pmn = INT64_MAX, pmx = INT64_MIN, imn = INT64_MAX, imx = INT64_MIN, dmx = 0;
  bool zoned = false;
  for (int n = lo + threadIdx.x; n < hi; n += kBlock) {
    if (gp(st.status)[n] != 0) continue;
    // PodTopologySpread
    int64_t ps = 0;
    if (pl.n_soft && !all_keys(st, pl.soft, pl.n_soft, n)) {
      ps = INT64_MIN;  // ignored node
    } else {
      double score = 0;
      for (int i = 0; i < pl.n_soft; ++i) {
        const TSpread& c = pl.soft[i];
        const int v = nval(st, c.key, n);
        int64_t cnt = c.is_hostname ? (int64_t)gp(st.mcnt)[(size_t)c.cls * st.N + n] : slot_ptr(st, pl, c.cslot)[v];
        if (cnt < c.max_skew) cnt = c.max_skew - 1;  // adjustForMaxSkew
        score += (double)cnt * w[i];
      }
      ps = (int64_t)score;
      pmn = min(pmn, ps);
      pmx = max(pmx, ps);
    }
    // InterPodAffinity: sum over the topologyScore keys the node carries
    int64_t is = 0;
    for (int s = 0; s < pl.n_slots; ++s) {
      if (pl.slot_kind[s] != kSlotTopo) continue;
      const int v = nval(st, pl.slot_key[s], n);
      if (v >= 0) is += slot_ptr(st, pl, s)[v];
    }
    imn = min(imn, is);
    imx = max(imx, is);
    // DefaultPodTopologySpread
    int64_t ds = 0;
    if (pl.dpts_cls >= 0) ds = gp(st.mcnt)[(size_t)pl.dpts_cls * st.N + n];
    dmx = max(dmx, ds);
    const int z = gp(st.zone_id)[n];
    if (z >= 0) {
      zoned = true;
      if (ds) add64(zone_sums(st) + z, ds);
    }
    gp(st.raw_pts)[n] = ps;
    gp(st.raw_ipa)[n] = is;
    gp(st.raw_dpts)[n] = ds;
    if (a.diag) {
      gp(st.diag_raw)[(size_t)KGPU_S_POD_TOPOLOGY_SPREAD * st.N + n] = ps == INT64_MIN ? 0 : ps;
      gp(st.diag_raw)[(size_t)KGPU_S_INTER_POD_AFFINITY * st.N + n] = is;
      gp(st.diag_raw)[(size_t)KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD * st.N + n] = pl.dpts_cls == -2 ? 0 : ds;
    }
  }
  pmn = wave_min_i64(pmn);
  pmx = wave_max_i64(pmx);
  imn = wave_min_i64(imn);
  imx = wave_max_i64(imx);
  dmx = wave_max_i64(dmx);
  const bool zw = __any(zoned);
  if (threadIdx.x == 0) {
    if (pmx != INT64_MIN) {
      amin64(&h->pts_min, pmn);
      amax64(&h->pts_max, pmx);
    }
    if (imx != INT64_MIN) {
      amin64(&h->ipa_min, imn);
      amax64(&h->ipa_max, imx);
    }
    if (dmx) amax64(&h->dpts_max, dmx);
    if (zw) h->have_zones = 1;
  }
}

// NormalizeScore of every plugin (framework.go:613-648), total, packed-key argmax per workgroup.
__device__ __forceinline__ void topo_final(const DevState* __restrict__ stp, PodArgs a, int stat_blocks) {
  const DevState& st = *stp;
  const QPlan& pl = st.plans[a.pod];
  const TopoHdr* h = hdr(st);
  int maxT = 0, maxNA = 0;
  // sharded: the maxima over the whole cluster's feasible set, one all-gathered record per rank
  const GAS BlkStat* sb = st.shard_stats ? gp(st.shard_stats) + (size_t)a.parity * kMaxRanks
                                         : gp(st.sbuf) + (size_t)a.parity * kMaxBlocks;
  if (st.shard_stats) stat_blocks = st.nranks;
  for (int b = threadIdx.x; b < stat_blocks; b += kBlock) {
    const BlkStat p = sb[b];
    maxT = max(maxT, p.max_taint);
    maxNA = max(maxNA, p.max_na);
  }
  maxT = wave_reduce_max(maxT);
  maxNA = wave_reduce_max(maxNA);
  // PTS (scoring.go:211-257): min / max over the non-ignored nodes
  const int64_t pmx0 = read_max(&h->pts_max), pmn0 = read_min(&h->pts_min);
  const int64_t pmx = pmx0 == INT64_MIN ? 0 : max(pmx0, (int64_t)0);
  const int64_t pmn = pmn0;
  // IPA (scoring.go:241-272): min and max start at 0
  const int64_t imx = max(read_max(&h->ipa_max), (int64_t)0), imn = min(read_min(&h->ipa_min), (int64_t)0);
  const int64_t idiff = imx - imn;
  // DPTS (default_pod_topology_spread.go:109-163)
  const int64_t dmax_node = max(read_max(&h->dpts_max), (int64_t)0);
  int64_t dmax_zone = 0;
  if (pl.dpts_cls >= 0 && h->have_zones)
    for (int z = threadIdx.x; z < st.n_zones; z += kBlock) dmax_zone = max(dmax_zone, zone_sums(st)[z]);
  dmax_zone = wave_max_i64(dmax_zone);
  const double M = 100.0, zwt = 2.0 / 3.0;
  int lo, hi;
  chunk_of(st.N, lo, hi);
  const uint64_t tk = pod_tie_key(st.seed, a.seq);
  uint64_t best = 0;
  int best_i = -1, bf = 0;
  for (int n = lo + threadIdx.x; n < hi; n += kBlock) {
    if (gp(st.status)[n] != 0) continue;
    ++bf;
    const int taint = gp(st.raw_taint)[n], na = gp(st.raw_na)[n];
    const int64_t vt = maxT == 0 ? 100 : 100 - (100 * (int64_t)taint) / maxT;
    const int64_t vn = maxNA == 0 ? (int64_t)na : (100 * (int64_t)na) / maxNA;
    const int64_t ps = gp(st.raw_pts)[n];
    int64_t vp;
    if (ps == INT64_MIN) vp = 0;
    else if (pmx == 0) vp = 100;
    else vp = 100 * (pmx + pmn - ps) / pmx;
    const int64_t is = gp(st.raw_ipa)[n];
    const int64_t vi = idiff > 0 ? (int64_t)(M * ((double)(is - imn) / (double)idiff)) : 0;
    int64_t vd = 0;
    if (pl.dpts_cls != -2) {
      const int64_t ds = gp(st.raw_dpts)[n];
      double f = M;
      if (dmax_node > 0) f = M * ((double)(dmax_node - ds) / (double)dmax_node);
      const int z = gp(st.zone_id)[n];
      if (h->have_zones && z >= 0) {
        double zs = M;
        if (dmax_zone > 0) zs = M * ((double)(dmax_zone - zone_sums(st)[z]) / (double)dmax_zone);
        f = (f * (1.0 - zwt)) + (zwt * zs);
      }
      vd = (int64_t)f;
    }
    int64_t total = gp(st.partial)[n] + vt * st.w_of[KGPU_S_TAINT_TOLERATION] + vn * st.w_of[KGPU_S_NODE_AFFINITY] +
                    vp * st.w_of[KGPU_S_POD_TOPOLOGY_SPREAD] + vi * st.w_of[KGPU_S_INTER_POD_AFFINITY] +
                    vd * st.w_of[KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD];
    if (st.n_scores == 0) total = 1;
    const uint64_t key = ((uint64_t)total << 40) | rank40(tk, (uint64_t)(st.node_base + n), st.tie_mode);
    key_max(best, best_i, key, n);
    if (a.diag) {
      // the normalized and topology plugins only (run_scores wrote the others' normalized rows)
      for (int i = 0; i < st.n_scores; ++i) {
        const int s = st.scores[i];
        int64_t v;
        if (s == KGPU_S_TAINT_TOLERATION) v = vt;
        else if (s == KGPU_S_NODE_AFFINITY) v = vn;
        else if (s == KGPU_S_POD_TOPOLOGY_SPREAD) v = vp;
        else if (s == KGPU_S_INTER_POD_AFFINITY) v = vi;
        else if (s == KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD) v = vd;
        else continue;
        gp(st.diag_norm)[(size_t)s * st.N + n] = v;
      }
    }
  }
  wave_reduce_key(best, best_i);
  bf = wave_reduce_sum(bf);
  if (threadIdx.x == 0) gp(st.kbuf)[(size_t)a.parity * kMaxBlocks + blockIdx.x] = BlkKey{best, best_i, bf};
}

// selectHost + assume of the topology pod, then zero the next topology pod's scratch.
__device__ __forceinline__ void topo_resolve(const DevState* __restrict__ stp, PodArgs a,
                                                         int64_t next_scratch) {
  const DevState& st = *stp;
  int lo, hi;
  chunk_of(st.N, lo, hi);
  int gidx;
  const Winner w = prev_winner(st, a, &gidx);
  const kgpu_pod_query pq = *cp(st.queries + a.prev);
  const int idx = settle_prev(st, a, pq, w, gidx, blockIdx.x == 0 && threadIdx.x == 0);
  if (idx >= lo && idx < hi && ((idx - lo) % kBlock) == (int)threadIdx.x) {
    NodeRes r = load_res(st, idx);
    assume_row(st, pq, r, idx);
    assume_counts(st, a.prev, idx);
  }
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < next_scratch; i += (int64_t)gridDim.x * kBlock)
    st.scratch[i] = 0;
}

// Node-sharded topology pods: topoSize of each ScheduleAnyway key (scoring.go:92-99) as the number of
// registered pairs, counted after the ranks' registration slots were summed.
__global__ __launch_bounds__(kBlock) void k_topo_ssize(const DevState* __restrict__ stp, PodArgs a) {
  const DevState& st = *stp;
  const QPlan& pl = st.plans[a.pod];
  TopoHdr* h = hdr(st);
  for (int i = 0; i < pl.n_soft; ++i) {
    const TSpread& c = pl.soft[i];
    if (c.is_hostname || !c.first_of_key || c.key < 0) continue;
    const int nv = gp(st.key_n_values)[c.key];
    const int64_t* reg = slot_ptr(st, pl, c.rslot);
    int k = 0;
    for (int v = blockIdx.x * kBlock + threadIdx.x; v < nv; v += gridDim.x * kBlock) k += reg[v] != 0;
    k = wave_reduce_sum(k);
    if (threadIdx.x == 0 && k) add64(&h->ssize[i], k);
  }
}

__global__ __launch_bounds__(kBlock) void k_topo_pre(const DevState* __restrict__ stp, PodArgs a) { topo_pre(stp, a); }
__global__ __launch_bounds__(kBlock) void k_topo_min(const DevState* __restrict__ stp, PodArgs a) { topo_min(stp, a); }
__global__ __launch_bounds__(kBlock) void k_topo_filter(const DevState* __restrict__ stp, PodArgs a) { topo_filter(stp, a); }
__global__ __launch_bounds__(kBlock) void k_topo_score(const DevState* __restrict__ stp, PodArgs a) { topo_score(stp, a); }
__global__ __launch_bounds__(kBlock) void k_topo_reg(const DevState* __restrict__ stp, PodArgs a) { topo_reg(stp, a); }
__global__ __launch_bounds__(kBlock) void k_topo_final(const DevState* __restrict__ stp, PodArgs a, int stat_blocks) { topo_final(stp, a, stat_blocks); }
__global__ __launch_bounds__(kBlock) void k_topo_resolve(const DevState* __restrict__ stp, PodArgs a,
                                                         int64_t next_scratch) {
  topo_resolve(stp, a, next_scratch);
}

// The whole per-pod topology pipeline in ONE cooperative launch: the six phases above separated
// by grid-wide barriers instead of kernel boundaries (the grid is <= kMaxBlocks one-wave
// workgroups; hipLaunchCooperativeKernel refuses a grid that cannot be co-resident).
// Grid barrier on a counter that only ever grows: the host passes the number of arrivals before
// this launch (`base`), so barrier i of the launch waits for base + i * gridDim.x.  Agent-scope
// fences publish / acquire the phase's writes across XCDs; the polling load is an agent-scope
// atomic, so it is served coherently and never from a stale cache line.
__device__ __forceinline__ void grid_barrier(unsigned long long* ctr, unsigned long long target) {
  __threadfence();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
  __threadfence();
}

__global__ __launch_bounds__(kBlock) void k_topo_fused(const DevState* __restrict__ stp, PodArgs a, int do_min,
                                                       int64_t next_scratch, unsigned long long* bar,
                                                       unsigned long long base) {
  const unsigned long long g = gridDim.x;
  unsigned long long t = base;
  topo_pre(stp, a);
  grid_barrier(bar, t += g);
  if (do_min) {
    topo_min(stp, a);
    grid_barrier(bar, t += g);
  }
  topo_filter(stp, a);
  grid_barrier(bar, t += g);
  topo_score(stp, a);
  grid_barrier(bar, t += g);
  topo_final(stp, a, (int)gridDim.x);
  grid_barrier(bar, t += g);
  PodArgs r = a;
  r.prev = a.pod;
  r.prev_blocks = (int)gridDim.x;
  r.prev_parity = a.parity;
  topo_resolve(stp, r, next_scratch);
}

// Pod class membership of the pod-table rows (labels.Selector.Matches, selector.go:198-242;
// util/topologies.go:40-49), accumulated into fresh mcnt columns.
__device__ bool pod_item_match(const DevState& st, const ClassItem& it, int p) {
  const int ns = gp(st.pod_ns)[p];
  bool in_ns = false;
  for (int i = 0; i < it.ns.count; ++i) in_ns |= (st.cints[it.ns.begin + i] == ns);
  if (!in_ns || it.sel.kind != KGPU_SEL_AND) return false;
  for (int i = 0; i < it.sel.reqs.count; ++i) {
    const kgpu_req rq = st.creqs[it.sel.reqs.begin + i];
    const int v = (rq.key >= 0 && rq.key < st.PKcap) ? gp(st.pod_lab)[(size_t)rq.key * st.Pcap + p] : -1;
    bool in = false;
    for (int j = 0; j < rq.vals.count; ++j) in |= (st.cints[rq.vals.begin + j] == v);
    switch (rq.op) {
      case KGPU_OP_IN: if (!(v >= 0 && in)) return false; break;
      case KGPU_OP_NOTIN: if (v >= 0 && in) return false; break;
      case KGPU_OP_EXISTS: if (v < 0) return false; break;
      case KGPU_OP_DNE: if (v >= 0) return false; break;
      default: return false;
    }
  }
  return true;
}

__global__ void k_class_init(const DevState* __restrict__ stp, int c0, int nc, int n_pods) {
  const DevState& st = *stp;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pods) return;
  const uint32_t fl = gp(st.pod_flags)[p];
  if (!(fl & KGPU_PF_ACTIVE)) return;
  const int n = gp(st.pod_node)[p] - st.node_base;
  if (n < 0 || n >= st.N) return;
  for (int c = c0; c < c0 + nc; ++c) {
    const ClassRec cr = st.classes[c];
    if (cr.excl_terminating && (fl & KGPU_PF_TERMINATING)) continue;
    bool ok = cr.n_items > 0;
    for (int i = 0; i < cr.n_items && ok; ++i) ok = pod_item_match(st, st.class_items[cr.item0 + i], p);
    if (ok) atomicAdd(gp(st.mcnt) + (size_t)c * st.N + n, 1);
  }
}

__global__ void k_vict_prep(const DevState* __restrict__ stp, const PreemptArgs* __restrict__ ap);
__global__ void k_victims(const DevState* __restrict__ stp, const PreemptArgs* __restrict__ ap);

int launch_topo(const DevState* st, PodArgs a, int blocks, int64_t min_values, int64_t next_scratch,
                bool fused, unsigned long long* bar, unsigned long long bar_base, int n_filters, void* stream,
                const PreemptArgs* nom, int N) {
  hipStream_t s = (hipStream_t)stream;
  if (fused && !a.cut && !nom) {
    int do_min = min_values > 0 ? 1 : 0;
    void* args[] = {(void*)&st, (void*)&a, (void*)&do_min, (void*)&next_scratch, (void*)&bar, (void*)&bar_base};
    return hipLaunchCooperativeKernel((const void*)k_topo_fused, dim3(blocks), dim3(kBlock), args, 0, s) == hipSuccess
               ? 0 : -1;
  }
  hipLaunchKernelGGL(k_topo_pre, dim3(blocks), dim3(kBlock), 0, s, st, a);
  if (min_values > 0) {
    int64_t mb = (min_values + kBlock - 1) / kBlock;
    if (mb > kMaxBlocks) mb = kMaxBlocks;
    hipLaunchKernelGGL(k_topo_min, dim3((int)mb), dim3(kBlock), 0, s, st, a);
  }
  if (nom) {  // nominated pods: pass 1 on the PreFilter histograms, before the filter phase reads it
    hipLaunchKernelGGL(k_vict_prep, dim3(kMaxSpread + 1), dim3(256), 0, s, st, nom);
    hipLaunchKernelGGL(k_victims, dim3((N + 63) / 64), dim3(64), 0, s, st, nom);
  }
  hipLaunchKernelGGL(k_topo_filter, dim3(blocks), dim3(kBlock), 0, s, st, a);
  if (a.cut) {
    hipLaunchKernelGGL(k_cut, dim3(1), dim3(kCutThreads), 0, s, st, a, blocks, n_filters);
    hipLaunchKernelGGL(k_topo_reg, dim3(blocks), dim3(kBlock), 0, s, st, a);
  }
  hipLaunchKernelGGL(k_topo_score, dim3(blocks), dim3(kBlock), 0, s, st, a);
  hipLaunchKernelGGL(k_topo_final, dim3(blocks), dim3(kBlock), 0, s, st, a, blocks);
  PodArgs r = a;
  r.prev = a.pod;
  r.prev_blocks = blocks;
  r.prev_parity = a.parity;
  hipLaunchKernelGGL(k_topo_resolve, dim3(blocks), dim3(kBlock), 0, s, st, r, next_scratch);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// One phase of the per-pod topology pipeline, for the node-sharded sequence the host interleaves
// with RCCL exchanges (kgpu_api.cpp run_topo_sharded).  extra: min_values (phase 1), stat blocks
// (5), next pod's scratch length (6).
int launch_topo_phase(const DevState* st, const PodArgs& a, int phase, int blocks, int64_t extra, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (phase) {
    case 0: hipLaunchKernelGGL(k_topo_pre, dim3(blocks), dim3(kBlock), 0, s, st, a); break;
    case 1: {
      int64_t mb = (extra + kBlock - 1) / kBlock;
      if (mb > kMaxBlocks) mb = kMaxBlocks;
      if (mb > 0) hipLaunchKernelGGL(k_topo_min, dim3((int)mb), dim3(kBlock), 0, s, st, a);
      break;
    }
    case 2: hipLaunchKernelGGL(k_topo_filter, dim3(blocks), dim3(kBlock), 0, s, st, a); break;
    case 3: hipLaunchKernelGGL(k_topo_ssize, dim3(blocks), dim3(kBlock), 0, s, st, a); break;
    case 4: hipLaunchKernelGGL(k_topo_score, dim3(blocks), dim3(kBlock), 0, s, st, a); break;
    case 5: hipLaunchKernelGGL(k_topo_final, dim3(blocks), dim3(kBlock), 0, s, st, a, (int)extra); break;
    default: {
      PodArgs r = a;
      r.prev = a.pod;
      r.prev_blocks = blocks;
      r.prev_parity = a.parity;
      hipLaunchKernelGGL(k_topo_resolve, dim3(blocks), dim3(kBlock), 0, s, st, r, extra);
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_debug_broken_linear(const kgpu_shape_point* pts, int n_pts, const int64_t* p, int64_t* out, int n,
                               void* stream) {
  if (n_pts <= 0 || n_pts > 16 || n <= 0) return -1;
  ShapeProbe s{};
  for (int i = 0; i < n_pts; ++i) s.pts[i] = pts[i];
  s.n = n_pts;
  hipLaunchKernelGGL(k_dbg_broken_linear, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, s, p, out, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_class_init(const DevState* st, int c0, int nc, int n_pods, void* stream) {
  if (n_pods <= 0 || nc <= 0) return 0;
  hipLaunchKernelGGL(k_class_init, dim3((n_pods + 255) / 256), dim3(256), 0, (hipStream_t)stream, st, c0, nc, n_pods);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------- persistent topology kernel
// (kgpu_internal.h "persistent topology kernel").  Reference semantics, per plugin:
//   PodTopologySpread  PreFilter/Filter podtopologyspread/filtering.go:146-328 (TpPairToMatchNum,
//                      criticalPaths, skew), PreScore/Score/Normalize scoring.go:59-257
//   InterPodAffinity   PreFilter/Filter interpodaffinity/filtering.go:166-396,
//                      PreScore/Score/Normalize scoring.go:47-272
//   DefaultPodTopologySpread default_pod_topology_spread.go:75-163
// Every per-cycle map of those plugins is read from a domain histogram (THist) instead of being
// rebuilt: TpPairToMatchNum[(k, v)] = sum over the pod's DoNotSchedule constraints on k of
// H[v] (+ the key-missing bin when v is "", since node.Labels[k] of a missing key is ""), the
// affinity maps are H[...] > 0, topologyScore[k][v] = sum of weight * H[v].

__device__ __forceinline__ bool tb_elig(const TBatchArgs& ta, int sig, int n) {
  const TSig sg = cp(ta.sigs)[sig];
  return (gp(ta.elig)[sg.elig_word + (n >> 5)] >> (n & 31)) & 1u;
}

// One pass per node at the start of a run:
//  * signature bitmaps: nodes a pod's nodeSelector / required NodeAffinity admits that carry every key
//    of the signature (filtering.go:229-238, scoring.go:143-150), and the DoNotSchedule pair
//    registrations of each (signature, key) (filtering.go:239-243);
//  * domain histograms (and their totals over the nodes carrying the key) from the columns, counted
//    only over the nodes the histogram's signature admits -- read from the node's own bits in a
//    register (a run has at most 64 signatures), not back from the bitmap.
__device__ __forceinline__ const int32_t* tb_col(const DevState& st, const THist& h) {
  return (h.col_kind == 0 ? st.mcnt : st.tcnt) + (size_t)h.col * st.N;
}

// Wave-aggregated atomics: the lanes targeting one word combine through a DPP reduction and one lane
// issues the atomic -- every node of a cluster hits the same few words (signature flags, the pair
// registrations and histogram bins of a few topology domains), which per-lane atomics serialize.
// Called by every lane of the wave (pend: this lane has a contribution).
__device__ __forceinline__ void or_agg(uint32_t* base, int word, uint32_t bits, bool pend) {
  const int lane = threadIdx.x & 63;
  for (;;) {
    const uint64_t m = __ballot(pend);
    if (!m) return;
    const int leader = (int)__builtin_ctzll(m);
    const int w0 = __builtin_amdgcn_readlane(word, leader);
    const bool mine = pend && word == w0;
    const uint32_t acc = (uint32_t)wave_red64(mine ? bits : 0u, OpOrU64{});
    if (lane == leader) atomicOr(base + w0, acc);
    if (mine) pend = false;
  }
}
__device__ __forceinline__ void add_agg(int32_t* base, int idx, int val, bool pend) {
  const int lane = threadIdx.x & 63;
  for (;;) {
    const uint64_t m = __ballot(pend);
    if (!m) return;
    const int leader = (int)__builtin_ctzll(m);
    const int i0 = __builtin_amdgcn_readlane(idx, leader);
    const bool mine = pend && idx == i0;
    const uint32_t acc = wave_sum32(mine ? (uint32_t)val : 0u);
    if (lane == leader) atomicAdd(base + i0, (int)acc);
    if (mine) pend = false;
  }
}

// The kernel is one short pass per node, so its time is the chain of dependent loads: the
// histogram columns and their label values (independent of the signature pass) are issued for the
// first kInitPre histograms before anything else and land while the signatures evaluate.
constexpr int kInitPre = 8;

// LH: the histogram bins and totals are first summed in the workgroup's LDS (lds_bins + n_hists
// int32, zeroed here) and flushed with one global atomic per non-zero bin -- a zone histogram gives
// every wave as many distinct bins as there are zones, which the wave-aggregated form serializes.
// Without LH (bins beyond kInitLdsBins) the wave-aggregated atomics go straight to global memory.
constexpr int kInitLdsBins = 16384;

template <bool LH>
__global__ void k_tbatch_init(const DevState* __restrict__ stp, TBatchArgs ta) {
  const DevState& st = *stp;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const bool on = n < st.N;  // every lane stays in the wave-wide aggregations
  const int lane = threadIdx.x & 63;
  extern __shared__ int32_t lh[];  // LH: [lds_bins] bins | [n_hists] totals
  const int nlh = ta.lds_bins + ta.n_hists;
  if constexpr (LH) {
    for (int b = threadIdx.x; b < nlh; b += blockDim.x) lh[b] = 0;
  }
  int pc[kInitPre], pv[kInitPre];
#pragma unroll
  for (int i = 0; i < kInitPre; ++i) {
    pc[i] = 0;
    pv[i] = -1;
    if (i < ta.n_hists && on) {
      const THist h = cp(ta.hists)[i];
      pc[i] = gp(tb_col(st, h))[n];
      if (h.key >= 0) pv[i] = gp(st.label_val)[(size_t)h.key * st.N + n];
    }
  }
  uint64_t em = 0;
  for (int s = 0; s < ta.n_sigs; ++s) {
    // through the constant pointer: a local copy's keys[k] at a run-time k lived in scratch
    const CAS TSig* sg = cp(ta.sigs) + s;
    bool ok = on && sg->n_keys >= 0 && node_affinity_ok(st, *cp(st.queries + sg->rep), n);
    for (int k = 0; k < sg->n_keys && ok; ++k) {
      const int key = sg->keys[k];
      ok = key >= 0 && gp(st.label_val)[(size_t)key * st.N + n] >= 0;
    }
    if (ok) em |= 1ull << s;
    or_agg(gp(ta.elig) + sg->elig_word, n >> 5, 1u << (n & 31), ok);
    const uint64_t any = __ballot(ok);
    if (any && lane == (int)__builtin_ctzll(any))
      __hip_atomic_store(gp(ta.sig_any) + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int r = 0; r < ta.n_regs; ++r) {
      const TReg rg = cp(ta.regs)[r];
      if (rg.sig != s) continue;  // uniform
      const int v = ok ? gp(st.label_val)[(size_t)rg.key * st.N + n] : 0;
      or_agg(gp(ta.reg_init) + rg.word, v >> 5, 1u << (v & 31), ok);
    }
  }
  if constexpr (LH) __syncthreads();  // the zeroed bins (the signature pass above hid the wait)
  auto hist = [&](int i, const THist& h, int c, int v) {
    const bool cnt = c != 0 && (h.sig < 0 || ((em >> h.sig) & 1u));
    if (!cnt) v = -1;
    if constexpr (LH) {
      if (cnt && h.off >= 0) atomicAdd(lh + h.off + (v >= 0 ? v : h.D), c);
      if (cnt && v >= 0) atomicAdd(lh + ta.lds_bins + i, c);
    } else {
      add_agg(gp(ta.hist_init), h.off + (v >= 0 ? v : h.D), c, cnt && h.off >= 0);
      add_agg(gp(ta.tot_init), i, c, cnt && v >= 0);
    }
  };
#pragma unroll
  for (int i = 0; i < kInitPre; ++i) {
    if (i >= ta.n_hists) break;  // uniform
    hist(i, cp(ta.hists)[i], pc[i], pv[i]);
  }
  for (int i = kInitPre; i < ta.n_hists; ++i) {
    const THist h = cp(ta.hists)[i];
    const int c = on ? gp(tb_col(st, h))[n] : 0;
    hist(i, h, c, (c != 0 && h.key >= 0) ? gp(st.label_val)[(size_t)h.key * st.N + n] : -1);
  }
  if constexpr (LH) {
    __syncthreads();
    for (int b = threadIdx.x; b < nlh; b += blockDim.x) {
      const int x = lh[b];
      if (x) atomicAdd(b < ta.lds_bins ? gp(ta.hist_init) + b : gp(ta.tot_init) + (b - ta.lds_bins), x);
    }
  }
}

// 63-bit order-preserving payloads of the statistics granules
constexpr int64_t kEncBias = 1ll << 62;
__device__ __forceinline__ uint64_t enc_stat(int64_t x) { return kGValid | (uint64_t)(x + kEncBias); }
__device__ __forceinline__ int64_t dec_stat(uint64_t g) { return (int64_t)(g & ~kGValid) - kEncBias; }
enum { kOpSum = 0, kOpMax, kOpMin, kOpOr };
__device__ __forceinline__ int tstat_op(int r) {
  switch (r) {
    case kTMaxT: case kTMaxNA: case kTAdjMax: case kTIpaMax: case kTDptsMax: case kTZoned: return kOpMax;
    case kTAdjMin: case kTIpaMin: return kOpMin;
    case kTFeas: case kTNonIgn: return kOpSum;
    default: return r < kTFixed + kTMaxSoftWords ? kOpOr : kOpSum;  // resolved by the caller's layout
  }
}
__device__ __forceinline__ int64_t tcombine(int op, int64_t a, int64_t b) {
  switch (op) {
    case kOpSum: return a + b;
    case kOpMax: return a > b ? a : b;
    case kOpMin: return a < b ? a : b;
    default: return a | b;
  }
}
__device__ __forceinline__ int64_t wave_op_i64(int op, int64_t x) {
  switch (op) {
    case kOpSum: return wave_sum_i64(x);
    case kOpMax: return wave_max_i64(x);
    case kOpMin: return wave_min_i64(x);
    default: return (int64_t)wave_red64((uint64_t)x, OpOrU64{});
  }
}
// identities of the statistics operations: beyond every real value, and inside the +-2^58 range the
// cross-rank records carry (kTXBias)
__device__ __forceinline__ int64_t tident(int op) {
  return op == kOpMax ? -(1ll << 56) : (op == kOpMin ? (1ll << 56) : 0);
}

struct TMisc {
  int64_t pmin[kTMaxTabs];   // criticalPaths[0].MatchNum per kind-0 table (MaxInt32 when none)
  uint64_t wkey;             // winning key of the pod (0: no feasible node)
  int32_t wg, wnode;         // its workgroup, its global node index
  int32_t abort, pad;
  uint64_t akey[16];         // per-wave argmax partials
  int32_t aidx[16];
  int32_t wlab[64];          // the winner's value of each key the run's deltas read (-1 absent)
  int32_t welig[64];         // the winner's eligibility under each signature
  // statistics accumulated across the waves (LDS atomics), kTFixed slots
  int32_t acc32[8];          // kTFeas, kTMaxT, kTMaxNA, kTNonIgn, kTAdjMin (as ~min), kTAdjMax, kTDptsMax, kTZoned
  int64_t acc64[2];          // kTIpaMin, kTIpaMax
  double logw[8];            // math.Log table entries logb .. logb + 7, loaded while the statistics travel
  int32_t logb, pad2;
};
static_assert(sizeof(TMisc) <= 1024, "kTMiscBytes (kgpu_api.cpp) holds TMisc");

__device__ __forceinline__ int tslot_op(int rr, int soft_words) {
  return rr < kTFixed ? tstat_op(rr) : (rr < kTFixed + soft_words ? kOpOr : kOpSum);
}
// Wave `w` polls statistics slots w, w + waves, ... of pod row `row`: every workgroup's granule
// of the slot, combined with the slot's operation.  False on timeout / abort.
__device__ __forceinline__ bool tpoll_slot(const uint64_t* row, int G, const int32_t* abort_word, int op,
                                           int64_t& out) {
  const int lane = threadIdx.x & 63;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool all = true;
    int64_t acc = tident(op);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int g = lane + 64 * j;
      if (g < G) {
        const uint64_t v = load_sc1(row + g);
        if (!(v & kGValid)) all = false;
        else acc = tcombine(op, acc, dec_stat(v));
      }
    }
    const int ab = load_sc1(abort_word);  // with the sweep: one round trip per retry
    if (__all(all)) {
      out = wave_op_i64(op, acc);
      return true;
    }
    if (ab != 0 || __builtin_amdgcn_s_memrealtime() - t0 > kSpinTimeout) return false;
  }
}

// Wave `wave` polls ALL of its statistics slots (wave, wave + W, ... below R, at most MS of them) in
// one sweep, NJ granules per lane and slot, and reduces each slot once every
// granule of every slot is there.  Polling the slots one after another costs a wave with two slots a
// second memory round trip after the data has landed.  Writes STAT[rr]; false on timeout / abort.
// NJ granules per lane and slot (G <= 64 * NJ).
// Wave `wave` polls ALL of its statistics slots (wave, wave + W, ... below R, at most MS of them) in
// one sweep, NJ granules per lane and slot (G <= 64 * NJ), and reduces each slot once every granule of
// every slot is there.  Polling the slots one after another costs a wave with two slots a second memory
// round trip after the data has landed.  The abort word is loaded with each sweep (loaded only after a
// failed sweep, it made every retry two round trips).  SLEEP (KGPU_OPT_TBATCH_POLL_SLEEP): a short
// s_sleep between sweeps -- every wave of every workgroup polls the same few granule lines, and less
// polling traffic measured 0.5-1 % faster per pod (more -- two sweeps in flight -- 1.5-2 % slower;
// DESIGN.md 4.4).  Writes STAT[rr]; false on timeout / abort.
template <int MS, int NJ, bool SLEEP>
__device__ __forceinline__ bool tpoll_slots(const uint64_t* srow, int G, int R, int W, int soft_words,
                                            const int32_t* abort_word, int64_t* STAT) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    uint64_t v[MS][NJ];
    bool all = true;
#pragma unroll
    for (int k = 0; k < MS; ++k) {
      const int rr = wave + k * W;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int gg = lane + 64 * j;
        v[k][j] = (rr < R && gg < G) ? load_sc1(srow + (size_t)rr * G + gg) : kGValid;
        if (!(v[k][j] & kGValid)) all = false;
      }
    }
    const int ab = load_sc1(abort_word);
    if (__all(all)) {
#pragma unroll
      for (int k = 0; k < MS; ++k) {
        const int rr = wave + k * W;
        if (rr >= R) break;  // uniform
        const int op = tslot_op(rr, soft_words);
        int64_t acc = tident(op);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          if (lane + 64 * j < G) acc = tcombine(op, acc, dec_stat(v[k][j]));
        const int64_t x = wave_op_i64(op, acc);
        if (lane == 0) STAT[rr] = x;
      }
      return true;
    }
    if (ab != 0 || __builtin_amdgcn_s_memrealtime() - t0 > kSpinTimeout) return false;
    if constexpr (SLEEP) __builtin_amdgcn_s_sleep(2);
  }
}

// ---- node sharding over xGMI (k_tbatch XG): the topology mailbox ring (kgpu_internal.h TX row)
constexpr uint64_t kTagMask = 0xFull << 60;
constexpr uint64_t kPayload60 = (1ull << 60) - 1;
__device__ __forceinline__ void store_sys(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void store_sys(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t load_sys(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int32_t load_sys(const int32_t* p) {
  return __hip_atomic_load(const_cast<int32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int32_t* tx_info(uint64_t* row, int nranks, int r) {
  return reinterpret_cast<int32_t*>(row + (size_t)nranks * (kTXRCap + 1)) + (size_t)r * kTXInfo;
}
// Every rank's record of one statistics slot (`base` = the slot of rank 0 in this pod's row),
// combined with the slot's operation; the record of rank r is at base + r * kTXRCap.  False on timeout
// or abort.
__device__ __forceinline__ bool xpoll_stat(const uint64_t* base, int nranks, const int32_t* abort_word, int op,
                                           uint64_t tag, int64_t& out) {
  const int lane = threadIdx.x & 63;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ok = true;
    int64_t v = tident(op);
    if (lane < nranks) {
      const uint64_t u = load_sys(base + (size_t)lane * kTXRCap);
      if ((u & kTagMask) != tag) ok = false;
      else v = (int64_t)(u & kPayload60) - kTXBias;
    }
    if (__all(ok)) {
      out = wave_op_i64(op, v);
      return true;
    }
    if (load_sc1(abort_word) != 0 || __builtin_amdgcn_s_memrealtime() - t0 > kSpinTimeout) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ int64_t tcol(const DevState& st, const TLook& t, int n) {
  return gp((t.col_kind == 0 ? st.mcnt : st.tcnt) + (size_t)t.col * st.N)[n];
}

// H[col][key][v] of one lookup at node n (v = label(key, n) >= 0)
__device__ __forceinline__ int64_t tval(const DevState& st, const int32_t* H, const TLook& t, int v, int n) {
  return t.off >= 0 ? (int64_t)H[t.off + v] : tcol(st, t, n);
}

// Score plugins of the pod outside the topology three (which k_tbatch normalizes itself).
constexpr uint32_t kTopoSM = (1u << KGPU_S_POD_TOPOLOGY_SPREAD) | (1u << KGPU_S_INTER_POD_AFFINITY) |
                             (1u << KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD);
// reg_taint: the raw TaintToleration score comes from the register-resident taint words (the
// caller adds it), not from the columns.
template <uint32_t SM, bool kDef>
__device__ __forceinline__ void tscores(const DevState& st, const kgpu_pod_query& q, const NodeRes& r, int n, NodeEval& e,
                                        bool reg_taint, bool diag, int64_t* dv = nullptr) {
  if constexpr (SM == kRuntime) {
    int64_t p = 0;
    for (int si = 0; si < st.n_scores; ++si) {
      const int s = cp(st.scores)[si];
      if ((kTopoSM >> s) & 1u) continue;
      if (s == KGPU_S_TAINT_TOLERATION && reg_taint) continue;
      const int64_t v = score_one<kDef>(s, st, q, r, n, e);
      if (diag) {
        gp(st.diag_raw)[(size_t)s * st.N + n] = v;
        if (!normalized(s)) gp(st.diag_norm)[(size_t)s * st.N + n] = v;
      }
      if (!normalized(s)) p += v * cp(st.w_of)[s];
    }
    e.partial = p;
  } else {
    if (reg_taint) run_scores<SM & ~kTopoSM & ~(1u << KGPU_S_TAINT_TOLERATION)>(st, q, r, n, e, diag, dv);
    else run_scores<SM & ~kTopoSM>(st, q, r, n, e, diag, dv);
  }
}

// One node of the pod: filters in profile order (PodTopologySpread / InterPodAffinity read the
// pod's LDS tables) and the raw scores.  Returns the status word.
struct TRow {
  int64_t part, adj, ipa;
  int32_t taint, na, ds, pad;
};
// Per-node data that never changes inside a run, loaded once with the resource row: the
// NodeUnschedulable flag, the taint bitsets (up to two words) and the zone.
struct TStatic {
  uint64_t tns[2], tpr[2];
  int32_t unsched, zone;
  uint64_t em;  // eligibility of the node under each of the run's signatures (bit s), from ta.elig
};
// The node's own match counts a pod reads from the columns (the ScheduleAnyway count of a node-unique
// key, the DefaultPodTopologySpread count), kept in registers across the run: only this lane's assume
// changes them (k_tbatch owns the columns during the run), so a column read once is exact after.
struct TCnt {
  int32_t col[2];  // cached column (class id) per purpose: 0 ScheduleAnyway, 1 DPTS; -1 none
  int32_t v[2];
};
__device__ __forceinline__ int32_t tcnt_get(const DevState& st, TCnt& c, int slot, int col, int n) {
  if (c.col[slot] != col) {
    c.col[slot] = col;
    c.v[slot] = gp(st.mcnt)[(size_t)col * st.N + n];
  }
  return c.v[slot];
}
// criticalPaths[0].MatchNum of a kind-0 table (MaxInt32 when no registered pair; filtering.go:93-121)
__device__ __forceinline__ int64_t pmin_of(const TMisc& M, int tab) {
  const int64_t x = M.pmin[tab];
  return x == INT64_MAX ? 2147483647 : x;
}

template <uint32_t FM, uint32_t SM, bool kDef>
__device__ __forceinline__ uint32_t trow_eval(const DevState& st, const TBatchArgs& ta, const kgpu_pod_query& q,
                                         const TPlan& tp, const NodeRes& r, int n, const int32_t* H,
                                         const int64_t* PT, const TMisc& M, bool pany, bool aff_any,
                                         const int32_t* LAB, int li, const TStatic& sr, TCnt& cc, TRow& o,
                                         bool diag, int64_t* dv = nullptr) {
  // node label value ids from the workgroup's LDS copy (keys < lab_keys), else from the column
  auto nval = [&](int key) -> int {
    if (key < 0) return -1;
    return key < ta.lab_keys ? LAB[key * ta.per + li] : gp(st.label_val)[(size_t)key * st.N + n];
  };
  auto pts = [&]() -> uint32_t {  // filtering.go:276-328
    if (!pany) return 0;
    for (int c = 0; c < tp.n_hard; ++c) {
      const THard hc = tp.hard[c];
      const int v = nval(hc.key);
      if (v < 0) return KGPU_CODE_UNSCHEDULABLE << 8;
      if (PT[hc.pt_off + v] + hc.self_match - pmin_of(M, hc.tab) > hc.max_skew) return KGPU_CODE_UNSCHEDULABLE << 8;
    }
    return 0;
  };
  auto ipa = [&]() -> uint32_t {  // filtering.go:314-396
    bool exist = true;
    for (int a = 0; a < tp.n_aff; ++a) {
      const TLook t = tp.aff[a];
      const int v = nval(t.key);
      if (v < 0) return (KGPU_CODE_UNRESOLVABLE << 8) | (1u << 16);
      if (tval(st, H, t, v, n) <= 0) exist = false;
    }
    if (!exist && !(!aff_any && tp.self_all)) return (KGPU_CODE_UNRESOLVABLE << 8) | (1u << 16);
    for (int a = 0; a < tp.n_anti; ++a) {
      const TLook t = tp.anti[a];
      const int v = nval(t.key);
      if (v >= 0 && tval(st, H, t, v, n) > 0) return (KGPU_CODE_UNSCHEDULABLE << 8) | (2u << 16);
    }
    for (int k = 0; k < tp.n_exa_tabs; ++k) {
      const TTab tb = cp(ta.tabs)[tp.tabs.begin + tp.tabs.count - tp.n_exa_tabs + k];
      const int v = nval(tb.key);
      if (v >= 0 && PT[tb.off + v] > 0) return (KGPU_CODE_UNSCHEDULABLE << 8) | (3u << 16);
    }
    for (int e = 0; e < tp.exa_u.count; ++e) {
      const TLook t = cp(ta.looks)[tp.exa_u.begin + e];
      if (nval(t.key) >= 0 && tcol(st, t, n) > 0) return (KGPU_CODE_UNSCHEDULABLE << 8) | (3u << 16);
    }
    return 0;
  };
  // NodeAffinity (node_affinity.go:53-62): the pod's selector program was evaluated once per run for
  // every node (k_tbatch_init); here it is one bit
  auto one = [&](int f) -> uint32_t {
    if (f == KGPU_F_POD_TOPOLOGY_SPREAD) return pts();
    if (f == KGPU_F_INTER_POD_AFFINITY) return ipa();
    if (f == KGPU_F_NODE_AFFINITY) return ((sr.em >> tp.aff_sig) & 1u) ? 0 : KGPU_CODE_UNRESOLVABLE << 8;
    if (f == KGPU_F_NODE_UNSCHEDULABLE)  // node_unschedulable.go:51-65
      return (sr.unsched && !(q.flags & KGPU_Q_TOLERATES_UNSCHEDULABLE)) ? KGPU_CODE_UNRESOLVABLE << 8 : 0;
    if (f == KGPU_F_TAINT_TOLERATION && st.TW <= 2) {  // taint_toleration.go:54-72
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        if (w >= st.TW) break;
        const uint64_t tol = w < q.tol_nosched.count ? cp(st.qp.words)[q.tol_nosched.begin + w] : 0ull;
        if (sr.tns[w] & ~tol) return KGPU_CODE_UNRESOLVABLE << 8;
      }
      return 0;
    }
    return filter_one(f, st, q, r, n);
  };
  uint32_t status = 0;
  if constexpr (FM == kRuntime) {
    for (int fi = 0; fi < st.n_filters && !status; ++fi) {
      status = one(cp(st.filters)[fi]);
      if (status) status |= (uint32_t)(fi + 1);
    }
  } else {
    // the default order: ascending plugin id (select_spec picks this instantiation only then)
    uint32_t pos = 0;
#pragma unroll
    for (int f = 0; f < KGPU_NUM_FILTERS; ++f) {
      if (!((FM >> f) & 1u)) continue;
      ++pos;
      if (status) continue;
      status = one(f);
      if (status) status |= pos;
    }
  }
  if (status) return status;
  NodeEval e{0, 0, 0, 0};
  tscores<SM, kDef>(st, q, r, n, e, st.TW <= 2, diag, dv);
  if (st.TW <= 2 && st.w_of[KGPU_S_TAINT_TOLERATION] && st.any_prefer_taint) {  // taint_toleration.go:123-152
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      if (w >= st.TW) break;
      const uint64_t tol = w < q.tol_prefer.count ? cp(st.qp.words)[q.tol_prefer.begin + w] : 0ull;
      e.taint += __popcll(sr.tpr[w] & ~tol);
    }
    if (diag && dv) dv[KGPU_S_TAINT_TOLERATION] = e.taint;
    else if (diag) gp(st.diag_raw)[(size_t)KGPU_S_TAINT_TOLERATION * st.N + n] = e.taint;
  }
  o.part = e.partial;
  o.taint = e.taint;
  o.na = e.na;
  // PodTopologySpread ScheduleAnyway (scoring.go:75-102,174-208): INT64_MIN = ignored node
  o.adj = 0;
  if (tp.n_soft) {
    const int v = nval(tp.soft_key);
    if (v < 0) {
      o.adj = INT64_MIN;
    } else {
      int64_t cnt;
      if (tp.soft_mode == 0) cnt = H[tp.soft_off + v];
      else if (tp.soft_mode == 1) cnt = tcnt_get(st, cc, 0, tp.soft_col, n);
      else cnt = ((sr.em >> tp.soft_sig) & 1u) ? tcnt_get(st, cc, 0, tp.soft_col, n) : 0;
      o.adj = cnt < tp.soft_max_skew ? tp.soft_max_skew - 1 : cnt;  // adjustForMaxSkew
    }
  }
  // InterPodAffinity topologyScore (scoring.go:217-236)
  int64_t is = 0;
  if (tp.need_ipa) {
    for (int k = 0; k < tp.tabs.count - tp.n_exa_tabs; ++k) {
      const TTab tb = cp(ta.tabs)[tp.tabs.begin + k];
      if (tb.kind != 2) continue;
      const int v = nval(tb.key);
      if (v >= 0) is += PT[tb.off + v];
    }
    for (int e2 = 0; e2 < tp.score_u.count; ++e2) {
      const TLook t = cp(ta.looks)[tp.score_u.begin + e2];
      if (nval(t.key) >= 0) is += (int64_t)t.weight * tcol(st, t, n);
    }
  }
  o.ipa = is;
  o.ds = tp.dpts_cls >= 0 ? tcnt_get(st, cc, 1, tp.dpts_cls, n) : 0;
  return 0;
}

// trow_eval in two parts, for the pods of a run after its first (not diagnostic: only feasibility and
// the raw scores matter, not the first failing filter's position).
//  * trow_ind: every filter and score outside PodTopologySpread / InterPodAffinity (and DPTS).  These
//    read the node's register row and node-static columns only, so k_tbatch evaluates them for pod
//    i+1 while pod i's exchanges are in flight; pod i's assume changes them on one row (its winner),
//    which is evaluated again -- on a copy of the candidate row with pod i applied -- before the key
//    round ends.  False when a filter fails.
//  * trow_topo: the topology filters and raw topology scores, after pod i's histogram deltas.
template <uint32_t FM, uint32_t SM, bool kDef>
__device__ __forceinline__ bool trow_ind(const DevState& st, const TBatchArgs& ta, const kgpu_pod_query& q,
                                         const TPlan& tp, const NodeRes& r, int n, const TStatic& sr, TRow& o) {
  auto one = [&](int f) -> bool {
    if (f == KGPU_F_POD_TOPOLOGY_SPREAD || f == KGPU_F_INTER_POD_AFFINITY) return true;
    if (f == KGPU_F_NODE_AFFINITY) return ((sr.em >> tp.aff_sig) & 1u) != 0;
    if (f == KGPU_F_NODE_UNSCHEDULABLE) return !(sr.unsched && !(q.flags & KGPU_Q_TOLERATES_UNSCHEDULABLE));
    if (f == KGPU_F_TAINT_TOLERATION && st.TW <= 2) {
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        if (w >= st.TW) break;
        const uint64_t tol = w < q.tol_nosched.count ? cp(st.qp.words)[q.tol_nosched.begin + w] : 0ull;
        if (sr.tns[w] & ~tol) return false;
      }
      return true;
    }
    return filter_one(f, st, q, r, n) == 0;
  };
  bool ok = true;
  if constexpr (FM == kRuntime) {
    for (int fi = 0; fi < st.n_filters && ok; ++fi) ok = one(cp(st.filters)[fi]);
  } else {
#pragma unroll
    for (int f = 0; f < KGPU_NUM_FILTERS; ++f) {
      if (!((FM >> f) & 1u)) continue;
      if (ok) ok = one(f);
    }
  }
  if (!ok) return false;
  NodeEval e{0, 0, 0, 0};
  tscores<SM, kDef>(st, q, r, n, e, st.TW <= 2, false);
  if (st.TW <= 2 && st.w_of[KGPU_S_TAINT_TOLERATION] && st.any_prefer_taint) {  // taint_toleration.go:123-152
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      if (w >= st.TW) break;
      const uint64_t tol = w < q.tol_prefer.count ? cp(st.qp.words)[q.tol_prefer.begin + w] : 0ull;
      e.taint += __popcll(sr.tpr[w] & ~tol);
    }
  }
  o.part = e.partial;
  o.taint = e.taint;
  o.na = e.na;
  return true;
}

// The topology half: PodTopologySpread and InterPodAffinity Filter (podtopologyspread/filtering.go:276-328,
// interpodaffinity/filtering.go:314-396), then the raw topology scores as in trow_eval.  False when a
// filter fails.
template <uint32_t FM>
__device__ __forceinline__ bool trow_topo(const DevState& st, const TBatchArgs& ta, const TPlan& tp, int n,
                                          const int32_t* H, const int64_t* PT, const TMisc& M, bool pany,
                                          bool aff_any, const int32_t* LAB, int li, const TStatic& sr, TCnt& cc,
                                          TRow& o) {
  auto nval = [&](int key) -> int {
    if (key < 0) return -1;
    return key < ta.lab_keys ? LAB[key * ta.per + li] : gp(st.label_val)[(size_t)key * st.N + n];
  };
  bool has_pts = ((FM >> KGPU_F_POD_TOPOLOGY_SPREAD) & 1u) != 0, has_ipa = ((FM >> KGPU_F_INTER_POD_AFFINITY) & 1u) != 0;
  if constexpr (FM == kRuntime) {
    has_pts = has_ipa = false;
    for (int fi = 0; fi < st.n_filters; ++fi) {
      has_pts |= st.filters[fi] == KGPU_F_POD_TOPOLOGY_SPREAD;
      has_ipa |= st.filters[fi] == KGPU_F_INTER_POD_AFFINITY;
    }
  }
  if (has_pts && pany) {
    for (int c = 0; c < tp.n_hard; ++c) {
      const THard hc = tp.hard[c];
      const int v = nval(hc.key);
      if (v < 0) return false;
      if (PT[hc.pt_off + v] + hc.self_match - pmin_of(M, hc.tab) > hc.max_skew) return false;
    }
  }
  if (has_ipa) {
    bool exist = true;
    for (int a = 0; a < tp.n_aff; ++a) {
      const TLook t = tp.aff[a];
      const int v = nval(t.key);
      if (v < 0) return false;
      if (tval(st, H, t, v, n) <= 0) exist = false;
    }
    if (!exist && !(!aff_any && tp.self_all)) return false;
    for (int a = 0; a < tp.n_anti; ++a) {
      const TLook t = tp.anti[a];
      const int v = nval(t.key);
      if (v >= 0 && tval(st, H, t, v, n) > 0) return false;
    }
    for (int k = 0; k < tp.n_exa_tabs; ++k) {
      const TTab tb = cp(ta.tabs)[tp.tabs.begin + tp.tabs.count - tp.n_exa_tabs + k];
      const int v = nval(tb.key);
      if (v >= 0 && PT[tb.off + v] > 0) return false;
    }
    for (int e = 0; e < tp.exa_u.count; ++e) {
      const TLook t = cp(ta.looks)[tp.exa_u.begin + e];
      if (nval(t.key) >= 0 && tcol(st, t, n) > 0) return false;
    }
  }
  o.adj = 0;
  if (tp.n_soft) {
    const int v = nval(tp.soft_key);
    if (v < 0) {
      o.adj = INT64_MIN;
    } else {
      int64_t cnt;
      if (tp.soft_mode == 0) cnt = H[tp.soft_off + v];
      else if (tp.soft_mode == 1) cnt = tcnt_get(st, cc, 0, tp.soft_col, n);
      else cnt = ((sr.em >> tp.soft_sig) & 1u) ? tcnt_get(st, cc, 0, tp.soft_col, n) : 0;
      o.adj = cnt < tp.soft_max_skew ? tp.soft_max_skew - 1 : cnt;  // adjustForMaxSkew
    }
  }
  int64_t is = 0;
  if (tp.need_ipa) {
    for (int k = 0; k < tp.tabs.count - tp.n_exa_tabs; ++k) {
      const TTab tb = cp(ta.tabs)[tp.tabs.begin + k];
      if (tb.kind != 2) continue;
      const int v = nval(tb.key);
      if (v >= 0) is += PT[tb.off + v];
    }
    for (int e2 = 0; e2 < tp.score_u.count; ++e2) {
      const TLook t = cp(ta.looks)[tp.score_u.begin + e2];
      if (nval(t.key) >= 0) is += (int64_t)t.weight * tcol(st, t, n);
    }
  }
  o.ipa = is;
  o.ds = tp.dpts_cls >= 0 ? tcnt_get(st, cc, 1, tp.dpts_cls, n) : 0;
  return true;
}

template <int B, int K, uint32_t FM, uint32_t SM, bool kDef, bool XG>
__global__ __launch_bounds__(B) void k_tbatch(const DevState* __restrict__ stp, TBatchArgs ta) {
  const DevState& st = *stp;
  __shared__ uint64_t* sh_ptx[XG ? kMaxRanks : 1];  // every rank's TX ring base (XG)
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  int32_t* H = reinterpret_cast<int32_t*>(lds_raw);
  uint32_t* REG = reinterpret_cast<uint32_t*>(lds_raw + ta.o_reg);
  int32_t* TOT = reinterpret_cast<int32_t*>(lds_raw + ta.o_tot);
  int32_t* SANY = reinterpret_cast<int32_t*>(lds_raw + ta.o_sany);
  int64_t* STAT = reinterpret_cast<int64_t*>(lds_raw + ta.o_stat);
  uint32_t* SMASK = reinterpret_cast<uint32_t*>(lds_raw + ta.o_smask);
  int32_t* ZSUM = reinterpret_cast<int32_t*>(lds_raw + ta.o_zsum);
  int64_t* PT = reinterpret_cast<int64_t*>(lds_raw + ta.o_pt);
  int32_t* LAB = reinterpret_cast<int32_t*>(lds_raw + ta.o_lab);  // [lab_keys][per] label value ids
  TMisc& M = *reinterpret_cast<TMisc*>(lds_raw + ta.o_misc);
  constexpr int W = B / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = gridDim.x, g = blockIdx.x;
  // every workgroup leaves through here, aborted or not (the pod loop only breaks): the last one to
  // leave copies the run's abort word into the caller's pinned block
  auto leave = [&]() {
    if (ta.abort_out) {
      // the host completes a one-pod cycle on abort_out: every wave's stores (records, diagnostic rows,
      // the resident state's write-back) reach L2 before thread 0's release writes it back and counts the
      // workgroup out (one write-back per workgroup: a fence in every wave cost a 100k-node cycle 38 us)
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
    if (ta.abort_out && tid == 0) {
      // release only (a full __threadfence() adds an L1 invalidate whose wait every workgroup paid): the last
      // workgroup reads nothing the others wrote but the abort word (an sc1 load), and its completion store
      // carries its own system-scope release
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      if (atomicAdd(ta.done, 1) == G - 1)
        __hip_atomic_store(ta.abort_out, load_sc1(ta.abort), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  };
  if (g == ta.hold) {  // KGPU_OPT_HOLD_GROUP: a workgroup that never became resident
    leave();
    return;
  }
  const int lo = g * ta.per;
  // run stamps (KGPU_OPT_PHASE_TRACE) in the trace's spare last row: entry, pod loop start, exit
  const bool trun = ta.trace && tid == 0 && (g == 0 || g == G - 1);
  int64_t* trun_row = ta.trace ? ta.trace + (size_t)ta.count * 16 + (g == 0 ? 0 : 8) : nullptr;
  if (trun) trun_row[0] = (int64_t)__builtin_amdgcn_s_memrealtime();
  // the resident state's spare buffer, zeroed for the next miss (nothing in this run reads it)
  for (int i = g * B + tid; i < ta.zero_n16; i += G * B) gp(ta.zero_buf)[i] = TBatchArgs::Z16{0, 0};

  // LDS replicas and the workgroup's label values: eight independent loads in flight per thread
  // and round (a one-pod run pays this start-up in full; a strided loop would wait for each load)
  constexpr int kU = 8;
  for (int base = 0; base < ta.lds_bins; base += kU * B) {
    int32_t v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = base + u * B + tid;
      v[u] = i < ta.lds_bins ? gp(ta.hist_init)[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (base + u * B + tid < ta.lds_bins) H[base + u * B + tid] = v[u];
  }
  for (int i = tid; i < ta.reg_words; i += B) REG[i] = gp(ta.reg_init)[i];
  for (int i = tid; i < ta.n_hists; i += B) TOT[i] = gp(ta.tot_init)[i];
  for (int i = tid; i < ta.n_sigs; i += B) SANY[i] = gp(ta.sig_any)[i];
  const int nlab = ta.lab_keys * ta.per;
  for (int base = 0; base < nlab; base += kU * B) {
    int32_t v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = base + u * B + tid;
      const int k = i / ta.per, n = lo + i % ta.per;
      v[u] = (i < nlab && n < st.N) ? gp(st.label_val)[(size_t)k * st.N + n] : -1;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (base + u * B + tid < nlab) LAB[base + u * B + tid] = v[u];
  }
  // every node's delta-key labels (ta.wlab): the winner's come from here in the assume phase
  int32_t* WLAB = reinterpret_cast<int32_t*>(lds_raw + ta.o_wlab);
  if (!XG && ta.wlab) {
    const int nw = ta.n_keys * st.N;
    for (int base = 0; base < nw; base += kU * B) {
      int32_t v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int i = base + u * B + tid;
        v[u] = i < nw ? gp(st.label_val)[i] : -1;  // label_val is [K][N]: the same layout
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (base + u * B + tid < nw) WLAB[base + u * B + tid] = v[u];
    }
  }
  if (tid == 0) M.abort = 0;
  if constexpr (XG) {
    if (tid < ta.nranks) sh_ptx[tid] = ta.ptx[tid];
  }
  const int64_t txw = XG ? tx_row_words(ta.nranks) : 0;
  NodeRes r[K];
  TStatic sr[K];
  TCnt cc[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int n = lo + j * B + tid;
    r[j] = NodeRes{};
    sr[j] = TStatic{{0, 0}, {0, 0}, 0, -1, 0};
    cc[j] = TCnt{{-1, -1}, {0, 0}};
    if (n < st.N) {
      // the node's eligibility bits (k_tbatch_init's bitmaps): one load per signature, all in flight
      uint64_t em = 0;
      for (int s0 = 0; s0 < ta.n_sigs; s0 += 8) {
        uint32_t w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          w[u] = s0 + u < ta.n_sigs ? gp(ta.elig)[cp(ta.sigs)[s0 + u].elig_word + (n >> 5)] : 0u;
#pragma unroll
        for (int u = 0; u < 8; ++u) em |= (uint64_t)((w[u] >> (n & 31)) & 1u) << (s0 + u);
      }
      sr[j].em = em;
    }
    if (n < st.N) {
      if (ta.diag && !(K == 1 && SM != kRuntime)) {
        // a diagnostic (kgpu_schedule_one) run: this node's per-plugin raw / normalized rows start at
        // 0 (this lane's later stores of them follow in program order; kDefer runs store every row
        // once at the end instead)
        for (int si = 0; si < st.n_scores; ++si) {  // the profile's plugins (the others stay 0)
          const int sc = cp(st.scores)[si];
          gp(st.diag_raw)[(size_t)sc * st.N + n] = 0;
          gp(st.diag_norm)[(size_t)sc * st.N + n] = 0;
        }
      }
      r[j] = load_res(st, n);
      if constexpr (kDef) set_recips(r[j]);
      sr[j].unsched = gp(st.unsched)[n];
      sr[j].zone = gp(st.zone_id)[n];
      // constant indices only: a dynamically indexed private array lives in scratch memory
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        if (w >= st.TW) break;
        sr[j].tns[w] = gp(st.taint_nosched)[(size_t)w * st.N + n];
        sr[j].tpr[w] = gp(st.taint_prefer)[(size_t)w * st.N + n];
      }
    }
  }
  const int R = ta.R;
  const bool trc = ta.trace && tid == 0 && (g == 0 || g == G - 1);
  int64_t* trow = ta.trace ? ta.trace + (g == 0 ? 0 : 8) : nullptr;
#define KGPU_TSTAMP(k) \
  if (trc) trow[(size_t)i * 16 + (k)] = (int64_t)__builtin_amdgcn_s_memrealtime()
#define KGPU_WSTAMP(k) \
  if (ta.trace_wg && tid == 0) ta.trace_wg[((size_t)i * G + g) * 8 + (k)] = (int64_t)__builtin_amdgcn_s_memrealtime()
  // Evaluation ahead (one row per lane): the next pod's non-topology filters and scores (trow_ind) run
  // while this pod's statistics round is in flight; the candidate lane evaluates them again on its row
  // with this pod applied while the key round is in flight, for the case its workgroup wins.
  constexpr bool kAhead = K == 1;
  // kDefer (diagnostic runs of a compile-time profile, one row per lane): the cycle's status word, raw
  // and normalized scores stay in registers until the pod is resolved, then every row of the lane's
  // node is stored once -- stores issued during the pod would hold every later load and the exchanges'
  // polls behind them (vmcnt counts stores too)
  constexpr bool kDefer = K == 1 && SM != kRuntime;
  int64_t dv[KGPU_NUM_SCORES];
  int64_t dn[5], dt[3];  // normalized TT, NA, PTS, IPA, DPTS; raw PTS, IPA, DPTS
  uint32_t dstat = 0;
  bool ind_have = false;                     // (uniform) ind_* hold this pod's trow_ind of the lane's row
  bool ind_next = false;                     // (uniform) ... and nx_* the next pod's
  bool ind_ok = false, nx_ok = false, vb_ok = false;
  int log_guess = 2;                         // (uniform) math.Log index of the last pod's topology size
  TRow ind_o{}, nx_o{}, vb_o{};              // part / taint / na only
  if (trun) trun_row[1] = (int64_t)__builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < ta.count; ++i) {
    KGPU_TSTAMP(0);
    KGPU_WSTAMP(0);
    if (i == ta.abort_at && g == 0 && tid == 0) __hip_atomic_store(ta.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int pod = ta.first + i;
    if (kDefer && ta.diag) {
#pragma unroll
      for (int k = 0; k < KGPU_NUM_SCORES; ++k) dv[k] = 0;
#pragma unroll
      for (int k = 0; k < 5; ++k) dn[k] = 0;
#pragma unroll
      for (int k = 0; k < 3; ++k) dt[k] = 0;
    }
    // warm the next pod's query record (its first touch would otherwise put a memory round trip at
    // the head of the next pod); the load is consumed at the end of this pod, so nothing waits for it
    uint4 qwarm{};
    if (wave == W - 1 && i + 1 < ta.count && lane < (int)(sizeof(kgpu_pod_query) / 16))
      qwarm = reinterpret_cast<const GAS uint4*>(gp(st.queries + pod + 1))[lane];
    const kgpu_pod_query& q = *cp(st.queries + pod);
    const TPlan& tp = *cp(ta.plans + cp(ta.plan_of)[i]);
    const uint64_t tk = pod_tie_key(st.seed, ta.seq0 + i);
    // ---- the pod's lookup tables and PreFilter state (every workgroup, from its LDS replicas)
    for (int w = tid; w < ta.soft_words; w += B) SMASK[w] = 0;
    for (int z = tid; z < ta.zones; z += B) ZSUM[z] = 0;
    if (tid < kTMaxTabs) M.pmin[tid] = INT64_MAX;
    if (tid < 8) M.acc32[tid] = 0;
    if (tid < 2) M.acc64[tid] = tid == 0 ? INT64_MAX : INT64_MIN;
    __syncthreads();
    if (ta.trace_mode == 3) KGPU_TSTAMP(1);  // trace mode 3: the pod's records loaded, LDS accumulators reset
    for (int k = 0; k < tp.tabs.count; ++k) {
      const TTab tb = cp(ta.tabs)[tp.tabs.begin + k];
      for (int v = tid; v < tb.D; v += B) {
        int64_t x = 0;
        for (int t = 0; t < tb.terms.count; ++t) {
          const TLook lk = cp(ta.looks)[tb.terms.begin + t];
          x += (int64_t)(tb.kind == 2 ? lk.weight : 1) * H[lk.off + v];
          if (tb.kind == 0 && v == tb.empty_v) x += H[lk.off + lk.D];  // node.Labels[key] of a missing key is ""
        }
        if (tb.kind == 0) {
          const TReg rg = cp(ta.regs)[tb.reg];
          if ((REG[rg.word + (v >> 5)] >> (v & 31)) & 1u) atomicMin(reinterpret_cast<long long*>(&M.pmin[k]), (long long)x);
          else x = 0;  // an unregistered pair has no TpPairToMatchNum entry
        }
        PT[tb.off + v] = x;
      }
    }
    KGPU_WSTAMP(7);
    if (ta.trace_mode == 3) KGPU_TSTAMP(2);  // ... and its lookup tables built (before the barrier)
    const bool pany = tp.n_hard > 0 && SANY[tp.hard_sig] != 0;
    bool aff_any = false;
    for (int a = 0; a < tp.n_aff; ++a) aff_any |= tp.aff_hist[a] >= 0 && TOT[tp.aff_hist[a]] > 0;
    __syncthreads();  // (readers map an unset minimum to MaxInt32: pmin_of)
    if (ta.trace_mode < 2) KGPU_TSTAMP(1);
    // ---- Filter + raw scores of this workgroup's rows
    bool feas[K];
    TRow o[K];
    uint32_t sf = 0, smaxT = 0, smaxNA = 0, snon = 0, sadjmin = 0xFFFFFFFFu, sadjmax = 0, sdmax = 0, szoned = 0;
    int64_t simin = INT64_MAX, simax = INT64_MIN;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int n = lo + j * B + tid;
      feas[j] = false;
      if (n >= st.N) continue;
      if (kAhead && ind_have) {
        // the non-topology half was evaluated ahead; the topology half reads this pod's tables
        if (!ind_ok) continue;
        o[j] = ind_o;
        if (!trow_topo<FM>(st, ta, tp, n, H, PT, M, pany, aff_any, LAB, j * B + tid, sr[j], cc[j], o[j])) continue;
      } else {
        const uint32_t sw = trow_eval<FM, SM, kDef>(st, ta, q, tp, r[j], n, H, PT, M, pany, aff_any, LAB, j * B + tid,
                                                    sr[j], cc[j], o[j], ta.diag, kDefer ? dv : (int64_t*)nullptr);
        if (kDefer && ta.diag) dstat = sw;
        else if (ta.diag) gp(st.status)[n] = sw;  // kgpu_schedule_one: the cycle's Filter verdicts
        if (sw) continue;
      }
      feas[j] = true;
      ++sf;
      smaxT = max(smaxT, (uint32_t)o[j].taint);
      smaxNA = max(smaxNA, (uint32_t)o[j].na);
      if (o[j].adj != INT64_MIN && tp.n_soft) {
        ++snon;
        sadjmin = min(sadjmin, (uint32_t)o[j].adj);
        sadjmax = max(sadjmax, (uint32_t)o[j].adj);
        if (tp.soft_mode == 0) {
          const int v = tp.soft_key < ta.lab_keys ? LAB[tp.soft_key * ta.per + j * B + tid] : nval(st, tp.soft_key, n);
          atomicOr(SMASK + (v >> 5), 1u << (v & 31));
        }
      }
      simin = min(simin, o[j].ipa);
      simax = max(simax, o[j].ipa);
      sdmax = max(sdmax, (uint32_t)o[j].ds);
      const int z = sr[j].zone;
      if (z >= 0) {
        szoned = 1;
        if (o[j].ds && z < ta.zones) atomicAdd(ZSUM + z, o[j].ds);
      }
    }
    if (ta.trace_mode < 2) KGPU_TSTAMP(2);
    KGPU_WSTAMP(1);
    // ---- statistics round: wave reductions (DPP), workgroup (LDS atomics), granules, every workgroup
    sf = wave_sum32(sf);
    smaxT = wave_max32u(smaxT);
    smaxNA = wave_max32u(smaxNA);
    if (tp.n_soft) {
      snon = wave_sum32(snon);
      sadjmin = ~wave_max32u(~sadjmin);
      sadjmax = wave_max32u(sadjmax);
    }
    if (tp.need_ipa) {
      simin = wave_min_i64(simin);
      simax = wave_max_i64(simax);
    }
    if (tp.dpts_cls >= 0) {
      sdmax = wave_max32u(sdmax);
      szoned = wave_max32u(szoned);
    }
    if (lane == 0) {
      atomicAdd(&M.acc32[0], (int)sf);
      atomicMax(reinterpret_cast<unsigned*>(&M.acc32[1]), smaxT);
      atomicMax(reinterpret_cast<unsigned*>(&M.acc32[2]), smaxNA);
      if (tp.n_soft) {
        atomicAdd(&M.acc32[3], (int)snon);
        atomicMax(reinterpret_cast<unsigned*>(&M.acc32[4]), ~sadjmin);
        atomicMax(reinterpret_cast<unsigned*>(&M.acc32[5]), sadjmax);
      }
      if (tp.need_ipa) {
        atomicMin(reinterpret_cast<long long*>(&M.acc64[0]), (long long)simin);
        atomicMax(reinterpret_cast<long long*>(&M.acc64[1]), (long long)simax);
      }
      if (tp.dpts_cls >= 0) {
        atomicMax(reinterpret_cast<unsigned*>(&M.acc32[6]), sdmax);
        atomicMax(reinterpret_cast<unsigned*>(&M.acc32[7]), szoned);
      }
    }
    __syncthreads();
    KGPU_WSTAMP(4);
    uint64_t* srow = ta.gran + (size_t)i * (R + 1) * G;  // [R][G] statistics granules | [G] keys
    // one slot per thread.  Every thread reads its candidate words first -- clamped addresses, one LDS
    // round trip -- and then selects: a switch over the slot puts an LDS read and its wait in each of a
    // dozen divergent branches, which the wave runs one after another (0.7 us per pod).  The selection is
    // a chain of selects, not an if / else chain: ROCm 7.2's gfx950 backend lowers the if / else chain (a
    // switch whose default, the zero extension, is reached from both sides of a divergent branch) to code
    // that never assigns the default's value to the lanes of slots kTDptsMax and kTZoned -- they publish
    // stale registers.  The LLVM IR is right; the machine code is not (reproducer
    // tools/repro/stat_select.hip).  Whether it shows depended on the surrounding code: the lambda form
    // miscompiled inside k_tbatch, the written-out if / else chain did not, both do in the reproducer.
    if (tid < R) {
      const int i32 = tid < 6 ? tid : (tid == kTDptsMax ? 6 : 7);
      const uint32_t w32 = (uint32_t)M.acc32[i32];
      const int64_t w64 = M.acc64[tid == kTIpaMax ? 1 : 0];
      const int vi = tid - kTFixed;
      const int voff = vi < 0 ? ta.o_smask : (vi < ta.soft_words ? ta.o_smask + 4 * vi : ta.o_zsum + 4 * (vi - ta.soft_words));
      const int32_t wv = *reinterpret_cast<const int32_t*>(lds_raw + voff);
      int64_t x = (int64_t)w32;  // kTMaxT, kTMaxNA, kTDptsMax, kTZoned
      x = (tid == kTFeas || tid == kTNonIgn) ? (int64_t)(int32_t)w32 : x;
      x = tid == kTAdjMax ? (tp.n_soft ? (int64_t)w32 : tident(kOpMax)) : x;
      x = tid == kTAdjMin ? (tp.n_soft ? (int64_t)(uint32_t)~w32 : tident(kOpMin)) : x;
      x = tid == kTIpaMax ? (w64 == INT64_MIN ? tident(kOpMax) : w64) : x;
      x = tid == kTIpaMin ? (w64 == INT64_MAX ? tident(kOpMin) : w64) : x;
      x = tid >= kTFixed ? (vi < ta.soft_words ? (int64_t)(uint32_t)wv : (int64_t)wv) : x;  // SMASK bits / ZSUM
      store_sc1(srow + (size_t)tid * G + g, enc_stat(x));
    }
    KGPU_TSTAMP(3);
    KGPU_WSTAMP(2);
    // the next pod's non-topology half while the statistics travel (the polls below start after it;
    // the round trip they wait for is longer than the evaluation)
    // the math.Log entries around the previous pod's topology size, issued before the evaluation
    // below and staged in LDS after it
    double logw_pre = 0.0;
    int logb_pre = 0;
    if (tp.n_soft && wave == W - 1 && lane < 8) {
      const int nl = st.n_total + 3;
      logb_pre = max(0, min(log_guess - 3, nl - 8));
      logw_pre = lane < nl ? st.log_table[logb_pre + lane] : 0.0;
    }
    const bool ahead = kAhead && ta.ahead && !ta.diag && i + 1 < ta.count;
    const kgpu_pod_query& qn = *cp(st.queries + pod + (ahead ? 1 : 0));
    const TPlan& tpn = *cp(ta.plans + cp(ta.plan_of)[ahead ? i + 1 : i]);
    if (ahead) {
      const int n = lo + tid;
      nx_ok = n < st.N && trow_ind<FM, SM, kDef>(st, ta, qn, tpn, r[0], n, sr[0], nx_o);
    }
    ind_next = ahead;
    // the math.Log entries around the previous pod's topology size (it changes by a few per pod): the
    // normalize pass reads its weight from LDS instead of a dependent global load
    if (tp.n_soft && wave == W - 1 && lane < 8) {
      M.logw[lane] = logw_pre;  // loaded before the evaluation above
      if (lane == 0) M.logb = logb_pre;
    }
    // this pod's tie-break ranks, for the keys formed once the statistics are in
    uint64_t rk[K];
#pragma unroll
    for (int j = 0; j < K; ++j) rk[j] = rank40(tk, (uint64_t)(st.node_base + lo + j * B + tid), st.tie_mode);
    // ---- NormalizeScore of every plugin under statistics S, weights, and the packed key of this
    // lane's best row; with write_diag, the cycle's per-plugin scores (as k_topo_score / k_topo_final)
    auto best_under = [&](const int64_t* S, bool write_diag, uint64_t& bkey, int& bidx) {
      const int maxT = (int)S[kTMaxT], maxNA = (int)S[kTMaxNA];
      int64_t pmx = 0, pmn = INT64_MAX;
      double wsoft = 0.0;
      if (tp.n_soft) {
        int64_t size = S[kTNonIgn];
        if (tp.soft_mode == 0) {
          size = 0;
          for (int w = 0; w < tp.soft_words; ++w) size += __popc((uint32_t)S[kTFixed + w]);
        }
        // topologyNormalizingWeight (scoring.go:286-288): math.Log(size + 2)
        const int64_t li = size + 2 - M.logb;
        wsoft = (li >= 0 && li < 8) ? M.logw[li] : st.log_table[size + 2];
        log_guess = (int)(size + 2);
        if (S[kTNonIgn] > 0) {
          // int64(cnt * w) does not decrease with cnt: the extremes come from the extreme counts
          pmn = (int64_t)((double)S[kTAdjMin] * wsoft);
          pmx = max((int64_t)((double)S[kTAdjMax] * wsoft), (int64_t)0);
        }
      }
      const int64_t imx = max(S[kTIpaMax], (int64_t)0), imn = min(S[kTIpaMin], (int64_t)0);
      const int64_t idiff = imx - imn;
      const int64_t dmax_node = max(S[kTDptsMax], (int64_t)0);
      int64_t dmax_zone = 0;
      for (int z = 0; z < ta.zones; ++z) dmax_zone = max(dmax_zone, S[kTFixed + ta.soft_words + z]);
      const bool have_zones = S[kTZoned] != 0;
      const double Mx = 100.0, zwt = 2.0 / 3.0;
      // DefaultNormalizeScore / PTS normalize quotients are 0..100 with this pod's (uniform) maxima
      // as divisors: one reciprocal each, and ratio100's exact quotient per node
      const double invT = maxT > 0 ? 1.0 / (double)maxT : 0.0, invNA = maxNA > 0 ? 1.0 / (double)maxNA : 0.0;
      const double invP = (pmx > 0 && pmx < (1ll << 52)) ? 1.0 / (double)pmx : 0.0;
      // the 32-bit quotients apply (maxima below 2^24: every quotient's dividend is below 2^31)
      const bool small = maxT >= 0 && maxT < (1 << 24) && maxNA >= 0 && maxNA < (1 << 24) && pmx >= 0 && pmx < (1 << 24);
      bkey = 0;
      bidx = -1;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        if (!feas[j]) continue;
        const int n = lo + j * B + tid;
        // DefaultNormalizeScore (helper/normalize_score.go:26-54): non-negative operands, exact
        // through div_nonneg
        const int64_t ps = (o[j].adj != INT64_MIN && tp.n_soft) ? (int64_t)((double)o[j].adj * wsoft) : 0;
        bool s1 = false, s2 = false, s3 = false;
        // scoring.go:248-256; pmn <= ps <= pmx, so the dividend is non-negative
        const bool pdiv = o[j].adj != INT64_MIN && pmx != 0;  // pmn is set whenever pmx is
        int64_t qt, qn, qp;
        if (small) {
          // every dividend below 2^31 (0 <= taint <= maxT, na <= maxNA, pmx + pmn - ps <= pmx < 2^24)
          qt = ratio100_32(100 * o[j].taint, maxT > 0 ? maxT : 1, invT);
          qn = ratio100_32(100 * o[j].na, maxNA > 0 ? maxNA : 1, invNA);
          qp = ratio100_32(pdiv ? 100 * (int32_t)(pmx + pmn - ps) : 0, pmx > 0 ? (int32_t)pmx : 1, invP);
        } else {
          qt = ratio100(100 * (int64_t)o[j].taint, maxT, invT, s1);
          qn = ratio100(100 * (int64_t)o[j].na, maxNA, invNA, s2);
          qp = ratio100(pdiv ? 100 * (pmx + pmn - ps) : 0, pmx, invP, s3);
        }
        const int64_t vt = maxT == 0 ? 100 : 100 - (s1 ? div_nonneg(100 * (int64_t)o[j].taint, maxT) : qt);
        const int64_t vn = maxNA == 0 ? (int64_t)o[j].na : (s2 ? div_nonneg(100 * (int64_t)o[j].na, maxNA) : qn);
        const int64_t vp = o[j].adj == INT64_MIN ? 0 : (pmx == 0 ? 100 : (s3 ? div_nonneg(100 * (pmx + pmn - ps), pmx) : qp));
        const int64_t vi = idiff > 0 ? (int64_t)(Mx * ((double)(o[j].ipa - imn) / (double)idiff)) : 0;
        int64_t vd = 0;
        if (tp.dpts_cls != -2) {
          double f = Mx;
          if (dmax_node > 0) f = Mx * ((double)(dmax_node - o[j].ds) / (double)dmax_node);
          const int z = sr[j].zone;
          if (have_zones && z >= 0) {
            double zs = Mx;
            if (dmax_zone > 0) zs = Mx * ((double)(dmax_zone - S[kTFixed + ta.soft_words + z]) / (double)dmax_zone);
            f = (f * (1.0 - zwt)) + (zwt * zs);
          }
          vd = (int64_t)f;
        }
        int64_t total = o[j].part + vt * st.w_of[KGPU_S_TAINT_TOLERATION] + vn * st.w_of[KGPU_S_NODE_AFFINITY] +
                        vp * st.w_of[KGPU_S_POD_TOPOLOGY_SPREAD] + vi * st.w_of[KGPU_S_INTER_POD_AFFINITY] +
                        vd * st.w_of[KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD];
        if (st.n_scores == 0) total = 1;
        const uint64_t key = ((uint64_t)(total + 1) << 40) | rk[j];
        if (key > bkey) {
          bkey = key;
          bidx = j * B + tid;
        }
        if (write_diag && kDefer) {
          dn[0] = vt; dn[1] = vn; dn[2] = vp; dn[3] = vi; dn[4] = vd;
          dt[0] = (o[j].adj == INT64_MIN || !tp.n_soft) ? 0 : (int64_t)((double)o[j].adj * wsoft);
          dt[1] = o[j].ipa;
          dt[2] = tp.dpts_cls == -2 ? 0 : o[j].ds;
        } else if (write_diag) {
          const size_t N = (size_t)st.N;
          gp(st.diag_raw)[KGPU_S_POD_TOPOLOGY_SPREAD * N + n] =
              (o[j].adj == INT64_MIN || !tp.n_soft) ? 0 : (int64_t)((double)o[j].adj * wsoft);
          gp(st.diag_raw)[KGPU_S_INTER_POD_AFFINITY * N + n] = o[j].ipa;
          gp(st.diag_raw)[KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD * N + n] = tp.dpts_cls == -2 ? 0 : o[j].ds;
          // the normalized and topology plugins only (tscores wrote the others' normalized rows)
          for (int si = 0; si < st.n_scores; ++si) {
            const int s = cp(st.scores)[si];
            int64_t v;
            switch (s) {
              case KGPU_S_TAINT_TOLERATION: v = vt; break;
              case KGPU_S_NODE_AFFINITY: v = vn; break;
              case KGPU_S_POD_TOPOLOGY_SPREAD: v = vp; break;
              case KGPU_S_INTER_POD_AFFINITY: v = vi; break;
              case KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD: v = vd; break;
              default: continue;
            }
            gp(st.diag_norm)[(size_t)s * N + n] = v;
          }
        }
      }
    };
    // the workgroup's best key: wave partials through LDS, combined by wave 0 (every wave calls it)
    auto wg_best = [&](uint64_t bkey, int bidx, uint64_t& bk, int& bi) {
      wave_argmax(bkey, bidx);
      if (lane == 0) {
        M.akey[wave] = bkey;
        M.aidx[wave] = bidx;
      }
      __syncthreads();
      bk = lane < W ? M.akey[lane] : 0;
      bi = lane < W ? M.aidx[lane] : -1;
      wave_argmax(bk, bi);
    };
    bool ok = true;
    // XG: this pod's TX row and record tag (ring lap in bits 60-62)
    uint64_t* txrow = nullptr;
    uint64_t txtag = 0;
    if constexpr (XG) {
      txrow = sh_ptx[ta.rank] + (size_t)((ta.xseq0 + i) % kTXRing) * txw;
      txtag = kGValid | ((uint64_t)(((ta.xseq0 + i) / kTXRing) & 7) << 60);
    }
    if (!XG && G <= 64 && R <= 4 * W) {
      ok = ta.poll_sleep ? tpoll_slots<4, 1, true>(srow, G, R, W, ta.soft_words, ta.abort, STAT)
                         : tpoll_slots<4, 1, false>(srow, G, R, W, ta.soft_words, ta.abort, STAT);
    } else if (!XG && G <= 256 && R <= 2 * W) {
      ok = ta.poll_sleep ? tpoll_slots<2, 4, true>(srow, G, R, W, ta.soft_words, ta.abort, STAT)
                         : tpoll_slots<2, 4, false>(srow, G, R, W, ta.soft_words, ta.abort, STAT);
    } else for (int rr = wave; rr < R; rr += W) {
      const int op = tslot_op(rr, ta.soft_words);
      int64_t x;
      if (!tpoll_slot(srow + (size_t)rr * G, G, ta.abort, op, x)) { ok = false; break; }
      if constexpr (XG) {
        // this rank's combined slot: workgroup 0 publishes it into every rank's ring
        if (g == 0 && lane < ta.nranks) {
          const size_t off = (size_t)(txrow - sh_ptx[ta.rank]) + (size_t)ta.rank * kTXRCap + rr;
          store_sys(sh_ptx[lane] + off, txtag | (uint64_t)(x + kTXBias));
        }
      }
      if (lane == 0) STAT[rr] = x;
    }
    if constexpr (XG) {
      // every rank's record of the wave's slots, combined: the cluster-wide statistics
      for (int rr = wave; ok && rr < R; rr += W) {
        const int op = tslot_op(rr, ta.soft_words);
        int64_t x;
        if (!xpoll_stat(txrow + rr, ta.nranks, ta.abort, op, txtag, x)) { ok = false; break; }
        if (lane == 0) STAT[rr] = x;
      }
    }
    // pod 0's statistics never came: no workgroup resolved a pod of this run
    const int32_t acode = (i == 0 && !XG) ? kAbortClean : kAbortDirty;
    if (!ok && lane == 0) {
      __hip_atomic_fetch_or(ta.abort, acode, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      M.abort = 1;
    }
    __syncthreads();
    if (M.abort) break;
    KGPU_TSTAMP(4);
    KGPU_WSTAMP(5);
    const int64_t feas_total = STAT[kTFeas];
    uint64_t* arow = srow + (size_t)R * G;
    // ---- NormalizeScore of every plugin, weights, packed-key argmax
    uint64_t bkey0, bk;
    int bidx0, bi;
    best_under(STAT, ta.diag != 0, bkey0, bidx0);
    if (ta.trace_mode == 2) KGPU_TSTAMP(1);  // trace mode 2: normalize + keys of the lane's rows done
    wg_best(bkey0, bidx0, bk, bi);
    if (ta.trace_mode == 2) KGPU_TSTAMP(2);  // ... and the workgroup's best key known
    if (wave == 0 && lane == 0) store_sc1(arow + g, kGValid | bk);
    // the candidate row with this pod applied, for the next pod (used when this workgroup wins; a pod
    // with host ports or extended resources changes memory columns: its winner is evaluated again
    // after the assume instead)
    const bool vb_fast = q.scalars.count == 0 && q.ports.count == 0;
    if (ind_next && ta.assume && bk != 0 && vb_fast && tid == bi) {
      NodeRes t = r[0];
      assume_regs(q, t);
      vb_ok = trow_ind<FM, SM, kDef>(st, ta, qn, tpn, t, lo + tid, sr[0], vb_o);
    }
    if (wave == 0) {
      KGPU_TSTAMP(5);
      KGPU_WSTAMP(3);
      uint64_t wkey = 0;
      int wg = -1;
      bool pok = poll_row<4, false>(arow, G, ta.abort, kGValid, kGValid, wkey, wg);
      if constexpr (XG) {
        // this rank's best: its local winner publishes the record -- the winning node's label values
        // and signature bits first, then (after a system-scope release) the key; workgroup 0 publishes
        // a key-0 record when no node of this rank is feasible
        const size_t roff = (size_t)(txrow - sh_ptx[ta.rank]);
        if (pok && (wg >= 0 ? wg == g : g == 0)) {
          if (wkey) {
            const int wl = (int)rank40_inv(tk, wkey & kMask40, st.tie_mode) - st.node_base;
            const int lab = lane < ta.n_keys ? (lane < ta.lab_keys ? LAB[lane * ta.per + (wl - lo)]
                                                                  : gp(st.label_val)[(size_t)lane * st.N + wl])
                                             : -1;
            const uint64_t eb = __ballot(lane < ta.n_sigs && tb_elig(ta, lane, wl));
            for (int rk = 0; rk < ta.nranks; ++rk) {
              int32_t* inf = tx_info(sh_ptx[rk] + roff, ta.nranks, ta.rank);
              store_sys(inf + lane, lab);
              if (lane < 2) store_sys(inf + 64 + lane, (int32_t)(uint32_t)(eb >> (32 * lane)));
            }
            __threadfence_system();
          }
          if (lane < ta.nranks) store_sys(sh_ptx[lane] + roff + (size_t)ta.nranks * kTXRCap + ta.rank, txtag | wkey);
        }
        // every rank's best: the cluster-wide winner and its rank's record
        uint64_t gk = 0;
        int gr = -1;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (pok) {
          bool all = true;
          uint64_t k = 0;
          if (lane < ta.nranks) {
            const uint64_t u = load_sys(txrow + (size_t)ta.nranks * kTXRCap + lane);
            if ((u & kTagMask) != txtag) all = false;
            else k = u & kPayload60;
          }
          if (__all(all)) {
            int li = lane;
            wave_argmax(k, li);
            gk = k;
            gr = k ? li : -1;
            break;
          }
          if (load_sc1(ta.abort) != 0 || __builtin_amdgcn_s_memrealtime() - t0 > kSpinTimeout) pok = false;
          else __builtin_amdgcn_s_sleep(1);
        }
        if (pok && gk) {
          const int32_t* inf = tx_info(txrow, ta.nranks, gr);
          const int32_t lab = load_sys(inf + lane);
          const uint32_t ew = (uint32_t)load_sys(inf + 64 + (lane >> 5));
          if (lane < ta.n_keys) M.wlab[lane] = lab;
          if (lane < ta.n_sigs) M.welig[lane] = (int32_t)((ew >> (lane & 31)) & 1u);
        }
        if (lane == 0) {
          if (!pok) {
            __hip_atomic_store(ta.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            M.abort = 1;
          }
          M.wkey = gk;
          M.wg = (gr == ta.rank) ? wg : -1;  // the local winner applies the assume on the owning rank
          M.wnode = gk ? (int)rank40_inv(tk, gk & kMask40, st.tie_mode) : -1;
        }
      } else if (lane == 0) {
        if (!pok) {
          // a key-poll timeout is never clean: a workgroup that published its key late may still see
          // every key, resolve the pod and assume it (only the statistics phase of pod 0 is clean)
          __hip_atomic_fetch_or(ta.abort, kAbortDirty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          M.abort = 1;
        }
        M.wkey = wkey;
        M.wg = wg;
        M.wnode = wkey ? (int)rank40_inv(tk, wkey & kMask40, st.tie_mode) : -1;
      }
    }
    __syncthreads();
    if (M.abort) break;
    KGPU_TSTAMP(6);
    KGPU_WSTAMP(6);
    // ---- outcome (generic_scheduler.go:171-208) and assume (types.go:456-480)
    const int wnode = M.wnode;  // global index
    const bool error = (q.flags & KGPU_Q_SCORE_ERROR) && feas_total >= 2;
    const bool placed = feas_total > 0 && !error;
    // the record: unsharded by the winning workgroup; XG by workgroup 0 of every rank (every rank
    // returns the same records)
    if (tid == 0 && (XG ? g == 0 : ((M.wg >= 0 && M.wg == g) || (M.wg < 0 && g == 0)))) {
      kgpu_result res;
      res.node = placed ? wnode : (error ? -2 : -1);
      res.feasible = (int32_t)feas_total;
      res.evaluated = st.n_total;
      res.scored = (placed && feas_total >= 2) ? 1 : 0;
      res.score = res.scored ? (int64_t)(M.wkey >> 40) - 1 : 0;
      gp(st.results)[pod] = res;
    }
    if (placed && ta.assume) {
      const int wl = wnode - st.node_base;
      // the winner's label values and signature bits, staged once for every delta (XG: from the
      // winning rank's record, staged by wave 0)
      if constexpr (!XG) {
        if (tid < ta.n_keys) M.wlab[tid] = ta.wlab ? WLAB[tid * st.N + wl] : gp(st.label_val)[(size_t)tid * st.N + wl];
        else if (tid >= 64 && tid - 64 < ta.n_sigs) M.welig[tid - 64] = tb_elig(ta, tid - 64, wl) ? 1 : 0;
        __syncthreads();
      }
      for (int d = tid; d < tp.deltas.count; d += B) {
        const TDelta dl = cp(ta.deltas)[tp.deltas.begin + d];
        if (dl.sig >= 0 && !M.welig[dl.sig]) continue;
        const int v = dl.key >= 0 ? M.wlab[dl.key] : -1;
        // LDS atomics: a pod whose terms repeat one term carries one delta per term, on the same words
        if (dl.off >= 0) atomicAdd(&H[dl.off + (v >= 0 ? v : dl.D)], 1);
        if (v >= 0) atomicAdd(&TOT[dl.hist], 1);
      }
      if (M.wg == g) {
        const int local = wl - lo;
#pragma unroll
        for (int j = 0; j < K; ++j)
          if (local == j * B + tid) {
            assume_row(st, q, r[j], wl);
            for (int a = 0; a < tp.assume_cls.count; ++a) {
              const int col = cp(ta.aux)[tp.assume_cls.begin + a];
              gp(st.mcnt)[(size_t)col * st.N + wl] += 1;
              cc[j].v[0] += cc[j].col[0] == col ? 1 : 0;
              cc[j].v[1] += cc[j].col[1] == col ? 1 : 0;
            }
            for (int a = 0; a < tp.own_tcls.count; ++a)
              gp(st.tcnt)[(size_t)cp(ta.aux)[tp.own_tcls.begin + a] * st.N + wl] += 1;
            if (kAhead && ind_next) {
              if (vb_fast) {
                nx_ok = vb_ok;
                nx_o = vb_o;
              } else {
                nx_ok = trow_ind<FM, SM, kDef>(st, ta, qn, tpn, r[0], wl, sr[0], nx_o);
              }
            }
          }
      }
    }
    ind_have = ind_next;
    ind_ok = nx_ok;
    ind_o = nx_o;
    asm volatile("" ::"v"(qwarm.x));
    __syncthreads();
    KGPU_TSTAMP(7);
    if (kDefer && ta.diag) {
      // the cycle's rows of this lane's node, once (zeros for plugins outside the profile and for a
      // node that failed a filter)
      const int n = lo + tid;
      if (n < st.N) {
        const size_t N = (size_t)st.N;
        gp(st.status)[n] = dstat;
#pragma unroll
        for (int k = 0; k < KGPU_NUM_SCORES; ++k) {
          if (!((SM >> k) & 1u)) continue;  // outside the profile: rows no kernel writes, zero since allocation
          int64_t raw = 0, nrm = 0;
          if (k == KGPU_S_POD_TOPOLOGY_SPREAD) { raw = dt[0]; nrm = dn[2]; }
          else if (k == KGPU_S_INTER_POD_AFFINITY) { raw = dt[1]; nrm = dn[3]; }
          else if (k == KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD) { raw = dt[2]; nrm = dn[4]; }
          else if (k == KGPU_S_TAINT_TOLERATION) { raw = dv[k]; nrm = dn[0]; }
          else if (k == KGPU_S_NODE_AFFINITY) { raw = dv[k]; nrm = dn[1]; }
          else { raw = dv[k]; nrm = dv[k]; }
          gp(st.diag_raw)[(size_t)k * N + n] = raw;
          gp(st.diag_norm)[(size_t)k * N + n] = nrm;
        }
      }
    }
  }
#undef KGPU_TSTAMP
#undef KGPU_WSTAMP
  // The run's final histograms for the next run with the same tables (TCache): every workgroup loaded
  // hist_init before it published pod 0's statistics, which workgroup 0 waited for, so nobody reads
  // these words any more.  An aborted run leaves them (the host invalidates the mirror).
  if (ta.writeback && g == 0 && !M.abort) {
    for (int b = tid; b < ta.lds_bins; b += B) gp(ta.hist_init)[b] = H[b];
    for (int h = tid; h < ta.n_hists; h += B) gp(ta.tot_init)[h] = TOT[h];
  }
  if (trun) trun_row[2] = (int64_t)__builtin_amdgcn_s_memrealtime();
  leave();
}

// ---------------------------------------------------------------- cross-rank init reduction
// A node-sharded persistent topology run starts from cluster-wide histograms: every rank's partial
// (k_tbatch_init over its own nodes) is summed -- and its pair registrations / signature flags OR-ed --
// over the ranks through the init mailbox (kgpu_internal.h XReduce).  Three launches on the stream:
// k_xput copies the partial into every rank's mailbox slot of this rank, k_xflag raises this rank's
// arrival flag everywhere after a system-scope release, k_xsum waits for every rank's flag and reduces
// the nranks partials in its own mailbox into the local buffer.  Parity-indexed slots: a rank reaches
// reduction s + 2 only after every rank finished reading reduction s.
__global__ void k_xput(XReduce x) {
  const int n = x.n_sum + x.n_or;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int32_t v = x.buf[i];
    for (int r = 0; r < x.nranks; ++r)
      store_sys(x.pinit[r] + ((size_t)x.parity * x.nranks + x.rank) * kXInitCap + i, v);
  }
}
__device__ __forceinline__ uint64_t* xflags(int32_t* base, int nranks) {
  return reinterpret_cast<uint64_t*>(base + 2 * (size_t)nranks * kXInitCap);
}
__global__ void k_xflag(XReduce x) {
  __threadfence_system();
  for (int r = 0; r < x.nranks; ++r) store_sys(xflags(x.pinit[r], x.nranks) + x.parity * x.nranks + x.rank, x.seq);
}
__global__ void k_xsum(XReduce x) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    const uint64_t* f = xflags(x.pinit[x.rank], x.nranks) + x.parity * x.nranks;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    ok = 1;
    for (int r = 0; r < x.nranks && ok; ++r)
      while (load_sys(f + r) != x.seq) {
        if (load_sc1(x.abort) != 0 || __builtin_amdgcn_s_memrealtime() - t0 > kSpinTimeout) {
          __hip_atomic_store(x.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
  }
  __syncthreads();
  if (!ok) return;
  const int n = x.n_sum + x.n_or;
  const int32_t* own = x.pinit[x.rank] + (size_t)x.parity * x.nranks * kXInitCap;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int32_t acc = 0;
    for (int r = 0; r < x.nranks; ++r) {
      const int32_t v = load_sys(own + (size_t)r * kXInitCap + i);
      acc = i < x.n_sum ? acc + v : (acc | v);
    }
    x.buf[i] = acc;
  }
}

int launch_xreduce(const XReduce& x, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int n = x.n_sum + x.n_or;
  if (n <= 0 || n > kXInitCap || x.nranks < 1 || x.nranks > kMaxRanks) return -1;
  const int nb = std::min((n + 255) / 256, 256);
  hipLaunchKernelGGL(k_xput, dim3(nb), dim3(256), 0, s, x);
  hipLaunchKernelGGL(k_xflag, dim3(1), dim3(1), 0, s, x);
  hipLaunchKernelGGL(k_xsum, dim3(std::min(nb, 64)), dim3(256), 0, s, x);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------- profile instantiations
constexpr uint32_t bit(int i) { return 1u << i; }
// config (b) of BASELINE.json: NodeResourcesFit + BalancedAllocation + LeastAllocated
constexpr uint32_t kFitFM = bit(KGPU_F_NODE_RESOURCES_FIT);
constexpr uint32_t kFitSM = bit(KGPU_S_BALANCED_ALLOCATION) | bit(KGPU_S_LEAST_ALLOCATED) | kDefRes;
// the default provider (algorithmprovider/registry.go:71-155)
constexpr uint32_t kDefaultFM = (1u << KGPU_NUM_FILTERS) - 1;
constexpr uint32_t kProviderSM = (1u << (KGPU_S_MOST_ALLOCATED + 1)) - 1;  // the provider-era score plugins
constexpr uint32_t kDefaultSM = (kProviderSM & ~bit(KGPU_S_MOST_ALLOCATED)) | kDefRes;
// the ClusterAutoscalerProvider (registry.go:157-165): MostAllocated instead of LeastAllocated
constexpr uint32_t kAutoscalerSM = (kProviderSM & ~bit(KGPU_S_LEAST_ALLOCATED)) | kDefRes;

// persistent topology kernel instantiations: [profile spec][geometry] (kgpu_internal.h)
struct TGeo {
  int B, K;
};
// 512 threads x 1 or 2 rows per lane (two waves per SIMD, no VGPR spills): up to 262,144 nodes per
// GPU in 256 workgroups; larger shards take the per-pod topology launches.
// 256 x 1: one wave per SIMD, up to 65,536 nodes per GPU (KGPU_OPT_TBATCH_GEO 0; it measured equal
// to 512 x 1 at 5k nodes -- the per-pod phases are latency chains, not issue-bound -- so the default
// starts at 512 x 1).
constexpr TGeo kTGeo[] = {{256, 1}, {512, 1}, {512, 2}};
constexpr int kNumTGeo = 3;
using TBatchFn = void (*)(const DevState*, TBatchArgs);
template <uint32_t FM, uint32_t SM, bool kDef, bool XG>
struct TBatchRow {
  static constexpr TBatchFn fn[kNumTGeo] = {k_tbatch<256, 1, FM, SM, kDef, XG>, k_tbatch<512, 1, FM, SM, kDef, XG>,
                                            k_tbatch<512, 2, FM, SM, kDef, XG>};
};
// rows: 0 generic, 1 generic with Least/Most over {cpu:1, memory:1}, 2 default provider,
// 3 ClusterAutoscaler provider; [1]: the node-sharded (xGMI) instantiations
static const TBatchFn* const kTBatch[2][4] = {
    {TBatchRow<kRuntime, kRuntime, false, false>::fn, TBatchRow<kRuntime, kRuntime, true, false>::fn,
     TBatchRow<kDefaultFM, kDefaultSM, true, false>::fn, TBatchRow<kDefaultFM, kAutoscalerSM, true, false>::fn},
    {TBatchRow<kRuntime, kRuntime, false, true>::fn, TBatchRow<kRuntime, kRuntime, true, true>::fn,
     TBatchRow<kDefaultFM, kDefaultSM, true, true>::fn, TBatchRow<kDefaultFM, kAutoscalerSM, true, true>::fn}};

int64_t kernel_layout_sig() { return layout_sig_of(); }

int tbatch_geometry(int N, int max_groups, int* per, int* groups, int first) {
  for (int gi = first < 0 ? 0 : first; gi < kNumTGeo; ++gi) {
    const int p = kTGeo[gi].B * kTGeo[gi].K;
    const int g = (N + p - 1) / p;
    if (g <= max_groups) {
      *per = p;
      *groups = g < 1 ? 1 : g;
      return gi;
    }
  }
  return -1;
}

// An ordinary launch of a persistent grid is only as good as its residency: the grid must fit the GPU at
// once (MI355X_MICROARCH.md coop-launch: a plain launch of a grid the cooperative check would accept has
// the same residency).  Queried once per kernel instantiation and block shape; false sends the launch
// through hipLaunchCooperativeKernel, which refuses a grid that cannot be co-resident.
static bool grid_fits(const void* fn, int threads, size_t lds, int groups) {
  static std::mutex mu;
  static std::map<std::tuple<const void*, int, size_t>, int> cap;  // workgroups the device holds at once
  std::lock_guard<std::mutex> lock(mu);
  auto key = std::make_tuple(fn, threads, lds);
  auto it = cap.find(key);
  if (it == cap.end()) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, lds) != hipSuccess) per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 0;
    it = cap.emplace(key, per_cu * cus).first;
  }
  return groups <= it->second;
}

int launch_tbatch_init(const DevState* st, const TBatchArgs& a, int groups, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int N = a.per * groups;  // >= st->N
  const int nb = (N + 255) / 256;
  const int nlh = a.lds_bins + a.n_hists;
  if (nlh <= kInitLdsBins)
    hipLaunchKernelGGL(k_tbatch_init<true>, dim3(nb), dim3(256), (unsigned)(sizeof(int32_t) * (size_t)std::max(nlh, 1)), s, st, a);
  else
    hipLaunchKernelGGL(k_tbatch_init<false>, dim3(nb), dim3(256), 0, s, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// spec: the k_eval profile instantiation (select_spec), def_res from the TBatchArgs
int launch_tbatch(const DevState* st, const TBatchArgs& a, int groups, int geo, int spec, bool xg, bool coop,
                  void* stream) {
  if (geo < 0 || geo >= kNumTGeo) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int row = spec == 2 ? 2 : (spec == 3 ? 3 : (a.def_res ? 1 : 0));
  const TBatchFn fn = kTBatch[xg ? 1 : 0][row][geo];
  static bool attr[2][4][kNumTGeo] = {};
  if (!attr[xg ? 1 : 0][row][geo]) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            kTLdsBudget) != hipSuccess)
      return -1;
    attr[xg ? 1 : 0][row][geo] = true;
  }
  // one workgroup per CU (>= 80 KB of LDS each); the cooperative launch checks co-residency
  TBatchArgs arg = a;
  const DevState* sp = st;
  void* args[] = {(void*)&sp, (void*)&arg};
  if (!coop && grid_fits(reinterpret_cast<const void*>(fn), kTGeo[geo].B, (size_t)a.lds_bytes, groups)) {
    hipLaunchKernelGGL(fn, dim3(groups), dim3(kTGeo[geo].B), (unsigned)a.lds_bytes, s, sp, arg);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  arg.hold = -1;
  return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(fn), dim3(groups), dim3(kTGeo[geo].B), args,
                                    (unsigned)a.lds_bytes, s) == hipSuccess
             ? 0
             : -1;
}

struct SpecEntry {
  uint32_t fm, sm;
  void (*fn)(const DevState*, PodArgs);
};
static const SpecEntry kSpecs[] = {
    {kRuntime, kRuntime, k_eval<kRuntime, kRuntime>},
    {kFitFM, kFitSM, k_eval<kFitFM, kFitSM>},
    {kDefaultFM, kDefaultSM, k_eval<kDefaultFM, kDefaultSM>},
    {kDefaultFM, kAutoscalerSM, k_eval<kDefaultFM, kAutoscalerSM>},
};
constexpr int kNumSpecs = sizeof(kSpecs) / sizeof(kSpecs[0]);

int select_spec(const int32_t* filters, int nf, const int32_t* scores, int ns, bool def_res) {
  uint32_t fm = 0, sm = 0;
  for (int i = 0; i < nf; ++i) {
    if (i > 0 && filters[i] <= filters[i - 1]) return 0;  // not in ascending (default) order
    fm |= bit(filters[i]);
  }
  for (int i = 0; i < ns; ++i) sm |= bit(scores[i]);
  const bool uses_res = (sm & (bit(KGPU_S_LEAST_ALLOCATED) | bit(KGPU_S_MOST_ALLOCATED))) != 0;
  if (uses_res) {
    if (!def_res) return 0;
    sm |= kDefRes;
  }
  for (int s = 1; s < kNumSpecs; ++s) {
    const uint32_t want = kSpecs[s].sm & (uses_res ? ~0u : ~kDefRes);
    if (kSpecs[s].fm == fm && want == sm) return s;
  }
  return 0;
}

// Persistent geometries: (threads per workgroup, rows per lane).  256 x 1 keeps small clusters
// on few workgroups; 1024 x 1 gives 4 waves per SIMD; 512 x 4 holds up to 524,288 nodes per GPU
// (256 workgroups x 2048 rows) with every row in registers and no spills.  Larger shards take the
// one-launch-per-pod path.
struct Geo {
  int B, K;
};
constexpr Geo kGeo[] = {{64, 1}, {128, 1}, {192, 1}, {448, 1}, {960, 1}, {512, 4}};  // B row threads (+ one communication wave), K slots per lane
constexpr int kNumGeo = 6;
constexpr int kBatchLdsPad = 96 * 1024;

template <uint32_t FM, uint32_t SM>
struct BatchRow {
  using Fn = void (*)(const DevState*, BatchArgs);
  static constexpr Fn fn[kNumGeo] = {k_batch<FM, SM, 1, 64, false>,  k_batch<FM, SM, 1, 128, false>,
                                     k_batch<FM, SM, 1, 192, false>, k_batch<FM, SM, 1, 448, false>,
                                     k_batch<FM, SM, 1, 960, false>, k_batch<FM, SM, 4, 512, false>};
  static constexpr Fn xfn[kNumGeo] = {k_batch<FM, SM, 1, 64, true>,  k_batch<FM, SM, 1, 128, true>,
                                      k_batch<FM, SM, 1, 192, true>, k_batch<FM, SM, 1, 448, true>,
                                      k_batch<FM, SM, 1, 960, true>, k_batch<FM, SM, 4, 512, true>};
};
using BatchFn = void (*)(const DevState*, BatchArgs);
// the helper-wave instantiation (HB) of config (b)'s profile on the one-row-wave geometry
template <uint32_t FM, uint32_t SM, bool E>
struct HelperFn {
  static constexpr BatchFn fn = nullptr;
};
template <uint32_t FM, uint32_t SM>
struct HelperFn<FM, SM, true> {
  static constexpr BatchFn fn = k_batch<FM, SM, 1, 64, false, true>;
};
static const BatchFn kBatchHelper[] = {
    nullptr,
    HelperFn<kFitFM, kFitSM, true>::fn,
    nullptr,
    nullptr,
};
static const BatchFn* const kBatch[] = {
    BatchRow<kRuntime, kRuntime>::fn,
    BatchRow<kFitFM, kFitSM>::fn,
    BatchRow<kDefaultFM, kDefaultSM>::fn,
    BatchRow<kDefaultFM, kAutoscalerSM>::fn,
};
static_assert(sizeof(kBatch) / sizeof(kBatch[0]) == kNumSpecs, "one k_batch row per profile instantiation");
static const BatchFn* const kBatchX[] = {
    BatchRow<kRuntime, kRuntime>::xfn,
    BatchRow<kFitFM, kFitSM>::xfn,
    BatchRow<kDefaultFM, kDefaultSM>::xfn,
    BatchRow<kDefaultFM, kAutoscalerSM>::xfn,
};

int batch_geometry(int N, int max_groups, int* per, int* groups, int first) {
  for (int gi = first < 0 ? 0 : first; gi < kNumGeo; ++gi) {
    const int p = kGeo[gi].B * kGeo[gi].K - 1;  // the last slot of the last lane is the spare
    const int g = (N + p - 1) / p;
    if (g <= max_groups) {
      *per = p;
      *groups = g < 1 ? 1 : g;
      return gi;
    }
  }
  return -1;
}

int launch_batch(const DevState* st, const BatchArgs& a, int groups, int geo, int spec, bool coop, bool helper,
                 void* stream) {
  if (spec < 0 || spec >= kNumSpecs) spec = 0;
  if (geo < 0 || geo >= kNumGeo) return -1;
  // One workgroup per CU: a dynamic LDS reservation above half a CU's 160 KB keeps the dispatcher
  // from stacking two persistent workgroups on one CU (they would share its SIMDs).
  const int x = a.R > 0 ? 1 : 0;  // node-sharded over xGMI mailboxes
  const bool hb = helper && !x && geo == 0 && kBatchHelper[spec] != nullptr;
  const BatchFn fn = hb ? kBatchHelper[spec] : (x ? kBatchX : kBatch)[spec][geo];
  const int threads = kGeo[geo].B + 64 + (hb ? 2 * kGeo[geo].B : 0);
  static bool attr_set[3][kNumSpecs][kNumGeo] = {};
  const int ai = hb ? 2 : x;
  if (!attr_set[ai][spec][geo]) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            kBatchLdsPad) != hipSuccess)
      return -1;
    attr_set[ai][spec][geo] = true;
  }
  // Cooperative: the runtime refuses a grid whose workgroups cannot all be resident at once, so
  // the granule exchange never waits on a workgroup that has not started.
  BatchArgs arg = a;
  const DevState* sp = st;
  void* args[] = {(void*)&sp, (void*)&arg};
  // (coop false, KGPU_OPT_COOPERATIVE: an ordinary launch of the same grid -- at most one workgroup per
  // CU on an otherwise idle device, so every workgroup is resident; were one not, the spins time out
  // into the abort word rather than hang)
  if (!coop && grid_fits(reinterpret_cast<const void*>(fn), threads, (size_t)kBatchLdsPad, groups)) {
    hipLaunchKernelGGL(fn, dim3(groups), dim3(threads), (unsigned)kBatchLdsPad, (hipStream_t)stream, sp, arg);
    if (hipGetLastError() != hipSuccess) return -1;
  } else {
    arg.hold = -1;  // every workgroup of a cooperative launch is resident
    if (hipLaunchCooperativeKernel(reinterpret_cast<const void*>(fn), dim3(groups), dim3(threads), args,
                                   (unsigned)kBatchLdsPad, (hipStream_t)stream) != hipSuccess)
      return -1;
  }
  hipLaunchKernelGGL(k_batch_fixup, dim3((a.count + 3) / 4), dim3(256), 0, (hipStream_t)stream, st, a, groups);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int eval_blocks(int N) {
  int b = (N + kBlock - 1) / kBlock;
  if (b > kMaxBlocks) b = kMaxBlocks;
  if (b < 1) b = 1;
  return b;
}

int launch_eval(const DevState* st, const PodArgs& a, int blocks, int spec, void* stream) {
  if (spec < 0 || spec >= kNumSpecs) spec = 0;
  hipLaunchKernelGGL(kSpecs[spec].fn, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_final(const DevState* st, const PodArgs& a, int blocks, int stat_blocks, void* stream) {
  hipLaunchKernelGGL(k_final, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, st, a, stat_blocks);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_cut(const DevState* st, const PodArgs& a, int blocks, int n_filters, void* stream) {
  hipLaunchKernelGGL(k_cut, dim3(1), dim3(kCutThreads), 0, (hipStream_t)stream, st, a, blocks, n_filters);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_resolve(const DevState* st, int N, const PodArgs& a, void* stream) {
  // same grid as the evaluation so that chunk ownership matches
  hipLaunchKernelGGL(k_resolve, dim3(eval_blocks(N)), dim3(kBlock), 0, (hipStream_t)stream, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_shard_pack(const DevState* st, int parity, int blocks, int what, void* stream) {
  hipLaunchKernelGGL(k_shard_pack, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, st, parity, blocks, what);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------- delta stream (kgpu_apply_delta)
// NodeInfo.AddPod / RemovePod (types.go:456-533) and SetNode (types.go:587-600) for a batch of
// cache events.  One workgroup per node walks that node's ops in batch order (an op's host ports
// depend on the previous op on the same node); rows of different nodes are disjoint, so the
// groups run in parallel.  Inside an op the lanes split the class columns, label keys and taints.
__global__ __launch_bounds__(kBlock) void k_delta(const DevState* __restrict__ stp, DeltaArgs a) {
  const DevState& st = *stp;
  const int lane = threadIdx.x;
  const size_t N = (size_t)st.N;
  const int o0 = a.group_off[blockIdx.x], o1 = a.group_off[blockIdx.x + 1];
  for (int o = o0; o < o1; ++o) {
    const DeltaOp op = a.ops[o];
    const int n = op.node;
    if (op.kind == kDSetNode) {
      const kgpu_node_row r = a.rows[op.item];
      if (lane == 0) {
        gp(st.alloc_cpu)[n] = r.alloc_cpu;
        gp(st.alloc_mem)[n] = r.alloc_mem;
        gp(st.alloc_eph)[n] = r.alloc_eph;
        gp(st.alloc_pods)[n] = r.alloc_pods;
        gp(st.unsched)[n] = (uint8_t)(r.unschedulable ? 1 : 0);
        gp(st.zone_id)[n] = r.zone_id;
      }
      for (int k = lane; k < st.K; k += kBlock) {
        int32_t v = -1;
        for (int j = 0; j + 1 < r.labels.count; j += 2)
          if (a.ints[r.labels.begin + j] == k) v = a.ints[r.labels.begin + j + 1];
        gp(st.label_val)[(size_t)k * N + n] = v;
      }
      for (int w = lane; w < st.TW; w += kBlock) {
        const bool has = r.taints.count >= 2 * st.TW;
        gp(st.taint_nosched)[(size_t)w * N + n] = has ? a.words[r.taints.begin + w] : 0ull;
        gp(st.taint_prefer)[(size_t)w * N + n] = has ? a.words[r.taints.begin + st.TW + w] : 0ull;
      }
      for (int sc = lane; sc < st.S; sc += kBlock)
        gp(st.alloc_scalar)[(size_t)sc * N + n] =
            sc < r.alloc_scalar.count ? (int64_t)a.words[r.alloc_scalar.begin + sc] : 0;
    } else {
      const kgpu_pod_query q = a.pods[op.item];
      const int64_t sg = op.kind == kDAddPod ? 1 : -1;
      if (lane == 0) {
        gp(st.req_cpu)[n] += sg * q.req[0];
        gp(st.req_mem)[n] += sg * q.req[1];
        gp(st.req_eph)[n] += sg * q.req[2];
        gp(st.nz_cpu)[n] += sg * q.nz[0];
        gp(st.nz_mem)[n] += sg * q.nz[1];
        gp(st.num_pods)[n] += (int32_t)sg;
        for (int i = 0; i < q.scalars.count; ++i) {
          const kgpu_scalar_req sr = a.scalars[q.scalars.begin + i];
          if (sr.col >= 0) gp(st.req_scalar)[(size_t)sr.col * N + n] += sg * sr.value;
        }
        // NodeInfo.UsedPorts is a set per (ip, protocol, port): Add is idempotent, Remove drops the
        // entry (types.go:728-745, HostPortInfo.Add/Remove host_ports.go)
        int pc = gp(st.port_count)[n];
        for (int i = 0; i < q.ports.count; ++i) {
          const kgpu_port w = a.ports[q.ports.begin + i];
          int at = -1;
          for (int s = 0; s < pc; ++s) {
            const kgpu_port p = gp(st.ports)[(size_t)s * N + n];
            if (p.ip == w.ip && p.proto == w.proto && p.port == w.port) at = s;
          }
          if (sg > 0) {
            if (at >= 0) continue;
            if (pc >= st.PS) {
              gp(st.port_overflow)[0] = 1;
              continue;
            }
            gp(st.ports)[(size_t)(pc++) * N + n] = w;
          } else if (at >= 0) {
            gp(st.ports)[(size_t)at * N + n] = gp(st.ports)[(size_t)(pc - 1) * N + n];
            --pc;
          }
        }
        gp(st.port_count)[n] = pc;
      }
      for (int i = lane; i < op.cls.count; i += kBlock)
        gp(st.mcnt)[(size_t)a.aux[op.cls.begin + i] * N + n] += (int32_t)sg;
      for (int i = lane; i < op.tcls.count; i += kBlock)
        gp(st.tcnt)[(size_t)a.aux[op.tcls.begin + i] * N + n] += (int32_t)sg;
    }
    __syncthreads();
  }
}

int launch_delta(const DevState* st, const DeltaArgs& a, void* stream) {
  if (a.n_ops <= 0 || a.n_groups <= 0) return 0;
  hipLaunchKernelGGL(k_delta, dim3(a.n_groups), dim3(kBlock), 0, (hipStream_t)stream, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Node-list rebuild: one grid-stride pass per column table (blockIdx.y), every element a
// coalesced load from its old row.
__global__ void k_remap(const RemapCol* __restrict__ cols, const int32_t* __restrict__ from, int old_n, int new_n) {
  const RemapCol c = cols[blockIdx.y];
  const size_t total = (size_t)c.ncols * (size_t)new_n;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const size_t col = e / (size_t)new_n, i = e - col * (size_t)new_n;
    const int f = from[i];
    const size_t so = col * (size_t)old_n + (size_t)(f < 0 ? 0 : f);
    switch (c.elem) {
      case 1: gp((uint8_t*)c.dst)[e] = f < 0 ? 0 : cp((const uint8_t*)c.src)[so]; break;
      case 4: gp((int32_t*)c.dst)[e] = f < 0 ? 0 : cp((const int32_t*)c.src)[so]; break;
      case 8: gp((int64_t*)c.dst)[e] = f < 0 ? 0 : cp((const int64_t*)c.src)[so]; break;
      default: {
        const kgpu_port z{0, 0, 0, 0};
        gp((kgpu_port*)c.dst)[e] = f < 0 ? z : cp((const kgpu_port*)c.src)[so];
      }
    }
  }
}

int launch_remap(const RemapCol* cols, int n_cols, const int32_t* from, int old_n, int new_n, void* stream) {
  if (n_cols <= 0 || new_n <= 0) return 0;
  const int blocks = (new_n + 255) / 256 < 1024 ? (new_n + 255) / 256 : 1024;
  hipLaunchKernelGGL(k_remap, dim3(blocks, n_cols), dim3(256), 0, (hipStream_t)stream, cols, from, old_n, new_n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------- nominated pods / preemption
// (kgpu_internal.h "nominated pods / preemption").  Reference semantics:
//   addNominatedPods / podPassesFiltersOnNode   core/generic_scheduler.go:526-615
//   selectVictimsOnNode                         core/generic_scheduler.go:921-1012
//   filterPodsWithPDBViolation                  core/generic_scheduler.go:878-919
//   PodTopologySpread AddPod / RemovePod        podtopologyspread/filtering.go:93-180 (criticalPaths)
//   InterPodAffinity AddPod / RemovePod         interpodaffinity/filtering.go:75-148, 277-296
// One thread per node re-runs the profile's filters on a private, delta-adjusted view of its own
// node: every pod added or removed by these paths sits on that node, so each plugin's state moves
// only at the node's own topology pairs.  NodeInfo.Requested / len(Pods) / UsedPorts are the node's
// row plus the deltas; TpPairToMatchNum and the three inter-pod affinity maps are the PreFilter
// histograms (k_topo_pre) plus the deltas at the node's pairs; criticalPaths[0] after any sequence of
// updates to one pair equals min(minimum over the key's other registered pairs, the pair's count)
// (k_vict_prep supplies the minimum and the runner-up).
enum { kVRemoved = 0, kVKept = 1, kVEvicted = 2, kVViolating = 4 };

struct VCtx {
  const DevState* st;
  const PreemptArgs* a;
  const kgpu_pod_query* q;
  const QPlan* pl;     // null: no topology state (PodTopologySpread / InterPodAffinity pass)
  int n;               // local node
  int v0, v1, m0, m1;  // victim / nominated ranges
  bool removal;        // the potential victims were removed (selectVictimsOnNode, first step done)
  bool pass1;          // nominated pods added
  int trial;           // victim being reprieved (-1 none)
  int step;            // reprieve steps processed before the trial (a->order[v0 .. v0 + step))
};

// sign of an effect in the current view: victims -1 while removed, nominated pods +1 in pass 1
__device__ __forceinline__ int v_sign(const VCtx& c, int v) {
  return (c.removal && (c.a->vstate[v] & 3) != kVKept) ? -1 : 0;
}

__device__ __forceinline__ bool port_eq(const kgpu_port& x, const kgpu_port& y) {
  return x.ip == y.ip && x.proto == y.proto && x.port == y.port;
}
__device__ __forceinline__ bool port_conflicts(const kgpu_port& e, const kgpu_port& w) {
  return e.port == w.port && e.proto == w.proto && (w.ip == 0 || e.ip == 0 || e.ip == w.ip);
}
__device__ __forceinline__ bool rec_has_port(const kgpu_pod_query& r, const kgpu_port* pool, const kgpu_port& e) {
  for (int i = 0; i < r.ports.count; ++i)
    if (port_eq(pool[r.ports.begin + i], e)) return true;
  return false;
}
__device__ __forceinline__ const kgpu_pod_query& vrec(const VCtx& c, int v) { return c.a->v_recs[c.a->veff[v].item]; }
__device__ __forceinline__ const kgpu_pod_query& nrec(const VCtx& c, int m) { return c.a->n_recs[c.a->neff[m].item]; }

// HostPortInfo membership of entry e on the adjusted node (types.go:726-756 set semantics): the
// last Add / Remove touching it wins -- removals of every potential victim, then the reprieve
// sequence (a kept pod re-adds its ports, an evicted one adds and removes them), then the trial
// pod and (pass 1) the nominated pods.
__device__ bool port_present(const VCtx& c, const kgpu_port& e) {
  const DevState& st = *c.st;
  if (c.pass1)
    for (int m = c.m0; m < c.m1; ++m)
      if (rec_has_port(nrec(c, m), c.a->n_ports, e)) return true;
  if (c.removal) {
    if (c.trial >= 0 && rec_has_port(vrec(c, c.trial), c.a->v_ports, e)) return true;
    for (int k = c.step - 1; k >= 0; --k) {
      const int v = c.a->order[c.v0 + k];
      if (rec_has_port(vrec(c, v), c.a->v_ports, e)) return (c.a->vstate[v] & 3) == kVKept;
    }
    for (int v = c.v0; v < c.v1; ++v)
      if (rec_has_port(vrec(c, v), c.a->v_ports, e)) return false;
  }
  const int have = gp(st.port_count)[c.n];
  for (int s = 0; s < have; ++s)
    if (port_eq(gp(st.ports)[(size_t)s * st.N + c.n], e)) return true;
  return false;
}

__device__ bool ports_conflict_adj(const VCtx& c) {
  const DevState& st = *c.st;
  const kgpu_pod_query& q = *c.q;
  for (int i = 0; i < q.ports.count; ++i) {
    const kgpu_port w = st.qp.ports[q.ports.begin + i];
    const int have = gp(st.port_count)[c.n];
    for (int s = 0; s < have; ++s) {
      const kgpu_port e = gp(st.ports)[(size_t)s * st.N + c.n];
      if (port_conflicts(e, w) && port_present(c, e)) return true;
    }
    for (int v = c.v0; v < c.v1; ++v) {
      const kgpu_pod_query& r = vrec(c, v);
      for (int j = 0; j < r.ports.count; ++j) {
        const kgpu_port e = c.a->v_ports[r.ports.begin + j];
        if (port_conflicts(e, w) && port_present(c, e)) return true;
      }
    }
    if (c.pass1)
      for (int m = c.m0; m < c.m1; ++m) {
        const kgpu_pod_query& r = nrec(c, m);
        for (int j = 0; j < r.ports.count; ++j) {
          const kgpu_port e = c.a->n_ports[r.ports.begin + j];
          if (port_conflicts(e, w) && port_present(c, e)) return true;
        }
      }
  }
  return false;
}

// NodeResourcesFit on the adjusted NodeInfo (fit.go:194-267): Requested and len(Pods) move by the
// added / removed pods' requests (NodeInfo.AddPod / RemovePod, types.go:456-533).
__device__ uint32_t fit_adj(const VCtx& c) {
  const DevState& st = *c.st;
  const kgpu_pod_query& q = *c.q;
  NodeRes r = load_res(st, c.n);
  for (int v = c.v0; v < c.v1; ++v) {
    const int sg = v_sign(c, v);
    if (!sg) continue;
    const kgpu_pod_query& p = vrec(c, v);
    r.rc += sg * p.req[0]; r.rm += sg * p.req[1]; r.re += sg * p.req[2]; r.np += sg;
  }
  if (c.pass1)
    for (int m = c.m0; m < c.m1; ++m) {
      const kgpu_pod_query& p = nrec(c, m);
      r.rc += p.req[0]; r.rm += p.req[1]; r.re += p.req[2]; r.np += 1;
    }
  uint32_t d = 0;
  if (r.np + 1 > r.ap) d |= 1u;
  if (!(q.flags & KGPU_Q_FIT_ALL_ZERO)) {
    if (r.ac < q.req[0] + r.rc) d |= 2u;
    if (r.am < q.req[1] + r.rm) d |= 4u;
    if (r.ae < q.req[2] + r.re) d |= 8u;
    for (int i = 0; i < q.scalars.count; ++i) {
      const kgpu_scalar_req s = st.qp.scalars[q.scalars.begin + i];
      if (!s.check) continue;
      const int64_t alloc = s.col >= 0 ? gp(st.alloc_scalar)[(size_t)s.col * st.N + c.n] : 0;
      int64_t used = s.col >= 0 ? gp(st.req_scalar)[(size_t)s.col * st.N + c.n] : 0;
      if (s.col >= 0) {
        for (int v = c.v0; v < c.v1; ++v) {
          const int sg = v_sign(c, v);
          if (!sg) continue;
          const kgpu_pod_query& p = vrec(c, v);
          for (int j = 0; j < p.scalars.count; ++j) {
            const kgpu_scalar_req t = c.a->v_scalars[p.scalars.begin + j];
            if (t.col == s.col) used += sg * t.value;
          }
        }
        if (c.pass1)
          for (int m = c.m0; m < c.m1; ++m) {
            const kgpu_pod_query& p = nrec(c, m);
            for (int j = 0; j < p.scalars.count; ++j) {
              const kgpu_scalar_req t = c.a->n_scalars[p.scalars.begin + j];
              if (t.col == s.col) used += t.value;
            }
          }
      }
      if (alloc < s.value + used) d |= 16u << (i < 11 ? i : 11);
    }
  }
  return d ? (KGPU_CODE_UNSCHEDULABLE << 8) | (d << 16) : 0;
}

// Sum of the signed effects selected by `pick(PEff)` (victims then nominated pods).
template <class Pick>
__device__ __forceinline__ int64_t eff_sum(const VCtx& c, Pick pick) {
  int64_t s = 0;
  for (int v = c.v0; v < c.v1; ++v) {
    const int sg = v_sign(c, v);
    if (sg) s += sg * (int64_t)pick(c.a->veff[v]);
  }
  if (c.pass1)
    for (int m = c.m0; m < c.m1; ++m) s += (int64_t)pick(c.a->neff[m]);
  return s;
}

// PodTopologySpread Filter (filtering.go:276-328) after updateWithPod of the effects (:123-143).
__device__ uint32_t pts_adj(const VCtx& c) {
  const DevState& st = *c.st;
  const QPlan& pl = *c.pl;
  if (pl.n_hard == 0) return 0;
  const TopoHdr* h = hdr(st);
  const bool keys = all_keys(st, pl.hard, pl.n_hard, c.n);  // nodeLabelsMatchSpreadConstraints
  int64_t d[kMaxSpread];
  bool any = h->pany != 0;
  for (int i = 0; i < pl.n_hard; ++i) {
    d[i] = 0;
    if (!keys) continue;
    // TpPairToMatchNum is keyed by (key, value): constraints on the same key share the pair
    for (int j = 0; j < pl.n_hard; ++j)
      if (pl.hard[j].key == pl.hard[i].key) d[i] += eff_sum(c, [j](const PEff& e) { return (e.pts_mask >> j) & 1u; });
    const int v = nval(st, pl.hard[i].key, c.n);
    if (d[i] != 0 && !slot_ptr(st, pl, pl.hard[i].rslot)[v]) any = true;  // a pair no eligible node registered
  }
  if (!any) return 0;
  for (int i = 0; i < pl.n_hard; ++i) {
    const TSpread& t = pl.hard[i];
    const int v = nval(st, t.key, c.n);
    if (v < 0) return KGPU_CODE_UNSCHEDULABLE << 8;
    const bool reg = slot_ptr(st, pl, t.rslot)[v] != 0;
    const int64_t cnt = (reg ? slot_ptr(st, pl, t.cslot)[v] : 0) + d[i];
    const int64_t* pr = c.a->prep + 3 * i;
    const int64_t mo = (reg && v == pr[1]) ? pr[2] : pr[0];
    int64_t mn = (reg || d[i] != 0) ? min(mo, cnt) : pr[0];
    if (mn == INT64_MAX) mn = 2147483647;  // criticalPaths initial MatchNum
    if (cnt + t.self_match - mn > t.max_skew) return KGPU_CODE_UNSCHEDULABLE << 8;
  }
  return 0;
}

// InterPodAffinity Filter (filtering.go:314-396) after updateWithPod of the effects (:75-90).
__device__ uint32_t ipa_adj(const VCtx& c) {
  const DevState& st = *c.st;
  const QPlan& pl = *c.pl;
  const TopoHdr* h = hdr(st);
  if (pl.n_aff) {  // satisfyPodAffinity
    const int64_t ad = eff_sum(c, [](const PEff& e) { return e.aff_all; });
    bool exist = true;
    int64_t nz = c.a->prep[3 * kMaxSpread];  // len(topologyToMatchedAffinityTerms) before the effects
    for (int i = 0; i < pl.n_aff; ++i) {
      const int v = nval(st, pl.aff[i].key, c.n);
      if (v < 0) return (KGPU_CODE_UNRESOLVABLE << 8) | (1u << 16);
      int mult = 0, first = i;
      for (int j = 0; j < pl.n_aff; ++j)
        if (pl.aff[j].slot == pl.aff[i].slot) {
          ++mult;
          if (j < first) first = j;
        }
      const int64_t b = slot_ptr(st, pl, pl.aff[i].slot)[v];
      const int64_t val = b + ad * mult;
      if (val <= 0) exist = false;
      if (first == i) nz += (val != 0) - (b != 0);
    }
    if (!exist && !(nz == 0 && pl.self_all)) return (KGPU_CODE_UNRESOLVABLE << 8) | (1u << 16);
  }
  for (int i = 0; i < pl.n_anti; ++i) {  // satisfyPodAntiAffinity
    const int v = nval(st, pl.anti[i].key, c.n);
    if (v < 0) continue;
    int64_t val = slot_ptr(st, pl, pl.anti[i].slot)[v];
    for (int j = 0; j < pl.n_anti; ++j)
      if (pl.anti[j].slot == pl.anti[i].slot) val += eff_sum(c, [j](const PEff& e) { return (e.anti_mask >> j) & 1u; });
    if (val > 0) return (KGPU_CODE_UNSCHEDULABLE << 8) | (2u << 16);
  }
  // satisfyExistingPodsAntiAffinity: every node label pair; only the node's own pairs move
  auto key_delta = [&](int key) -> int64_t {
    int64_t s = 0;
    for (int v = c.v0; v < c.v1; ++v) {
      const int sg = v_sign(c, v);
      if (!sg) continue;
      const PEff& e = c.a->veff[v];
      for (int k = 0; k < e.exa.count; ++k) s += sg * (c.a->aux[e.exa.begin + k] == key);
    }
    if (c.pass1)
      for (int m = c.m0; m < c.m1; ++m) {
        const PEff& e = c.a->neff[m];
        for (int k = 0; k < e.exa.count; ++k) s += (c.a->aux[e.exa.begin + k] == key);
      }
    return s;
  };
  for (int s = 0; s < pl.n_slots; ++s) {
    if (pl.slot_kind[s] != kSlotExA) continue;
    const int v = nval(st, pl.slot_key[s], c.n);
    if (v >= 0 && (h->ex_any ? slot_ptr(st, pl, s)[v] : 0) + key_delta(pl.slot_key[s]) > 0)
      return (KGPU_CODE_UNSCHEDULABLE << 8) | (3u << 16);
  }
  // keys of the effects' terms that no existing pod's term registered a histogram for
  auto key_checked = [&](int key) {
    for (int s = 0; s < pl.n_slots; ++s)
      if (pl.slot_kind[s] == kSlotExA && pl.slot_key[s] == key) return true;
    return false;
  };
  auto scan = [&](const PEff& e) -> bool {
    for (int k = 0; k < e.exa.count; ++k) {
      const int key = c.a->aux[e.exa.begin + k];
      if (key_checked(key) || nval(st, key, c.n) < 0) continue;
      if (key_delta(key) > 0) return true;
    }
    return false;
  };
  for (int v = c.v0; v < c.v1; ++v)
    if (v_sign(c, v) && scan(c.a->veff[v])) return (KGPU_CODE_UNSCHEDULABLE << 8) | (3u << 16);
  if (c.pass1)
    for (int m = c.m0; m < c.m1; ++m)
      if (scan(c.a->neff[m])) return (KGPU_CODE_UNSCHEDULABLE << 8) | (3u << 16);
  return 0;
}

// RunFilterPlugins + Merge on the adjusted view, profile order, first failure wins -- or, with
// runAllFilters, every plugin's word merged (and, with `all`, stored in status_all: the nominated pass
// 1 that becomes the cycle's verdict on the node).
__device__ uint32_t eval_adj(const VCtx& c, bool all = false) {
  const DevState& st = *c.st;
  const NodeRes r0 = load_res(st, c.n);
  uint32_t acc = 0;
  for (int i = 0; i < st.n_filters; ++i) {
    const int f = st.filters[i];
    uint32_t code;
    switch (f) {
      case KGPU_F_NODE_RESOURCES_FIT: code = fit_adj(c); break;
      case KGPU_F_NODE_PORTS: code = (c.q->ports.count && ports_conflict_adj(c)) ? KGPU_CODE_UNSCHEDULABLE << 8 : 0; break;
      case KGPU_F_POD_TOPOLOGY_SPREAD: code = c.pl ? pts_adj(c) : 0; break;
      case KGPU_F_INTER_POD_AFFINITY: code = c.pl ? ipa_adj(c) : 0; break;
      default: code = filter_one(f, st, *c.q, r0, c.n); break;  // NodeInfo-independent of pods
    }
    const uint32_t w = code ? code | (uint32_t)(i + 1) : 0u;
    if (!st.run_all) {
      if (w) return w;
      continue;
    }
    if (all) gp(st.status_all)[(size_t)i * st.N + c.n] = w;
    acc = w ? merge_status(acc, w) : acc;
  }
  return acc;
}

// podPassesFiltersOnNode: pass 1 with the nominated pods (only when some were added), pass 2 without.
__device__ uint32_t check_two_pass(VCtx& c) {
  if (c.m1 > c.m0) {
    c.pass1 = true;
    const uint32_t s = eval_adj(c);
    c.pass1 = false;
    if (s) return s;
  }
  return eval_adj(c);
}

__global__ __launch_bounds__(64) void k_victims(const DevState* __restrict__ stp, const PreemptArgs* __restrict__ ap) {
  const DevState& st = *stp;
  const PreemptArgs& a = *ap;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= st.N) return;
  VCtx c;
  c.st = stp;
  c.a = ap;
  c.q = st.queries + a.pod;
  c.pl = st.plans ? st.plans + a.pod : nullptr;
  c.n = n;
  c.v0 = a.v_off[n];
  c.v1 = a.v_off[n + 1];
  c.m0 = a.n_off[n];
  c.m1 = a.n_off[n + 1];
  c.removal = false;
  c.pass1 = false;
  c.trial = -1;
  c.step = 0;
  if (!a.preempt) {  // nominated pass 1 of a scheduling cycle
    if (c.m1 > c.m0) {
      c.pass1 = true;
      a.nom_status[n] = eval_adj(c, true);
    }
    return;
  }
  kgpu_node_victims out{0, 0, 0, c.v0};
  // nodesWherePreemptionMightHelp: the cycle's own verdict on the node
  const uint32_t base = check_two_pass(c);
  if (((base >> 8) & 3u) == KGPU_CODE_UNRESOLVABLE) {
    a.out[n] = out;
    return;
  }
  for (int v = c.v0; v < c.v1; ++v) a.vstate[v] = kVRemoved;
  c.removal = true;
  if (check_two_pass(c)) {
    a.out[n] = out;
    return;
  }
  // filterPodsWithPDBViolation over the victims in MoreImportantPod order (host-sorted)
  int32_t allowed[64];
  for (int j = 0; j < a.n_pdbs; ++j) allowed[j] = a.pdb_allowed[j];
  int k = 0;
  for (int v = c.v0; v < c.v1; ++v) {
    uint64_t m = a.veff[v].pdb_mask;
    bool viol = false;
    while (m) {
      const int j = __builtin_ctzll(m);
      m &= m - 1;
      if (allowed[j] <= 0) {
        viol = true;
        break;
      }
      --allowed[j];
    }
    if (viol) {
      a.vstate[v] = kVRemoved | kVViolating;
      a.order[c.v0 + k++] = v;
    }
  }
  for (int v = c.v0; v < c.v1; ++v)
    if (!(a.vstate[v] & kVViolating)) a.order[c.v0 + k++] = v;
  // reprieve: violating victims first, then the others, most important first
  int nv = 0, cnt = 0;
  for (int s = 0; s < c.v1 - c.v0; ++s) {
    const int v = a.order[c.v0 + s];
    const uint8_t viol = a.vstate[v] & kVViolating;
    a.vstate[v] = kVKept | viol;
    c.trial = v;
    c.step = s;
    if (check_two_pass(c)) {
      a.vstate[v] = kVEvicted | viol;
      a.out_victims[c.v0 + cnt++] = v;
      if (viol) ++nv;
    }
  }
  out.fits = 1;
  out.n_victims = cnt;
  out.num_pdb_violations = nv;
  a.out[n] = out;
}

// Per DoNotSchedule constraint: minimum count over the key's registered pairs, the pair holding it
// (lowest value id) and the minimum over the others; then the number of non-zero entries of the
// affinity map.  One workgroup per item.
__global__ __launch_bounds__(256) void k_vict_prep(const DevState* __restrict__ stp, const PreemptArgs* __restrict__ ap) {
  const DevState& st = *stp;
  const PreemptArgs& a = *ap;
  const QPlan& pl = st.plans[a.pod];
  __shared__ int64_t sv[4];
  __shared__ int32_t si[4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  auto block_min = [&](int64_t v, int idx, int64_t& ov, int& oi) {
    for (int o = 32; o; o >>= 1) {
      const int64_t v2 = __shfl_xor(v, o);
      const int i2 = __shfl_xor(idx, o);
      if (v2 < v || (v2 == v && i2 < idx)) {
        v = v2;
        idx = i2;
      }
    }
    if (lane == 0) {
      sv[w] = v;
      si[w] = idx;
    }
    __syncthreads();
    ov = sv[0];
    oi = si[0];
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
      if (sv[k] < ov || (sv[k] == ov && si[k] < oi)) {
        ov = sv[k];
        oi = si[k];
      }
    __syncthreads();
  };
  const int b = blockIdx.x;
  if (b < pl.n_hard) {
    const TSpread& t = pl.hard[b];
    const int nv = t.key >= 0 ? gp(st.key_n_values)[t.key] : 0;
    const int64_t* reg = slot_ptr(st, pl, t.rslot);
    const int64_t* cnt = slot_ptr(st, pl, t.cslot);
    int64_t m1 = INT64_MAX;
    int i1 = INT32_MAX;
    for (int v = threadIdx.x; v < nv; v += blockDim.x)
      if (reg[v] && cnt[v] < m1) {
        m1 = cnt[v];
        i1 = v;
      }
    int64_t mn;
    int mi;
    block_min(m1, i1, mn, mi);
    int64_t m2 = INT64_MAX;
    for (int v = threadIdx.x; v < nv; v += blockDim.x)
      if (reg[v] && v != mi && cnt[v] < m2) m2 = cnt[v];
    int64_t mn2;
    int dummy;
    block_min(m2, 0, mn2, dummy);
    if (threadIdx.x == 0) {
      a.prep[3 * b] = mn;
      a.prep[3 * b + 1] = mi == INT32_MAX ? -1 : mi;
      a.prep[3 * b + 2] = mn2;
    }
  } else if (b == kMaxSpread) {
    int64_t nz = 0;
    for (int i = 0; i < pl.n_aff; ++i) {
      bool first = true;
      for (int j = 0; j < i; ++j) first &= pl.aff[j].slot != pl.aff[i].slot;
      if (!first || pl.aff[i].key < 0) continue;
      const int nv = gp(st.key_n_values)[pl.aff[i].key];
      const int64_t* h = slot_ptr(st, pl, pl.aff[i].slot);
      for (int v = threadIdx.x; v < nv; v += blockDim.x) nz += h[v] != 0;
    }
    __shared__ int64_t ssum;
    if (threadIdx.x == 0) ssum = 0;
    __syncthreads();
    atomicAdd(reinterpret_cast<unsigned long long*>(&ssum), (unsigned long long)nz);
    __syncthreads();
    if (threadIdx.x == 0) a.prep[3 * kMaxSpread] = ssum;
  }
}

int launch_vict_prep(const DevState* st, const PreemptArgs* a, void* stream) {
  hipLaunchKernelGGL(k_vict_prep, dim3(kMaxSpread + 1), dim3(256), 0, (hipStream_t)stream, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_victims(const DevState* st, const PreemptArgs* a, int N, void* stream) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(k_victims, dim3((N + 63) / 64), dim3(64), 0, (hipStream_t)stream, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace kgpu
