// libkgpu.so host runtime: the C ABI of include/kgpu.h over HIP.
//
// One context = one scheduler profile on one GPU.  The snapshot lives in device-resident SoA
// arrays (Snapshot.List() order); a batch of compiled pod queries is copied once, then every
// pod is one node-evaluation launch (plus a normalize launch when a DefaultNormalizeScore
// maximum is needed) on a single stream, with the previous pod's selectHost + assume folded
// into the head of the next launch (kgpu_kernels.hip).  The host never waits between pods.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "kgpu_internal.h"

using kgpu::BlkKey;
using kgpu::BlkStat;
using kgpu::DevState;
using kgpu::PodArgs;

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct kgpu_ctx {
  kgpu_config cfg{};
  std::string err;
  int device = 0;
  hipStream_t stream = nullptr;
  DevState st{};
  std::vector<void*> snap_allocs;
  std::vector<void*> work_allocs;
  int64_t generation = -1;
  bool uploaded = false;
  // grow-only batch buffers
  DevBuf queries, reqs, ints, words, node_terms, pref_terms, spreads, pod_terms, scalars, ports, results;
  DevBuf dstate;     // device copy of the DevState used by the kernels of the current batch
  DevState st_batch{};  // its host source (kept alive for the async copy)
  bool timing = false;
  bool persistent = true;  // KGPU_OPT_PERSISTENT
  int n_cus = 0;
  int max_groups = 0;  // KGPU_OPT_PERSIST_GROUPS (0 = n_cus)
  DevBuf gran;        // persistent-kernel granules + abort word
  int32_t abort_host = 0;
  bool phase_trace = false;
  DevBuf trace;
  std::vector<int64_t> trace_host;
  int spec = 0;      // k_eval instantiation for the profile (kgpu::select_spec)
  std::vector<uint64_t> prefer_union;  // PreferNoSchedule taint ids present on any node
  // pods assumed through this context (slot -> record), for kgpu_forget_pod
  struct Assumed {
    int node;
    kgpu_pod_query q;
    std::vector<kgpu_scalar_req> sc;
    std::vector<kgpu_port> ports;
    bool active;
  };
  std::vector<Assumed> assumed;
  int32_t n_snapshot_pods = 0;
  bool last_diag = false;
  std::vector<hipEvent_t> ev_pool;
};

namespace {

int fail(kgpu_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIP_OK(c, x)                                                                           \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess)                                                                      \
      return fail((c), KGPU_E_DEVICE, std::string(#x ": ") + hipGetErrorString(e_));           \
  } while (0)

template <class T>
int dalloc(kgpu_ctx* c, std::vector<void*>& reg, T** out, size_t n) {
  *out = nullptr;
  if (n == 0) n = 1;
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, n * sizeof(T));
  if (e != hipSuccess) return fail(c, KGPU_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  reg.push_back(p);
  *out = static_cast<T*>(p);
  return KGPU_OK;
}

template <class T>
int dcopy(kgpu_ctx* c, std::vector<void*>& reg, T** out, const T* src, size_t n, size_t cap = 0) {
  int rc = dalloc(c, reg, out, std::max(n, cap));
  if (rc) return rc;
  if (n && src) HIP_OK(c, hipMemcpy(*out, src, n * sizeof(T), hipMemcpyHostToDevice));
  if (cap > n) HIP_OK(c, hipMemset(*out + n, 0, (cap - n) * sizeof(T)));
  return KGPU_OK;
}

void free_all(std::vector<void*>& reg) {
  for (void* p : reg) (void)hipFree(p);
  reg.clear();
}

int ensure(kgpu_ctx* c, DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 8;
  if (b.bytes >= bytes) return KGPU_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  HIP_OK(c, hipMalloc(&b.p, bytes));
  b.bytes = bytes;
  return KGPU_OK;
}

template <class T>
int upload_pool(kgpu_ctx* c, DevBuf& b, const T* src, int32_t n, const T** dst) {
  int rc = ensure(c, b, sizeof(T) * (size_t)std::max(n, 1));
  if (rc) return rc;
  if (n > 0) HIP_OK(c, hipMemcpyAsync(b.p, src, sizeof(T) * (size_t)n, hipMemcpyHostToDevice, c->stream));
  *dst = static_cast<const T*>(b.p);
  return KGPU_OK;
}

int upload_pools(kgpu_ctx* c, const kgpu_pools* p) {
  kgpu_pools empty{};
  if (!p) p = &empty;
  kgpu::DevPools& q = c->st.qp;
  int rc;
  if ((rc = upload_pool(c, c->reqs, p->reqs, p->n_reqs, &q.reqs))) return rc;
  if ((rc = upload_pool(c, c->ints, p->ints, p->n_ints, &q.ints))) return rc;
  if ((rc = upload_pool(c, c->words, p->words, p->n_words, &q.words))) return rc;
  if ((rc = upload_pool(c, c->node_terms, p->node_terms, p->n_node_terms, &q.node_terms))) return rc;
  if ((rc = upload_pool(c, c->pref_terms, p->pref_terms, p->n_pref_terms, &q.pref_terms))) return rc;
  if ((rc = upload_pool(c, c->spreads, p->spreads, p->n_spreads, &q.spreads))) return rc;
  if ((rc = upload_pool(c, c->pod_terms, p->pod_terms, p->n_pod_terms, &q.pod_terms))) return rc;
  if ((rc = upload_pool(c, c->scalars, p->scalars, p->n_scalars, &q.scalars))) return rc;
  if ((rc = upload_pool(c, c->ports, p->ports, p->n_ports, &q.ports))) return rc;
  return KGPU_OK;
}

bool has_score(const kgpu_ctx* c, int s) {
  for (int i = 0; i < c->cfg.n_scores; ++i)
    if (c->cfg.scores[i] == s) return true;
  return false;
}

// Pods whose DefaultNormalizeScore maxima are not constant need the second (normalize) launch.
bool needs_norm(const kgpu_ctx* c, const kgpu_pod_query& q, const kgpu_pools* p) {
  if (has_score(c, KGPU_S_NODE_AFFINITY) && q.pref_terms.count > 0) return true;
  if (has_score(c, KGPU_S_TAINT_TOLERATION)) {
    for (size_t w = 0; w < c->prefer_union.size(); ++w) {
      uint64_t tol = (p && (int)w < q.tol_prefer.count) ? p->words[q.tol_prefer.begin + w] : 0ull;
      if (c->prefer_union[w] & ~tol) return true;
    }
  }
  return false;
}

// Tier check: features whose kernels are not in this build (the pod falls back to the caller).
const char* unsupported(const kgpu_ctx* c, const kgpu_pod_query& q) {
  if (q.pts_hard.count || q.pts_soft.count) return "PodTopologySpread constraints";
  if (q.dpts.kind != kgpu::kSelEmpty && !(q.flags & KGPU_Q_HAS_TSC) && has_score(c, KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD))
    return "DefaultPodTopologySpread selector";
  if (q.ipa_req_aff.count || q.ipa_req_anti.count || q.ipa_pref_aff.count || q.ipa_pref_anti.count)
    return "InterPodAffinity terms";
  return nullptr;
}

hipEvent_t get_event(kgpu_ctx* c, size_t i) {
  while (c->ev_pool.size() <= i) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    c->ev_pool.push_back(e);
  }
  return c->ev_pool[i];
}

int run_batch(kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools, int64_t first_seq,
              kgpu_result* results, kgpu_stats* stats, bool diag, int32_t assume) {
  if (!c->uploaded) return fail(c, KGPU_E_STATE, "no snapshot uploaded");
  if (n <= 0) return KGPU_OK;
  for (int32_t i = 0; i < n; ++i) {
    const char* why = unsupported(c, qs[i]);
    if (why) return fail(c, KGPU_E_UNSUPPORTED, std::string("pod ") + std::to_string(i) + ": " + why);
  }
  int rc;
  if ((rc = upload_pools(c, pools))) return rc;
  if ((rc = ensure(c, c->queries, sizeof(kgpu_pod_query) * (size_t)n))) return rc;
  HIP_OK(c, hipMemcpyAsync(c->queries.p, qs, sizeof(kgpu_pod_query) * (size_t)n, hipMemcpyHostToDevice, c->stream));
  if ((rc = ensure(c, c->results, sizeof(kgpu_result) * (size_t)n))) return rc;
  DevState st = c->st;
  st.queries = static_cast<const kgpu_pod_query*>(c->queries.p);
  st.results = static_cast<kgpu_result*>(c->results.p);
  if (!diag) {
    st.diag_raw = nullptr;
    st.diag_norm = nullptr;
  } else {
    HIP_OK(c, hipMemsetAsync(st.diag_raw, 0, sizeof(int64_t) * KGPU_NUM_SCORES * (size_t)st.N, c->stream));
    HIP_OK(c, hipMemsetAsync(st.diag_norm, 0, sizeof(int64_t) * KGPU_NUM_SCORES * (size_t)st.N, c->stream));
  }
  if ((rc = ensure(c, c->dstate, sizeof(DevState)))) return rc;
  c->st_batch = st;
  HIP_OK(c, hipMemcpyAsync(c->dstate.p, &c->st_batch, sizeof(DevState), hipMemcpyHostToDevice, c->stream));
  const DevState* dst = static_cast<const DevState*>(c->dstate.p);
  const int blocks = kgpu::eval_blocks(st.N);
  hipEvent_t t0 = get_event(c, 0), t1 = get_event(c, 1);
  HIP_OK(c, hipEventRecord(t0, c->stream));
  size_t ev = 2;
  int64_t timed_passes = 0;
  // Persistent geometry: one workgroup per CU at most, K node rows per lane in registers.
  int per = 0, groups = 0;
  const int kidx = (c->persistent && !diag) ? kgpu::batch_geometry(st.N, std::min(c->max_groups > 0 ? std::min(c->max_groups, c->n_cus) : c->n_cus, 256), &per, &groups) : -1;
  std::vector<uint8_t> norm((size_t)n);
  // pods that need the normalize pass or whose scoring fails take the one-launch-per-pod path
  for (int32_t i = 0; i < n; ++i)
    norm[(size_t)i] = (diag || needs_norm(c, qs[i], pools) || (qs[i].flags & KGPU_Q_SCORE_ERROR)) ? 1 : 0;
  bool used_persistent = false;
  int32_t i = 0;
  while (i < n) {
    int32_t j = i;
    if (kidx >= 0 && !norm[(size_t)i]) {
      // a run of pods with constant normalize maxima: one persistent launch
      while (j < n && !norm[(size_t)j]) ++j;
      const int32_t cnt = j - i;
      // layout: abort word (64 B) | granules [cnt][groups] u64 | feasible counts [cnt][groups] i32
      const size_t cells = (size_t)cnt * (size_t)groups;
      const size_t gbytes = 64 + sizeof(uint64_t) * cells + sizeof(int32_t) * cells;
      if ((rc = ensure(c, c->gran, gbytes))) return rc;
      HIP_OK(c, hipMemsetAsync(c->gran.p, 0, 64 + sizeof(uint64_t) * cells, c->stream));
      kgpu::BatchArgs ba{};
      ba.first = i;
      ba.count = cnt;
      ba.per = per;
      ba.assume = assume;
      ba.seq0 = first_seq + i;
      ba.gran = static_cast<uint64_t*>(c->gran.p) + 8;
      ba.feas = reinterpret_cast<int32_t*>(ba.gran + cells);
      ba.abort = static_cast<int32_t*>(c->gran.p);
      ba.trace = nullptr;
      if (c->phase_trace) {
        if ((rc = ensure(c, c->trace, sizeof(int64_t) * 16 * (size_t)(cnt + 1)))) return rc;
        HIP_OK(c, hipMemsetAsync(c->trace.p, 0, sizeof(int64_t) * 16 * (size_t)(cnt + 1), c->stream));
        ba.trace = static_cast<int64_t*>(c->trace.p);
        c->trace_host.assign((size_t)(cnt + 1) * 16, 0);
      }
      if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev), c->stream));
      if (kgpu::launch_batch(dst, ba, groups, kidx, c->spec, c->stream))
        return fail(c, KGPU_E_DEVICE, "k_batch launch failed");
      if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev + 1), c->stream));
      ev += 2;
      timed_passes += cnt;
      HIP_OK(c, hipMemcpyAsync(&c->abort_host, c->gran.p, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
      if (ba.trace)
        HIP_OK(c, hipMemcpyAsync(c->trace_host.data(), ba.trace, sizeof(int64_t) * 16 * (size_t)(cnt + 1),
                                 hipMemcpyDeviceToHost, c->stream));
      used_persistent = true;
    } else {
      // one launch per pod; the next launch resolves (and assumes) the previous pod's winner
      while (j < n && (kidx < 0 || norm[(size_t)j])) ++j;
      int prev = -1;
      for (int32_t k = i; k < j; ++k) {
        PodArgs a{};
        a.pod = k;
        a.prev = prev;
        a.prev_blocks = blocks;
        a.prev_parity = (k - 1) & 1;
        a.parity = k & 1;
        a.norm = (diag || needs_norm(c, qs[k], pools)) ? 1 : 0;
        a.assume = assume;
        a.diag = diag ? 1 : 0;
        a.seq = first_seq + k;
        if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev), c->stream));
        if (kgpu::launch_eval(dst, a, blocks, c->spec, c->stream))
          return fail(c, KGPU_E_DEVICE, "k_eval launch failed");
        if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev + 1), c->stream));
        ev += 2;
        ++timed_passes;
        if (a.norm && kgpu::launch_final(dst, a, blocks, blocks, c->stream))
          return fail(c, KGPU_E_DEVICE, "k_final launch failed");
        prev = k;
      }
      PodArgs r{};
      r.pod = -1;
      r.prev = prev;
      r.prev_blocks = blocks;
      r.prev_parity = prev & 1;
      r.assume = assume;
      if (kgpu::launch_resolve(dst, st.N, r, c->stream)) return fail(c, KGPU_E_DEVICE, "k_resolve launch failed");
    }
    i = j;
  }
  HIP_OK(c, hipEventRecord(t1, c->stream));
  HIP_OK(c, hipMemcpyAsync(results, st.results, sizeof(kgpu_result) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  if (used_persistent && c->abort_host)
    return fail(c, KGPU_E_DEVICE, "persistent batch kernel lost co-residency (workgroups not all resident)");
  if (stats) {
    float ms = 0.f;
    HIP_OK(c, hipEventElapsedTime(&ms, t0, t1));
    stats->pods += n;
    stats->device_ms += ms;
    int64_t placed = 0;
    for (int32_t i = 0; i < n; ++i) placed += results[i].node >= 0;
    stats->scheduled += placed;
    if (c->timing) {
      double sum = 0;
      for (size_t e = 2; e < ev; e += 2) {
        float k = 0.f;
        HIP_OK(c, hipEventElapsedTime(&k, c->ev_pool[e], c->ev_pool[e + 1]));
        sum += k;
      }
      stats->eval_kernel_ms += sum;
      stats->eval_launches += timed_passes;
    }
  }
  // keep host records of assumed pods for ForgetPod
  if (assume) {
    for (int32_t i = 0; i < n; ++i) {
      if (results[i].node < 0) continue;
      kgpu_ctx::Assumed a;
      a.node = results[i].node - c->st.node_base;
      a.q = qs[i];
      a.active = true;
      if (pools) {
        for (int k = 0; k < qs[i].scalars.count; ++k) a.sc.push_back(pools->scalars[qs[i].scalars.begin + k]);
        for (int k = 0; k < qs[i].ports.count; ++k) a.ports.push_back(pools->ports[qs[i].ports.begin + k]);
      }
      c->assumed.push_back(std::move(a));
    }
  }
  c->last_diag = diag;
  return KGPU_OK;
}

}  // namespace

extern "C" {

int kgpu_abi_version(void) { return KGPU_ABI_VERSION; }

int kgpu_struct_sizes(int32_t* out, int32_t n) {
  const int32_t s[] = {(int32_t)sizeof(kgpu_range),     (int32_t)sizeof(kgpu_req),
                       (int32_t)sizeof(kgpu_selector),  (int32_t)sizeof(kgpu_node_term),
                       (int32_t)sizeof(kgpu_pref_term), (int32_t)sizeof(kgpu_spread),
                       (int32_t)sizeof(kgpu_pod_term),  (int32_t)sizeof(kgpu_term),
                       (int32_t)sizeof(kgpu_scalar_req), (int32_t)sizeof(kgpu_port),
                       (int32_t)sizeof(kgpu_pod_query), (int32_t)sizeof(kgpu_pools),
                       (int32_t)sizeof(kgpu_resource_weight), (int32_t)sizeof(kgpu_config),
                       (int32_t)sizeof(kgpu_snapshot),  (int32_t)sizeof(kgpu_result),
                       (int32_t)sizeof(kgpu_stats)};
  const int32_t m = (int32_t)(sizeof(s) / sizeof(s[0]));
  for (int32_t i = 0; i < n && i < m; ++i) out[i] = s[i];
  return m;
}

int kgpu_create(const kgpu_config* cfg, kgpu_ctx** out) {
  if (!cfg || !out) return KGPU_E_INVAL;
  *out = nullptr;
  if (cfg->abi_version != KGPU_ABI_VERSION) return KGPU_E_INVAL;
  if (cfg->n_filters < 0 || cfg->n_filters > KGPU_NUM_FILTERS || cfg->n_scores < 0 ||
      cfg->n_scores > KGPU_NUM_SCORES || cfg->n_least < 0 || cfg->n_least > 8 || cfg->n_most < 0 || cfg->n_most > 8)
    return KGPU_E_INVAL;
  int64_t total = 0;
  for (int i = 0; i < cfg->n_scores; ++i) {
    if (cfg->scores[i] < 0 || cfg->scores[i] >= KGPU_NUM_SCORES) return KGPU_E_INVAL;
    for (int j = 0; j < i; ++j)
      if (cfg->scores[j] == cfg->scores[i]) return KGPU_E_INVAL;  // a plugin appears once per extension point
    total += std::max<int64_t>(cfg->score_weights[i], 1) * 100;
  }
  if (total >= (1ll << 23) - 1) return KGPU_E_UNSUPPORTED;  // packed argmax key: 23 bits hold score + 1
  for (int i = 0; i < cfg->n_filters; ++i) {
    if (cfg->filters[i] < 0 || cfg->filters[i] >= KGPU_NUM_FILTERS) return KGPU_E_INVAL;
    for (int j = 0; j < i; ++j)
      if (cfg->filters[j] == cfg->filters[i]) return KGPU_E_INVAL;
  }
  if (cfg->percentage_of_nodes_to_score > 0 && cfg->percentage_of_nodes_to_score < 100) return KGPU_E_UNSUPPORTED;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return KGPU_E_DEVICE;
  if (cfg->device < 0 || cfg->device >= ndev) return KGPU_E_INVAL;
  kgpu_ctx* c = new kgpu_ctx();
  c->cfg = *cfg;
  c->device = cfg->device;
  if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return KGPU_E_DEVICE;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return KGPU_E_DEVICE;
  }
  c->n_cus = prop.multiProcessorCount;
  DevState& st = c->st;
  st.n_filters = cfg->n_filters;
  std::memcpy(st.filters, cfg->filters, sizeof(st.filters));
  st.n_scores = cfg->n_scores;
  std::memcpy(st.scores, cfg->scores, sizeof(st.scores));
  for (int i = 0; i < KGPU_NUM_SCORES; ++i) st.weights[i] = std::max<int64_t>(cfg->score_weights[i], 1);
  for (int i = 0; i < KGPU_NUM_SCORES; ++i) st.w_of[i] = 0;
  for (int i = 0; i < cfg->n_scores; ++i) st.w_of[cfg->scores[i]] = st.weights[i];
  st.n_least = cfg->n_least;
  st.n_most = cfg->n_most;
  std::memcpy(st.least, cfg->least, sizeof(st.least));
  std::memcpy(st.most, cfg->most, sizeof(st.most));
  st.least_wsum = st.most_wsum = 0;
  for (int i = 0; i < cfg->n_least; ++i) st.least_wsum += cfg->least[i].weight;
  for (int i = 0; i < cfg->n_most; ++i) st.most_wsum += cfg->most[i].weight;
  if (st.least_wsum == 0) st.least_wsum = 1;
  if (st.most_wsum == 0) st.most_wsum = 1;
  st.tie_mode = cfg->tie_break_mode;
  st.seed = cfg->seed;
  // default requested-resource specs {cpu: 1, memory: 1} (noderesources/resource_allocation.go:36-39)
  auto def_spec = [](const kgpu_resource_weight* r, int n) {
    return n == 2 && r[0].resource == 0 && r[0].weight == 1 && r[1].resource == 1 && r[1].weight == 1;
  };
  const bool has_least = has_score(c, KGPU_S_LEAST_ALLOCATED), has_most = has_score(c, KGPU_S_MOST_ALLOCATED);
  const bool def_res = (!has_least || def_spec(cfg->least, cfg->n_least)) && (!has_most || def_spec(cfg->most, cfg->n_most));
  c->spec = kgpu::select_spec(cfg->filters, cfg->n_filters, cfg->scores, cfg->n_scores, def_res);
  *out = c;
  return KGPU_OK;
}

int kgpu_destroy(kgpu_ctx* c) {
  if (!c) return KGPU_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_all(c->snap_allocs);
  free_all(c->work_allocs);
  for (DevBuf* b : {&c->dstate, &c->queries, &c->reqs, &c->ints, &c->words, &c->node_terms, &c->pref_terms, &c->spreads,
                    &c->pod_terms, &c->scalars, &c->ports, &c->results, &c->gran, &c->trace})
    if (b->p) (void)hipFree(b->p);
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return KGPU_OK;
}

const char* kgpu_last_error(const kgpu_ctx* c) { return c ? c->err.c_str() : "null context"; }

int64_t kgpu_generation(const kgpu_ctx* c) { return c ? c->generation : -1; }

int kgpu_read_phase_trace(kgpu_ctx* c, int64_t* out, int32_t max_pods) {
  if (!c || !out || max_pods < 0) return KGPU_E_INVAL;
  const int32_t n = std::min<int32_t>(max_pods, (int32_t)(c->trace_host.size() / 16));
  std::memcpy(out, c->trace_host.data(), sizeof(int64_t) * 16 * (size_t)n);
  return n;
}

int kgpu_set_option(kgpu_ctx* c, int32_t option, int64_t value) {
  if (!c) return KGPU_E_INVAL;
  if (option == KGPU_OPT_KERNEL_TIMING) c->timing = value != 0;
  else if (option == KGPU_OPT_PERSISTENT) c->persistent = value != 0;
  else if (option == KGPU_OPT_PERSIST_GROUPS) c->max_groups = (int)std::max<int64_t>(value, 0);
  else if (option == KGPU_OPT_PHASE_TRACE) c->phase_trace = value != 0;
  else return KGPU_E_INVAL;
  return KGPU_OK;
}

int kgpu_upload_snapshot(kgpu_ctx* c, const kgpu_snapshot* s, int64_t generation) {
  if (!c || !s) return KGPU_E_INVAL;
  if (s->n_nodes < 0 || s->n_label_keys < 0 || s->n_scalar < 0 || s->taint_words < 0 || s->port_slots < 0)
    return fail(c, KGPU_E_INVAL, "negative snapshot dimension");
  if (s->n_nodes > 0 && (!s->alloc_cpu || !s->alloc_mem || !s->alloc_eph || !s->alloc_pods || !s->req_cpu ||
                         !s->req_mem || !s->req_eph || !s->nz_cpu || !s->nz_mem || !s->num_pods ||
                         !s->unschedulable || !s->image_off || !s->avoid_off || !s->zone_id || !s->port_count))
    return fail(c, KGPU_E_INVAL, "missing node column");
  HIP_OK(c, hipSetDevice(c->device));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  free_all(c->snap_allocs);
  free_all(c->work_allocs);
  c->assumed.clear();
  c->uploaded = false;
  DevState& st = c->st;
  const size_t N = (size_t)s->n_nodes;
  st.N = s->n_nodes;
  st.node_base = s->node_base;
  st.n_total = s->n_total_nodes > 0 ? s->n_total_nodes : s->n_nodes;
  st.S = s->n_scalar;
  st.K = s->n_label_keys;
  st.TW = std::max(s->taint_words, 1);
  st.n_zones = s->n_zones;
  auto& R = c->snap_allocs;
  int rc = 0;
#define UP(field, src, count) \
  if ((rc = dcopy(c, R, &st.field, src, count))) return rc
  UP(alloc_cpu, s->alloc_cpu, N);
  UP(alloc_mem, s->alloc_mem, N);
  UP(alloc_eph, s->alloc_eph, N);
  UP(alloc_pods, s->alloc_pods, N);
  UP(req_cpu, s->req_cpu, N);
  UP(req_mem, s->req_mem, N);
  UP(req_eph, s->req_eph, N);
  UP(nz_cpu, s->nz_cpu, N);
  UP(nz_mem, s->nz_mem, N);
  UP(num_pods, s->num_pods, N);
  UP(alloc_scalar, s->alloc_scalar, (size_t)st.S * N);
  UP(req_scalar, s->req_scalar, (size_t)st.S * N);
  UP(unsched, s->unschedulable, N);
  UP(label_val, s->label_val, (size_t)st.K * N);
  UP(key_n_values, s->key_n_values, (size_t)st.K);
  UP(value_off, s->value_off, (size_t)st.K + 1);
  const size_t nvals = (st.K > 0 && s->value_off) ? (size_t)s->value_off[st.K] : 0;
  UP(value_int, s->value_int, nvals);
  UP(value_int_ok, s->value_int_ok, nvals);
  UP(key_empty_value, s->key_empty_value, (size_t)st.K);
  std::vector<uint64_t> zeros((size_t)st.TW * N, 0ull);
  UP(taint_nosched, s->taint_words > 0 ? s->taint_nosched : zeros.data(), (size_t)st.TW * N);
  UP(taint_prefer, s->taint_words > 0 ? s->taint_prefer : zeros.data(), (size_t)st.TW * N);
  c->prefer_union.assign(st.TW, 0ull);
  if (s->taint_words > 0)
    for (int w = 0; w < st.TW; ++w)
      for (size_t i = 0; i < N; ++i) c->prefer_union[w] |= s->taint_prefer[(size_t)w * N + i];
  // host ports: reserve room for assumed pods' ports
  st.PS = std::max(s->port_slots, 8);
  UP(port_count, s->port_count, N);
  {
    std::vector<kgpu_port> ports((size_t)st.PS * N);
    std::memset(ports.data(), 0, ports.size() * sizeof(kgpu_port));
    for (int sl = 0; sl < s->port_slots; ++sl)
      std::memcpy(&ports[(size_t)sl * N], &s->ports[(size_t)sl * N], N * sizeof(kgpu_port));
    UP(ports, ports.data(), ports.size());
  }
  UP(image_off, s->image_off, N + 1);
  const size_t nimg = s->image_off ? (size_t)s->image_off[N] : 0;
  UP(image_id, s->image_id, nimg);
  UP(image_score, s->image_score, nimg);
  UP(avoid_off, s->avoid_off, N + 1);
  const size_t navoid = s->avoid_off ? (size_t)s->avoid_off[N] : 0;
  UP(avoid_id, s->avoid_id, navoid);
  UP(zone_id, s->zone_id, N);
#undef UP
  // work buffers
  auto& W = c->work_allocs;
  if ((rc = dalloc(c, W, &st.status, N))) return rc;
  if ((rc = dalloc(c, W, &st.raw_taint, N))) return rc;
  if ((rc = dalloc(c, W, &st.raw_na, N))) return rc;
  if ((rc = dalloc(c, W, &st.partial, N))) return rc;
  if ((rc = dalloc(c, W, &st.sbuf, (size_t)2 * kgpu::kMaxBlocks))) return rc;
  if ((rc = dalloc(c, W, &st.kbuf, (size_t)2 * kgpu::kMaxBlocks))) return rc;
  if ((rc = dalloc(c, W, &st.diag_raw, (size_t)KGPU_NUM_SCORES * N))) return rc;
  if ((rc = dalloc(c, W, &st.diag_norm, (size_t)KGPU_NUM_SCORES * N))) return rc;
  HIP_OK(c, hipMemset(st.status, 0, sizeof(uint32_t) * std::max<size_t>(N, 1)));
  int anyp = 0;
  for (uint64_t w : c->prefer_union) anyp |= (w != 0);
  st.any_prefer_taint = anyp;
  c->n_snapshot_pods = s->n_pods;
  c->generation = generation;
  c->uploaded = true;
  HIP_OK(c, hipDeviceSynchronize());
  return KGPU_OK;
}

int kgpu_schedule_batch(kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools, int64_t first_seq,
                        kgpu_result* results, kgpu_stats* stats) {
  if (!c || (n > 0 && (!qs || !results))) return KGPU_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  return run_batch(c, qs, n, pools, first_seq, results, stats, false, 1);
}

int kgpu_schedule_one(kgpu_ctx* c, const kgpu_pod_query* q, const kgpu_pools* pools, int64_t pod_seq, int32_t assume,
                      kgpu_result* res, int32_t* assumed_slot) {
  if (!c || !q || !res) return KGPU_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  size_t before = c->assumed.size();
  int rc = run_batch(c, q, 1, pools, pod_seq, res, nullptr, true, assume);
  if (rc) return rc;
  if (assumed_slot)
    *assumed_slot = c->assumed.size() > before ? c->n_snapshot_pods + (int32_t)c->assumed.size() - 1 : -1;
  return KGPU_OK;
}

int kgpu_get_filter(kgpu_ctx* c, uint32_t* words) {
  if (!c || !words) return KGPU_E_INVAL;
  if (!c->last_diag) return fail(c, KGPU_E_STATE, "no kgpu_schedule_one cycle to report");
  HIP_OK(c, hipMemcpy(words, c->st.status, sizeof(uint32_t) * (size_t)c->st.N, hipMemcpyDeviceToHost));
  return KGPU_OK;
}

int kgpu_get_scores(kgpu_ctx* c, int32_t plugin, int64_t* raw, int64_t* normalized) {
  if (!c || plugin < 0 || plugin >= KGPU_NUM_SCORES) return KGPU_E_INVAL;
  if (!c->last_diag) return fail(c, KGPU_E_STATE, "no kgpu_schedule_one cycle to report");
  const size_t N = (size_t)c->st.N;
  if (raw) HIP_OK(c, hipMemcpy(raw, c->st.diag_raw + plugin * N, sizeof(int64_t) * N, hipMemcpyDeviceToHost));
  if (normalized)
    HIP_OK(c, hipMemcpy(normalized, c->st.diag_norm + plugin * N, sizeof(int64_t) * N, hipMemcpyDeviceToHost));
  return KGPU_OK;
}

int kgpu_read_nodes(kgpu_ctx* c, int64_t* req_cpu, int64_t* req_mem, int64_t* req_eph, int64_t* nz_cpu,
                    int64_t* nz_mem, int32_t* num_pods) {
  if (!c || !c->uploaded) return KGPU_E_INVAL;
  HIP_OK(c, hipStreamSynchronize(c->stream));
  const size_t N = (size_t)c->st.N;
  if (req_cpu) HIP_OK(c, hipMemcpy(req_cpu, c->st.req_cpu, 8 * N, hipMemcpyDeviceToHost));
  if (req_mem) HIP_OK(c, hipMemcpy(req_mem, c->st.req_mem, 8 * N, hipMemcpyDeviceToHost));
  if (req_eph) HIP_OK(c, hipMemcpy(req_eph, c->st.req_eph, 8 * N, hipMemcpyDeviceToHost));
  if (nz_cpu) HIP_OK(c, hipMemcpy(nz_cpu, c->st.nz_cpu, 8 * N, hipMemcpyDeviceToHost));
  if (nz_mem) HIP_OK(c, hipMemcpy(nz_mem, c->st.nz_mem, 8 * N, hipMemcpyDeviceToHost));
  if (num_pods) HIP_OK(c, hipMemcpy(num_pods, c->st.num_pods, 4 * N, hipMemcpyDeviceToHost));
  return KGPU_OK;
}

int kgpu_forget_pod(kgpu_ctx* c, int32_t slot) {
  if (!c) return KGPU_E_INVAL;
  const int32_t i = slot - c->n_snapshot_pods;
  if (i < 0) return fail(c, KGPU_E_UNSUPPORTED, "forget of a snapshot pod: re-upload the snapshot");
  if (i >= (int32_t)c->assumed.size() || !c->assumed[i].active) return fail(c, KGPU_E_INVAL, "no such assumed pod");
  kgpu_ctx::Assumed& a = c->assumed[i];
  HIP_OK(c, hipStreamSynchronize(c->stream));
  // NodeInfo.RemovePod (types.go:484-533): read-modify-write of one row (rare path).
  const size_t n = (size_t)a.node, N = (size_t)c->st.N;
  auto sub64 = [&](int64_t* col, int64_t d) -> int {
    int64_t v;
    HIP_OK(c, hipMemcpy(&v, col + n, 8, hipMemcpyDeviceToHost));
    v -= d;
    HIP_OK(c, hipMemcpy(col + n, &v, 8, hipMemcpyHostToDevice));
    return KGPU_OK;
  };
  int rc;
  if ((rc = sub64(c->st.req_cpu, a.q.req[0]))) return rc;
  if ((rc = sub64(c->st.req_mem, a.q.req[1]))) return rc;
  if ((rc = sub64(c->st.req_eph, a.q.req[2]))) return rc;
  if ((rc = sub64(c->st.nz_cpu, a.q.nz[0]))) return rc;
  if ((rc = sub64(c->st.nz_mem, a.q.nz[1]))) return rc;
  for (const kgpu_scalar_req& s : a.sc)
    if (s.col >= 0 && (rc = sub64(c->st.req_scalar + (size_t)s.col * N, s.value))) return rc;
  int32_t np;
  HIP_OK(c, hipMemcpy(&np, c->st.num_pods + n, 4, hipMemcpyDeviceToHost));
  np -= 1;
  HIP_OK(c, hipMemcpy(c->st.num_pods + n, &np, 4, hipMemcpyHostToDevice));
  if (!a.ports.empty()) {
    int32_t pc;
    HIP_OK(c, hipMemcpy(&pc, c->st.port_count + n, 4, hipMemcpyDeviceToHost));
    std::vector<kgpu_port> row(pc);
    for (int sl = 0; sl < pc; ++sl)
      HIP_OK(c, hipMemcpy(&row[sl], c->st.ports + (size_t)sl * N + n, sizeof(kgpu_port), hipMemcpyDeviceToHost));
    std::vector<kgpu_port> keep;
    for (const kgpu_port& p : row) {
      bool rm = false;
      for (const kgpu_port& w : a.ports) rm |= (p.ip == w.ip && p.proto == w.proto && p.port == w.port);
      if (!rm) keep.push_back(p);
    }
    for (size_t sl = 0; sl < keep.size(); ++sl)
      HIP_OK(c, hipMemcpy(c->st.ports + sl * N + n, &keep[sl], sizeof(kgpu_port), hipMemcpyHostToDevice));
    int32_t kc = (int32_t)keep.size();
    HIP_OK(c, hipMemcpy(c->st.port_count + n, &kc, 4, hipMemcpyHostToDevice));
  }
  a.active = false;
  return KGPU_OK;
}

int kgpu_comm_unique_id(uint8_t id[128]) {
  (void)id;
  return KGPU_E_UNSUPPORTED;
}

int kgpu_comm_init(kgpu_ctx* c, int32_t nranks, int32_t rank, const uint8_t id[128]) {
  (void)nranks;
  (void)rank;
  (void)id;
  return fail(c, KGPU_E_UNSUPPORTED, "sharded mode not built yet");
}

}  // extern "C"
