// libkgpu.so host runtime: the C ABI of include/kgpu.h over HIP.
//
// One context = one scheduler profile on one GPU.  The snapshot lives in device-resident SoA
// arrays (Snapshot.List() order); a batch of compiled pod queries is copied once, then every
// pod is one node-evaluation launch (plus a normalize launch when a DefaultNormalizeScore
// maximum is needed) on a single stream, with the previous pod's selectHost + assume folded
// into the head of the next launch (kgpu_kernels.hip).  The host never waits between pods.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <atomic>
#include <exception>
#include <memory>
#include <new>
#include <iterator>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <deque>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "kgpu_internal.h"
#include "kgpu_staging.h"
#include "kgpu_reasons.h"

// ---- RCCL, loaded on first use.  Only node sharding (kgpu_comm_unique_id / kgpu_comm_init) needs
// it, so a one-GPU process never maps librccl: RCCL's own exit-time teardown then cannot run after a
// profiler's finalization has shut the HSA runtime down (rocprofv3 runs faulted in exit handlers).
namespace {
struct Rccl {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclCommCount) CommCount = nullptr;        // kgpu_comm_info only (optional)
  decltype(&ncclCommUserRank) CommUserRank = nullptr;  // kgpu_comm_info only (optional)
  bool ok = false;
};
const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    x.GetUniqueId = reinterpret_cast<decltype(x.GetUniqueId)>(dlsym(h, "ncclGetUniqueId"));
    x.CommInitRank = reinterpret_cast<decltype(x.CommInitRank)>(dlsym(h, "ncclCommInitRank"));
    x.CommDestroy = reinterpret_cast<decltype(x.CommDestroy)>(dlsym(h, "ncclCommDestroy"));
    x.AllGather = reinterpret_cast<decltype(x.AllGather)>(dlsym(h, "ncclAllGather"));
    x.AllReduce = reinterpret_cast<decltype(x.AllReduce)>(dlsym(h, "ncclAllReduce"));
    x.GetErrorString = reinterpret_cast<decltype(x.GetErrorString)>(dlsym(h, "ncclGetErrorString"));
    x.CommCount = reinterpret_cast<decltype(x.CommCount)>(dlsym(h, "ncclCommCount"));
    x.CommUserRank = reinterpret_cast<decltype(x.CommUserRank)>(dlsym(h, "ncclCommUserRank"));
    x.ok = x.GetUniqueId && x.CommInitRank && x.CommDestroy && x.AllGather && x.AllReduce && x.GetErrorString;
    return x;
  }();
  return r;
}
}  // namespace

using kgpu::BlkKey;
using kgpu::BlkStat;
using kgpu::DevState;
using kgpu::PodArgs;

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  // host copy of the last pool uploaded into p (upload_pool skips an identical re-upload)
  std::vector<char> shadow;
  const void* shadow_p = nullptr;
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
  DevBuf queries, results;
  DevBuf dstate;     // device copy of the DevState used by the kernels of the current batch
  DevBuf ticket;     // k_final's last-workgroup ticket (zero between launches)
  DevState st_batch{};  // its host source (kept alive for the async copy)
  bool timing = false;
  bool persistent = true;  // KGPU_OPT_PERSISTENT
  bool topo_fused = false;  // KGPU_OPT_TOPO_FUSED (measured slower: DESIGN.md 4)
  DevBuf gbar;              // fused topology kernel: grid-barrier arrival counter
  unsigned long long bar_base = 0;
  int n_cus = 0;
  int max_groups = 0;  // KGPU_OPT_PERSIST_GROUPS (0 = n_cus)
  DevBuf gran;        // persistent-kernel granules + abort word
  int32_t abort_host = 0;
  int32_t abort_at = -1;  // KGPU_OPT_ABORT_AT: batch query index at which a persistent run aborts
  int32_t skip_release_at = -1;  // KGPU_OPT_SKIP_RELEASE_AT: batch query whose LDS hand-off is never released
  bool phase_trace = false;
  int phase_trace_mode = 0;         // the KGPU_OPT_PHASE_TRACE value
  DevBuf trace;
  std::vector<int64_t> trace_host;
  int spec = 0;      // k_eval instantiation for the profile (kgpu::select_spec)
  std::vector<uint64_t> prefer_union;  // PreferNoSchedule taint ids present on any node of this shard
  // node sharding: the union over every rank's shard (exchanged at kgpu_comm_init and after each
  // delta batch), so that every rank takes the same normalize decision for a pod
  std::vector<uint64_t> prefer_global;
  DevBuf pref_x;
  // Every pod on a device row, by pod-table slot (parallel to pod_rows): snapshot pods first, then
  // pods assumed by a schedule call or added by kgpu_apply_delta.  The resource record is what
  // NodeInfo.RemovePod subtracts for kgpu_forget_pod; snapshot pods have none (their removal goes
  // through a REMOVE_POD delta, which carries the pod).
  struct PodRec {
    int64_t uid = 0;
    bool has_uid = false;
    bool active = false;
    bool has_res = false;
    int32_t node = -1;  // global node index, -1: on no listed node (node removed)
    kgpu_pod_query q{};
    std::vector<kgpu_scalar_req> sc;
    std::vector<kgpu_port> ports;
  };
  std::vector<PodRec> recs;
  std::unordered_map<int64_t, int32_t> uid_slot;  // active pods with a UID
  int32_t n_snapshot_pods = 0;
  // host copies for incremental bookkeeping under SET_NODE deltas
  std::vector<int32_t> label_host;                 // [K][N] value ids
  std::vector<std::vector<int32_t>> val_nodes;     // [K][values] nodes carrying the value
  std::vector<int32_t> multi_values;               // [K] values carried by >= 2 nodes
  std::vector<uint64_t> prefer_host;               // [TW][N]
  std::vector<int32_t> prefer_cnt;                 // [TW * 64] nodes carrying PreferNoSchedule taint t
  int64_t port_bound = 0;                          // upper bound of any node's UsedPorts entries
  // Snapshot.List() may hold one NodeInfo at several positions: cache.go:283-291 takes numNodes
  // nodeTree.next() outputs, and after a node add the tree can restart its round-robin half way
  // through a pass.  Such rows are aliases: every change to the node is applied to all of them.
  std::vector<int32_t> row_canon;                  // [N] first row of the row's node (local index)
  std::unordered_map<int32_t, std::vector<int32_t>> alias_rows;  // canonical row -> all its rows
  bool has_alias = false;
  // ---- nominator (kgpu_set_nominated): owned copies of the records and of their pools
  struct Nominator {
    std::vector<kgpu_nominated> list;
    std::vector<kgpu_pod_query> recs;
    std::vector<kgpu_req> reqs;
    std::vector<int32_t> ints;
    std::vector<uint64_t> words;
    std::vector<kgpu_node_term> nterms;
    std::vector<kgpu_pref_term> pterms;
    std::vector<kgpu_spread> spreads;
    std::vector<kgpu_pod_term> pod_terms;
    std::vector<kgpu_scalar_req> scalars;
    std::vector<kgpu_port> ports;
    kgpu_pools pools{};
  } nom;
  // preemption / nominated-pass staging (device copies live until the stream is synchronized)
  DevBuf p_args, p_voff, p_veff, p_noff, p_neff, p_aux, p_vrecs, p_vsc, p_vports, p_nrecs, p_nsc, p_nports,
      p_vstate, p_order, p_out, p_outv, p_prep, p_nomstat, p_pdb;
  kgpu::PreemptArgs pa_host{};
  // ---- node sharding over xGMI (kgpu_xgmi_init): granule mailbox ring, peers' rings opened
  // through IPC handles, the common persistent geometry of every rank
  int32_t xg_nranks = 0, xg_rank = 0;
  DevBuf xg_box;                 // [kXgmiRing][GT] u64 granules | [kXgmiRing][GT] i32 feasible counts
  std::vector<void*> xg_open;    // peers' boxes (hipIpcOpenMemHandle), closed on destroy
  DevBuf xg_arr;                 // device array: nranks granule bases, then nranks feasible-count bases
  int xg_geo = -1, xg_per = 0, xg_groups = 0, xg_GT = 0;
  int64_t xg_seq = 0;            // ring sequence of the next pod (identical on every rank)
  // the persistent topology kernel's cross-rank exchange: TX ring (one row per pod) and the init
  // mailbox of the histogram reduction, both inside xg_box after the granule / feasible rings
  size_t xg_tx_off = 0, xg_init_off = 0;  // byte offsets in xg_box
  int64_t xt_seq = 0;            // TX ring sequence of the next topology pod (identical on every rank)
  uint64_t xr_seq = 0;           // init reductions issued (identical on every rank)
  bool xgmi = true;              // KGPU_OPT_XGMI
  DevBuf batch_ptrs;             // unsharded persistent runs: {gran, feas} per run
  DevBuf flags_buf;                                // DevState::port_overflow
  DevBuf d_stage, d_remap, d_from;
  kgpu::HostStage delta_stage;                     // pinned staging block of a delta launch
  void* cyc_host = nullptr;                        // pinned staging of a short cycle: DevState + queries
  void* res_pin = nullptr;                         // pinned coherent block the short cycle's kernels
  kgpu_result* res_dev = nullptr;                  // write their result records into (its device address)
  // pinned coherent block a one-launch cycle's k_eval reads the pod's query pools from (zero-copy: no copy
  // on the stream for pools that change with every pod), and its device address
  void* pool_pin = nullptr;
  const char* pool_pin_dev = nullptr;
  bool zc_pools = true;                            // KGPU_OPT_ZEROCOPY_POOLS
  // short-cycle arena (arena_put): bump offset and capacity in cyc_host / dstate, the byte range
  // still to be copied, and whether a copy from cyc_host may still be pending (kgpu_staging.h)
  kgpu::Arena ar;
  bool tb_abort_mapped = false;                    // the last k_tbatch run wrote its abort word to res_pin
  // Resident topology run state (TCache): the histograms, pair registrations, signature flags and
  // eligibility bitmaps of the last persistent topology run, as that run left them (k_tbatch writes
  // its final bins back).  The next run with the same tables starts from them instead of a
  // k_tbatch_init pass -- valid only while nothing else changed the mirror since: every other
  // writer of node state (upload, deltas, forget, the other evaluation paths' assumes, sharding)
  // drops it.
  // Two buffers: the run uses buf[cur] (a hit) or the other one (a miss), and zeroes the buffer it
  // does not use at kernel entry, so a miss finds its buffer zeroed without a memset (one stream
  // operation less per cycle where every pod brings other tables, config (d)).
  struct TCache {
    bool valid = false;
    std::string key;     // the run's hists, signature programs, registrations and geometry
    DevBuf buf[2];       // hist_init | tot_init | reg_init | sig_any | elig
    size_t dirty[2] = {0, 0};  // leading bytes of buf[i] that may be non-zero
    int cur = 0;
  } tc;
  uint64_t tc_hits = 0, tc_misses = 0;
  // KGPU_HOST_TRACE=1 (diagnostics): host time of a short cycle's steps, summed over cycles and printed
  // to stderr by kgpu_destroy (stamp k closes step k)
  bool htrace = false;
  static constexpr int kHt = 18;
  int64_t ht_last = 0, ht_cur[kHt] = {}, ht_n = 0;
  int ht_seen = 0;
  std::vector<std::array<int64_t, kHt>> ht_cycles;  // per short cycle: ns of each step (p50 / p99 at destroy)
  std::vector<std::array<int64_t, kHt>> ht_batches; // the same for longer calls (kgpu_schedule_batch)
  bool tc_on = true;                               // KGPU_OPT_TOPO_RESIDENT
  bool batch_helper = true;                        // KGPU_OPT_BATCH_HELPER
  bool topo_ahead = true;                          // KGPU_OPT_TOPO_AHEAD
  int tbatch_geo_first = 1;                        // KGPU_OPT_TBATCH_GEO (256 x 1 measured equal: 512 x 1 stays)
  size_t ar_limit = 1 << 20;                       // KGPU_OPT_ARENA_BYTES (bytes of arena items per cycle)
  DevState ds_last{};                              // the DevState image last uploaded by a short cycle
  const void* ds_ptr = nullptr;                    // ... into this dstate allocation (null: none)
  bool last_diag = false;
  std::vector<int64_t> trace_wg_host;             // k_tbatch per-workgroup stamps of the last traced run
  int32_t trace_wg_groups = 0;
  std::vector<hipEvent_t> ev_pool;
  // ---- topology state (kgpu_internal.h "topology plugins")
  std::map<std::vector<int64_t>, int> class_ids, tclass_ids;
  std::vector<kgpu::ClassRec> classes;
  std::vector<kgpu::ClassItem> citems;
  std::vector<kgpu::TermClassRec> tclasses;
  std::vector<kgpu_req> creqs;
  std::vector<int32_t> cints;
  int classes_init = 0;          // classes whose mcnt column is initialized on the device
  int Ccap = 0, TCcap = 0;
  DevBuf d_classes, d_citems, d_tclasses, d_creqs, d_cints, d_plans, d_aux, d_aux_terms, scratch, d_pods;
  // host mirror of the pod table (snapshot pods, then assumed pods in slot order)
  struct PodRow {
    int32_t node, ns;
    uint32_t flags;
    std::vector<int32_t> pairs;  // (pod label key id, value id)
    std::vector<int32_t> own_tcls;
  };
  std::vector<PodRow> pod_rows;
  int pod_rows_dev = -1;         // rows present in the device pod table (-1: rebuild it whole)
  std::vector<int32_t> pod_rows_dirty;  // slots below pod_rows_dev changed in place since (flags)
  std::vector<int32_t> key_n_values, key_empty;
  std::vector<uint8_t> key_unique;  // every value of the key sits on at most one node of THIS shard
  // kgpu_snapshot / kgpu_delta_batch.key_unique: the caller's cluster-wide view (empty: not given)
  std::vector<uint8_t> key_unique_caller;
  int64_t max_key_values = 1;
  // persistent topology runs (k_tbatch)
  bool tfast = true;                // KGPU_OPT_TOPO_PERSISTENT
  bool coop = false;                // KGPU_OPT_COOPERATIVE (ordinary launches of a co-resident grid)
  bool force_coop = false;          // a call issued again after a clean abort (every persistent launch
                                    // of it cooperative)
  int32_t hold_group = -1;          // KGPU_OPT_HOLD_GROUP test hook
  bool tbatch_wlab = true;          // KGPU_OPT_TBATCH_WLAB
  bool tbatch_sleep = true;         // KGPU_OPT_TBATCH_POLL_SLEEP
  bool run_all = false;             // KGPU_OPT_RUN_ALL_FILTERS
  bool last_run_all = false;        // the last diagnostic cycle wrote status_all
  int64_t n_coop_retry = 0, n_persist = 0, n_coop = 0;  // kgpu_debug_counters
  int64_t n_class_init = 0, n_pod_table_full = 0;       // ... k_class_init launches, whole pod-table uploads
  int state_launches = 0;           // launches of the current call that may change device state
  // pipelined batches (kgpu_schedule_batch_submit / _wait): two slots, each with its pinned staging block,
  // device block (DevState | queries | run pointers | abort word), granules and pinned result records
  struct PipeSlot {
    void* host = nullptr;         // pinned staging of the device block
    size_t host_cap = 0;
    DevBuf dev, gran;
    void* res = nullptr;          // pinned, mapped: the records and the abort word, written by k_batch_fixup
    void* res_dev = nullptr;
    size_t res_cap = 0;
    size_t gran_zeroed = 0;       // leading bytes of `gran` known to be zero
    hipEvent_t done = nullptr, t0 = nullptr, t1 = nullptr;
  };
  struct PipeBatch {
    int slot = 0;
    int32_t n = 0;
    kgpu_result* results = nullptr;
    kgpu_stats* stats = nullptr;
    std::vector<kgpu_pod_query> qs;           // for the assumed pods' records (ForgetPod)
    std::vector<int32_t> ints;                // the pools' label pairs ...
    std::vector<kgpu_scalar_req> scalars;     // ... and scalar requests those records keep
    int rc = KGPU_OK;                         // its outcome once done
    bool done = false;                        // completed (a batch the pipeline does not carry: in submit)
    bool timed = false;
  };
  PipeSlot pipe[2];
  std::deque<PipeBatch> pipe_q;
  int pipe_next = 0;
  bool unsettled = false;           // a short cycle returned on its completion word, before the stream's
                                    // own completion: settle() before anything that is not stream-ordered
  int batch_geo_first = 0;          // KGPU_OPT_BATCH_GEO
  DevBuf t_tables, t_zero, abort_buf;
  kgpu::HostStage table_stage;   // pinned staging of the runs' tables (bump-allocated, wraps after a sync)
  kgpu::HostStage batch_stage;   // pinned staging of a long batch's queries, DevState, run pointers and results
  DevBuf pool_blk;               // the call's query pools, packed (upload_pools)
  kgpu::HostStage pool_stage;    // ... and their pinned staging
  // ---- node sharding (kgpu_comm_init): this context holds one contiguous slice of the
  // snapshot; per pod the shard winners (and normalize maxima) are all-gathered over RCCL
  ncclComm_t comm = nullptr;
  int32_t nranks = 1, rank = 0;
  DevBuf shard;   // send key | send stat | keys [2][kMaxRanks] | stats [2][kMaxRanks]
  DevBuf cut_buf;  // DevState::cut_state (nextStartNodeIndex, last EvaluatedNodes)
  bool cut_init = false;
};

namespace {

int fail(kgpu_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

// ---- exception barrier: no C++ exception crosses the C ABI (include/kgpu.h conventions).  Every
// extern "C" entry is a function-try-block whose handler maps the exception in flight to a KGPU_E_*
// code and last_error.  A state-changing entry (upload, schedule, delta, forget) that throws may have
// left the host books and the device mirror apart, so its handler also invalidates the mirror: the
// engine then refuses cycles (KGPU_E_STATE) until the next kgpu_upload_snapshot.
std::atomic<int32_t> g_fail_alloc{0};  // kgpu_debug_fail_alloc countdown (0: off)

// A host allocation point the fault-injection hook can fail (std::bad_alloc, as operator new would).
void fail_point() {
  if (g_fail_alloc.load(std::memory_order_relaxed) > 0 && g_fail_alloc.fetch_sub(1) == 1) throw std::bad_alloc();
}

int on_exception(kgpu_ctx* c, bool invalidate) noexcept {
  int code = KGPU_E_STATE;
  const char* msg = "internal error (unknown exception)";
  std::string what;
  try {
    throw;
  } catch (const std::bad_alloc&) {
    code = KGPU_E_NOMEM;
    msg = "host memory allocation failed";
  } catch (const std::exception& e) {
    msg = "internal error";
    try {
      what = e.what();
    } catch (...) {
    }
  } catch (...) {
  }
  if (c) {
    if (invalidate) c->uploaded = false;
    try {
      c->err = std::string(msg) + (what.empty() ? "" : ": " + what) +
               (invalidate ? " (device mirror invalidated: upload the snapshot again)" : "");
    } catch (...) {
      c->err.clear();
    }
  }
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
  // a pipelined batch in flight may still read the old buffer (kgpu_schedule_batch_submit)
  if (b.p && !c->pipe_q.empty()) HIP_OK(c, hipStreamSynchronize(c->stream));
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  HIP_OK(c, hipMalloc(&b.p, bytes));
  b.bytes = bytes;
  return KGPU_OK;
}

// ensure() for buffers a cycle sizes from its own pods (plans, scratch, class tables): grown with headroom,
// so a run of pods that each need a little more does not pay a free + malloc on one cycle after another.
int ensure_grow(kgpu_ctx* c, DevBuf& b, size_t bytes) {
  if (b.bytes >= bytes) return KGPU_OK;
  return ensure(c, b, std::max<size_t>({bytes, 2 * b.bytes, (size_t)64 << 10}));
}

// ---- short-cycle arena.  A short cycle (kgpu_schedule_one, small batches) stages what it must send
// -- changed query pools, topology plans, DevState + queries, a one-pod persistent topology run's
// tables and zeroed words -- in the pinned block c->cyc_host, at the offsets they take in the device
// block c->dstate, and moves them with ONE copy (arena_flush, before the cycle's first launch that
// reads them): each stream operation saved is several microseconds of the per-cycle latency.  Items
// that do not fit take their own copies.  The arena is live only inside run_batch (ArenaScope).
constexpr size_t kArenaBytes = 1 << 20;
// Short cycles: at most kShortCycle pods.  Device block c->dstate = DevState | n queries (at
// kDsQueryOff) | the cycle's arena; pinned c->cyc_host = the same image.  The kernels write the
// result records into the pinned block c->res_pin (kCycResBytes), a k_tbatch run its abort word
// right after them.
constexpr int32_t kShortCycle = 64;
constexpr size_t kDsQueryOff = (sizeof(DevState) + 255) & ~(size_t)255;
constexpr size_t kCycHostBytes = kDsQueryOff + sizeof(kgpu_pod_query) * kShortCycle + kArenaBytes;
constexpr size_t kCycResBytes = sizeof(kgpu_result) * kShortCycle;
constexpr size_t kCycAbortOff = kCycResBytes;  // int32 in res_pin
constexpr size_t kCycDoneOff = kCycResBytes + 4;  // int32 in res_pin: k_final's completion word (PodArgs.done_out)

// The context's stream synchronize: every pending copy from the staging blocks has run
// (kgpu_staging.h), so they may be rewritten, regrown or freed.
int sync_stream(kgpu_ctx* c) {
  HIP_OK(c, hipStreamSynchronize(c->stream));
  c->pool_stage.synced();
  c->table_stage.synced();
  c->batch_stage.synced();
  c->delta_stage.synced();
  c->ar.synced();
  return KGPU_OK;
}
#define SYNC_OK(c)                 \
  do {                             \
    const int rs_ = sync_stream(c); \
    if (rs_) return rs_;           \
  } while (0)

int stage_sync(void* self) { return sync_stream(static_cast<kgpu_ctx*>(self)); }

// The stream's own completion of a short cycle that returned on its completion word.
int settle(kgpu_ctx* c) {
  if (!c->unsettled) return KGPU_OK;
  c->unsettled = false;
  return sync_stream(c);
}
int stage_alloc(void* self, void** p, size_t bytes) {
  kgpu_ctx* c = static_cast<kgpu_ctx*>(self);
  fail_point();
  HIP_OK(c, hipHostMalloc(p, bytes, hipHostMallocDefault));
  return KGPU_OK;
}
void stage_release(void*, void* p) { (void)hipHostFree(p); }
kgpu::StageOps stage_ops(kgpu_ctx* c) { return kgpu::StageOps{c, stage_sync, stage_alloc, stage_release}; }

// `bytes` of the arena: host and device addresses (false: no arena, or full)
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
// host trace stamp k of the current short cycle (k = 0 opens it)
inline void ht(kgpu_ctx* c, int k) {
  if (!c->htrace) return;
  const int64_t t = now_ns();
  if (k == 0) std::fill(c->ht_cur, c->ht_cur + kgpu_ctx::kHt, 0);
  if (k > 0) c->ht_cur[k] += t - c->ht_last;
  c->ht_last = t;
  c->ht_seen |= 1 << k;
}

bool arena_reserve(kgpu_ctx* c, size_t bytes, char** host, char** dev) {
  size_t o;
  if (!c->ar.reserve(bytes, &o)) return false;
  *host = static_cast<char*>(c->cyc_host) + o;
  *dev = static_cast<char*>(c->dstate.p) + o;
  return true;
}

// a copy of `src` (zeros when null) in the arena: its device address, or null
void* arena_put(kgpu_ctx* c, const void* src, size_t bytes) {
  char *h, *d;
  if (!arena_reserve(c, bytes, &h, &d)) return nullptr;
  if (src) std::memcpy(h, src, bytes);
  else std::memset(h, 0, bytes);
  return d;
}

int arena_flush(kgpu_ctx* c) {
  size_t lo, hi;
  if (c->ar.take_dirty(&lo, &hi))
    HIP_OK(c, hipMemcpyAsync(static_cast<char*>(c->dstate.p) + lo, static_cast<char*>(c->cyc_host) + lo, hi - lo,
                             hipMemcpyHostToDevice, c->stream));
  return KGPU_OK;
}

struct ArenaScope {
  kgpu_ctx* c;
  ~ArenaScope() { c->ar.end(); }
};

template <class T>
int upload_pool(kgpu_ctx* c, DevBuf& b, const T* src, int32_t n, const T** dst) {
  int rc = ensure_grow(c, b, sizeof(T) * (size_t)std::max(n, 1));
  if (rc) return rc;
  const size_t bytes = sizeof(T) * (size_t)std::max(n, 0);
  // A caller that passes the same pools every cycle (the batch's pools, one pod at a time) pays
  // one copy, not one per cycle: the device copy is current when the bytes equal the last upload
  // into this same allocation.  Pools above kPoolShadowMax are always copied.
  constexpr size_t kPoolShadowMax = 256 * 1024;
  const bool current = n > 0 && b.shadow_p == b.p && b.shadow.size() == bytes &&
                       std::memcmp(b.shadow.data(), src, bytes) == 0;
  if (n > 0 && !current) {
    HIP_OK(c, hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, c->stream));
    if (bytes <= kPoolShadowMax) {
      b.shadow.assign(reinterpret_cast<const char*>(src), reinterpret_cast<const char*>(src) + bytes);
      b.shadow_p = b.p;
    } else {
      b.shadow.clear();
      b.shadow_p = nullptr;
    }
  }
  *dst = static_cast<const T*>(b.p);
  return KGPU_OK;
}

// The query pools of a call, packed into one pinned block and moved with ONE copy (skipped when
// the bytes equal the last upload): a pageable copy per pool cost microseconds each on the per-pod
// (kgpu_schedule_one) path.  The staging block is rewritten only by the next call, after this call's
// stream synchronize.
constexpr size_t kPoolPinBytes = 64 * 1024;

// zero_copy: a one-pod cycle whose only kernel is k_eval (kgpu_schedule_one's one-launch and normalize
// cycles without topology state): pools that are not on the device already are read by the kernel from
// pinned host memory (each wave's reads are uniform: one transaction per wave and word) instead of
// riding in the cycle's arena copy -- the copy was one hipMemcpyAsync and one copyBuffer dispatch per
// cycle (profiles/r05_b5000_cycle_hip_stats.txt).  The block is rewritten only by the next cycle, after
// this one's kernel finished (the cycle returns on its completion word or its stream synchronize).
int upload_pools(kgpu_ctx* c, const kgpu_pools* p, bool zero_copy = false) {
  kgpu_pools empty{};
  if (!p) p = &empty;
  kgpu::DevPools& q = c->st.qp;
  size_t off = 0;
  auto place = [&](size_t bytes) {
    const size_t o = off;
    off += (std::max<size_t>(bytes, 16) + 15) & ~(size_t)15;
    return o;
  };
  auto nb = [](int32_t n, size_t sz) { return sz * (size_t)std::max(n, 0); };
  const size_t o_req = place(nb(p->n_reqs, sizeof(kgpu_req))), o_int = place(nb(p->n_ints, sizeof(int32_t))),
               o_wrd = place(nb(p->n_words, sizeof(uint64_t))), o_nt = place(nb(p->n_node_terms, sizeof(kgpu_node_term))),
               o_pt = place(nb(p->n_pref_terms, sizeof(kgpu_pref_term))), o_sp = place(nb(p->n_spreads, sizeof(kgpu_spread))),
               o_pd = place(nb(p->n_pod_terms, sizeof(kgpu_pod_term))), o_sc = place(nb(p->n_scalars, sizeof(kgpu_scalar_req))),
               o_po = place(nb(p->n_ports, sizeof(kgpu_port)));
  const size_t total = off;
  // the block is rewritten from offset 0: a copy from its previous contents still pending (a call
  // that left before its synchronize) is waited for first (kgpu_staging.h)
  char* h = nullptr;
  int rc0;
  const kgpu::StageOps ops = stage_ops(c);
  if ((rc0 = c->pool_stage.rewrite(ops, total, 64 * 1024, &h))) return rc0;
  std::memset(h, 0, total);
  auto put = [&](size_t o, const void* src, size_t bytes) {
    if (src && bytes) std::memcpy(h + o, src, bytes);
  };
  put(o_req, p->reqs, nb(p->n_reqs, sizeof(kgpu_req)));
  put(o_int, p->ints, nb(p->n_ints, sizeof(int32_t)));
  put(o_wrd, p->words, nb(p->n_words, sizeof(uint64_t)));
  put(o_nt, p->node_terms, nb(p->n_node_terms, sizeof(kgpu_node_term)));
  put(o_pt, p->pref_terms, nb(p->n_pref_terms, sizeof(kgpu_pref_term)));
  put(o_sp, p->spreads, nb(p->n_spreads, sizeof(kgpu_spread)));
  put(o_pd, p->pod_terms, nb(p->n_pod_terms, sizeof(kgpu_pod_term)));
  put(o_sc, p->scalars, nb(p->n_scalars, sizeof(kgpu_scalar_req)));
  put(o_po, p->ports, nb(p->n_ports, sizeof(kgpu_port)));
  int rc;
  if ((rc = ensure_grow(c, c->pool_blk, total))) return rc;
  const bool current = c->pool_blk.shadow_p == c->pool_blk.p && c->pool_blk.shadow.size() == total &&
                       std::memcmp(c->pool_blk.shadow.data(), h, total) == 0;
  const char* d = static_cast<const char*>(c->pool_blk.p);
  if (!current && zero_copy && c->zc_pools && total <= kPoolPinBytes) {
    if (!c->pool_pin) {
      HIP_OK(c, hipHostMalloc(&c->pool_pin, kPoolPinBytes, hipHostMallocCoherent | hipHostMallocMapped));
      void* dp = nullptr;
      HIP_OK(c, hipHostGetDevicePointer(&dp, c->pool_pin, 0));
      c->pool_pin_dev = static_cast<const char*>(dp);
    }
    std::memcpy(c->pool_pin, h, total);
    d = c->pool_pin_dev;
  } else if (!current) {
    // a short cycle's changed pools ride in its arena copy (pool_blk and its shadow stay as they were)
    if (const void* a = arena_put(c, h, total)) {
      d = static_cast<const char*>(a);
    } else {
      HIP_OK(c, hipMemcpyAsync(c->pool_blk.p, h, total, hipMemcpyHostToDevice, c->stream));
      c->pool_stage.enqueued();
      c->pool_blk.shadow.assign(h, h + total);
      c->pool_blk.shadow_p = c->pool_blk.p;
    }
  }
  q.reqs = reinterpret_cast<const kgpu_req*>(d + o_req);
  q.ints = reinterpret_cast<const int32_t*>(d + o_int);
  q.words = reinterpret_cast<const uint64_t*>(d + o_wrd);
  q.node_terms = reinterpret_cast<const kgpu_node_term*>(d + o_nt);
  q.pref_terms = reinterpret_cast<const kgpu_pref_term*>(d + o_pt);
  q.spreads = reinterpret_cast<const kgpu_spread*>(d + o_sp);
  q.pod_terms = reinterpret_cast<const kgpu_pod_term*>(d + o_pd);
  q.scalars = reinterpret_cast<const kgpu_scalar_req*>(d + o_sc);
  q.ports = reinterpret_cast<const kgpu_port*>(d + o_po);
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
    // sharded: the cluster-wide union, or ranks would disagree on the extra stat all-gather
    const std::vector<uint64_t>& u = c->comm ? c->prefer_global : c->prefer_union;
    for (size_t w = 0; w < u.size(); ++w) {
      uint64_t tol = (p && (int)w < q.tol_prefer.count) ? p->words[q.tol_prefer.begin + w] : 0ull;
      if (u[w] & ~tol) return true;
    }
  }
  return false;
}

// Cluster-wide PreferNoSchedule union: all-gather every rank's shard union (TW words) and OR them.
int sync_prefer_union(kgpu_ctx* c) {
  const size_t TW = c->prefer_union.size();
  const size_t bytes = sizeof(uint64_t) * TW * (size_t)(c->nranks + 1);
  int rc = ensure(c, c->pref_x, std::max<size_t>(bytes, 8));
  if (rc) return rc;
  uint64_t* d = static_cast<uint64_t*>(c->pref_x.p);
  if (TW) {
    HIP_OK(c, hipMemcpyAsync(d, c->prefer_union.data(), sizeof(uint64_t) * TW, hipMemcpyHostToDevice, c->stream));
    const ncclResult_t r = rccl().AllGather(d, d + TW, TW, ncclUint64, c->comm, c->stream);
    if (r != ncclSuccess) return fail(c, KGPU_E_DEVICE, std::string("ncclAllGather: ") + rccl().GetErrorString(r));
  }
  std::vector<uint64_t> all(TW * (size_t)c->nranks);
  if (TW) HIP_OK(c, hipMemcpyAsync(all.data(), d + TW, sizeof(uint64_t) * all.size(), hipMemcpyDeviceToHost, c->stream));
  SYNC_OK(c);
  c->prefer_global.assign(TW, 0ull);
  for (int r = 0; r < c->nranks; ++r)
    for (size_t w = 0; w < TW; ++w) c->prefer_global[w] |= all[(size_t)r * TW + w];
  return KGPU_OK;
}


// ---------------------------------------------------------------- topology: pod classes
// Classes are interned by content, so every pod with the same spread selector / term shares one
// match-count column.  Selector requirements and namespace sets are copied into the class pool.
bool topo_profile(const kgpu_ctx* c) {
  for (int i = 0; i < c->cfg.n_filters; ++i)
    if (c->cfg.filters[i] == KGPU_F_POD_TOPOLOGY_SPREAD || c->cfg.filters[i] == KGPU_F_INTER_POD_AFFINITY) return true;
  return has_score(c, KGPU_S_POD_TOPOLOGY_SPREAD) || has_score(c, KGPU_S_INTER_POD_AFFINITY) ||
         has_score(c, KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD);
}

bool has_filter(const kgpu_ctx* c, int f) {
  for (int i = 0; i < c->cfg.n_filters; ++i)
    if (c->cfg.filters[i] == f) return true;
  return false;
}

// A hostname-like key (every value on at most one node): its topology counts are read from the
// node's own column instead of a domain histogram.  Unique on this shard AND, when the caller gave its
// cluster-wide view, unique there; a node-sharded engine without that view treats the key as shared.
bool key_uniq(const kgpu_ctx* c, int k) {
  if (k < 0 || !c->key_unique[(size_t)k]) return false;
  if (!c->key_unique_caller.empty()) return c->key_unique_caller[(size_t)k] != 0;
  return c->comm == nullptr && c->xg_nranks <= 1 && c->st.n_total == c->st.N;
}

struct ItemSrc {
  std::vector<int32_t> ns;
  kgpu_selector sel;
  const kgpu_pools* p;
};

void key_push_item(std::vector<int64_t>& k, const ItemSrc& it) {
  std::vector<int32_t> ns = it.ns;
  std::sort(ns.begin(), ns.end());
  k.push_back((int64_t)ns.size());
  for (int32_t x : ns) k.push_back(x);
  k.push_back(it.sel.kind);
  const int nr = it.sel.kind == KGPU_SEL_AND ? it.sel.reqs.count : 0;
  k.push_back(nr);
  for (int i = 0; i < nr; ++i) {
    const kgpu_req& r = it.p->reqs[it.sel.reqs.begin + i];
    std::vector<int32_t> v(it.p->ints + r.vals.begin, it.p->ints + r.vals.begin + r.vals.count);
    std::sort(v.begin(), v.end());
    k.push_back(r.key);
    k.push_back(r.op);
    k.push_back(r.imm);
    k.push_back((int64_t)v.size());
    for (int32_t x : v) k.push_back(x);
  }
}

kgpu::ClassItem store_item(kgpu_ctx* c, const ItemSrc& it) {
  kgpu::ClassItem o{};
  o.ns.begin = (int32_t)c->cints.size();
  o.ns.count = (int32_t)it.ns.size();
  c->cints.insert(c->cints.end(), it.ns.begin(), it.ns.end());
  o.sel.kind = it.sel.kind;
  const int nr = it.sel.kind == KGPU_SEL_AND ? it.sel.reqs.count : 0;
  std::vector<kgpu_req> reqs;
  for (int i = 0; i < nr; ++i) {
    kgpu_req r = it.p->reqs[it.sel.reqs.begin + i];
    const int32_t b = (int32_t)c->cints.size();
    c->cints.insert(c->cints.end(), it.p->ints + r.vals.begin, it.p->ints + r.vals.begin + r.vals.count);
    r.vals.begin = b;
    reqs.push_back(r);
  }
  o.sel.reqs.begin = (int32_t)c->creqs.size();
  o.sel.reqs.count = nr;
  c->creqs.insert(c->creqs.end(), reqs.begin(), reqs.end());
  return o;
}

int intern_class(kgpu_ctx* c, int excl, const std::vector<ItemSrc>& items) {
  std::vector<int64_t> k{0, excl, (int64_t)items.size()};
  for (const ItemSrc& it : items) key_push_item(k, it);
  auto f = c->class_ids.find(k);
  if (f != c->class_ids.end()) return f->second;
  kgpu::ClassRec cr{};
  cr.item0 = (int32_t)c->citems.size();
  cr.n_items = (int32_t)items.size();
  cr.excl_terminating = excl;
  for (const ItemSrc& it : items) c->citems.push_back(store_item(c, it));
  const int id = (int)c->classes.size();
  c->classes.push_back(cr);
  c->class_ids[k] = id;
  return id;
}

int intern_tclass(kgpu_ctx* c, int kind, int weight, int topo_key, const ItemSrc& it) {
  std::vector<int64_t> k{1, kind, weight, topo_key};
  key_push_item(k, it);
  auto f = c->tclass_ids.find(k);
  if (f != c->tclass_ids.end()) return f->second;
  kgpu::TermClassRec t{};
  t.kind = kind;
  t.weight = weight;
  t.topo_key = topo_key;
  t.item = store_item(c, it);
  const int id = (int)c->tclasses.size();
  c->tclasses.push_back(t);
  c->tclass_ids[k] = id;
  return id;
}

ItemSrc term_item(const kgpu_pod_term& t, const kgpu_pools* p) {
  ItemSrc it;
  it.ns.assign(p->ints + t.ns.begin, p->ints + t.ns.begin + t.ns.count);
  it.sel = t.sel;
  it.p = p;
  return it;
}

// labels.Selector.Matches of a class item against a pod given as (key, value) pairs
// (selector.go:198-242; util/topologies.go:40-49).
bool item_matches(const kgpu_ctx* c, const kgpu::ClassItem& it, int32_t ns, const int32_t* pairs, int np) {
  bool in_ns = false;
  for (int i = 0; i < it.ns.count; ++i) in_ns |= c->cints[it.ns.begin + i] == ns;
  if (!in_ns || it.sel.kind != KGPU_SEL_AND) return false;
  for (int i = 0; i < it.sel.reqs.count; ++i) {
    const kgpu_req& r = c->creqs[it.sel.reqs.begin + i];
    int v = -1;
    for (int j = 0; j < np; ++j)
      if (pairs[2 * j] == r.key) v = pairs[2 * j + 1];
    if (r.key < 0) v = -1;
    bool in = false;
    for (int j = 0; j < r.vals.count; ++j) in |= c->cints[r.vals.begin + j] == v;
    switch (r.op) {
      case KGPU_OP_IN: if (!(v >= 0 && in)) return false; break;
      case KGPU_OP_NOTIN: if (v >= 0 && in) return false; break;
      case KGPU_OP_EXISTS: if (v < 0) return false; break;
      case KGPU_OP_DNE: if (v >= 0) return false; break;
      default: return false;
    }
  }
  return true;
}

bool class_matches(const kgpu_ctx* c, int cls, int32_t ns, uint32_t flags, const int32_t* pairs, int np) {
  const kgpu::ClassRec& cr = c->classes[cls];
  if (cr.excl_terminating && (flags & KGPU_PF_TERMINATING)) return false;
  if (cr.n_items == 0) return false;
  for (int i = 0; i < cr.n_items; ++i)
    if (!item_matches(c, c->citems[cr.item0 + i], ns, pairs, np)) return false;
  return true;
}

uint32_t query_pod_flags(const kgpu_pod_query& q) {
  return KGPU_PF_ACTIVE | ((q.flags & KGPU_Q_TERMINATING) ? KGPU_PF_TERMINATING : 0u) |
         ((q.flags & (KGPU_Q_HAS_POD_AFFINITY | KGPU_Q_HAS_POD_ANTI)) ? KGPU_PF_WITH_AFFINITY : 0u);
}

struct SlotAlloc {
  kgpu::QPlan* pl;
  const kgpu_ctx* c;
  int64_t off;
  int get(int kind, int key) {
    for (int s = 0; s < pl->n_slots; ++s)
      if (pl->slot_kind[s] == kind && pl->slot_key[s] == key) return s;
    if (pl->n_slots == kgpu::kMaxSlots) return -1;
    const int s = pl->n_slots++;
    pl->slot_kind[s] = kind;
    pl->slot_key[s] = key;
    pl->slot_off[s] = off;
    off += key >= 0 ? std::max<int64_t>(1, c->key_n_values[key]) : 1;
    return s;
  }
};

// Per-query plans of a batch: pass 1 interns every class / term class the batch needs, pass 2
// matches each pod against all of them (its assume increments and the existing terms it meets).
int build_plans(kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* p,
                std::vector<kgpu::QPlan>& plans, std::vector<int32_t>& aux, std::vector<kgpu::TTerm>& aux_terms,
                int64_t* max_scratch) {
  fail_point();
  const bool fp = has_filter(c, KGPU_F_POD_TOPOLOGY_SPREAD), fi = has_filter(c, KGPU_F_INTER_POD_AFFINITY);
  const bool sp = has_score(c, KGPU_S_POD_TOPOLOGY_SPREAD), si = has_score(c, KGPU_S_INTER_POD_AFFINITY);
  const bool sd = has_score(c, KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD);
  const int hw = c->cfg.hard_pod_affinity_weight;
  plans.assign((size_t)n, kgpu::QPlan{});
  std::vector<std::vector<int32_t>> own((size_t)n);
  for (int32_t i = 0; i < n; ++i) {
    const kgpu_pod_query& q = qs[i];
    kgpu::QPlan& pl = plans[(size_t)i];
    SlotAlloc sa{&pl, c, (int64_t)kgpu::kHdrWords + std::max(c->st.n_zones, 1)};
    auto spread = [&](const kgpu_spread& sp0, bool hard, kgpu::TSpread& o, int idx, const kgpu_spread* all) {
      ItemSrc it{{q.ns}, sp0.sel, p};
      o.cls = intern_class(c, 1, {it});
      o.key = sp0.key;
      o.max_skew = sp0.max_skew;
      o.self_match = sp0.self_match;
      o.is_hostname = sp0.is_hostname;
      o.first_of_key = 1;
      for (int j = 0; j < idx; ++j)
        if (all[j].key == sp0.key) o.first_of_key = 0;
      o.rslot = sa.get(hard ? kgpu::kSlotPReg : kgpu::kSlotSReg, sp0.key);
      o.cslot = sa.get(hard ? kgpu::kSlotPCnt : kgpu::kSlotSCnt, sp0.key);
      return o.rslot >= 0 && o.cslot >= 0;
    };
    if (fp && q.pts_hard.count) {
      if (q.pts_hard.count > kgpu::kMaxSpread) return fail(c, KGPU_E_UNSUPPORTED, "more than 4 DoNotSchedule constraints");
      pl.n_hard = q.pts_hard.count;
      for (int j = 0; j < pl.n_hard; ++j)
        if (!spread(p->spreads[q.pts_hard.begin + j], true, pl.hard[j], j, p->spreads + q.pts_hard.begin))
          return fail(c, KGPU_E_UNSUPPORTED, "too many topology histograms");
    }
    if (sp && q.pts_soft.count) {
      if (q.pts_soft.count > kgpu::kMaxSpread) return fail(c, KGPU_E_UNSUPPORTED, "more than 4 ScheduleAnyway constraints");
      pl.n_soft = q.pts_soft.count;
      for (int j = 0; j < pl.n_soft; ++j)
        if (!spread(p->spreads[q.pts_soft.begin + j], false, pl.soft[j], j, p->spreads + q.pts_soft.begin))
          return fail(c, KGPU_E_UNSUPPORTED, "too many topology histograms");
    }
    pl.dpts_cls = -1;
    if (sd) {
      if (q.flags & KGPU_Q_HAS_TSC) pl.dpts_cls = -2;
      else if (q.dpts.kind != kgpu::kSelEmpty) pl.dpts_cls = intern_class(c, 1, {ItemSrc{{q.ns}, q.dpts, p}});
    }
    if (fi) {
      if (q.ipa_req_aff.count > kgpu::kMaxIpa || q.ipa_req_anti.count > kgpu::kMaxIpa)
        return fail(c, KGPU_E_UNSUPPORTED, "more than 4 required (anti-)affinity terms");
      if (q.ipa_req_aff.count) {
        std::vector<ItemSrc> items;
        for (int j = 0; j < q.ipa_req_aff.count; ++j) items.push_back(term_item(p->pod_terms[q.ipa_req_aff.begin + j], p));
        pl.conj_cls = intern_class(c, 0, items);
        pl.n_aff = q.ipa_req_aff.count;
        for (int j = 0; j < pl.n_aff; ++j) {
          const kgpu_pod_term& t = p->pod_terms[q.ipa_req_aff.begin + j];
          pl.aff[j] = kgpu::TTerm{pl.conj_cls, t.topo_key, sa.get(kgpu::kSlotAff, t.topo_key), 0};
          if (pl.aff[j].slot < 0) return fail(c, KGPU_E_UNSUPPORTED, "too many topology histograms");
        }
      }
      pl.n_anti = q.ipa_req_anti.count;
      for (int j = 0; j < pl.n_anti; ++j) {
        const kgpu_pod_term& t = p->pod_terms[q.ipa_req_anti.begin + j];
        pl.anti[j] = kgpu::TTerm{intern_class(c, 0, {term_item(t, p)}), t.topo_key, sa.get(kgpu::kSlotAnti, t.topo_key), 0};
        if (pl.anti[j].slot < 0) return fail(c, KGPU_E_UNSUPPORTED, "too many topology histograms");
      }
      pl.self_all = (q.flags & KGPU_Q_SELF_MATCH_ALL_AFF) ? 1 : 0;
    }
    if (si) {
      for (int kind = 0; kind < 2; ++kind) {
        const kgpu_range r = kind == 0 ? q.ipa_pref_aff : q.ipa_pref_anti;
        for (int j = 0; j < r.count; ++j) {
          const kgpu_pod_term& t = p->pod_terms[r.begin + j];
          if (t.topo_key < 0) continue;
          if (pl.n_pref == kgpu::kMaxPref) return fail(c, KGPU_E_UNSUPPORTED, "more than 8 preferred pod terms");
          pl.pref[pl.n_pref++] = kgpu::TTerm{intern_class(c, 0, {term_item(t, p)}), t.topo_key,
                                             sa.get(kgpu::kSlotTopo, t.topo_key), kind == 0 ? t.weight : -t.weight};
          if (pl.pref[pl.n_pref - 1].slot < 0) return fail(c, KGPU_E_UNSUPPORTED, "too many topology histograms");
        }
      }
    }
    // the pod's own terms (PodInfo, types.go:92-160): term classes it adds on assume
    const kgpu_range tr[4] = {q.ipa_req_aff, q.ipa_req_anti, q.ipa_pref_aff, q.ipa_pref_anti};
    const int tk[4] = {KGPU_TERM_REQ_AFF, KGPU_TERM_REQ_ANTI, KGPU_TERM_PREF_AFF, KGPU_TERM_PREF_ANTI};
    for (int k = 0; k < 4; ++k)
      for (int j = 0; j < tr[k].count; ++j) {
        const kgpu_pod_term& t = p->pod_terms[tr[k].begin + j];
        own[(size_t)i].push_back(intern_tclass(c, tk[k], t.weight, t.topo_key, term_item(t, p)));
      }
    pl.scratch_len = sa.off;
  }
  // pass 2: matches against every class / term class
  for (int32_t i = 0; i < n; ++i) {
    const kgpu_pod_query& q = qs[i];
    kgpu::QPlan& pl = plans[(size_t)i];
    SlotAlloc sa{&pl, c, pl.scratch_len};
    const int32_t* pairs = q.labels.count ? p->ints + q.labels.begin : nullptr;
    const int np = q.labels.count / 2;
    const uint32_t fl = query_pod_flags(q);
    pl.assume_cls.begin = (int32_t)aux.size();
    for (int cl = 0; cl < (int)c->classes.size(); ++cl)
      if (class_matches(c, cl, q.ns, fl, pairs, np)) aux.push_back(cl);
    pl.assume_cls.count = (int32_t)aux.size() - pl.assume_cls.begin;
    pl.own_tcls.begin = (int32_t)aux.size();
    aux.insert(aux.end(), own[(size_t)i].begin(), own[(size_t)i].end());
    pl.own_tcls.count = (int32_t)own[(size_t)i].size();
    // existing pods' terms that match this pod: required anti-affinity first (filter), then the
    // score terms (scoring.go:109-124)
    pl.ex.begin = (int32_t)aux_terms.size();
    for (int pass = 0; pass < 2; ++pass) {
      for (int t = 0; t < (int)c->tclasses.size(); ++t) {
        const kgpu::TermClassRec& tc = c->tclasses[t];
        if (tc.topo_key < 0) continue;
        int w;
        if (pass == 0) {
          if (!fi || tc.kind != KGPU_TERM_REQ_ANTI) continue;
          w = 0;
        } else {
          if (!si) continue;
          if (tc.kind == KGPU_TERM_REQ_AFF) {
            if (hw <= 0) continue;
            w = hw;
          } else if (tc.kind == KGPU_TERM_PREF_AFF) {
            w = tc.weight;
          } else if (tc.kind == KGPU_TERM_PREF_ANTI) {
            w = -tc.weight;
          } else {
            continue;
          }
        }
        if (!item_matches(c, tc.item, q.ns, pairs, np)) continue;
        const int slot = sa.get(pass == 0 ? kgpu::kSlotExA : kgpu::kSlotTopo, tc.topo_key);
        if (slot < 0) return fail(c, KGPU_E_UNSUPPORTED, "too many topology histograms");
        aux_terms.push_back(kgpu::TTerm{t, tc.topo_key, slot, w});
      }
      if (pass == 0) pl.n_ex_anti = (int32_t)aux_terms.size() - pl.ex.begin;
    }
    pl.ex.count = (int32_t)aux_terms.size() - pl.ex.begin;
    pl.scratch_len = sa.off;
    pl.topo = (pl.n_hard || pl.n_soft || pl.dpts_cls >= 0 || pl.n_aff || pl.n_anti || pl.n_pref || pl.ex.count) ? 1 : 0;
    *max_scratch = std::max(*max_scratch, pl.scratch_len);
  }
  return KGPU_OK;
}

// Grow an int32 [cap][N] column table to hold `need` columns (existing columns kept).
int grow_columns(kgpu_ctx* c, int32_t** tab, int* cap, int need) {
  if (need <= *cap && *tab) return KGPU_OK;
  int nc = std::max(16, *cap);
  while (nc < need) nc *= 2;
  const size_t N = (size_t)std::max(c->st.N, 1);
  int32_t* t = nullptr;
  HIP_OK(c, hipMalloc(&t, sizeof(int32_t) * N * nc));
  HIP_OK(c, hipMemsetAsync(t, 0, sizeof(int32_t) * N * nc, c->stream));
  if (*tab && *cap) HIP_OK(c, hipMemcpyAsync(t, *tab, sizeof(int32_t) * N * (*cap), hipMemcpyDeviceToDevice, c->stream));
  SYNC_OK(c);
  if (*tab) (void)hipFree(*tab);
  *tab = t;
  *cap = nc;
  return KGPU_OK;
}

// A pod row changed in place (its flags): re-sent with the next table sync when already on the device.
void pod_row_dirty(kgpu_ctx* c, int32_t slot) {
  if (c->pod_rows_dev >= 0 && slot < c->pod_rows_dev) c->pod_rows_dirty.push_back(slot);
}

// The device pod table (node, ns, flags, dense labels; column-major with row capacity Pcap and key
// capacity PKcap) that k_class_init walks.  Incremental: the rows appended since the last sync and the
// rows changed in place go out as two strided copies (a new pod class on a cluster of 100k pods used to
// rebuild and send the whole table, ~4 MB, on the cycle that met it); a full rebuild only when a
// capacity is exceeded or the rows were renumbered (a node reorder).
int upload_pod_table(kgpu_ctx* c) {
  const int rows = (int)c->pod_rows.size();
  auto key_end = [&](int i) {
    int pk = 0;
    const auto& r = c->pod_rows[(size_t)i];
    for (size_t j = 0; j + 1 < r.pairs.size(); j += 2) pk = std::max(pk, r.pairs[j] + 1);
    return pk;
  };
  auto fill = [&](int32_t* col0, size_t stride, int i, int pkc) {  // row i into a (3 + pkc) x stride block
    const auto& r = c->pod_rows[(size_t)i];
    col0[0] = r.node;
    col0[stride] = r.ns;
    col0[2 * stride] = (int32_t)r.flags;
    for (int k = 0; k < pkc; ++k) col0[(3 + (size_t)k) * stride] = -1;
    for (size_t j = 0; j + 1 < r.pairs.size(); j += 2)
      if (r.pairs[j] >= 0 && r.pairs[j] < pkc) col0[(3 + (size_t)r.pairs[j]) * stride] = r.pairs[j + 1];
  };
  if (c->pod_rows_dev >= 0 && c->d_pods.p && rows <= c->st.Pcap) {
    int pk = 0;
    for (int i = c->pod_rows_dev; i < rows; ++i) pk = std::max(pk, key_end(i));
    for (int32_t sl : c->pod_rows_dirty) pk = std::max(pk, key_end(sl));
    if (pk <= c->st.PKcap) {
      const size_t P = (size_t)c->st.Pcap, H = 3 + (size_t)c->st.PKcap;
      int32_t* b = static_cast<int32_t*>(c->d_pods.p);
      const int nnew = rows - c->pod_rows_dev;
      std::vector<int32_t> buf(H * (size_t)std::max(nnew, 0) + H * c->pod_rows_dirty.size());
      if (nnew > 0) {
        for (int i = 0; i < nnew; ++i) fill(buf.data() + i, (size_t)nnew, c->pod_rows_dev + i, c->st.PKcap);
        HIP_OK(c, hipMemcpy2DAsync(b + c->pod_rows_dev, P * 4, buf.data(), (size_t)nnew * 4, (size_t)nnew * 4, H,
                                   hipMemcpyHostToDevice, c->stream));
      }
      int32_t* d = buf.data() + H * (size_t)std::max(nnew, 0);
      for (int32_t sl : c->pod_rows_dirty) {
        fill(d, 1, sl, c->st.PKcap);
        HIP_OK(c, hipMemcpy2DAsync(b + sl, P * 4, d, 4, 4, H, hipMemcpyHostToDevice, c->stream));
        d += H;
      }
      SYNC_OK(c);  // buf is pageable and local
      c->pod_rows_dev = rows;
      c->pod_rows_dirty.clear();
      return KGPU_OK;
    }
  }
  int pk = 0;
  for (int i = 0; i < rows; ++i) pk = std::max(pk, key_end(i));
  // capacities with room for the pods the next cycles assume and the label keys they bring
  const size_t R = (size_t)std::max(rows + rows / 2, 1024);
  const int pkc = std::max(pk + 4, 8);
  ++c->n_pod_table_full;
  std::vector<int32_t> buf(R * (3 + (size_t)pkc), -1);
  for (int i = 0; i < rows; ++i) fill(buf.data() + i, R, i, pkc);
  int rc;
  if ((rc = ensure(c, c->d_pods, sizeof(int32_t) * buf.size()))) return rc;
  HIP_OK(c, hipMemcpyAsync(c->d_pods.p, buf.data(), sizeof(int32_t) * buf.size(), hipMemcpyHostToDevice, c->stream));
  SYNC_OK(c);
  int32_t* b = static_cast<int32_t*>(c->d_pods.p);
  c->st.pod_node = b;
  c->st.pod_ns = b + R;
  c->st.pod_flags = reinterpret_cast<uint32_t*>(b + 2 * R);
  c->st.pod_lab = b + 3 * R;
  c->st.Pcap = (int32_t)R;
  c->st.PKcap = pkc;
  c->pod_rows_dev = rows;
  c->pod_rows_dirty.clear();
  return KGPU_OK;
}

template <class T>
int upload_vec(kgpu_ctx* c, DevBuf& b, const std::vector<T>& v, const T** dst) {
  if (!v.empty())
    if (const void* a = arena_put(c, v.data(), sizeof(T) * v.size())) {
      *dst = static_cast<const T*>(a);
      return KGPU_OK;
    }
  int rc = ensure_grow(c, b, sizeof(T) * std::max<size_t>(v.size(), 1));
  if (rc) return rc;
  if (!v.empty()) HIP_OK(c, hipMemcpyAsync(b.p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, c->stream));
  *dst = static_cast<const T*>(b.p);
  return KGPU_OK;
}

// Swap a registered device allocation for a new one (the old one is freed).
void swap_alloc(std::vector<void*>& reg, void* old_p, void* new_p) {
  for (void*& q : reg)
    if (q == old_p) {
      q = new_p;
      (void)hipFree(old_p);
      return;
    }
  reg.push_back(new_p);
  if (old_p) (void)hipFree(old_p);
}

// NodeInfo.UsedPorts has no cap (HostPortInfo.Add): before a batch that may add `extra` entries
// to one node, grow the [PS][N] slot table so that no entry can be lost.
int reserve_ports(kgpu_ctx* c, int64_t extra) {
  const int64_t need = c->port_bound + extra;
  DevState& st = c->st;
  if (need <= st.PS) return KGPU_OK;
  const int ps = (int)std::max<int64_t>(need, 2 * (int64_t)st.PS);
  const size_t N = (size_t)st.N;
  kgpu_port* np = nullptr;
  HIP_OK(c, hipMalloc(&np, sizeof(kgpu_port) * std::max<size_t>((size_t)ps * N, 1)));
  HIP_OK(c, hipMemsetAsync(np, 0, sizeof(kgpu_port) * (size_t)ps * N, c->stream));
  if (N) HIP_OK(c, hipMemcpyAsync(np, st.ports, sizeof(kgpu_port) * (size_t)st.PS * N, hipMemcpyDeviceToDevice, c->stream));
  SYNC_OK(c);
  swap_alloc(c->snap_allocs, st.ports, np);
  st.ports = np;
  st.PS = ps;
  return KGPU_OK;
}

// Go's math.Log (FreeBSD e_log.c, src/math/log.go) for the PodTopologySpread weight table.
double go_log(double x) {
  const double ln2hi = 6.93147180369123816490e-01, ln2lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (std::isnan(x) || std::isinf(x)) return x;
  if (x < 0) return NAN;
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = std::frexp(x, &ki);
  if (f1 < 0.70710678118654752440) {
    f1 *= 2;
    ki--;
  }
  const double f = f1 - 1, k = (double)ki;
  const double s = f / (2 + f), s2 = s * s, s4 = s2 * s2;
  const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const double R = t1 + t2, hfsq = 0.5 * f * f;
  return k * ln2hi - ((hfsq - (s * (hfsq + R) + k * ln2lo)) - f);
}

// numFeasibleNodesToFind (generic_scheduler.go:379-399): minFeasibleNodesToFind = 100,
// minFeasibleNodesPercentageToFind = 5, adaptive 50 - N/125 when the percentage is 0 (the default,
// apis/config/types.go:251).
int32_t num_feasible_nodes_to_find(int32_t n, int32_t pct) {
  if (n < 100 || pct >= 100) return n;
  int32_t adaptive = pct;
  if (adaptive <= 0) {
    adaptive = 50 - n / 125;
    if (adaptive < 5) adaptive = 5;
  }
  const int32_t k = (int32_t)((int64_t)n * adaptive / 100);
  return k < 100 ? 100 : k;
}

hipEvent_t get_event(kgpu_ctx* c, size_t i) {
  while (c->ev_pool.size() <= i) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    c->ev_pool.push_back(e);
  }
  return c->ev_pool[i];
}

// ---------------------------------------------------------------- persistent topology runs
// A run of consecutive topology pods is planned against ONE set of domain histograms
// (kgpu_internal.h "persistent topology kernel"): every (column, key, signature) the run's pods
// read becomes a THist, every nodeSelector / required-NodeAffinity program + key set a TSig.
// A pool whose ranges are interned by content: pods of one template share their records, so the
// persistent kernel reads cache-hot lines instead of fresh ones per pod.
template <class T>
struct RangePool {
  std::vector<T> v;
  std::map<std::string, kgpu_range> m;
  kgpu_range add(const std::vector<T>& items) {
    if (items.empty()) return kgpu_range{0, 0};
    std::string k(reinterpret_cast<const char*>(items.data()), items.size() * sizeof(T));
    auto f = m.find(k);
    if (f != m.end()) return f->second;
    const kgpu_range r{(int32_t)v.size(), (int32_t)items.size()};
    v.insert(v.end(), items.begin(), items.end());
    m[k] = r;
    return r;
  }
  void truncate(size_t n) {
    v.resize(n);
    for (auto it = m.begin(); it != m.end();)
      it = (size_t)(it->second.begin + it->second.count) > n ? m.erase(it) : std::next(it);
  }
};

struct TRun {
  std::vector<kgpu::THist> hists;
  std::map<std::array<int32_t, 4>, int> hist_ids;
  std::vector<kgpu::TSig> sigs;
  std::map<std::vector<int64_t>, int> sig_ids;
  std::vector<kgpu::TReg> regs;
  std::map<std::pair<int, int>, int> reg_ids;
  std::vector<kgpu::TPlan> plans;   // one per pod while planning; distinct ones after t_finish
  std::vector<int32_t> plan_of;     // plan index of each pod of the run (after t_finish)
  RangePool<int32_t> aux;
  RangePool<kgpu::TLook> looks;
  RangePool<kgpu::TTab> tabs;
  RangePool<kgpu::TDelta> deltas;
  std::vector<int32_t> pods;  // query index of each plan
  int lds_bins = 0, reg_words = 0, soft_words = 0, zones = 0, pt_max = 0;
};

void push_reqs(std::vector<int64_t>& k, const kgpu_pools* p, kgpu_range rr) {
  k.push_back(rr.count);
  for (int i = 0; i < rr.count; ++i) {
    const kgpu_req& r = p->reqs[rr.begin + i];
    std::vector<int32_t> v(p->ints + r.vals.begin, p->ints + r.vals.begin + r.vals.count);
    std::sort(v.begin(), v.end());
    k.push_back(r.key);
    k.push_back(r.op);
    k.push_back(r.imm);
    k.push_back((int64_t)v.size());
    for (int32_t x : v) k.push_back(x);
  }
}

// signature = PodMatchesNodeSelectorAndAffinityTerms program + the keys a node must carry
int t_sig(TRun& tr, const kgpu_pod_query& q, const kgpu_pools* p, int qi, const int32_t* keys, int nk) {
  std::vector<int64_t> k;
  push_reqs(k, p, q.node_selector);
  const bool req = (q.flags & KGPU_Q_REQ_NODE_AFFINITY) != 0;
  k.push_back(req ? 1 : 0);
  if (req) {
    k.push_back(q.req_terms.count);
    for (int t = 0; t < q.req_terms.count; ++t) {
      const kgpu_node_term& nt = p->node_terms[q.req_terms.begin + t];
      k.push_back(nt.never_match);
      k.push_back(nt.field_op);
      k.push_back(nt.field_node);
      push_reqs(k, p, nt.reqs);
    }
  }
  std::vector<int32_t> ks(keys, keys + std::max(nk, 0));
  std::sort(ks.begin(), ks.end());
  ks.erase(std::unique(ks.begin(), ks.end()), ks.end());
  k.push_back(nk < 0 ? -8 : -7);
  for (int32_t x : ks) k.push_back(x);
  auto f = tr.sig_ids.find(k);
  if (f != tr.sig_ids.end()) return f->second;
  kgpu::TSig sg{};
  sg.rep = qi;
  sg.n_keys = nk < 0 ? -1 : (int32_t)ks.size();  // -1: a key no node carries, nothing is eligible
  for (size_t i = 0; i < ks.size() && i < (size_t)kgpu::kMaxSpread; ++i) sg.keys[i] = ks[i];
  const int id = (int)tr.sigs.size();
  tr.sigs.push_back(sg);
  tr.sig_ids[k] = id;
  return id;
}

// histogram of (column, key, signature); off = -1 for a node-unique key (no LDS bins)
int t_hist(TRun& tr, const kgpu_ctx* c, int kind, int col, int key, int sig) {
  const std::array<int32_t, 4> k{kind, col, key, sig};
  auto f = tr.hist_ids.find(k);
  if (f != tr.hist_ids.end()) return f->second;
  kgpu::THist h{};
  h.col_kind = kind;
  h.col = col;
  h.key = key;
  h.sig = sig;
  h.D = key >= 0 ? c->key_n_values[(size_t)key] : 0;
  const bool uniq = key_uniq(c, key);
  h.off = uniq ? -1 : tr.lds_bins;
  if (!uniq) tr.lds_bins += h.D + 1;
  const int id = (int)tr.hists.size();
  tr.hists.push_back(h);
  tr.hist_ids[k] = id;
  return id;
}

int t_reg(TRun& tr, const kgpu_ctx* c, int sig, int key) {
  auto f = tr.reg_ids.find({sig, key});
  if (f != tr.reg_ids.end()) return f->second;
  kgpu::TReg r{sig, key, c->key_n_values[(size_t)key], tr.reg_words};
  tr.reg_words += (r.D + 31) / 32;
  const int id = (int)tr.regs.size();
  tr.regs.push_back(r);
  tr.reg_ids[{sig, key}] = id;
  return id;
}

size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }

constexpr size_t kTMiscBytes = 1024;

// LDS layout of a run (byte offsets into the dynamic region); returns the total
size_t t_layout(const TRun& tr, kgpu::TBatchArgs* a, int B, int lab_keys = 0, int per = 0, size_t wlab_n = 0) {
  size_t o = a16((size_t)tr.lds_bins * 4);
  const size_t o_reg = o;
  o = a16(o + (size_t)tr.reg_words * 4);
  const size_t o_tot = o;
  o = a16(o + tr.hists.size() * 4);
  const size_t o_sany = o;
  o = a16(o + tr.sigs.size() * 4);
  const int R = kgpu::kTFixed + tr.soft_words + tr.zones;
  const size_t o_stat = o;
  o = a16(o + (size_t)R * 8);
  const size_t o_smask = o;
  o = a16(o + (size_t)kgpu::kTMaxSoftWords * 4);
  const size_t o_zsum = o;
  o = a16(o + (size_t)std::max(tr.zones, 1) * 4);
  const size_t o_pt = o;
  o = a16(o + (size_t)std::max(tr.pt_max, 1) * 8);
  const size_t o_misc = o;
  o = a16(o + kTMiscBytes);
  const size_t o_lab = o;
  o = a16(o + (size_t)lab_keys * (size_t)per * 4);
  const size_t o_wlab = o;
  o = a16(o + wlab_n * 4);
  if (a) {
    a->o_wlab = (int32_t)o_wlab;
    a->wlab = wlab_n > 0 ? 1 : 0;
    a->o_lab = (int32_t)o_lab;
    a->lab_keys = lab_keys;
    a->o_reg = (int32_t)o_reg;
    a->o_tot = (int32_t)o_tot;
    a->o_sany = (int32_t)o_sany;
    a->o_stat = (int32_t)o_stat;
    a->o_smask = (int32_t)o_smask;
    a->o_zsum = (int32_t)o_zsum;
    a->o_pt = (int32_t)o_pt;
    a->o_misc = (int32_t)o_misc;
    a->R = R;
  }
  return o;
}

struct TRunMark {
  size_t hists, sigs, regs, plans, aux, looks, tabs;
  int lds_bins, reg_words, soft_words, zones, pt_max;
};

void t_rollback(TRun& tr, const TRunMark& m) {
  for (auto it = tr.hist_ids.begin(); it != tr.hist_ids.end();)
    it = it->second >= (int)m.hists ? tr.hist_ids.erase(it) : std::next(it);
  for (auto it = tr.sig_ids.begin(); it != tr.sig_ids.end();)
    it = it->second >= (int)m.sigs ? tr.sig_ids.erase(it) : std::next(it);
  for (auto it = tr.reg_ids.begin(); it != tr.reg_ids.end();)
    it = it->second >= (int)m.regs ? tr.reg_ids.erase(it) : std::next(it);
  tr.hists.resize(m.hists);
  tr.sigs.resize(m.sigs);
  tr.regs.resize(m.regs);
  tr.plans.resize(m.plans);
  tr.aux.truncate(m.aux);
  tr.looks.truncate(m.looks);
  tr.tabs.truncate(m.tabs);
  tr.lds_bins = m.lds_bins;
  tr.reg_words = m.reg_words;
  tr.soft_words = m.soft_words;
  tr.zones = m.zones;
  tr.pt_max = m.pt_max;
}

kgpu::TLook t_look(TRun& tr, const kgpu_ctx* c, int kind, int col, int key, int weight) {
  kgpu::TLook l{};
  l.key = key;
  l.weight = weight;
  l.col_kind = kind;
  l.col = col;
  l.off = -1;
  l.D = 0;
  if (key >= 0) {
    const kgpu::THist& h = tr.hists[(size_t)t_hist(tr, c, kind, col, key, -1)];
    l.off = h.off;
    l.D = h.D;
  }
  return l;
}

// Plan pod qi for the persistent topology kernel; false (run left unchanged) when the pod needs
// what the kernel does not carry: more than one ScheduleAnyway constraint, a DoNotSchedule
// constraint on a node-unique key (its criticalPaths minimum is a cluster-wide reduction per
// pod), a shared ScheduleAnyway key with more than 256 values, more than 32 zones for
// DefaultPodTopologySpread, more than 64 signatures, or tables beyond the LDS budget.
bool t_add(TRun& tr, const kgpu_ctx* c, const kgpu_pod_query& q, const kgpu::QPlan& pl, const kgpu_pools* p,
           const std::vector<int32_t>& aux, const std::vector<kgpu::TTerm>& aux_terms, int qi) {
  const TRunMark m{tr.hists.size(), tr.sigs.size(), tr.regs.size(), tr.plans.size(), tr.aux.v.size(),
                   tr.looks.v.size(), tr.tabs.v.size(), tr.lds_bins, tr.reg_words, tr.soft_words, tr.zones, tr.pt_max};
  auto fail_ = [&]() {
    t_rollback(tr, m);
    return false;
  };
  if (pl.n_soft > 1) return fail_();
  kgpu::TPlan tp;
  std::memset(&tp, 0, sizeof(tp));  // plans are interned by their bytes
  // the pod's tables: [kind 0 per DoNotSchedule key][kind 2 per score key][kind 1 per anti key],
  // each with its term list (shared-key histograms)
  struct Tab {
    kgpu::TTab t;
    std::vector<kgpu::TLook> terms;
  };
  std::vector<Tab> t0, t1, t2;
  auto tab_for = [&](std::vector<Tab>& v, int kind, int key) -> int {
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i].t.key == key) return (int)i;
    Tab t{};
    t.t.kind = kind;
    t.t.key = key;
    t.t.D = c->key_n_values[(size_t)key];
    t.t.reg = -1;
    t.t.empty_v = -1;
    v.push_back(t);
    return (int)v.size() - 1;
  };
  tp.aff_sig = t_sig(tr, q, p, qi, nullptr, 0);
  tp.n_hard = pl.n_hard;
  if (pl.n_hard) {
    int32_t keys[kgpu::kMaxSpread];
    bool missing = false;
    for (int h = 0; h < pl.n_hard; ++h) {
      keys[h] = pl.hard[h].key;
      missing |= keys[h] < 0;
    }
    tp.hard_sig = t_sig(tr, q, p, qi, keys, missing ? -1 : pl.n_hard);
    for (int h = 0; h < pl.n_hard; ++h) {
      const kgpu::TSpread& sp = pl.hard[h];
      kgpu::THard& th = tp.hard[h];
      th.key = sp.key;
      th.max_skew = sp.max_skew;
      th.self_match = sp.self_match;
      th.tab = -1;
      if (sp.key < 0) continue;  // nothing registers: the filter passes every node (pany == 0)
      if (key_uniq(c, sp.key)) return fail_();
      const int ti = tab_for(t0, 0, sp.key);
      t0[(size_t)ti].t.reg = t_reg(tr, c, tp.hard_sig, sp.key);
      t0[(size_t)ti].t.empty_v = c->key_empty[(size_t)sp.key];
      t0[(size_t)ti].terms.push_back(t_look(tr, c, 0, sp.cls, sp.key, 1));
      th.tab = ti;
    }
  }
  tp.n_soft = pl.n_soft;
  if (pl.n_soft) {
    const kgpu::TSpread& sp = pl.soft[0];
    tp.soft_key = sp.key;
    tp.soft_max_skew = sp.max_skew;
    tp.soft_col = sp.cls;
    tp.soft_off = -1;
    tp.soft_sig = -1;
    if (sp.is_hostname) {
      tp.soft_mode = 1;
    } else if (key_uniq(c, sp.key)) {
      tp.soft_mode = 2;
      int32_t k1 = sp.key;
      tp.soft_sig = t_sig(tr, q, p, qi, &k1, 1);
    } else {
      tp.soft_mode = 0;
      if (sp.key >= 0) {
        const int D = c->key_n_values[(size_t)sp.key];
        if (D > 32 * kgpu::kTMaxSoftWords) return fail_();
        int32_t k1 = sp.key;
        tp.soft_sig = t_sig(tr, q, p, qi, &k1, 1);
        tp.soft_off = tr.hists[(size_t)t_hist(tr, c, 0, sp.cls, sp.key, tp.soft_sig)].off;
        tp.soft_words = (D + 31) / 32;
        tr.soft_words = std::max(tr.soft_words, tp.soft_words);
      }
    }
  }
  tp.n_aff = pl.n_aff;
  tp.self_all = pl.self_all;
  for (int a = 0; a < pl.n_aff; ++a) {
    tp.aff[a] = t_look(tr, c, 0, pl.aff[a].cls, pl.aff[a].key, 0);
    tp.aff_hist[a] = pl.aff[a].key >= 0 ? t_hist(tr, c, 0, pl.aff[a].cls, pl.aff[a].key, -1) : -1;
  }
  tp.n_anti = pl.n_anti;
  for (int a = 0; a < pl.n_anti; ++a) tp.anti[a] = t_look(tr, c, 0, pl.anti[a].cls, pl.anti[a].key, 0);
  std::vector<kgpu::TLook> exa_u, score_u;
  auto add_term = [&](std::vector<Tab>& tabs, std::vector<kgpu::TLook>& uniq, int kind_tab, int col_kind, int col, int key,
                      int w) {
    if (key < 0) return;
    const kgpu::TLook l = t_look(tr, c, col_kind, col, key, w);
    if (l.off < 0) uniq.push_back(l);
    else tabs[(size_t)tab_for(tabs, kind_tab, key)].terms.push_back(l);
  };
  for (int e = 0; e < pl.n_ex_anti; ++e) {
    const kgpu::TTerm& t = aux_terms[(size_t)pl.ex.begin + e];
    add_term(t1, exa_u, 1, 1, t.cls, t.key, 1);
  }
  for (int e = 0; e < pl.n_pref; ++e) add_term(t2, score_u, 2, 0, pl.pref[e].cls, pl.pref[e].key, pl.pref[e].weight);
  for (int e = pl.n_ex_anti; e < pl.ex.count; ++e) {
    const kgpu::TTerm& t = aux_terms[(size_t)pl.ex.begin + e];
    add_term(t2, score_u, 2, 1, t.cls, t.key, t.weight);
  }
  tp.need_ipa = (!t2.empty() || !score_u.empty()) ? 1 : 0;
  tp.exa_u = tr.looks.add(exa_u);
  tp.score_u = tr.looks.add(score_u);
  // tables: kind 0, kind 2, kind 1 (the last n_exa_tabs)
  int pt = 0;
  std::vector<kgpu::TTab> tabs;
  for (std::vector<Tab>* v : {&t0, &t2, &t1})
    for (Tab& t : *v) {
      t.t.off = pt;
      pt += t.t.D;
      t.t.terms = tr.looks.add(t.terms);
      tabs.push_back(t.t);
    }
  tp.tabs = tr.tabs.add(tabs);
  tp.n_exa_tabs = (int32_t)t1.size();
  for (int h = 0; h < pl.n_hard; ++h)
    if (tp.hard[h].tab >= 0) tp.hard[h].pt_off = t0[(size_t)tp.hard[h].tab].t.off;
  if (tp.tabs.count > kgpu::kTMaxTabs) return fail_();
  tp.pt_words = pt;
  tr.pt_max = std::max(tr.pt_max, pt);
  tp.dpts_cls = pl.dpts_cls;
  if (pl.dpts_cls >= 0) {
    if (c->st.n_zones > kgpu::kTMaxZones) return fail_();
    tr.zones = c->st.n_zones;
  }
  tp.assume_cls = tr.aux.add(std::vector<int32_t>(aux.begin() + pl.assume_cls.begin,
                                                   aux.begin() + pl.assume_cls.begin + pl.assume_cls.count));
  tp.own_tcls = tr.aux.add(std::vector<int32_t>(aux.begin() + pl.own_tcls.begin,
                                                aux.begin() + pl.own_tcls.begin + pl.own_tcls.count));
  if (tr.sigs.size() > 64 || t_layout(tr, nullptr, 512) > (size_t)kgpu::kTLdsBudget) return fail_();
  tr.plans.push_back(tp);
  tr.pods.push_back(qi);
  return true;
}

// Histogram deltas of every planned pod (the run's histograms over the columns it increments),
// then the distinct plans: pods of one template share one plan record.  One delta per occurrence of the
// column in the pod's list: the assume increments the column once per entry (a pod whose affinity terms
// repeat one term counts it once per term, as processExistingPod does), and the run's histogram must move
// by as much (round 6: one delta per column left the in-run histogram 1 short after such a pod).
void t_finish(TRun& tr) {
  std::map<std::string, int> ids;
  std::vector<kgpu::TPlan> uniq;
  tr.plan_of.clear();
  for (kgpu::TPlan& tp : tr.plans) {
    std::vector<kgpu::TDelta> ds;
    for (int h = 0; h < (int)tr.hists.size(); ++h) {
      const kgpu::THist& hh = tr.hists[(size_t)h];
      const kgpu_range rr = hh.col_kind == 0 ? tp.assume_cls : tp.own_tcls;
      for (int i = 0; i < rr.count; ++i)
        if (tr.aux.v[(size_t)rr.begin + i] == hh.col) {
          kgpu::TDelta d;
          std::memset(&d, 0, sizeof(d));
          d.hist = h;
          d.off = hh.off;
          d.D = hh.D;
          d.key = hh.key;
          d.sig = hh.sig;
          ds.push_back(d);
        }
    }
    tp.deltas = tr.deltas.add(ds);
    const std::string k(reinterpret_cast<const char*>(&tp), sizeof(tp));
    auto f = ids.find(k);
    if (f == ids.end()) {
      f = ids.emplace(k, (int)uniq.size()).first;
      uniq.push_back(tp);
    }
    tr.plan_of.push_back(f->second);
  }
  tr.plans.swap(uniq);
}

// Upload a planned run and launch k_tbatch_init + k_tbatch on the engine's stream.
int run_tbatch(kgpu_ctx* c, TRun& tr, int first, int count, int64_t first_seq, int32_t assume, int per, int groups,
               int geo, int32_t* abort_word, bool xg, bool diag) {
  t_finish(tr);
  int rc;
  kgpu::TBatchArgs a{};
  a.diag = diag ? 1 : 0;
  a.first = first;
  a.count = count;
  a.per = per;
  a.assume = assume;
  a.seq0 = first_seq + first;
  a.n_hists = (int32_t)tr.hists.size();
  a.n_sigs = (int32_t)tr.sigs.size();
  a.n_regs = (int32_t)tr.regs.size();
  a.lds_bins = tr.lds_bins;
  a.reg_words = tr.reg_words;
  a.soft_words = tr.soft_words;
  a.zones = tr.zones;
  a.pt_words = tr.pt_max;
  a.n_keys = c->st.K;
  a.def_res = c->spec != 0 || (c->cfg.n_least == 2 && c->cfg.least[0].resource == 0 && c->cfg.least[0].weight == 1 &&
                                c->cfg.least[1].resource == 1 && c->cfg.least[1].weight == 1 && c->cfg.n_most == 2 &&
                                c->cfg.most[0].resource == 0 && c->cfg.most[0].weight == 1 &&
                                c->cfg.most[1].resource == 1 && c->cfg.most[1].weight == 1)
                  ? 1 : 0;
  // node labels of the workgroup's rows in LDS when they fit beside the histograms
  // (a one-pod run reads each label it needs once: copying the workgroup's label values into LDS first
  // would only add a round of loads to its start)
  int lab_keys = count == 1 ? 0 : std::min(c->st.K, 16);
  while (lab_keys > 0 && t_layout(tr, nullptr, 512, lab_keys, per) > (size_t)kgpu::kTLdsBudget) --lab_keys;
  // every node's label values of the delta keys, for the winner's (a batch run, when they fit too)
  size_t wlab_n = (count > 1 && !xg && c->st.K > 0 && c->tbatch_wlab) ? (size_t)c->st.K * (size_t)c->st.N : 0;
  if (wlab_n && t_layout(tr, nullptr, 512, lab_keys, per, wlab_n) > (size_t)kgpu::kTLdsBudget) wlab_n = 0;
  size_t lds = t_layout(tr, &a, 512, lab_keys, per, wlab_n);
  // at least half a CU's LDS: one persistent workgroup per CU (two would share its SIMDs)
  a.lds_bytes = (int32_t)std::max<size_t>(lds, 96 * 1024);
  const size_t N = (size_t)c->st.N;
  const size_t ew = (N + 31) / 32;
  for (size_t s = 0; s < tr.sigs.size(); ++s) tr.sigs[s].elig_word = (int32_t)(s * ew);
  // TCache: the init state of a run with these tables, left by the last run (unsharded engines; a
  // node-sharded run sums every rank's partial instead)
  const bool use_tc = !xg && c->tc_on;
  std::string tkey;
  if (use_tc) {
    auto put = [&](const void* p, size_t n) { tkey.append(static_cast<const char*>(p), n); };
    const int64_t geo[6] = {c->st.N, c->st.node_base, tr.lds_bins, tr.reg_words, (int64_t)tr.hists.size(),
                            (int64_t)tr.regs.size()};
    put(geo, sizeof(geo));
    put(tr.hists.data(), sizeof(kgpu::THist) * tr.hists.size());
    put(tr.regs.data(), sizeof(kgpu::TReg) * tr.regs.size());
    // signatures by content (their programs; `rep` is only where the kernel reads the program)
    std::vector<const std::vector<int64_t>*> progs(tr.sigs.size(), nullptr);
    for (const auto& kv : tr.sig_ids) progs[(size_t)kv.second] = &kv.first;
    for (const auto* pv : progs) {
      const int64_t len = pv ? (int64_t)pv->size() : -1;
      put(&len, sizeof(len));
      if (pv) put(pv->data(), sizeof(int64_t) * pv->size());
    }
  }
  const bool tc_hit = use_tc && c->tc.valid && c->tc.key == tkey;
  c->tc.valid = false;  // until this run is launched
  // Every table of the run in one pinned block and ONE copy: a copy from pageable memory costs
  // microseconds each, and nine of them dominated a one-pod (kgpu_schedule_one) run.  The pinned
  // block is bump-allocated per run; it wraps only after a stream synchronize, so no staged bytes are
  // overwritten before their copy ran.
  size_t toff = 0;
  auto place = [&](size_t bytes) {
    const size_t o = toff;
    toff += a16(std::max<size_t>(bytes, 16));
    return o;
  };
  const size_t o_pl = place(sizeof(kgpu::TPlan) * tr.plans.size()), o_ax = place(sizeof(int32_t) * tr.aux.v.size()),
               o_po = place(sizeof(int32_t) * tr.plan_of.size()), o_lk = place(sizeof(kgpu::TLook) * tr.looks.v.size()),
               o_h = place(sizeof(kgpu::THist) * tr.hists.size()), o_tb = place(sizeof(kgpu::TTab) * tr.tabs.v.size()),
               o_dl = place(sizeof(kgpu::TDelta) * tr.deltas.v.size()), o_sg = place(sizeof(kgpu::TSig) * tr.sigs.size()),
               o_rg = place(sizeof(kgpu::TReg) * tr.regs.size());
  const size_t tbytes = toff;
  // a short cycle's tables ride in its arena copy
  char* th = nullptr;
  char* tdev = nullptr;
  const bool t_arena = arena_reserve(c, tbytes, &th, &tdev);
  if (!t_arena && (rc = c->table_stage.reserve(stage_ops(c), tbytes, 1 << 20, &th))) return rc;
  auto stage = [&](size_t o, const auto& v) {
    if (!v.empty()) std::memcpy(th + o, v.data(), sizeof(v[0]) * v.size());
  };
  stage(o_pl, tr.plans);
  stage(o_ax, tr.aux.v);
  stage(o_po, tr.plan_of);
  stage(o_lk, tr.looks.v);
  stage(o_h, tr.hists);
  stage(o_tb, tr.tabs.v);
  stage(o_dl, tr.deltas.v);
  stage(o_sg, tr.sigs);
  stage(o_rg, tr.regs);
  if (!t_arena) {
    if ((rc = ensure(c, c->t_tables, tbytes))) return rc;
    HIP_OK(c, hipMemcpyAsync(c->t_tables.p, th, tbytes, hipMemcpyHostToDevice, c->stream));
    c->table_stage.enqueued();
    tdev = static_cast<char*>(c->t_tables.p);
  }
  const char* td = tdev;
  const kgpu::TPlan* dpl = reinterpret_cast<const kgpu::TPlan*>(td + o_pl);
  const int32_t* dax = reinterpret_cast<const int32_t*>(td + o_ax);
  const int32_t* dpo = reinterpret_cast<const int32_t*>(td + o_po);
  const kgpu::TLook* dlk = reinterpret_cast<const kgpu::TLook*>(td + o_lk);
  const kgpu::THist* dh = reinterpret_cast<const kgpu::THist*>(td + o_h);
  const kgpu::TTab* dtb = reinterpret_cast<const kgpu::TTab*>(td + o_tb);
  const kgpu::TDelta* ddl = reinterpret_cast<const kgpu::TDelta*>(td + o_dl);
  const kgpu::TSig* dsg = reinterpret_cast<const kgpu::TSig*>(td + o_sg);
  const kgpu::TReg* drg = reinterpret_cast<const kgpu::TReg*>(td + o_rg);
  a.plans = dpl;
  a.plan_of = dpo;
  a.aux = dax;
  a.looks = dlk;
  a.tabs = dtb;
  a.deltas = ddl;
  a.hists = dh;
  a.sigs = dsg;
  a.regs = drg;
  // zeroed region: hist_init | tot_init | reg_init | sig_any | elig | granules
  const size_t b_hist = a16((size_t)std::max(tr.lds_bins, 1) * 4), b_tot = a16(std::max<size_t>(tr.hists.size(), 1) * 4);
  const size_t b_reg = a16((size_t)std::max(tr.reg_words, 1) * 4), b_sany = a16(std::max<size_t>(tr.sigs.size(), 1) * 4);
  const size_t b_elig = a16(std::max<size_t>(tr.sigs.size() * ew, 1) * 4);
  const size_t b_gran = (size_t)count * (size_t)(a.R + 1) * (size_t)groups * 8;
  const size_t b_init = b_hist + b_tot + b_reg + b_sany + b_elig;
  char* zinit = nullptr;  // the init region in TCache's buffer (use_tc), else in the zeroed region
  int tc_use = 0;  // the TCache buffer this run uses; the other is zeroed by the kernel
  if (use_tc) {
    tc_use = tc_hit ? c->tc.cur : 1 - c->tc.cur;
    DevBuf& tb = c->tc.buf[tc_use];
    if (tb.bytes < b_init) {
      if ((rc = ensure(c, tb, b_init))) return rc;
      c->tc.dirty[tc_use] = tb.bytes;  // fresh memory: zeroed below
    }
    zinit = static_cast<char*>(tb.p);
    if (!tc_hit && c->tc.dirty[tc_use]) HIP_OK(c, hipMemsetAsync(zinit, 0, c->tc.dirty[tc_use], c->stream));
    c->tc.dirty[tc_use] = std::max(tc_hit ? c->tc.dirty[tc_use] : 0, b_init);
    ++(tc_hit ? c->tc_hits : c->tc_misses);
  }
  const size_t total = (use_tc ? 0 : b_init) + b_gran;
  // abort_word null: a one-pod run of a short cycle -- its own abort word and workgroup counter after
  // the zeroed region, and the abort word copied to res_pin by the kernel (run_batch reads it there)
  const bool own_abort = abort_word == nullptr;
  char* z = own_abort ? static_cast<char*>(arena_put(c, nullptr, total + 16)) : nullptr;
  c->tb_abort_mapped = z != nullptr;
  if (!z) {
    if ((rc = ensure(c, c->t_zero, total))) return rc;
    HIP_OK(c, hipMemsetAsync(c->t_zero.p, 0, total, c->stream));
    z = static_cast<char*>(c->t_zero.p);
    if (own_abort) {
      HIP_OK(c, hipMemsetAsync(c->abort_buf.p, 0, 64, c->stream));
      abort_word = static_cast<int32_t*>(c->abort_buf.p);
    }
  }
  char* zi = use_tc ? zinit : z;
  a.hist_init = reinterpret_cast<int32_t*>(zi);
  a.tot_init = reinterpret_cast<int32_t*>(zi + b_hist);
  a.reg_init = reinterpret_cast<uint32_t*>(zi + b_hist + b_tot);
  a.sig_any = reinterpret_cast<int32_t*>(zi + b_hist + b_tot + b_reg);
  a.elig = reinterpret_cast<uint32_t*>(zi + b_hist + b_tot + b_reg + b_sany);
  a.gran = reinterpret_cast<uint64_t*>(use_tc ? z : z + b_init);
  a.writeback = use_tc ? 1 : 0;
  a.zero_n16 = 0;
  a.zero_buf = nullptr;
  if (use_tc && c->tc.dirty[1 - tc_use]) {
    a.zero_n16 = (int32_t)((c->tc.dirty[1 - tc_use] + 15) / 16);
    a.zero_buf = static_cast<kgpu::TBatchArgs::Z16*>(c->tc.buf[1 - tc_use].p);
  }
  a.ahead = c->topo_ahead ? 1 : 0;
  if (c->tb_abort_mapped) {
    abort_word = reinterpret_cast<int32_t*>(z + total);
    a.done = abort_word + 1;
    int32_t* out = reinterpret_cast<int32_t*>(static_cast<char*>(c->res_pin) + kCycAbortOff);
    __atomic_store_n(out, -1, __ATOMIC_RELEASE);  // overwritten by the kernel's last workgroup
    a.abort_out = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(c->res_dev) + kCycAbortOff);
  }
  a.abort = abort_word;
  a.abort_at = c->abort_at >= first && c->abort_at < first + count ? c->abort_at - first : -1;
  a.trace = nullptr;
  a.trace_wg = nullptr;
  if (c->phase_trace) {
    const size_t tw = 16 * (size_t)(count + 1), ww = (size_t)count * (size_t)groups * 8;
    if ((rc = ensure(c, c->trace, sizeof(int64_t) * (tw + ww)))) return rc;
    HIP_OK(c, hipMemsetAsync(c->trace.p, 0, sizeof(int64_t) * (tw + ww), c->stream));
    a.trace = static_cast<int64_t*>(c->trace.p);
    a.trace_wg = a.trace + tw;
    a.trace_mode = c->phase_trace_mode;
    c->trace_host.assign(tw, 0);
    c->trace_wg_host.assign(ww, 0);
    c->trace_wg_groups = groups;
  }
  if (c->ar.on) ht(c, 5);  // 5: tables staged, resident-state key, layout
  if ((rc = arena_flush(c))) return rc;  // the short cycle's one copy: DevState, queries, pools, tables, zeros
  if (c->ar.on) ht(c, 6);  // 6: the copy (API call)
  const DevState* dst = static_cast<const DevState*>(c->dstate.p);
  if (!tc_hit && kgpu::launch_tbatch_init(dst, a, groups, c->stream))
    return fail(c, KGPU_E_DEVICE, "k_tbatch_init launch failed");
  if (xg) {
    // node-sharded run: cluster-wide histograms from every rank's partial, then the
    // XG kernel exchanges one record per rank per pod through the topology ring
    void* const* arr = static_cast<void* const*>(c->xg_arr.p);
    a.ptx = reinterpret_cast<uint64_t* const*>(arr + 2 * (size_t)c->xg_nranks);
    a.nranks = c->xg_nranks;
    a.rank = c->xg_rank;
    a.xseq0 = c->xt_seq;
    c->xt_seq += count;
    kgpu::XReduce x{};
    x.pinit = reinterpret_cast<int32_t* const*>(arr + 3 * (size_t)c->xg_nranks);
    x.nranks = c->xg_nranks;
    x.rank = c->xg_rank;
    x.seq = ++c->xr_seq;
    x.parity = (int32_t)(x.seq & 1);
    x.buf = a.hist_init;
    x.n_sum = (int32_t)((b_hist + b_tot) / 4);     // hist_init | tot_init: summed
    x.n_or = (int32_t)((b_reg + b_sany) / 4);      // reg_init | sig_any: OR-ed
    x.abort = abort_word;
    if (kgpu::launch_xreduce(x, c->stream)) return fail(c, KGPU_E_DEVICE, "cross-rank histogram reduction launch failed");
  }
  // Ordinary dispatch unless KGPU_OPT_COOPERATIVE (or the retry of a clean abort) asks otherwise: the
  // cooperative launch's residency check costs tens of microseconds of host wall time (a one-pod run's
  // synchronize returned 57 us after the launch against a 24 us run), and the grid -- at most one
  // workgroup per CU (the LDS reservation), at most 256 -- is resident on an idle device either way;
  // were it not, the spin timeouts raise the abort word instead of hanging.
  const bool coop = (c->coop && !(count == 1 && !xg)) || c->force_coop;
  a.hold = coop ? -1 : c->hold_group;
  a.poll_sleep = c->tbatch_sleep ? 1 : 0;
  ++c->n_persist;
  c->n_coop += coop ? 1 : 0;
  ++c->state_launches;
  if (kgpu::launch_tbatch(dst, a, groups, geo, c->spec, xg, coop, c->stream))
    return fail(c, KGPU_E_DEVICE, std::string("k_tbatch launch failed: ") + hipGetErrorString(hipGetLastError()));
  if (c->ar.on) ht(c, 7);  // 7: the launch (API call)
  if (use_tc) {
    c->tc.valid = true;  // what this run leaves behind (an aborted run invalidates the mirror)
    c->tc.key.swap(tkey);
    c->tc.cur = tc_use;
    c->tc.dirty[1 - tc_use] = 0;  // zeroed by this run
  }
  if (a.trace) {
    HIP_OK(c, hipMemcpyAsync(c->trace_host.data(), a.trace, sizeof(int64_t) * 16 * (size_t)(count + 1),
                             hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipMemcpyAsync(c->trace_wg_host.data(), a.trace_wg, sizeof(int64_t) * c->trace_wg_host.size(),
                             hipMemcpyDeviceToHost, c->stream));
  }
  return KGPU_OK;
}

int copy_to_aliases(kgpu_ctx* c, int32_t* cols, int ncols);
int assume_via_delta(kgpu_ctx* c, const kgpu_pod_query& q, const kgpu_pools* pools, int32_t gnode);


// ---------------------------------------------------------------- nominated pods / preemption (host)
// labels.Selector.Matches + namespace membership of a pod term held in a query's pools
// (util/topologies.go:40-49 PodMatchesTermsNamespaceAndSelector).
bool pool_term_matches(const kgpu_pools* p, const kgpu_pod_term& t, int32_t ns, const int32_t* pairs, int np) {
  bool in_ns = false;
  for (int i = 0; i < t.ns.count; ++i) in_ns |= p->ints[t.ns.begin + i] == ns;
  if (!in_ns || t.sel.kind != KGPU_SEL_AND) return false;
  for (int i = 0; i < t.sel.reqs.count; ++i) {
    const kgpu_req& r = p->reqs[t.sel.reqs.begin + i];
    int v = -1;
    for (int j = 0; j < np; ++j)
      if (pairs[2 * j] == r.key) v = pairs[2 * j + 1];
    if (r.key < 0) v = -1;
    bool in = false;
    for (int j = 0; j < r.vals.count; ++j) in |= p->ints[r.vals.begin + j] == v;
    switch (r.op) {
      case KGPU_OP_IN: if (!(v >= 0 && in)) return false; break;
      case KGPU_OP_NOTIN: if (v >= 0 && in) return false; break;
      case KGPU_OP_EXISTS: if (v < 0) return false; break;
      case KGPU_OP_DNE: if (v >= 0) return false; break;
      default: return false;
    }
  }
  return true;
}

// A pod added to / removed from a node, resolved against the pod being scheduled `q`
// (kgpu_internal.h PEff): which of its PreFilter states the AddPod / RemovePod extensions move.
// exa_keys receives the topology keys of the pod's own required anti-affinity terms that match q.
kgpu::PEff build_effect(const kgpu_ctx* c, const kgpu::QPlan* pl, int32_t ens, const int32_t* epairs, int enp) {
  kgpu::PEff e{};
  if (!pl) return e;
  for (int i = 0; i < pl->n_hard; ++i)  // updateWithPod counts terminating pods too
    if (class_matches(c, pl->hard[i].cls, ens, KGPU_PF_ACTIVE, epairs, enp)) e.pts_mask |= 1u << i;
  for (int i = 0; i < pl->n_anti; ++i)
    if (class_matches(c, pl->anti[i].cls, ens, KGPU_PF_ACTIVE, epairs, enp)) e.anti_mask |= 1u << i;
  e.aff_all = (pl->n_aff > 0 && class_matches(c, pl->conj_cls, ens, KGPU_PF_ACTIVE, epairs, enp)) ? 1 : 0;
  return e;
}

// Nominated pods of equal or higher priority (and another UID) on this shard's nodes, as pass-1
// effects for `q`, grouped by local node in nomination order (addNominatedPods, generic_scheduler.go:526-551).
void stage_nominated(const kgpu_ctx* c, const kgpu_pod_query& q, const kgpu_pools* qp, const kgpu::QPlan* pl,
                     std::vector<int32_t>& n_off, std::vector<kgpu::PEff>& neff, std::vector<int32_t>& aux) {
  const int N = c->st.N;
  std::vector<std::vector<kgpu::PEff>> by(N);
  const int32_t* qpairs = (qp && q.labels.count) ? qp->ints + q.labels.begin : nullptr;
  const int qnp = q.labels.count / 2;
  const kgpu_ctx::Nominator& nm = c->nom;
  for (const kgpu_nominated& e : nm.list) {
    const kgpu_pod_query& r = nm.recs[(size_t)e.item];
    const int local = e.node - c->st.node_base;
    if (local < 0 || local >= N || r.priority < q.priority || r.uid == q.uid) continue;
    const int32_t* pairs = r.labels.count ? nm.pools.ints + r.labels.begin : nullptr;
    kgpu::PEff f = build_effect(c, pl, r.ns, pairs, r.labels.count / 2);
    f.item = e.item;
    f.prio = r.priority;
    f.exa.begin = (int32_t)aux.size();
    for (int j = 0; j < r.ipa_req_anti.count; ++j) {
      const kgpu_pod_term& t = nm.pools.pod_terms[r.ipa_req_anti.begin + j];
      if (t.topo_key >= 0 && pool_term_matches(&nm.pools, t, q.ns, qpairs, qnp)) aux.push_back(t.topo_key);
    }
    f.exa.count = (int32_t)aux.size() - f.exa.begin;
    by[(size_t)local].push_back(f);
  }
  n_off.assign((size_t)N + 1, 0);
  for (int n = 0; n < N; ++n) {
    n_off[(size_t)n + 1] = n_off[(size_t)n] + (int32_t)by[(size_t)n].size();
    neff.insert(neff.end(), by[(size_t)n].begin(), by[(size_t)n].end());
  }
}

// Upload the effect tables and the PreemptArgs record; returns its device address in *dev.
struct PreemptStage {
  std::vector<int32_t> v_off, n_off, aux;
  std::vector<kgpu::PEff> veff, neff;
  std::vector<kgpu_pod_query> vrecs;
};
int upload_preempt(kgpu_ctx* c, const PreemptStage& ps, const kgpu_pools* vpools, int preempt, int n_pdbs,
                   const int32_t* pdb_allowed_dev, const kgpu::PreemptArgs** dev) {
  kgpu::PreemptArgs& a = c->pa_host;
  a = kgpu::PreemptArgs{};
  a.pod = 0;
  a.preempt = preempt;
  const int N = c->st.N;
  const size_t nv = std::max<size_t>(ps.veff.size(), 1);
  int rc;
  std::vector<int32_t> zero_off((size_t)N + 1, 0);
  if ((rc = upload_vec(c, c->p_voff, ps.v_off.empty() ? zero_off : ps.v_off, &a.v_off)) ||
      (rc = upload_vec(c, c->p_noff, ps.n_off.empty() ? zero_off : ps.n_off, &a.n_off)) ||
      (rc = upload_vec(c, c->p_veff, ps.veff, &a.veff)) || (rc = upload_vec(c, c->p_neff, ps.neff, &a.neff)) ||
      (rc = upload_vec(c, c->p_aux, ps.aux, &a.aux)) || (rc = upload_vec(c, c->p_vrecs, ps.vrecs, &a.v_recs)) ||
      (rc = upload_vec(c, c->p_nrecs, c->nom.recs, &a.n_recs)) ||
      (rc = upload_vec(c, c->p_nsc, c->nom.scalars, &a.n_scalars)) ||
      (rc = upload_vec(c, c->p_nports, c->nom.ports, &a.n_ports)))
    return rc;
  if (vpools) {
    if ((rc = upload_pool(c, c->p_vsc, vpools->scalars, vpools->n_scalars, &a.v_scalars)) ||
        (rc = upload_pool(c, c->p_vports, vpools->ports, vpools->n_ports, &a.v_ports)))
      return rc;
  }
  if ((rc = ensure(c, c->p_vstate, nv)) || (rc = ensure(c, c->p_order, sizeof(int32_t) * nv)) ||
      (rc = ensure(c, c->p_out, sizeof(kgpu_node_victims) * (size_t)std::max(N, 1))) ||
      (rc = ensure(c, c->p_outv, sizeof(int32_t) * nv)) || (rc = ensure(c, c->p_prep, sizeof(int64_t) * kgpu::kPrepWords)) ||
      (rc = ensure(c, c->p_nomstat, sizeof(uint32_t) * (size_t)std::max(N, 1))) ||
      (rc = ensure(c, c->p_args, sizeof(kgpu::PreemptArgs))))
    return rc;
  a.vstate = static_cast<uint8_t*>(c->p_vstate.p);
  a.order = static_cast<int32_t*>(c->p_order.p);
  a.out = static_cast<kgpu_node_victims*>(c->p_out.p);
  a.out_victims = static_cast<int32_t*>(c->p_outv.p);
  a.prep = static_cast<int64_t*>(c->p_prep.p);
  a.nom_status = static_cast<uint32_t*>(c->p_nomstat.p);
  a.n_pdbs = n_pdbs;
  a.pdb_allowed = pdb_allowed_dev;
  HIP_OK(c, hipMemsetAsync(a.nom_status, 0, sizeof(uint32_t) * (size_t)std::max(N, 1), c->stream));
  HIP_OK(c, hipMemsetAsync(a.prep, 0xFF, sizeof(int64_t) * kgpu::kPrepWords, c->stream));
  HIP_OK(c, hipMemcpyAsync(c->p_args.p, &c->pa_host, sizeof(kgpu::PreemptArgs), hipMemcpyHostToDevice, c->stream));
  *dev = static_cast<const kgpu::PreemptArgs*>(c->p_args.p);
  return KGPU_OK;
}

// scheduler.assume drops the assumed pod from the nominator (scheduler.go:448).
void drop_nominated(kgpu_ctx* c, int64_t uid) {
  auto& l = c->nom.list;
  l.erase(std::remove_if(l.begin(), l.end(), [&](const kgpu_nominated& e) { return c->nom.recs[(size_t)e.item].uid == uid; }),
          l.end());
}

// The interned classes / term classes on the device: count columns grown, class tables re-sent when they
// changed, and the columns of classes new since the last sync counted over the pod table (k_class_init).
int sync_classes(kgpu_ctx* c) {
  int rc;
  if ((rc = grow_columns(c, &c->st.mcnt, &c->Ccap, (int)c->classes.size()))) return rc;
  if ((rc = grow_columns(c, &c->st.tcnt, &c->TCcap, (int)c->tclasses.size()))) return rc;
  ht(c, 15);
  const kgpu::ClassRec* dcl;
  const kgpu::ClassItem* dci;
  const kgpu::TermClassRec* dtc;
  const kgpu_req* dcr;
  const int32_t* dcint;
  // the class tables only grow: re-sent when they changed since the last cycle (upload_pool)
  auto up = [&](DevBuf& b, const auto& v, auto** d) { return upload_pool(c, b, v.data(), (int32_t)v.size(), d); };
  if ((rc = up(c->d_classes, c->classes, &dcl)) || (rc = up(c->d_citems, c->citems, &dci)) ||
      (rc = up(c->d_tclasses, c->tclasses, &dtc)) || (rc = up(c->d_creqs, c->creqs, &dcr)) ||
      (rc = up(c->d_cints, c->cints, &dcint)))
    return rc;
  c->st.classes = dcl;
  c->st.class_items = dci;
  c->st.tclasses = dtc;
  c->st.creqs = dcr;
  c->st.cints = dcint;
  ht(c, 16);
  if (c->classes_init < (int)c->classes.size()) {
    // fresh mcnt columns: counted on the device over the pod table (snapshot + assumed pods)
    c->tc.valid = false;
    if ((c->pod_rows_dev != (int)c->pod_rows.size() || !c->pod_rows_dirty.empty()) && (rc = upload_pod_table(c)))
      return rc;
    if ((rc = ensure(c, c->dstate, sizeof(DevState)))) return rc;
    c->st_batch = c->st;
    c->ds_ptr = nullptr;  // the short cycle's cached DevState image is stale
    HIP_OK(c, hipMemcpyAsync(c->dstate.p, &c->st_batch, sizeof(DevState), hipMemcpyHostToDevice, c->stream));
    if (kgpu::launch_class_init(static_cast<const DevState*>(c->dstate.p), c->classes_init,
                                (int)c->classes.size() - c->classes_init, (int)c->pod_rows.size(), c->stream))
      return fail(c, KGPU_E_DEVICE, "k_class_init launch failed");
    ++c->n_class_init;
    if (c->has_alias && (rc = copy_to_aliases(c, c->st.mcnt + (size_t)c->classes_init * c->st.N,
                                              (int)c->classes.size() - c->classes_init)))
      return rc;
    SYNC_OK(c);
    c->classes_init = (int)c->classes.size();
  }
  ht(c, 17);
  return KGPU_OK;
}

// Topology plugins of a batch: plans, class columns, pools (kgpu_internal.h "topology plugins").
struct Staged {
  std::vector<kgpu::QPlan> plans;
  std::vector<int32_t> aux;
  std::vector<kgpu::TTerm> aux_terms;
  int64_t max_scratch = 0;
  bool topo_on = false;
};
int stage_topology(kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools, Staged& sg) {
  std::vector<kgpu::QPlan>& plans = sg.plans;
  std::vector<int32_t>& aux = sg.aux;
  std::vector<kgpu::TTerm>& aux_terms = sg.aux_terms;
  int64_t& max_scratch = sg.max_scratch;
  int rc;
  sg.topo_on = topo_profile(c);
  if (sg.topo_on) {
    kgpu_pools empty{};
    if ((rc = build_plans(c, qs, n, pools ? pools : &empty, plans, aux, aux_terms, &max_scratch))) return rc;
    ht(c, 12);  // (host trace: topology staging split into 12, 13, 14 and the rest in 1)
    if ((rc = sync_classes(c))) return rc;
    ht(c, 13);
    const kgpu::QPlan* dpl;
    const int32_t* dax;
    const kgpu::TTerm* dat;
    if ((rc = upload_vec(c, c->d_plans, plans, &dpl)) || (rc = upload_vec(c, c->d_aux, aux, &dax)) ||
        (rc = upload_vec(c, c->d_aux_terms, aux_terms, &dat)))
      return rc;
    c->st.plans = dpl;
    c->st.aux = dax;
    c->st.aux_terms = dat;
    ht(c, 14);
    if ((rc = ensure_grow(c, c->scratch, sizeof(int64_t) * (size_t)std::max<int64_t>(max_scratch, 1)))) return rc;
    c->st.scratch = static_cast<int64_t*>(c->scratch.p);
  } else {
    c->st.plans = nullptr;
  }
  return KGPU_OK;
}

int run_batch(kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools, int64_t first_seq,
              kgpu_result* results, kgpu_stats* stats, bool diag, int32_t assume);

// A long batch's host-to-device copy through the pinned batch block: a copy from pageable memory is
// staged by the runtime itself and costs the call far more (the queries of a 1000-pod batch are
// 0.3 MB).
int stage_h2d(kgpu_ctx* c, void* dst, const void* src, size_t bytes) {
  char* h = nullptr;
  int rc;
  if ((rc = c->batch_stage.reserve(stage_ops(c), bytes, 1 << 20, &h))) return rc;
  std::memcpy(h, src, bytes);
  HIP_OK(c, hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, c->stream));
  c->batch_stage.enqueued();
  return KGPU_OK;
}

// internal: run_batch_once's persistent run aborted before resolving any pod and was the call's only
// state-changing launch (never returned to a caller)
constexpr int kCleanAbort = 1000;

int run_batch_once(kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools, int64_t first_seq,
                   kgpu_result* results, kgpu_stats* stats, bool diag, int32_t assume) {
  if (!c->uploaded) return fail(c, KGPU_E_STATE, "no snapshot uploaded");
  if (n <= 0) return KGPU_OK;
  int rc;
  fail_point();
  if (c->has_alias && assume) {
    // A node listed twice: the device assume updates one row only, so place pods one at a time
    // and apply NodeInfo.AddPod to every row of the chosen node through k_delta.
    for (int32_t i = 0; i < n; ++i) {
      if ((rc = run_batch(c, qs + i, 1, pools, first_seq + i, results + i, stats, diag, 0))) return rc;
      if (results[i].node >= 0 && (rc = assume_via_delta(c, qs[i], pools, results[i].node))) return rc;
      if (results[i].node >= 0) drop_nominated(c, qs[i].uid);
    }
    return KGPU_OK;
  }
  if (!c->nom.list.empty()) {
    if (c->comm)
      return fail(c, KGPU_E_UNSUPPORTED, "nominated pods on a node-sharded engine (the two-pass filter runs unsharded)");
    if (n > 1) {
      // the nominator changes as pods are assumed: one cycle at a time
      for (int32_t i = 0; i < n; ++i)
        if ((rc = run_batch(c, qs + i, 1, pools, first_seq + i, results + i, stats, diag, assume))) return rc;
      return KGPU_OK;
    }
  }
  // A short cycle (kgpu_schedule_one, small batches) moves what it sends -- DevState, queries and the
  // items of its arena -- with ONE copy from pinned memory into one device block, and its kernels
  // write the result records straight into pinned host memory: every stream operation saved is
  // several microseconds of the per-cycle latency.
  const bool short_cycle = n <= kShortCycle;
  ArenaScope arena_scope{c};
  if (short_cycle) {
    if (!c->cyc_host) HIP_OK(c, hipHostMalloc(&c->cyc_host, kCycHostBytes, hipHostMallocDefault));
    if ((rc = ensure(c, c->dstate, kCycHostBytes))) return rc;
    if (!c->res_pin) {
      HIP_OK(c, hipHostMalloc(&c->res_pin, kCycResBytes + 64, hipHostMallocCoherent | hipHostMallocMapped));
      void* d = nullptr;
      HIP_OK(c, hipHostGetDevicePointer(&d, c->res_pin, 0));
      c->res_dev = static_cast<kgpu_result*>(d);
    }
    // the previous cycle's arena copy may still read cyc_host when that cycle failed before its
    // stream synchronize
    if (c->ar.inflight) SYNC_OK(c);
    const size_t first = (kDsQueryOff + sizeof(kgpu_pod_query) * (size_t)n + 255) & ~(size_t)255;
    c->ar.begin(first, c->ar_limit > 0 ? std::min(kCycHostBytes, first + c->ar_limit) : 0);
    // every record the kernels write overwrites this: the host trace's "record landed" step, and the
    // second half of a one-pod cycle's completion (its word and its record)
    for (int32_t i = 0; i < n; ++i)
      __atomic_store_n(&static_cast<kgpu_result*>(c->res_pin)[i].evaluated, INT32_MIN, __ATOMIC_RELAXED);
  }
  c->tb_abort_mapped = false;
  ht(c, 0);
  Staged sg;
  if ((rc = stage_topology(c, qs, n, pools, sg))) return rc;
  ht(c, 1);  // 1: topology staging (QPlan, classes)
  std::vector<kgpu::QPlan>& plans = sg.plans;
  std::vector<int32_t>& aux = sg.aux;
  std::vector<kgpu::TTerm>& aux_terms = sg.aux_terms;
  const bool topo_on = sg.topo_on;
  int64_t batch_ports = 0;
  if (assume)
    for (int32_t i = 0; i < n; ++i) batch_ports += qs[i].ports.count;
  if ((rc = reserve_ports(c, batch_ports))) return rc;
  // the cycles whose only kernel is k_eval (inline_q below): their pools may stay in pinned memory
  const bool zc = short_cycle && n == 1 && diag && !topo_on && c->comm == nullptr && !(c->xg_nranks > 1) &&
                  c->st.cut_state == nullptr && c->nom.list.empty() && !c->timing && !c->phase_trace;
  if ((rc = upload_pools(c, pools, zc))) return rc;
  ht(c, 2);  // 2: ports, pools
  if (!short_cycle) {
    if ((rc = ensure(c, c->queries, sizeof(kgpu_pod_query) * (size_t)n))) return rc;
    if ((rc = stage_h2d(c, c->queries.p, qs, sizeof(kgpu_pod_query) * (size_t)n))) return rc;
    if ((rc = ensure(c, c->results, sizeof(kgpu_result) * (size_t)n))) return rc;
  }
  if (!c->ticket.p) {  // resolve_tail's counters: the top one and 8 group counters, a 64-byte line each
    if ((rc = ensure(c, c->ticket, 9 * 64))) return rc;
    HIP_OK(c, hipMemset(c->ticket.p, 0, 9 * 64));
  }
  DevState st = c->st;
  st.ticket = static_cast<int32_t*>(c->ticket.p);
  // runAllFilters: a diagnostic cycle's statuses merge every failing plugin (k_eval's runtime profile,
  // k_topo_filter, k_victims' nominated pass); placements do not depend on it
  st.run_all = (diag && c->run_all) ? 1 : 0;
  st.queries = short_cycle ? reinterpret_cast<const kgpu_pod_query*>(static_cast<char*>(c->dstate.p) + kDsQueryOff)
                           : static_cast<const kgpu_pod_query*>(c->queries.p);
  // a short cycle's records go straight to pinned host memory (no read-back copy)
  st.results = short_cycle ? c->res_dev : static_cast<kgpu_result*>(c->results.p);
  // Per-plugin scores of a diagnostic cycle: every pod of a batch without topology pods goes
  // through k_eval, which then zeroes each node's rows itself; a one-pod persistent topology run's
  // k_tbatch does too; otherwise one memset does, issued before the first launch that needs it.
  const bool zero_diag = diag && !topo_on && c->comm == nullptr;
  bool diag_zeroed = !diag || zero_diag;
  if (!diag) {
    st.diag_raw = nullptr;
    st.diag_norm = nullptr;
  }
  auto zero_diag_rows = [&]() -> int {
    if (!diag_zeroed) {
      HIP_OK(c, hipMemsetAsync(c->st.diag_raw, 0, sizeof(int64_t) * 2 * KGPU_NUM_SCORES * (size_t)c->st.N, c->stream));
      diag_zeroed = true;
    }
    return KGPU_OK;
  };
  // nominated pods that apply to this pod: pass 1 runs in k_victims before the filter phase
  PreemptStage nps;
  const kgpu::PreemptArgs* nom_dev = nullptr;
  if (!c->nom.list.empty()) {
    stage_nominated(c, qs[0], pools, topo_on ? &plans[0] : nullptr, nps.n_off, nps.neff, nps.aux);
    if (!nps.neff.empty()) {
      if ((rc = upload_preempt(c, nps, nullptr, 0, 0, nullptr, &nom_dev))) return rc;
      st.nom_status = c->pa_host.nom_status;
    }
  }
  if ((rc = ensure(c, c->dstate, sizeof(DevState)))) return rc;
  c->st_batch = st;
  // A one-pod diagnostic cycle on k_eval + k_final (kgpu_schedule_one) passes its query in the
  // launch arguments; its DevState is re-sent only when it differs from the image already there.
  const bool inline_q = short_cycle && n == 1 && diag && !topo_on && c->comm == nullptr && !(c->xg_nranks > 1) &&
                        c->st.cut_state == nullptr && nom_dev == nullptr;
  if (short_cycle) {
    char* h = static_cast<char*>(c->cyc_host);
    const bool ds_same = c->ds_ptr == c->dstate.p && std::memcmp(&c->ds_last, &c->st_batch, sizeof(DevState)) == 0;
    // staged only: the arena copy (arena_flush, below or in run_tbatch) moves it
    if (!inline_q) {
      std::memcpy(h, &c->st_batch, sizeof(DevState));
      std::memcpy(h + kDsQueryOff, qs, sizeof(kgpu_pod_query) * (size_t)n);
      c->ar.mark(0, kDsQueryOff + sizeof(kgpu_pod_query) * (size_t)n);
    } else if (!ds_same) {
      std::memcpy(h, &c->st_batch, sizeof(DevState));
      c->ar.mark(0, sizeof(DevState));
    }
    c->ds_last = c->st_batch;
    c->ds_ptr = c->dstate.p;
  } else {
    c->ds_ptr = nullptr;
    if ((rc = stage_h2d(c, c->dstate.p, &c->st_batch, sizeof(DevState)))) return rc;
    ht(c, 3);  // 3: queries and DevState copies (API calls)
  }
  const DevState* dst = static_cast<const DevState*>(c->dstate.p);
  const int blocks = kgpu::eval_blocks(st.N);
  hipEvent_t t0 = get_event(c, 0), t1 = get_event(c, 1);
  const bool timed = stats != nullptr || c->timing;  // the cycle's device time is reported in stats only
  if (timed) HIP_OK(c, hipEventRecord(t0, c->stream));
  size_t ev = 2;
  int64_t timed_passes = 0;
  // Persistent geometry: one workgroup per CU at most, K node rows per lane in registers.
  int per = 0, groups = 0;
  const bool xg = c->xg_nranks > 1 && c->xgmi;  // persistent runs exchange granules over xGMI
  const bool sharded = c->comm != nullptr || xg;
  const bool cut = c->st.cut_state != nullptr;  // percentageOfNodesToScore trims the feasible set
  if (cut && sharded)
    return fail(c, KGPU_E_UNSUPPORTED, "percentageOfNodesToScore < 100 on a node-sharded engine (nextStartNodeIndex "
                                       "rotates over the whole cluster): use 100 when sharding");
  int kidx = -1;
  if (c->persistent && !diag && !cut && !nom_dev) {
    if (xg) {
      kidx = c->xg_geo;
      per = c->xg_per;
      groups = c->xg_groups;
    } else if (!sharded) {
      kidx = kgpu::batch_geometry(st.N, std::min(c->max_groups > 0 ? std::min(c->max_groups, c->n_cus) : c->n_cus, 256),
                                  &per, &groups, c->batch_geo_first);
    }
  }
  std::deque<std::array<void*, 2>> run_ptrs;  // kept until the stream is synchronized
  if (kidx >= 0 && !xg && (rc = ensure(c, c->batch_ptrs, sizeof(void*) * 2 * (size_t)(n + 1)))) return rc;
  std::vector<uint8_t> norm((size_t)n), topo((size_t)n, 0);
  // pods that need the normalize pass or whose scoring fails take the one-launch-per-pod path;
  // pods with topology state take the topology pipeline
  for (int32_t i = 0; i < n; ++i) {
    norm[(size_t)i] = (diag || needs_norm(c, qs[i], pools) || (qs[i].flags & KGPU_Q_SCORE_ERROR)) ? 1 : 0;
    if (topo_on) topo[(size_t)i] = plans[(size_t)i].topo ? 1 : 0;
  }
  // Sharded: after the evaluation (and normalize) of pod k, pack this shard's record and
  // all-gather it on the same stream; the next launch resolves pod k over every rank's record.
  auto exchange = [&](int parity, int what) -> int {
    if (!c->comm)
      return fail(c, KGPU_E_STATE, "this pod needs the per-pod RCCL exchange: call kgpu_comm_init (xGMI mailboxes "
                                   "carry persistent runs only)");
    if (kgpu::launch_shard_pack(dst, parity, blocks, what, c->stream))
      return fail(c, KGPU_E_DEVICE, "k_shard_pack launch failed");
    const ncclResult_t r =
        what == 0 ? rccl().AllGather(c->st.shard_send_key, c->st.shard_keys + (size_t)parity * kgpu::kMaxRanks,
                                  sizeof(BlkKey) / 8, ncclUint64, c->comm, c->stream)
                  : rccl().AllGather(c->st.shard_send_stat, c->st.shard_stats + (size_t)parity * kgpu::kMaxRanks,
                                  sizeof(BlkStat) / 4, ncclInt32, c->comm, c->stream);
    if (r != ncclSuccess) return fail(c, KGPU_E_DEVICE, std::string("ncclAllGather: ") + rccl().GetErrorString(r));
    return KGPU_OK;
  };
  bool used_persistent = false;
  int32_t* done_word = nullptr;  // the pinned completion word of the call's last kernel (one-pod cycles)
  // one abort word for every persistent run of this batch (OR-ed on the device)
  int rc_abort = ensure(c, c->abort_buf, 64);
  if (rc_abort) return rc_abort;
  int32_t* abort_word = static_cast<int32_t*>(c->abort_buf.p);
  int tper = 0, tgroups = 0;
  // node-sharded engines take the persistent topology kernel over the xGMI mailboxes (the XG
  // instantiation); without them, the per-pod RCCL pipeline
  // a diagnostic cycle (kgpu_schedule_one: status words and per-plugin scores) of one topology pod
  // runs as a one-pod persistent run too
  const int tgeo = (topo_on && c->tfast && (!diag || (n == 1 && !st.run_all)) && (!sharded || xg) && !cut && !nom_dev &&
                    st.K <= 64)
                       ? kgpu::tbatch_geometry(st.N, std::min(c->max_groups > 0 ? std::min(c->max_groups, c->n_cus) : c->n_cus, 256),
                                               &tper, &tgroups, c->tbatch_geo_first)
                       : -1;
  // A one-pod persistent topology run (kgpu_schedule_one of a topology pod) keeps its abort word in
  // the arena, and k_tbatch copies it into res_pin at exit: no memset, no read-back copy.
  const bool tb_arena = short_cycle && n == 1 && topo[0] && tgeo >= 0 && !xg && c->ar.on;
  // zeroed only when a persistent run can start (a one-launch-per-pod cycle never reads it)
  if (kidx >= 0 || (tgeo >= 0 && !tb_arena)) HIP_OK(c, hipMemsetAsync(c->abort_buf.p, 0, 64, c->stream));
  std::deque<TRun> runs;
  int32_t scratch_zeroed_for = -1;
  int32_t i = 0;
  while (i < n) {
    int32_t j = i;
    if (topo[(size_t)i] && tgeo >= 0) {
      runs.emplace_back();  // kept until the stream is synchronized (async copies read its vectors)
      TRun& tr = runs.back();
      kgpu_pools empty{};
      const kgpu_pools* pp = pools ? pools : &empty;
      ht(c, 3);  // 3: DevState / queries staged, geometry
      while (j < n && topo[(size_t)j] && t_add(tr, c, qs[j], plans[(size_t)j], pp, aux, aux_terms, j)) ++j;
      ht(c, 4);  // 4: the run's tables planned (t_add)
      if (j > i) {
        if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev), c->stream));
        if ((rc = run_tbatch(c, tr, i, j - i, first_seq, assume, tper, tgroups, tgeo, tb_arena ? nullptr : abort_word, xg,
                             diag)))
          return rc;
        // the one-pod run's last workgroup copies the abort word into pinned memory after everything is
        // written back: the call's completion word
        done_word = (c->tb_abort_mapped && !c->timing && !c->phase_trace)
                        ? reinterpret_cast<int32_t*>(static_cast<char*>(c->res_pin) + kCycAbortOff)
                        : nullptr;
        if (diag) diag_zeroed = true;  // k_tbatch zeroed the rows (a diagnostic run is one pod)
        if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev + 1), c->stream));
        ev += 2;
        timed_passes += j - i;
        used_persistent = true;
        i = j;
        continue;
      }
    }
    if ((rc = arena_flush(c))) return rc;  // every other launch reads DevState / queries / pools from it
    c->tc.valid = false;                     // ... and may assume outside a persistent topology run
    if (topo[(size_t)i]) {
      ++c->state_launches;  // the per-pod topology pipeline
      if ((rc = zero_diag_rows())) return rc;
      const kgpu::QPlan& pl = plans[(size_t)i];
      // the previous pod's resolve launch zeroes this pod's scratch only when it went through this
      // pipeline too (a persistent topology run in between leaves it dirty)
      if (scratch_zeroed_for != i)
        HIP_OK(c, hipMemsetAsync(c->st.scratch, 0, sizeof(int64_t) * (size_t)pl.scratch_len, c->stream));
      int64_t min_values = 0;
      for (int k = 0; k < pl.n_hard; ++k)
        if (pl.hard[k].key >= 0) min_values = std::max<int64_t>(min_values, c->key_n_values[pl.hard[k].key]);
      const int64_t next = (i + 1 < n && topo[(size_t)i + 1]) ? plans[(size_t)i + 1].scratch_len : 0;
      PodArgs a{};
      a.pod = i;
      a.prev = -1;
      a.parity = i & 1;
      a.norm = 1;
      a.assume = assume;
      a.diag = diag ? 1 : 0;
      a.cut = cut ? 1 : 0;
      a.seq = first_seq + i;
      if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev), c->stream));
      if (sharded) {
        // Node-sharded topology pod: every rank builds the histograms of
        // its shard; RCCL sums them (and ORs / mins / maxes the header) between the phases, so
        // every rank filters and scores against the cluster-wide TpPairToMatchNum, topology
        // scores, sizes and normalize extremes; the winner exchange is the non-topology one.
        if (!c->comm) return fail(c, KGPU_E_STATE, "topology pods on a sharded engine need kgpu_comm_init");
        int64_t* sc = c->st.scratch;
        auto ar = [&](void* buf, size_t cnt, ncclDataType_t t, ncclRedOp_t op) -> int {
          if (!cnt) return KGPU_OK;
          const ncclResult_t r = rccl().AllReduce(buf, buf, cnt, t, op, c->comm, c->stream);
          return r == ncclSuccess ? KGPU_OK : fail(c, KGPU_E_DEVICE, std::string("ncclAllReduce: ") + rccl().GetErrorString(r));
        };
        auto phase = [&](int ph, int64_t extra) -> int {
          return kgpu::launch_topo_phase(dst, a, ph, blocks, extra, c->stream) ? fail(c, KGPU_E_DEVICE, "topology phase launch failed")
                                                                                : KGPU_OK;
        };
        if ((rc = phase(0, 0)) || (rc = ar(sc, (size_t)pl.scratch_len, ncclInt64, ncclSum))) return rc;
        if (min_values > 0 && (rc = phase(1, min_values))) return rc;
        if ((rc = phase(2, 0))) return rc;
        bool soft_sizes = false;
        for (int k = 0; k < pl.n_soft; ++k) {
          const kgpu::TSpread& t = pl.soft[k];
          if (t.is_hostname || t.key < 0) continue;
          if ((rc = ar(sc + pl.slot_off[t.rslot], (size_t)std::max(c->key_n_values[(size_t)t.key], 1), ncclInt64, ncclSum)))
            return rc;
          soft_sizes |= t.first_of_key != 0;
        }
        int32_t* h32 = reinterpret_cast<int32_t*>(sc);
        const size_t i_feas = offsetof(kgpu::TopoHdr, feas_nonign) / 4, i_zones = offsetof(kgpu::TopoHdr, have_zones) / 4;
        if (pl.n_soft && (rc = ar(h32 + i_feas, 1, ncclInt32, ncclSum))) return rc;
        if (soft_sizes && (rc = phase(3, 0))) return rc;
        if ((rc = phase(4, 0))) return rc;
        // score extremes are max-encoded words (pts_min .. dpts_max), zone sums add, have_zones ORs
        if ((rc = ar(sc + offsetof(kgpu::TopoHdr, pts_min) / 8, 5, ncclUint64, ncclMax)) ||
            (rc = ar(h32 + i_zones, 1, ncclInt32, ncclMax)) ||
            (rc = ar(sc + kgpu::kHdrWords, (size_t)std::max(c->st.n_zones, 0), ncclInt64, ncclSum)) ||
            (rc = exchange(a.parity, 1)) || (rc = phase(5, blocks)) || (rc = exchange(a.parity, 0)) ||
            (rc = phase(6, next)))
          return rc;
        scratch_zeroed_for = next > 0 ? i + 1 : -1;
        if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev + 1), c->stream));
        ev += 2;
        ++timed_passes;
        i = i + 1;
        continue;
      }
      if (c->topo_fused && !c->gbar.p) {
        if ((rc = ensure(c, c->gbar, 64))) return rc;
        HIP_OK(c, hipMemsetAsync(c->gbar.p, 0, 64, c->stream));
        c->bar_base = 0;
      }
      if (kgpu::launch_topo(dst, a, blocks, min_values, next, c->topo_fused,
                            static_cast<unsigned long long*>(c->gbar.p), c->bar_base, c->cfg.n_filters, c->stream,
                            nom_dev, st.N))
        return fail(c, KGPU_E_DEVICE, "topology pipeline launch failed");
      if (c->topo_fused && !cut && !nom_dev) c->bar_base += (unsigned long long)kgpu::topo_barriers(min_values) * (unsigned long long)blocks;
      scratch_zeroed_for = next > 0 ? i + 1 : -1;
      if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev + 1), c->stream));
      ev += 2;
      ++timed_passes;
      i = i + 1;
      continue;
    }
    if (kidx >= 0 && !norm[(size_t)i]) {
      // a run of pods with constant normalize maxima: one persistent launch
      while (j < n && !norm[(size_t)j] && !topo[(size_t)j] && (!xg || j - i < kgpu::kXgmiRing / 2)) ++j;
      const int32_t cnt = j - i;
      kgpu::BatchArgs ba{};
      if (xg) {
        // every rank's mailbox ring (kgpu_xgmi_init); rows are addressed by the ring sequence
        const size_t cells = (size_t)kgpu::kXgmiRing * (size_t)c->xg_GT;
        ba.gran = static_cast<uint64_t*>(c->xg_box.p);
        ba.feas = reinterpret_cast<int32_t*>(ba.gran + cells);
        ba.pgran = static_cast<uint64_t* const*>(c->xg_arr.p);
        ba.pfeas = reinterpret_cast<int32_t* const*>(static_cast<uint64_t* const*>(c->xg_arr.p) + c->xg_nranks);
        ba.nranks = c->xg_nranks;
        ba.rank = c->xg_rank;
        ba.GT = c->xg_GT;
        ba.R = kgpu::kXgmiRing;
        ba.xseq0 = c->xg_seq;
        c->xg_seq += cnt;
      } else {
        // layout: granules [cnt][groups] u64 | feasible counts [cnt][groups] i32
        const size_t cells = (size_t)cnt * (size_t)groups;
        const size_t gbytes = sizeof(uint64_t) * cells + sizeof(int32_t) * cells;
        if ((rc = ensure(c, c->gran, gbytes))) return rc;
        HIP_OK(c, hipMemsetAsync(c->gran.p, 0, sizeof(uint64_t) * cells, c->stream));
        ba.gran = static_cast<uint64_t*>(c->gran.p);
        ba.feas = reinterpret_cast<int32_t*>(ba.gran + cells);
        run_ptrs.push_back({ba.gran, ba.feas});
        void** slot = static_cast<void**>(c->batch_ptrs.p) + 2 * (run_ptrs.size() - 1);
        if ((rc = stage_h2d(c, slot, run_ptrs.back().data(), sizeof(void*) * 2))) return rc;
        ba.pgran = reinterpret_cast<uint64_t* const*>(slot);
        ba.pfeas = reinterpret_cast<int32_t* const*>(slot + 1);
        ba.nranks = 1;
        ba.rank = 0;
        ba.GT = groups;
        ba.R = 0;
      }
      ba.first = i;
      ba.count = cnt;
      ba.per = per;
      ba.assume = assume;
      ba.seq0 = first_seq + i;
      ba.abort = abort_word;
      ba.abort_at = c->abort_at >= i && c->abort_at < i + cnt ? c->abort_at - i : -1;
      ba.skip_release_at = c->skip_release_at >= i && c->skip_release_at < i + cnt ? c->skip_release_at - i : -1;
      ba.trace = nullptr;
      if (c->phase_trace) {
        if ((rc = ensure(c, c->trace, sizeof(int64_t) * 16 * (size_t)(cnt + 1)))) return rc;
        HIP_OK(c, hipMemsetAsync(c->trace.p, 0, sizeof(int64_t) * 16 * (size_t)(cnt + 1), c->stream));
        ba.trace = static_cast<int64_t*>(c->trace.p);
        c->trace_host.assign((size_t)(cnt + 1) * 16, 0);
      }
      if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev), c->stream));
      const bool coop = c->coop || c->force_coop;
      ba.hold = coop ? -1 : c->hold_group;
      ++c->n_persist;
      c->n_coop += coop ? 1 : 0;
      ++c->state_launches;
      if (kgpu::launch_batch(dst, ba, groups, kidx, c->spec, coop, c->batch_helper, c->stream))
        return fail(c, KGPU_E_DEVICE, "k_batch launch failed");
      if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev + 1), c->stream));
      ev += 2;
      timed_passes += cnt;
      if (ba.trace)
        HIP_OK(c, hipMemcpyAsync(c->trace_host.data(), ba.trace, sizeof(int64_t) * 16 * (size_t)(cnt + 1),
                                 hipMemcpyDeviceToHost, c->stream));
      used_persistent = true;
    } else {
      // one launch per pod; the next launch resolves (and assumes) the previous pod's winner
      while (j < n && (kidx < 0 || norm[(size_t)j]) && !topo[(size_t)j]) ++j;
      int prev = -1;
      bool resolved_in_final = false;
      for (int32_t k = i; k < j; ++k) {
        PodArgs a{};
        a.pod = k;
        a.prev = prev;
        a.prev_blocks = blocks;
        a.prev_parity = (k - 1) & 1;
        a.parity = k & 1;
        // a one-pod diagnostic cycle of a pod without a normalize pass takes one launch: k_eval's last
        // workgroup resolves it (resolve_tail) and writes the normalized rows k_final would
        const bool one_launch = short_cycle && n == 1 && diag && !sharded && !cut &&
                                !(qs[k].flags & KGPU_Q_SCORE_ERROR) && !needs_norm(c, qs[k], pools);
        a.norm = (!one_launch && (diag || cut || needs_norm(c, qs[k], pools))) ? 1 : 0;
        a.assume = assume;
        a.diag = diag ? 1 : 0;
        a.zero_diag = zero_diag ? 1 : 0;
        a.cut = cut ? 1 : 0;
        a.seq = first_seq + k;
        // the chain's last pod with a normalize pass: k_final's last workgroup resolves it (k_eval's, for a
        // one-launch cycle)
        a.resolve_self = (k == j - 1 && (a.norm || one_launch) && !sharded) ? 1 : 0;
        resolved_in_final = a.resolve_self != 0;
        if (inline_q) {
          a.q_inline = 1;
          a.q = qs[k];
        }
        // a one-pod diagnostic cycle ends on k_final's (k_eval's) resolving workgroup: it raises a pinned
        // completion word once everything is written back, and the host returns on it
        if (a.resolve_self && short_cycle && n == 1 && !sharded && !c->timing && !c->phase_trace) {
          int32_t* dw = reinterpret_cast<int32_t*>(static_cast<char*>(c->res_pin) + kCycDoneOff);
          __atomic_store_n(dw, -1, __ATOMIC_RELEASE);
          a.done_out = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(c->res_dev) + kCycDoneOff);
          done_word = dw;
        }
        if ((rc = zero_diag_rows())) return rc;
        ++c->state_launches;
        if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev), c->stream));
        if (nom_dev && kgpu::launch_victims(dst, nom_dev, st.N, c->stream))
          return fail(c, KGPU_E_DEVICE, "k_victims launch failed");
        if (kgpu::launch_eval(dst, a, blocks, st.run_all ? 0 : c->spec, c->stream))  // run-all: the runtime profile
          return fail(c, KGPU_E_DEVICE, "k_eval launch failed");
        if (cut && kgpu::launch_cut(dst, a, blocks, c->cfg.n_filters, c->stream))
          return fail(c, KGPU_E_DEVICE, "k_cut launch failed");
        if (c->timing) HIP_OK(c, hipEventRecord(get_event(c, ev + 1), c->stream));
        ev += 2;
        ++timed_passes;
        if (sharded && a.norm && (rc = exchange(a.parity, 1))) return rc;
        if (a.norm && kgpu::launch_final(dst, a, blocks, blocks, c->stream))
          return fail(c, KGPU_E_DEVICE, "k_final launch failed");
        if (sharded && (rc = exchange(a.parity, 0))) return rc;
        prev = k;
      }
      if (!resolved_in_final) {
        PodArgs r{};
        r.pod = -1;
        r.prev = prev;
        r.prev_blocks = blocks;
        r.prev_parity = prev & 1;
        r.assume = assume;
        r.cut = cut ? 1 : 0;
        if (kgpu::launch_resolve(dst, st.N, r, c->stream)) return fail(c, KGPU_E_DEVICE, "k_resolve launch failed");
      }
    }
    i = j;
  }
  if (timed) HIP_OK(c, hipEventRecord(t1, c->stream));
  ht(c, 8);  // 8: launches issued (after run_tbatch's 5-7)
  // a long batch's records land in the pinned batch block (read back after the synchronize, before the
  // block can be reused)
  kgpu_result* res_host = static_cast<kgpu_result*>(c->res_pin);
  if (!short_cycle) {
    char* h = nullptr;
    if ((rc = c->batch_stage.reserve(stage_ops(c), sizeof(kgpu_result) * (size_t)n, 1 << 20, &h))) return rc;
    res_host = reinterpret_cast<kgpu_result*>(h);
    HIP_OK(c, hipMemcpyAsync(res_host, st.results, sizeof(kgpu_result) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    c->batch_stage.enqueued();
  }
  if (used_persistent && !c->tb_abort_mapped)
    HIP_OK(c, hipMemcpyAsync(&c->abort_host, abort_word, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  int32_t port_overflow = 0;
  if (batch_ports) HIP_OK(c, hipMemcpyAsync(&port_overflow, c->st.port_overflow, 4, hipMemcpyDeviceToHost, c->stream));
  // A one-pod cycle whose last kernel raises a completion word, with no stream operation after it,
  // returns once the word lands (bounded: 2 s, then the synchronize below): the stream's own completion
  // signal reaches the host about 8 us later (profiles/r05_host_trace.txt).  The copies that fed the
  // kernel ran before it, so the staging blocks are free; settle() synchronizes before any operation
  // that is not ordered on the stream.
  bool landed = false;
  if (done_word && short_cycle && n == 1 && !batch_ports && !timed && (!used_persistent || c->tb_abort_mapped)) {
    const int64_t t_end = now_ns() + 2000000000ll;
    const int32_t* ev = &static_cast<kgpu_result*>(c->res_pin)[0].evaluated;
    // a non-zero word is an abort code: the run wrote no record, so stop at once and let the
    // synchronize below complete the stream (an aborted cycle used to spin the full 2 s)
    for (;;) {
      const int32_t w = __atomic_load_n(done_word, __ATOMIC_ACQUIRE);
      if (w > 0) break;
      if (w == 0 && __atomic_load_n(ev, __ATOMIC_ACQUIRE) != INT32_MIN) {
        landed = true;
        break;
      }
      if (now_ns() >= t_end) break;
    }
  }
  if (landed && c->htrace) ht(c, 11);
  if (!landed && short_cycle && c->htrace) {
    // 11: until the kernels' records are visible in pinned memory (bounded: 2 s); the synchronize after it
    // is then the completion signal's own latency
    const int64_t t_end = now_ns() + 2000000000ll;
    for (int32_t i = 0; i < n; ++i)
      while (__atomic_load_n(&static_cast<kgpu_result*>(c->res_pin)[i].evaluated, __ATOMIC_ACQUIRE) == INT32_MIN &&
             now_ns() < t_end) {
      }
    ht(c, 11);
  }
  if (landed) {
    c->pool_stage.synced();
    c->table_stage.synced();
    c->delta_stage.synced();
    c->batch_stage.synced();
    c->ar.synced();
    c->unsettled = true;
  } else {
    SYNC_OK(c);
  }
  ht(c, 9);  // 9: synchronize
  std::memcpy(results, res_host, sizeof(kgpu_result) * (size_t)n);
  if (used_persistent && c->tb_abort_mapped) {
    // k_tbatch's last workgroup wrote the abort word (-1 left by the host: the run never finished)
    const int32_t w = __atomic_load_n(reinterpret_cast<int32_t*>(static_cast<char*>(c->res_pin) + kCycAbortOff),
                                      __ATOMIC_ACQUIRE);
    c->abort_host = w == -1 ? kgpu::kAbortDirty : w;
  }
  if (used_persistent && c->abort_host == kgpu::kAbortClean && c->state_launches == 1 && !c->force_coop && !xg) {
    // A workgroup never started before the run resolved its first pod, and that run was the call's
    // only state-changing launch: nothing on the device changed.  The resident topology state's spare
    // buffer may be half zeroed: both buffers are recomputed from zeros by the next run.
    c->tc.valid = false;
    for (int k = 0; k < 2; ++k) c->tc.dirty[k] = c->tc.buf[k].bytes;
    return kCleanAbort;
  }
  c->port_bound += batch_ports;
  if (port_overflow) {
    c->uploaded = false;
    return fail(c, KGPU_E_DEVICE, "a node's host-port slots ran out during assume: re-upload the snapshot");
  }
  if (used_persistent && c->abort_host) {
    // Pods resolved before the abort have already been assumed on the device, but their results
    // were never returned: the mirror no longer matches the caller's records.  Refuse further
    // cycles until the snapshot is uploaded again.
    c->uploaded = false;
    return fail(c, KGPU_E_DEVICE, "persistent kernel gave up waiting for a workgroup (lost co-residency); the device "
                                  "mirror is invalid: re-upload the snapshot");
  }
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
  if (assume && !c->nom.list.empty())
    for (int32_t i = 0; i < n; ++i)
      if (results[i].node >= 0) drop_nominated(c, qs[i].uid);
  // keep host records of assumed pods for ForgetPod (and the pod table for later classes)
  if (assume) {
    for (int32_t i = 0; i < n; ++i) {
      if (results[i].node < 0) continue;
      {
        kgpu_ctx::PodRow row;
        row.node = results[i].node;
        row.ns = qs[i].ns;
        row.flags = query_pod_flags(qs[i]);
        if (pools && qs[i].labels.count)
          row.pairs.assign(pools->ints + qs[i].labels.begin, pools->ints + qs[i].labels.begin + qs[i].labels.count);
        if (topo_on) {
          const kgpu_range ot = plans[(size_t)i].own_tcls;
          row.own_tcls.assign(aux.begin() + ot.begin, aux.begin() + ot.begin + ot.count);
        }
        c->pod_rows.push_back(std::move(row));
      }
      kgpu_ctx::PodRec a;
      a.node = results[i].node;  // global: the row lives on this shard or on another rank's
      a.q = qs[i];
      a.active = true;
      a.has_res = true;
      if (pools) {
        for (int k = 0; k < qs[i].scalars.count; ++k) a.sc.push_back(pools->scalars[qs[i].scalars.begin + k]);
        for (int k = 0; k < qs[i].ports.count; ++k) a.ports.push_back(pools->ports[qs[i].ports.begin + k]);
      }
      c->recs.push_back(std::move(a));
    }
  }
  c->last_diag = diag;
  c->last_run_all = diag && c->run_all;
  if (c->htrace) {
    ht(c, 10);  // 10: records, assumed-pod bookkeeping
    std::array<int64_t, kgpu_ctx::kHt> row{};
    std::copy(c->ht_cur, c->ht_cur + kgpu_ctx::kHt, row.begin());
    (short_cycle ? c->ht_cycles : c->ht_batches).push_back(row);
    c->ht_n += short_cycle ? 1 : 0;
  }
  return KGPU_OK;
}

// Per-node work buffers, the percentageOfNodesToScore cut and the math.Log table: everything
// sized by the node count that carries no state across cycles (upload and node-list rebuilds).
int alloc_node_work(kgpu_ctx* c) {
  DevState& st = c->st;
  const size_t N = (size_t)st.N;
  free_all(c->work_allocs);
  auto& W = c->work_allocs;
  int rc;
  if ((rc = dalloc(c, W, &st.status, N))) return rc;
  if ((rc = dalloc(c, W, &st.status_all, (size_t)KGPU_NUM_FILTERS * N))) return rc;
  if ((rc = dalloc(c, W, &st.raw_taint, N))) return rc;
  if ((rc = dalloc(c, W, &st.raw_na, N))) return rc;
  if ((rc = dalloc(c, W, &st.partial, N))) return rc;
  if ((rc = dalloc(c, W, &st.sbuf, (size_t)2 * kgpu::kMaxBlocks))) return rc;
  if ((rc = dalloc(c, W, &st.kbuf, (size_t)2 * kgpu::kMaxBlocks))) return rc;
  // raw | normalized in one block: a diagnostic cycle zeroes both with one memset
  if ((rc = dalloc(c, W, &st.diag_raw, (size_t)2 * KGPU_NUM_SCORES * N))) return rc;
  st.diag_norm = st.diag_raw + (size_t)KGPU_NUM_SCORES * N;
  // the rows of plugins outside the profile are never written: zero from here on (the kernels zero only
  // the profile's rows per diagnostic cycle)
  if (N) HIP_OK(c, hipMemset(st.diag_raw, 0, sizeof(int64_t) * 2 * KGPU_NUM_SCORES * N));
  HIP_OK(c, hipMemset(st.status, 0, sizeof(uint32_t) * std::max<size_t>(N, 1)));
  if ((rc = dalloc(c, W, &st.raw_pts, N))) return rc;
  if ((rc = dalloc(c, W, &st.raw_ipa, N))) return rc;
  if ((rc = dalloc(c, W, &st.raw_dpts, N))) return rc;
  // percentageOfNodesToScore: nextStartNodeIndex lives with the generic scheduler, not the snapshot
  // (generic_scheduler.go:451,487), so it carries over a re-upload (taken mod N on use)
  st.to_find = num_feasible_nodes_to_find(st.n_total, c->cfg.percentage_of_nodes_to_score);
  if (st.to_find < st.n_total) {
    if ((rc = ensure(c, c->cut_buf, 16))) return rc;
    if (!c->cut_init) {
      HIP_OK(c, hipMemset(c->cut_buf.p, 0, 16));
      c->cut_init = true;
    }
    st.cut_state = static_cast<int32_t*>(c->cut_buf.p);
  } else {
    st.cut_state = nullptr;
  }
  // math.Log(x) for x = 0 .. n_total + 2 (PodTopologySpread weights, scoring.go:286-288)
  std::vector<double> lt((size_t)st.n_total + 3);
  for (size_t x = 0; x < lt.size(); ++x) lt[x] = go_log((double)x);
  return dcopy(c, W, &st.log_table, lt.data(), lt.size());
}

// key_unique (hostname-like keys) and the PreferNoSchedule union from the host copies.
void rebuild_node_books(kgpu_ctx* c) {
  const DevState& st = c->st;
  const size_t N = (size_t)st.N;
  c->val_nodes.assign((size_t)st.K, {});
  c->multi_values.assign((size_t)st.K, 0);
  c->key_unique.assign((size_t)st.K, 0);
  for (int k = 0; k < st.K; ++k) {
    auto& vn = c->val_nodes[(size_t)k];
    vn.assign((size_t)std::max(c->key_n_values[(size_t)k], 1), 0);
    for (size_t i = 0; i < N; ++i) {
      const int32_t v = c->label_host[(size_t)k * N + i];
      if (v < 0) continue;
      if (v >= (int32_t)vn.size()) vn.resize((size_t)v + 1, 0);
      if (++vn[(size_t)v] == 2) c->multi_values[(size_t)k] += 1;
    }
    // a key is node-unique when no value labels two nodes (and no node's value is "", which a node
    // missing the key also stands for in PodTopologySpread's counts)
    c->key_unique[(size_t)k] = (c->key_empty[(size_t)k] < 0 && c->multi_values[(size_t)k] == 0) ? 1 : 0;
  }
  c->prefer_cnt.assign((size_t)st.TW * 64, 0);
  for (int w = 0; w < st.TW; ++w)
    for (size_t i = 0; i < N; ++i) {
      uint64_t b = c->prefer_host[(size_t)w * N + i];
      while (b) {
        c->prefer_cnt[(size_t)w * 64 + (size_t)__builtin_ctzll(b)] += 1;
        b &= b - 1;
      }
    }
  c->prefer_union.assign((size_t)st.TW, 0ull);
  for (size_t t = 0; t < c->prefer_cnt.size(); ++t)
    if (c->prefer_cnt[t]) c->prefer_union[t / 64] |= 1ull << (t % 64);
  int anyp = 0;
  for (uint64_t w : c->prefer_union) anyp |= (w != 0);
  c->st.any_prefer_taint = anyp;
}


// ---------------------------------------------------------------- delta stream
// Ops resolved on the host (slot, classes, term classes), launched as one k_delta.
struct DeltaBuild {
  std::vector<kgpu::DeltaOp> ops;
  std::vector<int32_t> aux;
};

// The pod's side of the topology columns: classes it matches (mcnt) and the term classes it owns
// (tcnt) -- the same sets an assume increments (assume_counts).
void pod_op(kgpu_ctx* c, DeltaBuild& b, int kind, int local_node, int item, int slot) {
  kgpu::DeltaOp op{};
  op.kind = kind;
  op.node = local_node;
  op.item = item;
  op.slot = -1;
  op.cls.begin = (int32_t)b.aux.size();
  const kgpu_ctx::PodRow& row = c->pod_rows[(size_t)slot];
  if (c->st.mcnt)
    for (int cl = 0; cl < c->classes_init; ++cl)
      if (class_matches(c, cl, row.ns, row.flags | KGPU_PF_ACTIVE, row.pairs.data(), (int)row.pairs.size() / 2))
        b.aux.push_back(cl);
  op.cls.count = (int32_t)b.aux.size() - op.cls.begin;
  op.tcls.begin = (int32_t)b.aux.size();
  if (c->st.tcnt) b.aux.insert(b.aux.end(), row.own_tcls.begin(), row.own_tcls.end());
  op.tcls.count = (int32_t)b.aux.size() - op.tcls.begin;
  b.ops.push_back(op);
}

template <class T>
int upload_span(kgpu_ctx* c, DevBuf& buf, const T* src, size_t n, const T** dst) {
  int rc = ensure(c, buf, sizeof(T) * std::max<size_t>(n, 1));
  if (rc) return rc;
  if (n && src) HIP_OK(c, hipMemcpyAsync(buf.p, src, sizeof(T) * n, hipMemcpyHostToDevice, c->stream));
  *dst = static_cast<const T*>(buf.p);
  return KGPU_OK;
}

int launch_ops(kgpu_ctx* c, const DeltaBuild& b, const kgpu_pod_query* pods, int n_pods, const kgpu_node_row* rows,
               int n_rows, const int32_t* ints, int n_ints, const uint64_t* words, int n_words,
               const kgpu_scalar_req* scalars, int n_scalars, const kgpu_port* ports, int n_ports) {
  if (b.ops.empty()) return KGPU_OK;
  c->tc.valid = false;  // node state changes outside a persistent topology run
  // group the ops by node (stable: batch order within a node), one workgroup per group
  std::vector<int32_t> idx(b.ops.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int32_t)i;
  std::stable_sort(idx.begin(), idx.end(), [&](int32_t x, int32_t y) { return b.ops[(size_t)x].node < b.ops[(size_t)y].node; });
  std::vector<kgpu::DeltaOp> ops(b.ops.size());
  std::vector<int32_t> goff;
  for (size_t i = 0; i < idx.size(); ++i) {
    ops[i] = b.ops[(size_t)idx[i]];
    if (i == 0 || ops[i].node != ops[i - 1].node) goff.push_back((int32_t)i);
  }
  goff.push_back((int32_t)ops.size());
  // One pinned staging block, one copy: DevState | ops | aux | pods | rows | ints | words | scalars | ports | groups
  // (a delta batch is latency-bound: one H2D, one launch, one 4-byte readback).
  struct Part {
    const void* src;
    size_t bytes;
  };
  const Part parts[] = {{&c->st, sizeof(DevState)},
                        {ops.data(), sizeof(kgpu::DeltaOp) * ops.size()},
                        {b.aux.data(), sizeof(int32_t) * b.aux.size()},
                        {pods, sizeof(kgpu_pod_query) * (size_t)n_pods},
                        {rows, sizeof(kgpu_node_row) * (size_t)n_rows},
                        {ints, sizeof(int32_t) * (size_t)n_ints},
                        {words, sizeof(uint64_t) * (size_t)n_words},
                        {scalars, sizeof(kgpu_scalar_req) * (size_t)n_scalars},
                        {ports, sizeof(kgpu_port) * (size_t)n_ports},
                        {goff.data(), sizeof(int32_t) * goff.size()}};
  constexpr int kParts = (int)(sizeof(parts) / sizeof(parts[0]));
  size_t off[kParts], total = 0;
  for (int i = 0; i < kParts; ++i) {
    off[i] = total;
    total += (parts[i].bytes + 63) & ~(size_t)63;
  }
  const size_t need = total + 64;  // + the overflow readback word
  int rc;
  char* h = nullptr;
  if ((rc = c->delta_stage.rewrite(stage_ops(c), need, 64 * 1024, &h))) return rc;
  if ((rc = ensure(c, c->d_stage, total))) return rc;
  for (int i = 0; i < kParts; ++i)
    if (parts[i].bytes && parts[i].src) std::memcpy(h + off[i], parts[i].src, parts[i].bytes);
  HIP_OK(c, hipMemcpyAsync(c->d_stage.p, h, total, hipMemcpyHostToDevice, c->stream));
  c->delta_stage.enqueued();
  char* d = static_cast<char*>(c->d_stage.p);
  kgpu::DeltaArgs a{};
  a.n_ops = (int32_t)ops.size();
  a.n_groups = (int32_t)goff.size() - 1;
  a.group_off = reinterpret_cast<const int32_t*>(d + off[9]);
  a.ops = reinterpret_cast<const kgpu::DeltaOp*>(d + off[1]);
  a.aux = reinterpret_cast<const int32_t*>(d + off[2]);
  a.pods = reinterpret_cast<const kgpu_pod_query*>(d + off[3]);
  a.rows = reinterpret_cast<const kgpu_node_row*>(d + off[4]);
  a.ints = reinterpret_cast<const int32_t*>(d + off[5]);
  a.words = reinterpret_cast<const uint64_t*>(d + off[6]);
  a.scalars = reinterpret_cast<const kgpu_scalar_req*>(d + off[7]);
  a.ports = reinterpret_cast<const kgpu_port*>(d + off[8]);
  if (kgpu::launch_delta(reinterpret_cast<const DevState*>(d), a, c->stream))
    return fail(c, KGPU_E_DEVICE, "k_delta launch failed");
  int32_t* ov = reinterpret_cast<int32_t*>(h + total);
  HIP_OK(c, hipMemcpyAsync(ov, c->st.port_overflow, 4, hipMemcpyDeviceToHost, c->stream));
  SYNC_OK(c);
  if (*ov) return fail(c, KGPU_E_DEVICE, "a node's host-port slots ran out while applying deltas");
  return KGPU_OK;
}

// SET_NODE bookkeeping on the host copies (labels -> key_unique, PreferNoSchedule union).
int set_node_books(kgpu_ctx* c, int n, const kgpu_node_row& r, const kgpu_pools& p) {
  DevState& st = c->st;
  const size_t N = (size_t)st.N;
  if (r.labels.count % 2 || (r.labels.count && (!p.ints || r.labels.begin + r.labels.count > p.n_ints)))
    return fail(c, KGPU_E_INVAL, "node row labels out of the pool");
  if (r.taints.count && (r.taints.count != 2 * st.TW || !p.words || r.taints.begin + r.taints.count > p.n_words))
    return fail(c, KGPU_E_INVAL, "node row taints must be 2 x taint_words words of the pool");
  if (r.alloc_scalar.count > st.S || (r.alloc_scalar.count && (!p.words || r.alloc_scalar.begin + r.alloc_scalar.count > p.n_words)))
    return fail(c, KGPU_E_INVAL, "node row scalars out of range");
  std::vector<int32_t> nv((size_t)st.K, -1);
  for (int j = 0; j < r.labels.count; j += 2) {
    const int32_t k = p.ints[r.labels.begin + j], v = p.ints[r.labels.begin + j + 1];
    if (k < 0 || k >= st.K) return fail(c, KGPU_E_INVAL, "node label key outside the snapshot's keys: re-upload");
    if (v < 0 || v >= c->key_n_values[(size_t)k])
      return fail(c, KGPU_E_INVAL, "node label value outside the key's dictionary (send key_n_values)");
    nv[(size_t)k] = v;
  }
  for (int k = 0; k < st.K; ++k) {
    int32_t& cur = c->label_host[(size_t)k * N + (size_t)n];
    if (cur == nv[(size_t)k]) continue;
    auto& vn = c->val_nodes[(size_t)k];
    if (cur >= 0 && --vn[(size_t)cur] == 1) c->multi_values[(size_t)k] -= 1;
    cur = nv[(size_t)k];
    if (cur >= 0) {
      if (cur >= (int32_t)vn.size()) vn.resize((size_t)cur + 1, 0);
      if (++vn[(size_t)cur] == 2) c->multi_values[(size_t)k] += 1;
    }
    c->key_unique[(size_t)k] = (c->key_empty[(size_t)k] < 0 && c->multi_values[(size_t)k] == 0) ? 1 : 0;
  }
  for (int w = 0; w < st.TW; ++w) {
    uint64_t& cur = c->prefer_host[(size_t)w * N + (size_t)n];
    const uint64_t nw = r.taints.count ? p.words[r.taints.begin + st.TW + w] : 0ull;
    for (uint64_t b = cur & ~nw; b; b &= b - 1) c->prefer_cnt[(size_t)w * 64 + (size_t)__builtin_ctzll(b)] -= 1;
    for (uint64_t b = nw & ~cur; b; b &= b - 1) c->prefer_cnt[(size_t)w * 64 + (size_t)__builtin_ctzll(b)] += 1;
    cur = nw;
  }
  c->prefer_union.assign((size_t)st.TW, 0ull);
  int anyp = 0;
  for (size_t t = 0; t < c->prefer_cnt.size(); ++t)
    if (c->prefer_cnt[t]) {
      c->prefer_union[t / 64] |= 1ull << (t % 64);
      anyp = 1;
    }
  st.any_prefer_taint = anyp;
  if (r.zone_id >= st.n_zones) st.n_zones = r.zone_id + 1;
  return KGPU_OK;
}

// Snapshot.List() rebuild after node adds / removes (cache.go:278-301): every node column is
// gathered on the device into the new order; new rows start empty (their SET_NODE follows).
int reorder_nodes(kgpu_ctx* c, const kgpu_delta_batch* b) {
  DevState& st = c->st;
  if (c->comm) return fail(c, KGPU_E_UNSUPPORTED, "node-list rebuild on a node-sharded engine: re-upload the shards");
  if (!b->image_off || !b->avoid_off)
    return fail(c, KGPU_E_INVAL, "a node-list rebuild needs the ImageLocality / NodePreferAvoidPods CSR");
  const int oldN = st.N, newN = b->n_order;
  std::vector<int32_t> from((size_t)newN), inv((size_t)std::max(oldN, 1), -1);
  std::unordered_map<int32_t, int32_t> first;  // order value -> first new position (aliases share it)
  std::vector<int32_t> canon((size_t)newN);
  for (int i = 0; i < newN; ++i) {
    const int32_t o = b->order[i];
    if (o >= oldN) return fail(c, KGPU_E_INVAL, "order names a node index past the old list");
    // an old row keeps the canonical row of its node (old aliases collapse onto one node)
    const int32_t key = o >= 0 ? c->row_canon[(size_t)o] : o;
    auto it = first.emplace(key, i).first;
    canon[(size_t)i] = it->second;
    if (o >= 0 && inv[(size_t)o] < 0) inv[(size_t)o] = i;
    from[(size_t)i] = o >= 0 ? o : -1;
  }
  // every old row of a node maps to the node's first new row
  for (int o = 0; o < oldN; ++o) {
    auto it = first.find(c->row_canon[(size_t)o]);
    inv[(size_t)o] = it == first.end() ? -1 : it->second;
  }
  struct Col {
    void** field;
    int elem, ncols;
    bool registered;
  };
  const std::vector<Col> cols = {
      {(void**)&st.alloc_cpu, 8, 1, true},      {(void**)&st.alloc_mem, 8, 1, true},
      {(void**)&st.alloc_eph, 8, 1, true},      {(void**)&st.alloc_pods, 4, 1, true},
      {(void**)&st.req_cpu, 8, 1, true},        {(void**)&st.req_mem, 8, 1, true},
      {(void**)&st.req_eph, 8, 1, true},        {(void**)&st.nz_cpu, 8, 1, true},
      {(void**)&st.nz_mem, 8, 1, true},         {(void**)&st.num_pods, 4, 1, true},
      {(void**)&st.alloc_scalar, 8, st.S, true}, {(void**)&st.req_scalar, 8, st.S, true},
      {(void**)&st.unsched, 1, 1, true},        {(void**)&st.label_val, 4, st.K, true},
      {(void**)&st.taint_nosched, 8, st.TW, true}, {(void**)&st.taint_prefer, 8, st.TW, true},
      {(void**)&st.port_count, 4, 1, true},     {(void**)&st.ports, 16, st.PS, true},
      {(void**)&st.zone_id, 4, 1, true},        {(void**)&st.mcnt, 4, c->Ccap, false},
      {(void**)&st.tcnt, 4, c->TCcap, false}};
  std::vector<kgpu::RemapCol> desc;
  std::vector<void*> fresh(cols.size(), nullptr);
  for (size_t i = 0; i < cols.size(); ++i) {
    const size_t bytes = (size_t)cols[i].elem * (size_t)std::max(cols[i].ncols, 0) * (size_t)newN;
    HIP_OK(c, hipMalloc(&fresh[i], std::max<size_t>(bytes, 16)));
    if (bytes && *cols[i].field && oldN > 0) desc.push_back({*cols[i].field, fresh[i], cols[i].elem, cols[i].ncols});
    else if (bytes) HIP_OK(c, hipMemsetAsync(fresh[i], 0, bytes, c->stream));
  }
  const int32_t* dfrom;
  const kgpu::RemapCol* ddesc;
  int rc;
  if ((rc = upload_span(c, c->d_from, from.data(), from.size(), &dfrom)) ||
      (rc = upload_span(c, c->d_remap, desc.data(), desc.size(), &ddesc)))
    return rc;
  if (kgpu::launch_remap(ddesc, (int)desc.size(), dfrom, oldN, newN, c->stream))
    return fail(c, KGPU_E_DEVICE, "k_remap launch failed");
  SYNC_OK(c);
  for (size_t i = 0; i < cols.size(); ++i) {
    if (cols[i].registered) swap_alloc(c->snap_allocs, *cols[i].field, fresh[i]);
    else if (*cols[i].field) (void)hipFree(*cols[i].field);
    *cols[i].field = fresh[i];
  }
  // CSR lists over the new order
  const size_t nimg = (size_t)b->image_off[newN], navoid = (size_t)b->avoid_off[newN];
  auto recopy = [&](auto** field, const auto* src, size_t n) -> int {
    using T = std::remove_cv_t<std::remove_pointer_t<std::remove_pointer_t<decltype(field)>>>;
    T* np = nullptr;
    HIP_OK(c, hipMalloc(&np, sizeof(T) * std::max<size_t>(n, 1)));
    if (n) HIP_OK(c, hipMemcpy(np, src, sizeof(T) * n, hipMemcpyHostToDevice));
    swap_alloc(c->snap_allocs, (void*)*field, np);
    *field = np;
    return KGPU_OK;
  };
  if ((rc = recopy(&st.image_off, b->image_off, (size_t)newN + 1)) || (rc = recopy(&st.image_id, b->image_id, nimg)) ||
      (rc = recopy(&st.image_score, b->image_score, nimg)) ||
      (rc = recopy(&st.avoid_off, b->avoid_off, (size_t)newN + 1)) || (rc = recopy(&st.avoid_id, b->avoid_id, navoid)))
    return rc;
  // host copies and pod records follow the rows
  std::vector<int32_t> lab((size_t)st.K * newN, -1);
  std::vector<uint64_t> pref((size_t)st.TW * newN, 0ull);
  for (int i = 0; i < newN; ++i) {
    const int f = from[(size_t)i];
    if (f < 0) continue;
    for (int k = 0; k < st.K; ++k) lab[(size_t)k * newN + i] = c->label_host[(size_t)k * oldN + f];
    for (int w = 0; w < st.TW; ++w) pref[(size_t)w * newN + i] = c->prefer_host[(size_t)w * oldN + f];
  }
  c->label_host.swap(lab);
  c->prefer_host.swap(pref);
  for (size_t sl = 0; sl < c->recs.size(); ++sl) {
    kgpu_ctx::PodRec& r = c->recs[sl];
    const int nn = (r.node >= 0 && r.node < oldN) ? inv[(size_t)r.node] : -1;
    if (nn < 0 && r.active) {
      // cache.RemoveNode drops the NodeInfo with its pods (cache.go:626-640)
      r.active = false;
      c->pod_rows[sl].flags &= ~KGPU_PF_ACTIVE;
      if (r.has_uid) c->uid_slot.erase(r.uid);
    }
    r.node = nn;
    c->pod_rows[sl].node = nn;
  }
  c->pod_rows_dev = -1;  // renumbered rows: the table is rebuilt
  c->pod_rows_dirty.clear();
  c->row_canon.swap(canon);
  c->alias_rows.clear();
  c->has_alias = false;
  for (int i = 0; i < newN; ++i)
    if (c->row_canon[(size_t)i] != i) {
      auto& v = c->alias_rows[c->row_canon[(size_t)i]];
      if (v.empty()) v.push_back(c->row_canon[(size_t)i]);
      v.push_back(i);
      c->has_alias = true;
    }
  st.N = newN;
  st.n_total = newN;
  if ((rc = alloc_node_work(c))) return rc;
  rebuild_node_books(c);
  return KGPU_OK;
}

// Class columns counted on canonical rows only (k_class_init walks the pod table): copy them to
// the alias rows, in place (alias rows read their canonical row, which maps to itself).
int copy_to_aliases(kgpu_ctx* c, int32_t* cols, int ncols) {
  if (ncols <= 0) return KGPU_OK;
  const kgpu::RemapCol d{cols, cols, 4, ncols};
  const int32_t* dfrom;
  const kgpu::RemapCol* ddesc;
  int rc;
  if ((rc = upload_span(c, c->d_from, c->row_canon.data(), c->row_canon.size(), &dfrom)) ||
      (rc = upload_span(c, c->d_remap, &d, 1, &ddesc)))
    return rc;
  if (kgpu::launch_remap(ddesc, 1, dfrom, c->st.N, c->st.N, c->stream)) return fail(c, KGPU_E_DEVICE, "k_remap launch failed");
  return KGPU_OK;
}

// Every row of the node that local row `r` belongs to.
std::vector<int32_t> node_rows(const kgpu_ctx* c, int32_t r) {
  const int32_t cr = c->row_canon.empty() ? r : c->row_canon[(size_t)r];
  auto it = c->alias_rows.find(cr);
  if (it == c->alias_rows.end()) return {cr};
  return it->second;
}

// Label dictionary growth (new values of existing keys).
int update_key_meta(kgpu_ctx* c, const kgpu_delta_batch* b) {
  DevState& st = c->st;
  if (!b->key_n_values) return KGPU_OK;
  if (!b->value_off || !b->value_int || !b->value_int_ok || !b->key_empty_value)
    return fail(c, KGPU_E_INVAL, "label dictionary update needs every key metadata array");
  const int K = st.K;
  for (int k = 0; k < K; ++k)
    if (b->key_n_values[k] < c->key_n_values[(size_t)k]) return fail(c, KGPU_E_INVAL, "label dictionaries only grow");
  const size_t nv = (size_t)b->value_off[K];
  auto recopy = [&](auto** field, const auto* src, size_t n) -> int {
    using T = std::remove_cv_t<std::remove_pointer_t<std::remove_pointer_t<decltype(field)>>>;
    T* np = nullptr;
    HIP_OK(c, hipMalloc(&np, sizeof(T) * std::max<size_t>(n, 1)));
    if (n) HIP_OK(c, hipMemcpy(np, src, sizeof(T) * n, hipMemcpyHostToDevice));
    swap_alloc(c->snap_allocs, (void*)*field, np);
    *field = np;
    return KGPU_OK;
  };
  int rc;
  if ((rc = recopy(&st.key_n_values, b->key_n_values, (size_t)K)) || (rc = recopy(&st.value_off, b->value_off, (size_t)K + 1)) ||
      (rc = recopy(&st.value_int, b->value_int, nv)) || (rc = recopy(&st.value_int_ok, b->value_int_ok, nv)) ||
      (rc = recopy(&st.key_empty_value, b->key_empty_value, (size_t)K)))
    return rc;
  st.key_empty = st.key_empty_value;
  c->key_n_values.assign(b->key_n_values, b->key_n_values + K);
  c->key_empty.assign(b->key_empty_value, b->key_empty_value + K);
  for (int k = 0; k < K; ++k) {
    c->val_nodes[(size_t)k].resize((size_t)std::max(c->key_n_values[(size_t)k], 1), 0);
    c->key_unique[(size_t)k] = (c->key_empty[(size_t)k] < 0 && c->multi_values[(size_t)k] == 0) ? 1 : 0;
  }
  return KGPU_OK;
}

int update_csr(kgpu_ctx* c, const kgpu_delta_batch* b) {
  DevState& st = c->st;
  const size_t N = (size_t)st.N;
  auto recopy = [&](auto** field, const auto* src, size_t n) -> int {
    using T = std::remove_cv_t<std::remove_pointer_t<std::remove_pointer_t<decltype(field)>>>;
    T* np = nullptr;
    HIP_OK(c, hipMalloc(&np, sizeof(T) * std::max<size_t>(n, 1)));
    if (n) HIP_OK(c, hipMemcpy(np, src, sizeof(T) * n, hipMemcpyHostToDevice));
    swap_alloc(c->snap_allocs, (void*)*field, np);
    *field = np;
    return KGPU_OK;
  };
  int rc;
  if (b->image_off) {
    const size_t ni = (size_t)b->image_off[N];
    if ((rc = recopy(&st.image_off, b->image_off, N + 1)) || (rc = recopy(&st.image_id, b->image_id, ni)) ||
        (rc = recopy(&st.image_score, b->image_score, ni)))
      return rc;
  }
  if (b->avoid_off) {
    const size_t na = (size_t)b->avoid_off[N];
    if ((rc = recopy(&st.avoid_off, b->avoid_off, N + 1)) || (rc = recopy(&st.avoid_id, b->avoid_id, na))) return rc;
  }
  return KGPU_OK;
}

int apply_delta(kgpu_ctx* c, const kgpu_delta_batch* b, int32_t* slots) {
  DevState& st = c->st;
  int rc;
  // Any delta batch may change what the resident topology state was computed from -- a reorder moves
  // rows without a single op, key metadata and CSR updates change no row either -- so it is dropped
  // before anything is touched (an order-only batch kept it valid).
  c->tc.valid = false;
  if (b->n_order > 0 && (rc = reorder_nodes(c, b))) return rc;
  fail_point();
  if ((rc = update_key_meta(c, b))) return rc;
  if (b->key_unique) c->key_unique_caller.assign(b->key_unique, b->key_unique + st.K);
  if (b->n_order <= 0 && (rc = update_csr(c, b))) return rc;
  if (b->n_zones > st.n_zones) st.n_zones = b->n_zones;
  const kgpu_pools& P = b->pools;
  const bool topo = topo_profile(c);
  DeltaBuild db;
  for (int i = 0; i < b->n_deltas; ++i) {
    const kgpu_delta& d = b->deltas[i];
    if (slots) slots[i] = -1;
    int local = d.node - st.node_base;
    const bool mine = d.node >= 0 && local >= 0 && local < st.N;
    if (mine) local = c->row_canon[(size_t)local];
    const int32_t gnode = mine ? local + st.node_base : d.node;  // the node's canonical (first) row
    if (d.op == KGPU_D_SET_NODE) {
      if (d.item < 0 || d.item >= b->n_rows) return fail(c, KGPU_E_INVAL, "SET_NODE row index out of range");
      if (d.node < 0 || d.node >= st.n_total) return fail(c, KGPU_E_INVAL, "SET_NODE node index out of range");
      if (!mine) continue;
      for (int32_t r : node_rows(c, local)) {
        if ((rc = set_node_books(c, r, b->rows[d.item], P))) return rc;
        db.ops.push_back(kgpu::DeltaOp{kgpu::kDSetNode, r, d.item, -1, {0, 0}, {0, 0}});
      }
      continue;
    }
    if (d.op != KGPU_D_ADD_POD && d.op != KGPU_D_REMOVE_POD) return fail(c, KGPU_E_INVAL, "unknown delta op");
    if (d.item < 0 || d.item >= b->n_pods) return fail(c, KGPU_E_INVAL, "pod delta item out of range");
    const kgpu_pod_query& q = b->pods[d.item];
    if (q.scalars.count && q.scalars.begin + q.scalars.count > P.n_scalars) return fail(c, KGPU_E_INVAL, "pod scalars out of the pool");
    if (q.ports.count && q.ports.begin + q.ports.count > P.n_ports) return fail(c, KGPU_E_INVAL, "pod ports out of the pool");
    if (q.labels.count && q.labels.begin + q.labels.count > P.n_ints) return fail(c, KGPU_E_INVAL, "pod labels out of the pool");
    for (int k = 0; k < q.scalars.count; ++k)
      if (P.scalars[q.scalars.begin + k].col >= st.S)
        return fail(c, KGPU_E_INVAL, "pod scalar resource outside the snapshot's scalar columns: re-upload");
    if (d.op == KGPU_D_ADD_POD) {
      if (d.node < 0 || d.node >= st.n_total) return fail(c, KGPU_E_INVAL, "ADD_POD on a node outside Snapshot.List()");
      if (c->uid_slot.count(d.uid)) return fail(c, KGPU_E_STATE, "ADD_POD: the pod uid is already on a node");
      const int32_t slot = (int32_t)c->recs.size();
      kgpu_ctx::PodRec rec;
      rec.uid = d.uid;
      rec.has_uid = true;
      rec.active = true;
      rec.has_res = true;
      rec.node = gnode;
      rec.q = q;
      for (int k = 0; k < q.scalars.count; ++k) rec.sc.push_back(P.scalars[q.scalars.begin + k]);
      for (int k = 0; k < q.ports.count; ++k) rec.ports.push_back(P.ports[q.ports.begin + k]);
      kgpu_ctx::PodRow row;
      row.node = gnode;
      row.ns = q.ns;
      row.flags = query_pod_flags(q);
      if (q.labels.count) row.pairs.assign(P.ints + q.labels.begin, P.ints + q.labels.begin + q.labels.count);
      if (topo) {
        const kgpu_range tr[4] = {q.ipa_req_aff, q.ipa_req_anti, q.ipa_pref_aff, q.ipa_pref_anti};
        const int tk[4] = {KGPU_TERM_REQ_AFF, KGPU_TERM_REQ_ANTI, KGPU_TERM_PREF_AFF, KGPU_TERM_PREF_ANTI};
        for (int k = 0; k < 4; ++k)
          for (int j = 0; j < tr[k].count; ++j) {
            const kgpu_pod_term& t = P.pod_terms[tr[k].begin + j];
            row.own_tcls.push_back(intern_tclass(c, tk[k], t.weight, t.topo_key, term_item(t, &P)));
          }
      }
      c->recs.push_back(std::move(rec));
      c->pod_rows.push_back(std::move(row));
      c->uid_slot.emplace(d.uid, slot);
      if (slots) slots[i] = slot;
      if (mine) {
        if (topo && (rc = grow_columns(c, &st.tcnt, &c->TCcap, (int)c->tclasses.size()))) return rc;
        if ((rc = reserve_ports(c, q.ports.count))) return rc;
        c->port_bound += q.ports.count;
        for (int32_t r : node_rows(c, local)) pod_op(c, db, kgpu::kDAddPod, r, d.item, slot);
      }
    } else {
      auto it = c->uid_slot.find(d.uid);
      if (it == c->uid_slot.end()) return fail(c, KGPU_E_STATE, "REMOVE_POD: no pod with this uid on a node");
      const int32_t slot = it->second;
      kgpu_ctx::PodRec& rec = c->recs[(size_t)slot];
      if (rec.node != gnode) return fail(c, KGPU_E_STATE, "REMOVE_POD: the pod is on another node");
      if (mine)
        for (int32_t r : node_rows(c, local)) pod_op(c, db, kgpu::kDRemovePod, r, d.item, slot);
      rec.active = false;
      c->pod_rows[(size_t)slot].flags &= ~KGPU_PF_ACTIVE;
      pod_row_dirty(c, slot);
      c->uid_slot.erase(it);
    }
  }
  return launch_ops(c, db, b->pods, b->n_pods, b->rows, b->n_rows, P.ints, P.n_ints, P.words, P.n_words, P.scalars,
                    P.n_scalars, P.ports, P.n_ports);
}
// Reserve-time assume of a pod placed by a schedule call, through k_delta on every row of the
// chosen node (the aliased-list path of run_batch).
int assume_via_delta(kgpu_ctx* c, const kgpu_pod_query& q, const kgpu_pools* pools, int32_t gnode) {
  kgpu_pools empty{};
  const kgpu_pools& P = pools ? *pools : empty;
  const int32_t slot = (int32_t)c->recs.size();
  kgpu_ctx::PodRec rec;
  rec.active = true;
  rec.has_res = true;
  rec.q = q;
  for (int k = 0; k < q.scalars.count; ++k) rec.sc.push_back(P.scalars[q.scalars.begin + k]);
  for (int k = 0; k < q.ports.count; ++k) rec.ports.push_back(P.ports[q.ports.begin + k]);
  kgpu_ctx::PodRow row;
  row.ns = q.ns;
  row.flags = query_pod_flags(q);
  if (q.labels.count) row.pairs.assign(P.ints + q.labels.begin, P.ints + q.labels.begin + q.labels.count);
  if (topo_profile(c)) {
    const kgpu_range tr[4] = {q.ipa_req_aff, q.ipa_req_anti, q.ipa_pref_aff, q.ipa_pref_anti};
    const int tk[4] = {KGPU_TERM_REQ_AFF, KGPU_TERM_REQ_ANTI, KGPU_TERM_PREF_AFF, KGPU_TERM_PREF_ANTI};
    for (int k = 0; k < 4; ++k)
      for (int j = 0; j < tr[k].count; ++j) {
        const kgpu_pod_term& t = P.pod_terms[tr[k].begin + j];
        row.own_tcls.push_back(intern_tclass(c, tk[k], t.weight, t.topo_key, term_item(t, &P)));
      }
  }
  int local = gnode - c->st.node_base;
  const bool mine = local >= 0 && local < c->st.N;
  if (mine) local = c->row_canon[(size_t)local];
  rec.node = mine ? local + c->st.node_base : gnode;
  row.node = rec.node;
  c->recs.push_back(std::move(rec));
  c->pod_rows.push_back(std::move(row));  // appended: the next table sync sends it
  if (!mine) return KGPU_OK;
  int rc;
  if (topo_profile(c) && (rc = grow_columns(c, &c->st.tcnt, &c->TCcap, (int)c->tclasses.size()))) return rc;
  if ((rc = reserve_ports(c, q.ports.count))) return rc;
  c->port_bound += q.ports.count;
  kgpu_ctx::PodRec& r = c->recs[(size_t)slot];
  kgpu_pod_query qq = q;
  qq.scalars = kgpu_range{0, (int32_t)r.sc.size()};
  qq.ports = kgpu_range{0, (int32_t)r.ports.size()};
  DeltaBuild db;
  for (int32_t rr : node_rows(c, local)) pod_op(c, db, kgpu::kDAddPod, rr, 0, slot);
  return launch_ops(c, db, &qq, 1, nullptr, 0, nullptr, 0, nullptr, 0, r.sc.data(), (int)r.sc.size(), r.ports.data(),
                    (int)r.ports.size());
}

// One scheduling call.  Its persistent kernels go out as ordinary launches; when a run's workgroups were
// not all resident before it resolved its first pod and nothing else of the call touched the device
// (kCleanAbort), the call is issued once more with cooperative launches, which wait for the whole grid
// (KGPU_OPT_COOPERATIVE, ADVICE r4: transient contention no longer forces a full re-upload).
int run_batch(kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools, int64_t first_seq,
              kgpu_result* results, kgpu_stats* stats, bool diag, int32_t assume) {
  c->state_launches = 0;
  int rc = run_batch_once(c, qs, n, pools, first_seq, results, stats, diag, assume);
  if (rc != kCleanAbort) return rc;
  ++c->n_coop_retry;
  c->force_coop = true;
  c->state_launches = 0;
  rc = run_batch_once(c, qs, n, pools, first_seq, results, stats, diag, assume);
  c->force_coop = false;
  if (rc == kCleanAbort) {  // unreachable: a forced cooperative call never reports a clean abort
    c->uploaded = false;
    return fail(c, KGPU_E_DEVICE, "persistent run aborted twice before its first pod");
  }
  return rc;
}

// ---------------------------------------------------------------- pipelined batches
// kgpu_schedule_batch_submit stages and launches a batch and returns; kgpu_schedule_batch_wait completes
// the oldest one.  Batch k+1's host work (the caller's, staging, the launch) then runs while batch k's
// kernel does, and the stream carries three operations per batch -- one copy (DevState, queries, run
// pointers, a zeroed abort word), k_batch, k_batch_fixup (records and abort word into pinned memory, the
// other slot's granules zeroed) -- where a synchronous call pays a staging gap, six operations and a
// synchronize (0.19 ms of each 1.75 ms config-(b) step outside the kernel).  Batches alternate
// between two slots; slot s is reused by batch k+2 only after batch k completed.
bool pipe_eligible(const kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools) {
  if (!c->uploaded || !c->persistent || n <= kShortCycle || c->comm || c->xg_nranks > 1 || c->has_alias ||
      !c->nom.list.empty() || c->st.cut_state || topo_profile(c) || c->phase_trace || c->abort_at >= 0 ||
      c->skip_release_at >= 0 || c->hold_group >= 0)
    return false;
  for (int32_t i = 0; i < n; ++i)
    if (qs[i].ports.count || needs_norm(c, qs[i], pools) || (qs[i].flags & KGPU_Q_SCORE_ERROR)) return false;
  return true;
}

int pipe_finish(kgpu_ctx* c, kgpu_ctx::PipeBatch& b);
int pipe_in_flight(const kgpu_ctx* c) {
  int k = 0;
  for (const auto& b : c->pipe_q) k += b.done ? 0 : 1;
  return k;
}

int pipe_submit(kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools, int64_t first_seq,
                kgpu_result* results, kgpu_stats* stats) {
  int rc;
  if (!pipe_eligible(c, qs, n, pools)) {
    // not carried: complete what is in flight (each keeps its outcome for its own wait), run it
    // synchronously, queue its outcome for its wait
    for (auto& b : c->pipe_q)
      if (!b.done) pipe_finish(c, b);
    kgpu_ctx::PipeBatch b;
    b.rc = c->uploaded ? run_batch(c, qs, n, pools, first_seq, results, stats, false, 1)
                       : fail(c, KGPU_E_STATE, "no snapshot uploaded");
    b.done = true;
    c->pipe_q.push_back(std::move(b));
    return KGPU_OK;
  }
  if (pipe_in_flight(c) >= 2) {
    for (auto& b : c->pipe_q)
      if (!b.done) {
        pipe_finish(c, b);
        break;
      }
  }
  int per = 0, groups = 0;
  const int kidx = kgpu::batch_geometry(c->st.N, std::min(c->max_groups > 0 ? std::min(c->max_groups, c->n_cus) : c->n_cus, 256),
                                        &per, &groups, c->batch_geo_first);
  if (kidx < 0) return fail(c, KGPU_E_UNSUPPORTED, "no persistent geometry for this node count");
  // the pools ride on the stream like every other copy (ordered after the batch in flight)
  if ((rc = upload_pools(c, pools))) return rc;
  if (!c->ticket.p) {  // resolve_tail's counters: the top one and 8 group counters, a 64-byte line each
    if ((rc = ensure(c, c->ticket, 9 * 64))) return rc;
    HIP_OK(c, hipMemset(c->ticket.p, 0, 9 * 64));
  }
  const int s = c->pipe_next;
  c->pipe_next ^= 1;
  kgpu_ctx::PipeSlot& ps = c->pipe[s];
  // device block: DevState | queries | [gran, feas] run pointers | abort word
  const size_t q_off = kDsQueryOff, q_bytes = sizeof(kgpu_pod_query) * (size_t)n;
  const size_t p_off = (q_off + q_bytes + 15) & ~(size_t)15, a_off = p_off + 16 * 2;
  const size_t bytes = a_off + 64;
  if ((rc = ensure(c, ps.dev, bytes))) return rc;
  if (ps.host_cap < bytes) {
    if (ps.host) HIP_OK(c, hipHostFree(ps.host));
    ps.host = nullptr;
    ps.host_cap = 0;
    HIP_OK(c, hipHostMalloc(&ps.host, bytes * 2, hipHostMallocDefault));
    ps.host_cap = bytes * 2;
  }
  const size_t cells = (size_t)n * (size_t)groups;
  const size_t gbytes = (sizeof(uint64_t) + sizeof(int32_t)) * cells;
  if (ps.gran.bytes < gbytes) {
    if ((rc = ensure(c, ps.gran, gbytes))) return rc;
    ps.gran_zeroed = 0;
  }
  if (ps.gran_zeroed < gbytes) {
    HIP_OK(c, hipMemsetAsync(ps.gran.p, 0, ps.gran.bytes, c->stream));
    ps.gran_zeroed = ps.gran.bytes;
  }
  const size_t rbytes = sizeof(kgpu_result) * (size_t)n + 64;
  if (ps.res_cap < rbytes) {
    if (ps.res) HIP_OK(c, hipHostFree(ps.res));
    ps.res = nullptr;
    ps.res_cap = 0;
    HIP_OK(c, hipHostMalloc(&ps.res, rbytes * 2, hipHostMallocCoherent | hipHostMallocMapped));
    HIP_OK(c, hipHostGetDevicePointer(&ps.res_dev, ps.res, 0));
    ps.res_cap = rbytes * 2;
  }
  for (hipEvent_t* e : {&ps.done, &ps.t0, &ps.t1})
    if (!*e) HIP_OK(c, hipEventCreateWithFlags(e, e == &ps.done ? hipEventDisableTiming : hipEventDefault));
  char* h = static_cast<char*>(ps.host);
  char* d = static_cast<char*>(ps.dev.p);
  DevState st = c->st;
  st.ticket = static_cast<int32_t*>(c->ticket.p);
  st.queries = reinterpret_cast<const kgpu_pod_query*>(d + q_off);
  if ((rc = ensure(c, c->results, sizeof(kgpu_result) * (size_t)n))) return rc;
  st.results = static_cast<kgpu_result*>(c->results.p);
  st.diag_raw = nullptr;
  st.diag_norm = nullptr;
  uint64_t* gran = static_cast<uint64_t*>(ps.gran.p);
  int32_t* feas = reinterpret_cast<int32_t*>(gran + cells);
  std::memcpy(h, &st, sizeof(DevState));
  std::memcpy(h + q_off, qs, q_bytes);
  void* ptrs[2] = {gran, feas};
  std::memcpy(h + p_off, ptrs, sizeof(ptrs));
  std::memset(h + a_off, 0, 64);
  HIP_OK(c, hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, c->stream));
  c->tc.valid = false;  // the batch assumes outside a persistent topology run
  kgpu::BatchArgs ba{};
  ba.gran = gran;
  ba.feas = feas;
  ba.pgran = reinterpret_cast<uint64_t* const*>(d + p_off);
  ba.pfeas = reinterpret_cast<int32_t* const*>(d + p_off + sizeof(void*));
  ba.nranks = 1;
  ba.rank = 0;
  ba.GT = groups;
  ba.R = 0;
  ba.first = 0;
  ba.count = n;
  ba.per = per;
  ba.assume = 1;
  ba.seq0 = first_seq;
  ba.abort = reinterpret_cast<int32_t*>(d + a_off);
  ba.abort_at = -1;
  ba.skip_release_at = -1;
  ba.trace = nullptr;
  ba.res_out = static_cast<kgpu_result*>(ps.res_dev);
  ba.abort_out = reinterpret_cast<int32_t*>(static_cast<char*>(ps.res_dev) + sizeof(kgpu_result) * (size_t)n);
  // the other slot's granules, zeroed by this batch's fixup for the batch after next
  kgpu_ctx::PipeSlot& po = c->pipe[s ^ 1];
  ba.zero_buf = static_cast<uint64_t*>(po.gran.p);
  ba.zero_n16 = po.gran.p ? (int64_t)(po.gran.bytes / 16) : 0;
  const bool coop = c->coop;
  ba.hold = -1;
  ++c->n_persist;
  c->n_coop += coop ? 1 : 0;
  *reinterpret_cast<int32_t*>(static_cast<char*>(ps.res) + sizeof(kgpu_result) * (size_t)n) = -1;
  const bool timed = stats != nullptr;
  if (timed) HIP_OK(c, hipEventRecord(ps.t0, c->stream));
  if (kgpu::launch_batch(reinterpret_cast<const DevState*>(d), ba, groups, kidx, c->spec, coop, c->batch_helper,
                         c->stream))
    return fail(c, KGPU_E_DEVICE, "k_batch launch failed");
  if (timed) HIP_OK(c, hipEventRecord(ps.t1, c->stream));
  HIP_OK(c, hipEventRecord(ps.done, c->stream));
  ps.gran_zeroed = 0;                 // this batch dirties its slot ...
  if (po.gran.p) po.gran_zeroed = po.gran.bytes;  // ... and its fixup zeroes the other
  kgpu_ctx::PipeBatch b;
  b.slot = s;
  b.n = n;
  b.results = results;
  b.stats = stats;
  b.timed = timed;
  b.qs.assign(qs, qs + n);
  if (pools) {
    if (pools->ints && pools->n_ints > 0) b.ints.assign(pools->ints, pools->ints + pools->n_ints);
    if (pools->scalars && pools->n_scalars > 0) b.scalars.assign(pools->scalars, pools->scalars + pools->n_scalars);
  }
  c->pipe_q.push_back(std::move(b));
  return KGPU_OK;
}

// Completes a batch in flight in place: its records, the assumed pods' bookkeeping, its stats; its
// outcome waits for its own kgpu_schedule_batch_wait.
int pipe_finish(kgpu_ctx* c, kgpu_ctx::PipeBatch& b) {
  b.done = true;
  b.rc = KGPU_OK;
  kgpu_ctx::PipeSlot& ps = c->pipe[b.slot];
  if (hipEventSynchronize(ps.done) != hipSuccess) {
    c->uploaded = false;
    return b.rc = fail(c, KGPU_E_DEVICE, "pipelined batch: event synchronize failed");
  }
  if (!c->uploaded) return b.rc = fail(c, KGPU_E_STATE, "the device mirror was invalidated by an earlier batch");
  const kgpu_result* res = static_cast<const kgpu_result*>(ps.res);
  const int32_t abort = __atomic_load_n(reinterpret_cast<const int32_t*>(res + b.n), __ATOMIC_ACQUIRE);
  if (abort != 0) {
    // no re-issue here: the next batch already ran on top of this one
    c->uploaded = false;
    return b.rc = fail(c, KGPU_E_DEVICE, "pipelined persistent run gave up waiting for a workgroup; the device "
                                         "mirror is invalid: re-upload the snapshot");
  }
  std::memcpy(b.results, res, sizeof(kgpu_result) * (size_t)b.n);
  if (b.stats) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ps.t0, ps.t1) != hipSuccess) ms = 0.f;
    b.stats->pods += b.n;
    b.stats->device_ms += ms;
    int64_t placed = 0;
    for (int32_t i = 0; i < b.n; ++i) placed += b.results[i].node >= 0;
    b.stats->scheduled += placed;
    if (c->timing) {
      b.stats->eval_kernel_ms += ms;
      b.stats->eval_launches += b.n;
    }
  }
  for (int32_t i = 0; i < b.n; ++i) {
    if (b.results[i].node < 0) continue;
    const kgpu_pod_query& q = b.qs[(size_t)i];
    kgpu_ctx::PodRow row;
    row.node = b.results[i].node;
    row.ns = q.ns;
    row.flags = query_pod_flags(q);
    if (q.labels.count && q.labels.begin + q.labels.count <= (int32_t)b.ints.size())
      row.pairs.assign(b.ints.begin() + q.labels.begin, b.ints.begin() + q.labels.begin + q.labels.count);
    c->pod_rows.push_back(std::move(row));
    kgpu_ctx::PodRec a;
    a.node = b.results[i].node;
    a.q = q;
    a.active = true;
    a.has_res = true;
    if (q.scalars.count && q.scalars.begin + q.scalars.count <= (int32_t)b.scalars.size())
      a.sc.assign(b.scalars.begin() + q.scalars.begin, b.scalars.begin() + q.scalars.begin + q.scalars.count);
    c->recs.push_back(std::move(a));
  }
  c->last_diag = false;
  return KGPU_OK;
}

// kgpu_schedule_batch_wait: the oldest batch submitted and not yet waited for.
int pipe_complete(kgpu_ctx* c) {
  if (c->pipe_q.empty()) return fail(c, KGPU_E_STATE, "no pipelined batch in flight");
  if (!c->pipe_q.front().done) pipe_finish(c, c->pipe_q.front());
  const int rc = c->pipe_q.front().rc;
  c->pipe_q.pop_front();
  return rc;
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
                       (int32_t)sizeof(kgpu_stats),     (int32_t)sizeof(kgpu_delta),
                       (int32_t)sizeof(kgpu_node_row),  (int32_t)sizeof(kgpu_delta_batch),
                       (int32_t)sizeof(kgpu_shape_point), (int32_t)sizeof(kgpu_nominated),
                       (int32_t)sizeof(kgpu_victim),    (int32_t)sizeof(kgpu_preempt_args),
                       (int32_t)sizeof(kgpu_node_victims), (int32_t)sizeof(kgpu_taint_ref),
                       (int32_t)sizeof(kgpu_reason_args)};
  const int32_t m = (int32_t)(sizeof(s) / sizeof(s[0]));
  for (int32_t i = 0; i < n && i < m; ++i) out[i] = s[i];
  return m;
}

// KGPU_SEGV_TRACE=1 (diagnostics): a host SIGSEGV prints this library's native backtrace to stderr
// before the default action (a Python faulthandler shows only the interpreter's frames).
// Each frame is printed with dladdr's library, symbol and offset from the library's load base, and the
// /proc/self/maps line that holds it, so a fault inside another library's exit handler names that
// library (diagnostics: formatting in a signal handler is not async-signal-safe).
static void segv_maps_line(const void* addr) {
  static char buf[1 << 17];
  const int fd = open("/proc/self/maps", O_RDONLY);
  if (fd < 0) return;
  const ssize_t n = read(fd, buf, sizeof(buf) - 1);
  close(fd);
  if (n <= 0) return;
  buf[n] = 0;
  char* save = nullptr;
  for (char* line = strtok_r(buf, "\n", &save); line; line = strtok_r(nullptr, "\n", &save)) {
    unsigned long lo = 0, hi = 0;
    if (std::sscanf(line, "%lx-%lx", &lo, &hi) == 2 && (unsigned long)addr >= lo && (unsigned long)addr < hi) {
      std::fprintf(stderr, "      maps: %s\n", line);
      return;
    }
  }
}

static void segv_trace(int sig, siginfo_t* si, void*) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  std::fprintf(stderr, "kgpu: signal %d, fault address %p, %d frames\n", sig, si ? si->si_addr : nullptr, n);
  for (int i = 0; i < n; ++i) {
    Dl_info d{};
    if (dladdr(fr[i], &d) && d.dli_fname)
      std::fprintf(stderr, "  #%d %p %s (%s+0x%lx) load base %p, offset 0x%lx\n", i, fr[i], d.dli_fname,
                   d.dli_sname ? d.dli_sname : "?",
                   d.dli_saddr ? (unsigned long)((const char*)fr[i] - (const char*)d.dli_saddr) : 0ul, d.dli_fbase,
                   (unsigned long)((const char*)fr[i] - (const char*)d.dli_fbase));
    else
      std::fprintf(stderr, "  #%d %p (no library)\n", i, fr[i]);
    segv_maps_line(fr[i]);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

int kgpu_create(const kgpu_config* cfg, kgpu_ctx** out) try {
  if (!cfg || !out) return KGPU_E_INVAL;
  if (const char* e = std::getenv("KGPU_SEGV_TRACE"))
    if (e[0] == '1') {
      struct sigaction sa {};
      sa.sa_sigaction = segv_trace;
      sa.sa_flags = SA_SIGINFO;
      sigaction(SIGSEGV, &sa, nullptr);
    }
  *out = nullptr;
  if (cfg->abi_version != KGPU_ABI_VERSION) return KGPU_E_INVAL;
  if (kgpu::kernel_layout_sig() != kgpu::layout_sig_of()) return KGPU_E_STATE;  // mixed-revision build
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
  if (cfg->percentage_of_nodes_to_score < 0 || cfg->percentage_of_nodes_to_score > 100) return KGPU_E_INVAL;
  for (int i = 0; i < cfg->n_scores; ++i)
    if (cfg->scores[i] == KGPU_S_REQUESTED_TO_CAPACITY_RATIO) {
      // ValidateRequestedToCapacityRatioArgs: a non-empty shape with strictly increasing utilization
      if (cfg->n_rtcr < 0 || cfg->n_rtcr > 8 || cfg->n_shape < 1 || cfg->n_shape > 16) return KGPU_E_INVAL;
      for (int j = 1; j < cfg->n_shape; ++j)
        if (cfg->shape[j].utilization <= cfg->shape[j - 1].utilization) return KGPU_E_INVAL;
    }
  fail_point();
  std::unique_ptr<kgpu_ctx> holder(new kgpu_ctx());  // freed on every early return and on a throw
  kgpu_ctx* c = holder.get();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return KGPU_E_DEVICE;
  if (cfg->device < 0 || cfg->device >= ndev) return KGPU_E_INVAL;
  c->cfg = *cfg;
  c->device = cfg->device;
  // KGPU_SYNC_SPIN=1: synchronizes spin instead of yielding (hipDeviceScheduleSpin: kgpu_schedule_one of a
  // topology pod 66.4 -> 63.4 us p50 at 5k nodes, profiles/r04_sync_spin_latency.txt).  Opt-in: the flag
  // is the device's, for every context and library of the process (a PyTorch or Go caller included), and
  // a spinning synchronize holds a CPU core for the length of a 100k-node batch.  It takes effect only if
  // no HIP context exists on the device yet (hipSetDeviceFlags fails otherwise; the failure is ignored).
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  {
    const char* e = std::getenv("KGPU_SYNC_SPIN");
    if (e && e[0] == '1') (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
  }
  if (const char* e = std::getenv("KGPU_HOST_TRACE")) c->htrace = e[0] == '1';
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
    return KGPU_E_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) {
    (void)hipStreamDestroy(c->stream);
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
  st.n_rtcr = cfg->n_rtcr;
  st.n_shape = cfg->n_shape;
  std::memcpy(st.rtcr, cfg->rtcr, sizeof(st.rtcr));
  std::memcpy(st.shape, cfg->shape, sizeof(st.shape));
  for (int i = 0; i < st.n_rtcr; ++i)
    if (st.rtcr[i].weight == 0) st.rtcr[i].weight = 1;  // requested_to_capacity_ratio.go:63-66
  // default requested-resource specs {cpu: 1, memory: 1} (noderesources/resource_allocation.go:36-39)
  auto def_spec = [](const kgpu_resource_weight* r, int n) {
    return n == 2 && r[0].resource == 0 && r[0].weight == 1 && r[1].resource == 1 && r[1].weight == 1;
  };
  const bool has_least = has_score(c, KGPU_S_LEAST_ALLOCATED), has_most = has_score(c, KGPU_S_MOST_ALLOCATED);
  const bool def_res = (!has_least || def_spec(cfg->least, cfg->n_least)) && (!has_most || def_spec(cfg->most, cfg->n_most));
  c->spec = kgpu::select_spec(cfg->filters, cfg->n_filters, cfg->scores, cfg->n_scores, def_res);
  *out = holder.release();
  return KGPU_OK;
} catch (...) {
  return on_exception(nullptr, false);
}

int kgpu_destroy(kgpu_ctx* c) try {
  if (!c) return KGPU_OK;
  if (c->htrace) {
    static const char* names[kgpu_ctx::kHt] = {"", "topology staging", "ports+pools", "state staged+geometry",
                                               "tables planned", "tables staged+key", "copy API", "launch API",
                                               "to end of issue", "synchronize", "records+bookkeeping", "record landed",
                                               "  topo: plans built", "  topo: classes synced", "  topo: plans staged",
                                               "    classes: columns", "    classes: tables", "    classes: counted"};
    // p50 and p99 of each step, and of the whole call, over the short cycles and over the longer calls
    auto pct = [](std::vector<int64_t> v, double q) {
      const size_t i = std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1) + 0.5));
      std::nth_element(v.begin(), v.begin() + (long)i, v.end());
      return (long long)v[i];
    };
    const std::vector<std::array<int64_t, kgpu_ctx::kHt>>* sets[2] = {&c->ht_cycles, &c->ht_batches};
    for (int si = 0; si < 2; ++si) {
      const auto& rows = *sets[si];
      if (rows.empty()) continue;
      std::fprintf(stderr, "kgpu host trace over %zu %s (ns per call: p50, p99, and the median over the calls at "
                   "or above the whole call's p99 -- what holds the tail):\n", rows.size(),
                   si == 0 ? "short cycles" : "batch calls");
      std::vector<int64_t> tot;
      for (const auto& r : rows) {
        int64_t t = 0;
        for (int k = 1; k < kgpu_ctx::kHt; ++k) t += r[(size_t)k];
        tot.push_back(t);
      }
      const long long t99 = pct(tot, 0.99);
      for (int k = 1; k < kgpu_ctx::kHt; ++k) {
        if (!(c->ht_seen & (1 << k))) continue;
        std::vector<int64_t> v, tail;
        for (size_t i = 0; i < rows.size(); ++i) {
          v.push_back(rows[i][(size_t)k]);
          if (tot[i] >= t99) tail.push_back(rows[i][(size_t)k]);
        }
        std::fprintf(stderr, "  %2d %-24s %9lld %9lld %9lld\n", k, names[k], pct(v, 0.5), pct(v, 0.99), pct(tail, 0.5));
      }
      std::fprintf(stderr, "     %-24s %9lld %9lld\n", "whole call", pct(tot, 0.5), t99);
    }
  }
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_all(c->snap_allocs);
  free_all(c->work_allocs);
  for (DevBuf* b : {&c->dstate, &c->ticket, &c->queries, &c->pool_blk, &c->results, &c->gran, &c->trace, &c->d_classes,
                    &c->d_citems, &c->d_tclasses, &c->d_creqs, &c->d_cints, &c->d_plans, &c->d_aux,
                    &c->d_aux_terms, &c->scratch, &c->d_pods, &c->gbar, &c->cut_buf, &c->t_tables, &c->t_zero,
                    &c->abort_buf, &c->flags_buf, &c->d_stage, &c->d_remap, &c->d_from,
                    &c->p_args, &c->p_voff, &c->p_veff, &c->p_noff, &c->p_neff, &c->p_aux, &c->p_vrecs,
                    &c->p_vsc, &c->p_vports, &c->p_nrecs, &c->p_nsc, &c->p_nports, &c->p_vstate, &c->p_order,
                    &c->p_out, &c->p_outv, &c->p_prep, &c->p_nomstat, &c->p_pdb, &c->xg_arr,
                    &c->batch_ptrs})
    if (b->p) (void)hipFree(b->p);
  if (c->pref_x.p) (void)hipFree(c->pref_x.p);
  for (void* q : c->xg_open)
    if (q) (void)hipIpcCloseMemHandle(q);
  if (c->xg_box.p) (void)hipFree(c->xg_box.p);
  {
    const kgpu::StageOps ops = stage_ops(c);
    c->delta_stage.release(ops);
    c->table_stage.release(ops);
    c->pool_stage.release(ops);
    c->batch_stage.release(ops);
  }
  for (auto& ps : c->pipe) {
    if (ps.host) (void)hipHostFree(ps.host);
    if (ps.res) (void)hipHostFree(ps.res);
    if (ps.dev.p) (void)hipFree(ps.dev.p);
    if (ps.gran.p) (void)hipFree(ps.gran.p);
    for (hipEvent_t e : {ps.done, ps.t0, ps.t1})
      if (e) (void)hipEventDestroy(e);
  }
  if (c->cyc_host) (void)hipHostFree(c->cyc_host);
  if (c->res_pin) (void)hipHostFree(c->res_pin);
  if (c->pool_pin) (void)hipHostFree(c->pool_pin);
  if (c->st.mcnt) (void)hipFree(c->st.mcnt);
  if (c->st.tcnt) (void)hipFree(c->st.tcnt);
  if (c->shard.p) (void)hipFree(c->shard.p);
  if (c->comm) (void)rccl().CommDestroy(c->comm);
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

const char* kgpu_last_error(const kgpu_ctx* c) { return c ? c->err.c_str() : "null context"; }

int64_t kgpu_generation(const kgpu_ctx* c) { return c ? c->generation : -1; }

int kgpu_read_phase_trace(kgpu_ctx* c, int64_t* out, int32_t max_pods) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !out || max_pods < 0) return KGPU_E_INVAL;
  const int32_t n = std::min<int32_t>(max_pods, (int32_t)(c->trace_host.size() / 16));
  std::memcpy(out, c->trace_host.data(), sizeof(int64_t) * 16 * (size_t)n);
  return n;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_debug_counters(const kgpu_ctx* c, int64_t* out, int32_t n) {
  if (!c || (n > 0 && !out)) return KGPU_E_INVAL;
  const int64_t v[5] = {c->n_coop_retry, c->n_persist, c->n_coop, c->n_class_init, c->n_pod_table_full};
  for (int32_t i = 0; i < n && i < 5; ++i) out[i] = v[i];
  return 5;
}

int kgpu_debug_topo_resident(const kgpu_ctx* c, int64_t out[2]) {
  if (!c || !out) return KGPU_E_INVAL;
  out[0] = (int64_t)c->tc_hits;
  out[1] = (int64_t)c->tc_misses;
  return KGPU_OK;
}

int kgpu_debug_wg_trace(kgpu_ctx* c, int64_t* out, int64_t max_words, int32_t* groups) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !out || !groups || max_words < 0) return KGPU_E_INVAL;
  const size_t n = std::min<size_t>((size_t)max_words, c->trace_wg_host.size());
  std::memcpy(out, c->trace_wg_host.data(), sizeof(int64_t) * n);
  *groups = c->trace_wg_groups;
  return (int)std::min<size_t>(n, INT32_MAX);
} catch (...) {
  return on_exception(c, false);
}

int kgpu_set_option(kgpu_ctx* c, int32_t option, int64_t value) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (!c) return KGPU_E_INVAL;
  if (option == KGPU_OPT_KERNEL_TIMING) c->timing = value != 0;
  else if (option == KGPU_OPT_PERSISTENT) c->persistent = value != 0;
  else if (option == KGPU_OPT_PERSIST_GROUPS) c->max_groups = (int)std::max<int64_t>(value, 0);
  else if (option == KGPU_OPT_PHASE_TRACE) {
    c->phase_trace = value != 0;
    c->phase_trace_mode = (int)std::min<int64_t>(std::max<int64_t>(value, 0), 3);
  }
  else if (option == KGPU_OPT_TOPO_FUSED) c->topo_fused = value != 0;
  else if (option == KGPU_OPT_TOPO_PERSISTENT) c->tfast = value != 0;
  else if (option == KGPU_OPT_COOPERATIVE) c->coop = value != 0;
  else if (option == KGPU_OPT_BATCH_GEO) c->batch_geo_first = (int)std::max<int64_t>(0, value);
  else if (option == KGPU_OPT_BATCH_HELPER) c->batch_helper = value != 0;
  else if (option == KGPU_OPT_TOPO_AHEAD) c->topo_ahead = value != 0;
  else if (option == KGPU_OPT_TBATCH_GEO) c->tbatch_geo_first = (int)std::min<int64_t>(std::max<int64_t>(value, 0), 2);
  else if (option == KGPU_OPT_TOPO_RESIDENT) {
    c->tc_on = value != 0;
    c->tc.valid = false;
  } else if (option == KGPU_OPT_ARENA_BYTES) c->ar_limit = (size_t)std::min<int64_t>(std::max<int64_t>(0, value), (int64_t)kArenaBytes);
  else if (option == KGPU_OPT_ABORT_AT) c->abort_at = value < 0 || value > INT32_MAX ? -1 : (int32_t)value;
  else if (option == KGPU_OPT_XGMI) c->xgmi = value != 0;
  else if (option == KGPU_OPT_TBATCH_WLAB) c->tbatch_wlab = value != 0;
  else if (option == KGPU_OPT_TBATCH_POLL_SLEEP) c->tbatch_sleep = value != 0;
  else if (option == KGPU_OPT_ZEROCOPY_POOLS) c->zc_pools = value != 0;
  else if (option == KGPU_OPT_RUN_ALL_FILTERS) c->run_all = value != 0;
  else if (option == KGPU_OPT_HOLD_GROUP) c->hold_group = value < 0 || value > INT32_MAX ? -1 : (int32_t)value;
  else if (option == KGPU_OPT_SKIP_RELEASE_AT) c->skip_release_at = value < 0 || value > INT32_MAX ? -1 : (int32_t)value;
  else return KGPU_E_INVAL;
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_upload_snapshot(kgpu_ctx* c, const kgpu_snapshot* s, int64_t generation) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !s) return KGPU_E_INVAL;
  c->tc.valid = false;
  if (s->n_nodes < 0 || s->n_label_keys < 0 || s->n_scalar < 0 || s->taint_words < 0 || s->port_slots < 0)
    return fail(c, KGPU_E_INVAL, "negative snapshot dimension");
  if (s->n_nodes > 0 && (!s->alloc_cpu || !s->alloc_mem || !s->alloc_eph || !s->alloc_pods || !s->req_cpu ||
                         !s->req_mem || !s->req_eph || !s->nz_cpu || !s->nz_mem || !s->num_pods ||
                         !s->unschedulable || !s->image_off || !s->avoid_off || !s->zone_id || !s->port_count))
    return fail(c, KGPU_E_INVAL, "missing node column");
  HIP_OK(c, hipSetDevice(c->device));
  SYNC_OK(c);
  free_all(c->snap_allocs);
  free_all(c->work_allocs);
  fail_point();
  c->recs.clear();
  c->uid_slot.clear();
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
  c->prefer_host.assign((size_t)st.TW * N, 0ull);
  if (s->taint_words > 0) std::memcpy(c->prefer_host.data(), s->taint_prefer, sizeof(uint64_t) * (size_t)st.TW * N);
  c->label_host.assign((size_t)st.K * N, -1);
  if (st.K > 0) std::memcpy(c->label_host.data(), s->label_val, sizeof(int32_t) * (size_t)st.K * N);
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
  if ((rc = alloc_node_work(c))) return rc;
  st.key_empty = st.key_empty_value;
  st.hard_pod_affinity_weight = c->cfg.hard_pod_affinity_weight;
  if ((rc = ensure(c, c->flags_buf, 64))) return rc;
  HIP_OK(c, hipMemset(c->flags_buf.p, 0, 64));
  st.port_overflow = static_cast<int32_t*>(c->flags_buf.p);
  // topology state: host copies of the key metadata, the pod table, existing pods' term classes
  c->key_n_values.assign(s->key_n_values ? s->key_n_values : nullptr, s->key_n_values ? s->key_n_values + st.K : nullptr);
  c->key_empty.assign(s->key_empty_value ? s->key_empty_value : nullptr,
                      s->key_empty_value ? s->key_empty_value + st.K : nullptr);
  rebuild_node_books(c);
  c->key_unique_caller.clear();
  if (s->key_unique) c->key_unique_caller.assign(s->key_unique, s->key_unique + st.K);
  c->class_ids.clear();
  c->tclass_ids.clear();
  c->classes.clear();
  c->citems.clear();
  c->tclasses.clear();
  c->creqs.clear();
  c->cints.clear();
  c->classes_init = 0;
  c->pod_rows.clear();
  c->pod_rows_dev = -1;
  c->pod_rows_dirty.clear();
  for (int i = 0; i < s->n_pods; ++i) {
    kgpu_ctx::PodRec rec;
    rec.node = s->pod_node[i];
    rec.active = (s->pod_flags[i] & KGPU_PF_ACTIVE) != 0;
    if (s->pod_uid) {
      rec.uid = s->pod_uid[i];
      rec.has_uid = true;
      if (rec.active && !c->uid_slot.emplace(rec.uid, i).second)
        return fail(c, KGPU_E_INVAL, "duplicate pod uid in the snapshot");
    }
    c->recs.push_back(std::move(rec));
    kgpu_ctx::PodRow row;
    row.node = s->pod_node[i];
    row.ns = s->pod_ns[i];
    row.flags = s->pod_flags[i];
    for (int k = 0; k < s->n_pod_label_keys; ++k) {
      const int32_t v = s->pod_label_val[(size_t)k * s->n_pods + i];
      if (v >= 0) {
        row.pairs.push_back(k);
        row.pairs.push_back(v);
      }
    }
    c->pod_rows.push_back(std::move(row));
  }
  if (c->st.mcnt) (void)hipFree(c->st.mcnt);
  if (c->st.tcnt) (void)hipFree(c->st.tcnt);
  st.mcnt = nullptr;
  st.tcnt = nullptr;
  c->Ccap = c->TCcap = 0;
  std::vector<std::pair<int, int>> term_cells;  // (term class, local node)
  for (int t = 0; t < s->n_terms; ++t) {
    const kgpu_term& tm = s->terms[t];
    const int tc = intern_tclass(c, tm.kind, tm.t.weight, tm.t.topo_key, term_item(tm.t, &s->pools));
    if (tm.pod < 0 || tm.pod >= s->n_pods || !(s->pod_flags[tm.pod] & KGPU_PF_ACTIVE)) continue;
    // the owner's PodInfo terms: what RemovePod / a preemption removal takes back out of tcnt
    c->pod_rows[(size_t)tm.pod].own_tcls.push_back(tc);
    const int ln = s->pod_node[tm.pod] - st.node_base;
    if (ln >= 0 && ln < st.N) term_cells.emplace_back(tc, ln);
  }
  if ((rc = grow_columns(c, &st.mcnt, &c->Ccap, 1))) return rc;
  if ((rc = grow_columns(c, &st.tcnt, &c->TCcap, (int)c->tclasses.size()))) return rc;
  if (!term_cells.empty()) {
    std::vector<int32_t> tc_host((size_t)c->TCcap * N, 0);
    for (auto& cell : term_cells) tc_host[(size_t)cell.first * N + cell.second] += 1;
    HIP_OK(c, hipMemcpy(st.tcnt, tc_host.data(), sizeof(int32_t) * tc_host.size(), hipMemcpyHostToDevice));
  }
  c->port_bound = 0;
  for (size_t i = 0; i < N; ++i) c->port_bound = std::max<int64_t>(c->port_bound, s->port_count[i]);
  c->row_canon.resize(N);
  for (size_t i = 0; i < N; ++i) c->row_canon[i] = (int32_t)i;
  c->alias_rows.clear();
  c->has_alias = false;
  c->n_snapshot_pods = s->n_pods;
  c->generation = generation;
  if (c->comm && (rc = sync_prefer_union(c))) return rc;  // every rank re-uploads its shard together
  c->uploaded = true;
  HIP_OK(c, hipDeviceSynchronize());
  return KGPU_OK;
} catch (...) {
  return on_exception(c, true);
}

int kgpu_schedule_batch(kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools, int64_t first_seq,
                        kgpu_result* results, kgpu_stats* stats) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || (n > 0 && (!qs || !results))) return KGPU_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  return run_batch(c, qs, n, pools, first_seq, results, stats, false, 1);
} catch (...) {
  return on_exception(c, true);
}

int kgpu_schedule_batch_submit(kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools,
                               int64_t first_seq, kgpu_result* results, kgpu_stats* stats) try {
  if (!c || (n > 0 && (!qs || !results))) return KGPU_E_INVAL;
  if (c->unsettled) {
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  return pipe_submit(c, qs, n, pools, first_seq, results, stats);
} catch (...) {
  c->pipe_q.clear();
  return on_exception(c, true);
}

int kgpu_schedule_batch_wait(kgpu_ctx* c) try {
  if (!c) return KGPU_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  return pipe_complete(c);
} catch (...) {
  c->pipe_q.clear();
  return on_exception(c, true);
}

int kgpu_pipelined(const kgpu_ctx* c) { return c ? (int)c->pipe_q.size() : 0; }

int kgpu_schedule_one(kgpu_ctx* c, const kgpu_pod_query* q, const kgpu_pools* pools, int64_t pod_seq, int32_t assume,
                      kgpu_result* res, int32_t* assumed_slot) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (!c || !q || !res) return KGPU_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  size_t before = c->recs.size();
  int rc = run_batch(c, q, 1, pools, pod_seq, res, nullptr, true, assume);
  if (rc) return rc;
  if (assumed_slot) *assumed_slot = c->recs.size() > before ? (int32_t)c->recs.size() - 1 : -1;
  return KGPU_OK;
} catch (...) {
  return on_exception(c, true);
}

int kgpu_set_nominated(kgpu_ctx* c, const kgpu_nominated* noms, int32_t n, const kgpu_pod_query* pods,
                       const kgpu_pools* pools) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || n < 0 || (n > 0 && (!noms || !pods))) return KGPU_E_INVAL;
  kgpu_ctx::Nominator nm;
  int32_t n_items = 0;
  for (int32_t i = 0; i < n; ++i) {
    if (noms[i].item < 0) return fail(c, KGPU_E_INVAL, "kgpu_set_nominated: negative record index");
    if (noms[i].node < 0 || noms[i].node >= std::max(c->st.n_total, c->st.N))
      return fail(c, KGPU_E_INVAL, "kgpu_set_nominated: node index out of range");
    n_items = std::max(n_items, noms[i].item + 1);
  }
  nm.list.assign(noms, noms + n);
  nm.recs.assign(pods, pods + n_items);
  if (pools) {  // owned copies: the records' ranges stay valid after the call
    auto cp = [](auto& v, const auto* src, int32_t cnt) {
      if (src && cnt > 0) v.assign(src, src + cnt);
    };
    cp(nm.reqs, pools->reqs, pools->n_reqs);
    cp(nm.ints, pools->ints, pools->n_ints);
    cp(nm.words, pools->words, pools->n_words);
    cp(nm.nterms, pools->node_terms, pools->n_node_terms);
    cp(nm.pterms, pools->pref_terms, pools->n_pref_terms);
    cp(nm.spreads, pools->spreads, pools->n_spreads);
    cp(nm.pod_terms, pools->pod_terms, pools->n_pod_terms);
    cp(nm.scalars, pools->scalars, pools->n_scalars);
    cp(nm.ports, pools->ports, pools->n_ports);
  }
  c->nom = std::move(nm);
  kgpu_pools& v = c->nom.pools;
  v = kgpu_pools{};
  v.reqs = c->nom.reqs.data(); v.n_reqs = (int32_t)c->nom.reqs.size();
  v.ints = c->nom.ints.data(); v.n_ints = (int32_t)c->nom.ints.size();
  v.words = c->nom.words.data(); v.n_words = (int32_t)c->nom.words.size();
  v.node_terms = c->nom.nterms.data(); v.n_node_terms = (int32_t)c->nom.nterms.size();
  v.pref_terms = c->nom.pterms.data(); v.n_pref_terms = (int32_t)c->nom.pterms.size();
  v.spreads = c->nom.spreads.data(); v.n_spreads = (int32_t)c->nom.spreads.size();
  v.pod_terms = c->nom.pod_terms.data(); v.n_pod_terms = (int32_t)c->nom.pod_terms.size();
  v.scalars = c->nom.scalars.data(); v.n_scalars = (int32_t)c->nom.scalars.size();
  v.ports = c->nom.ports.data(); v.n_ports = (int32_t)c->nom.ports.size();
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

// pickOneNodeForPreemption (generic_scheduler.go:718-843) over the nodes that fit, walked in
// Snapshot.List() order (the reference walks a map: any of the tied nodes).
static int32_t pick_one_node(const std::vector<int32_t>& cand, const kgpu_node_victims* out, const int32_t* vout,
                             const kgpu_preempt_args* a, const int32_t* prio) {
  if (cand.empty()) return -1;
  auto pods = [&](int32_t n) { return out[n].n_victims; };
  auto vict = [&](int32_t n, int k) { return vout[out[n].first + k]; };
  for (int32_t n : cand)
    if (pods(n) == 0) return n;
  auto narrow = [&](const std::vector<int32_t>& in, auto key) {  // nodes with the minimum key
    std::vector<int32_t> o;
    int64_t best = INT64_MAX;
    for (int32_t n : in) {
      const int64_t k = key(n);
      if (k < best) {
        best = k;
        o.clear();
      }
      if (k == best) o.push_back(n);
    }
    return o;
  };
  std::vector<int32_t> m = narrow(cand, [&](int32_t n) { return (int64_t)out[n].num_pdb_violations; });
  if (m.size() == 1) return m[0];
  m = narrow(m, [&](int32_t n) { return (int64_t)prio[vict(n, 0)]; });  // Victims.Pods[0]: the highest
  if (m.size() == 1) return m[0];
  m = narrow(m, [&](int32_t n) {
    int64_t sum = 0;
    for (int k = 0; k < pods(n); ++k) sum += (int64_t)prio[vict(n, k)] + (int64_t)2147483647 + 1;
    return sum;
  });
  if (m.size() == 1) return m[0];
  m = narrow(m, [&](int32_t n) { return (int64_t)pods(n); });
  if (m.size() == 1) return m[0];
  // latest earliest start time among each node's highest-priority victims (util.GetEarliestPodStartTime)
  auto earliest = [&](int32_t n) {
    int32_t v0 = vict(n, 0);
    int64_t t = a->victims[v0].start_time;
    int32_t mp = prio[v0];
    for (int k = 0; k < pods(n); ++k) {
      const int32_t v = vict(n, k);
      if (prio[v] == mp) {
        if (a->victims[v].start_time < t) t = a->victims[v].start_time;
      } else if (prio[v] > mp) {
        mp = prio[v];
        t = a->victims[v].start_time;
      }
    }
    return t;
  };
  int32_t ret = m[0];
  int64_t latest = earliest(m[0]);
  for (size_t i = 1; i < m.size(); ++i) {
    const int64_t t = earliest(m[i]);
    if (t > latest) {
      latest = t;
      ret = m[i];
    }
  }
  return ret;
}

int kgpu_select_victims(kgpu_ctx* c, const kgpu_pod_query* q, const kgpu_pools* pools, const kgpu_preempt_args* args,
                        kgpu_node_victims* nodes_out, int32_t* victims_out, int32_t* chosen) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !q || !args || !nodes_out || (args->n_victims > 0 && (!args->victims || !args->pods || !victims_out)))
    return KGPU_E_INVAL;
  if (args->n_victims < 0 || args->n_pdbs < 0 || (args->n_pdbs > 0 && !args->pdb_allowed)) return KGPU_E_INVAL;
  if (args->n_pdbs > 64) return fail(c, KGPU_E_CAPACITY, "more than 64 PodDisruptionBudgets");
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  if (!c->uploaded) return fail(c, KGPU_E_STATE, "no snapshot uploaded");
  if (c->comm) return fail(c, KGPU_E_UNSUPPORTED, "preemption on a node-sharded engine");
  const int N = c->st.N;
  int rc;
  Staged sg;
  if ((rc = stage_topology(c, q, 1, pools, sg))) return rc;
  const kgpu::QPlan* pl = sg.topo_on ? &sg.plans[0] : nullptr;
  if ((rc = upload_pools(c, pools))) return rc;
  if ((rc = ensure(c, c->queries, sizeof(kgpu_pod_query)))) return rc;
  HIP_OK(c, hipMemcpyAsync(c->queries.p, q, sizeof(kgpu_pod_query), hipMemcpyHostToDevice, c->stream));
  DevState st = c->st;
  st.queries = static_cast<const kgpu_pod_query*>(c->queries.p);
  st.diag_raw = nullptr;
  st.diag_norm = nullptr;
  // nodesWherePreemptionMightHelp reads the cycle's merged code (framework.go:494 runAllFilters)
  st.run_all = c->run_all ? 1 : 0;
  // potential victims per local node, MoreImportantPod order (stable over the caller's order)
  PreemptStage ps;
  std::vector<int32_t> pos_of;  // sorted position -> caller's victim index
  std::vector<std::vector<int32_t>> by((size_t)N);
  for (int32_t i = 0; i < args->n_victims; ++i) {
    const kgpu_victim& v = args->victims[i];
    const int local = v.node - c->st.node_base;
    if (local < 0 || local >= N) return fail(c, KGPU_E_INVAL, "kgpu_select_victims: victim node out of range");
    if (v.slot < 0 || v.slot >= (int32_t)c->pod_rows.size() || v.item < 0)
      return fail(c, KGPU_E_INVAL, "kgpu_select_victims: bad victim slot or record");
    if (args->pods[v.item].priority >= q->priority) continue;  // not a potential victim
    by[(size_t)local].push_back(i);
  }
  const int32_t* qpairs = (pools && q->labels.count) ? pools->ints + q->labels.begin : nullptr;
  const int qnp = q->labels.count / 2;
  ps.v_off.assign((size_t)N + 1, 0);
  for (int n = 0; n < N; ++n) {
    std::vector<int32_t>& l = by[(size_t)n];
    std::stable_sort(l.begin(), l.end(), [&](int32_t x, int32_t y) {
      const int32_t px = args->pods[args->victims[x].item].priority, py = args->pods[args->victims[y].item].priority;
      if (px != py) return px > py;
      return args->victims[x].start_time < args->victims[y].start_time;
    });
    for (int32_t i : l) {
      const kgpu_victim& v = args->victims[i];
      const kgpu_ctx::PodRow& row = c->pod_rows[(size_t)v.slot];
      kgpu::PEff f = build_effect(c, pl, row.ns, row.pairs.empty() ? nullptr : row.pairs.data(), (int)row.pairs.size() / 2);
      f.item = (int32_t)ps.vrecs.size();
      ps.vrecs.push_back(args->pods[v.item]);
      f.prio = args->pods[v.item].priority;
      f.start = v.start_time;
      f.pdb_mask = args->n_pdbs >= 64 ? v.pdb_mask : (v.pdb_mask & ((1ull << args->n_pdbs) - 1));
      f.exa.begin = (int32_t)ps.aux.size();
      for (int32_t t : row.own_tcls) {
        const kgpu::TermClassRec& tc = c->tclasses[(size_t)t];
        if (tc.kind == KGPU_TERM_REQ_ANTI && tc.topo_key >= 0 && item_matches(c, tc.item, q->ns, qpairs, qnp))
          ps.aux.push_back(tc.topo_key);
      }
      f.exa.count = (int32_t)ps.aux.size() - f.exa.begin;
      ps.veff.push_back(f);
      pos_of.push_back(i);
    }
    ps.v_off[(size_t)n + 1] = (int32_t)ps.veff.size();
  }
  stage_nominated(c, *q, pools, pl, ps.n_off, ps.neff, ps.aux);
  const kgpu::PreemptArgs* dev = nullptr;
  const int32_t* d_pdb = nullptr;
  if ((rc = upload_pool(c, c->p_pdb, args->pdb_allowed, args->n_pdbs, &d_pdb)) ||
      (rc = upload_preempt(c, ps, pools, 1, args->n_pdbs, d_pdb, &dev)))
    return rc;
  if ((rc = ensure(c, c->dstate, sizeof(DevState)))) return rc;
  c->ds_ptr = nullptr;  // the short cycle's cached DevState image is stale
  c->st_batch = st;
  HIP_OK(c, hipMemcpyAsync(c->dstate.p, &c->st_batch, sizeof(DevState), hipMemcpyHostToDevice, c->stream));
  const DevState* dst = static_cast<const DevState*>(c->dstate.p);
  if (pl && pl->topo) {  // the preemptor's PreFilter state: TpPairToMatchNum / criticalPaths / IPA maps
    HIP_OK(c, hipMemsetAsync(c->st.scratch, 0, sizeof(int64_t) * (size_t)pl->scratch_len, c->stream));
    PodArgs a{};
    a.pod = 0;
    a.prev = -1;
    int64_t min_values = 0;
    for (int k = 0; k < pl->n_hard; ++k)
      if (pl->hard[k].key >= 0) min_values = std::max<int64_t>(min_values, c->key_n_values[pl->hard[k].key]);
    const int blocks = kgpu::eval_blocks(N);
    if (kgpu::launch_topo_phase(dst, a, 0, blocks, 0, c->stream) ||
        (min_values > 0 && kgpu::launch_topo_phase(dst, a, 1, blocks, min_values, c->stream)) ||
        kgpu::launch_vict_prep(dst, dev, c->stream))
      return fail(c, KGPU_E_DEVICE, "preemption PreFilter launch failed");
  }
  if (kgpu::launch_victims(dst, dev, N, c->stream)) return fail(c, KGPU_E_DEVICE, "k_victims launch failed");
  std::vector<int32_t> vout(std::max<size_t>(ps.veff.size(), 1));
  HIP_OK(c, hipMemcpyAsync(nodes_out, c->pa_host.out, sizeof(kgpu_node_victims) * (size_t)N, hipMemcpyDeviceToHost,
                           c->stream));
  if (!ps.veff.empty())
    HIP_OK(c, hipMemcpyAsync(vout.data(), c->pa_host.out_victims, sizeof(int32_t) * ps.veff.size(),
                             hipMemcpyDeviceToHost, c->stream));
  SYNC_OK(c);
  // sorted positions -> the caller's victim indices; pick the node
  std::vector<int32_t> prio(std::max<int32_t>(args->n_victims, 1));
  for (int32_t i = 0; i < args->n_victims; ++i) prio[(size_t)i] = args->pods[args->victims[i].item].priority;
  std::vector<int32_t> cand;
  for (int n = 0; n < N; ++n) {
    kgpu_node_victims& o = nodes_out[n];
    for (int k = 0; k < o.n_victims; ++k) victims_out[o.first + k] = pos_of[(size_t)vout[(size_t)(o.first + k)]];
    if (o.fits) cand.push_back(n);
  }
  const int32_t pick = pick_one_node(cand, nodes_out, victims_out, args, prio.data());
  if (chosen) *chosen = pick >= 0 ? pick + c->st.node_base : -1;
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

// The per-pod topology phases of one pod on the engine's current state (diagnostics only): the
// histograms (k_topo_pre) always; for kind 0 the critical-path minima of hard constraint `constraint`
// (k_topo_min), for kind 1 the registrations of the filtered nodes (k_topo_filter).  The pod's
// scratch (TopoHdr + slots) comes back in sc, its plan in sg.
static int debug_topo_scratch(kgpu_ctx* c, const kgpu_pod_query* q, const kgpu_pools* pools, int32_t kind,
                              int32_t constraint, Staged& sg, std::vector<int64_t>& sc) {
  int rc;
  if ((rc = stage_topology(c, q, 1, pools, sg))) return rc;
  const kgpu::QPlan& pl = sg.plans[0];
  int64_t D = 0;
  if (kind == 0 || kind == 1) {
    if (constraint >= (kind == 0 ? pl.n_hard : pl.n_soft)) return fail(c, KGPU_E_INVAL, "no such constraint");
    const kgpu::TSpread& sp = kind == 0 ? pl.hard[constraint] : pl.soft[constraint];
    D = sp.key >= 0 ? c->key_n_values[(size_t)sp.key] : 0;
  }
  if ((rc = upload_pools(c, pools))) return rc;
  if ((rc = ensure(c, c->queries, sizeof(kgpu_pod_query)))) return rc;
  HIP_OK(c, hipMemcpyAsync(c->queries.p, q, sizeof(kgpu_pod_query), hipMemcpyHostToDevice, c->stream));
  DevState st = c->st;
  st.queries = static_cast<const kgpu_pod_query*>(c->queries.p);
  st.diag_raw = nullptr;
  st.diag_norm = nullptr;
  st.nom_status = nullptr;
  if ((rc = ensure(c, c->results, sizeof(kgpu_result)))) return rc;
  st.results = static_cast<kgpu_result*>(c->results.p);
  if ((rc = ensure(c, c->dstate, sizeof(DevState)))) return rc;
  c->ds_ptr = nullptr;  // the short cycle's cached DevState image is stale
  c->st_batch = st;
  HIP_OK(c, hipMemcpyAsync(c->dstate.p, &c->st_batch, sizeof(DevState), hipMemcpyHostToDevice, c->stream));
  const DevState* dst = static_cast<const DevState*>(c->dstate.p);
  HIP_OK(c, hipMemsetAsync(c->st.scratch, 0, sizeof(int64_t) * (size_t)pl.scratch_len, c->stream));
  PodArgs a{};
  a.pod = 0;
  a.prev = -1;
  const int blocks = kgpu::eval_blocks(c->st.N);
  if (kgpu::launch_topo_phase(dst, a, 0, blocks, 0, c->stream) ||
      (kind == 0 && D > 0 && kgpu::launch_topo_phase(dst, a, 1, blocks, D, c->stream)) ||
      (kind == 1 && kgpu::launch_topo_phase(dst, a, 2, blocks, 0, c->stream)))
    return fail(c, KGPU_E_DEVICE, "topology phase launch failed");
  sc.assign((size_t)pl.scratch_len, 0);
  HIP_OK(c, hipMemcpyAsync(sc.data(), c->st.scratch, sizeof(int64_t) * sc.size(), hipMemcpyDeviceToHost, c->stream));
  SYNC_OK(c);
  return KGPU_OK;
}

static int debug_topo_check(kgpu_ctx* c) {
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  if (!c->uploaded) return fail(c, KGPU_E_STATE, "no snapshot uploaded");
  if (c->comm || c->xg_nranks > 1)
    return fail(c, KGPU_E_UNSUPPORTED, "the topology state diagnostics read one engine's state: unsharded only");
  return KGPU_OK;
}

int kgpu_debug_pts_state(kgpu_ctx* c, const kgpu_pod_query* q, const kgpu_pools* pools, int32_t kind,
                         int32_t constraint, uint8_t* registered, int64_t* counts, int64_t* scalar) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !q || !registered || !counts || !scalar || (kind != 0 && kind != 1) || constraint < 0) return KGPU_E_INVAL;
  int rc;
  if ((rc = debug_topo_check(c))) return rc;
  if (!has_filter(c, KGPU_F_POD_TOPOLOGY_SPREAD) && kind == 0)
    return fail(c, KGPU_E_INVAL, "the profile has no PodTopologySpread filter");
  if (!has_score(c, KGPU_S_POD_TOPOLOGY_SPREAD) && kind == 1)
    return fail(c, KGPU_E_INVAL, "the profile has no PodTopologySpread score");
  Staged sg;
  std::vector<int64_t> sc;
  if ((rc = debug_topo_scratch(c, q, pools, kind, constraint, sg, sc))) return rc;
  const kgpu::QPlan& pl = sg.plans[0];
  const kgpu::TSpread& sp = kind == 0 ? pl.hard[constraint] : pl.soft[constraint];
  const int64_t D = sp.key >= 0 ? c->key_n_values[(size_t)sp.key] : 0;
  const kgpu::TopoHdr* h = reinterpret_cast<const kgpu::TopoHdr*>(sc.data());
  for (int64_t v = 0; v < D; ++v) {
    registered[v] = sc[(size_t)(pl.slot_off[sp.rslot] + v)] != 0 ? 1 : 0;
    counts[v] = sc[(size_t)(pl.slot_off[sp.cslot] + v)];
  }
  if (kind == 0) {
    // criticalPaths[0].MatchNum: MaxInt32 when no pair registered (filtering.go:86-90)
    const uint64_t u = static_cast<uint64_t>(h->pmin[constraint]);
    *scalar = u ? (int64_t)(~u ^ (1ull << 63)) : 2147483647;
  } else {
    // topologyNormalizingWeight's size (scoring.go:92-102): registered pairs of the key, or for
    // kubernetes.io/hostname the filtered nodes that carry every soft key
    *scalar = sp.is_hostname ? (int64_t)h->feas_nonign : (sp.first_of_key ? h->ssize[constraint] : -1);
  }
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_debug_ipa_state(kgpu_ctx* c, const kgpu_pod_query* q, const kgpu_pools* pools, int32_t max_maps,
                         int32_t max_values, int32_t* kinds, int32_t* keys, int64_t* counts, int32_t* n_maps) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !q || !kinds || !keys || !counts || !n_maps || max_maps < 0 || max_values < 0) return KGPU_E_INVAL;
  int rc;
  if ((rc = debug_topo_check(c))) return rc;
  if (!has_filter(c, KGPU_F_INTER_POD_AFFINITY))
    return fail(c, KGPU_E_INVAL, "the profile has no InterPodAffinity filter");
  Staged sg;
  std::vector<int64_t> sc;
  if ((rc = debug_topo_scratch(c, q, pools, 2, 0, sg, sc))) return rc;
  const kgpu::QPlan& pl = sg.plans[0];
  // preFilterState's three maps (interpodaffinity/filtering.go:166-271), one histogram per (map,
  // topology key): the terms of one map that share a key add into the same pairs, as they do there
  int m = 0;
  for (int s = 0; s < pl.n_slots; ++s) {
    const int k = pl.slot_kind[s];
    const int kind = k == kgpu::kSlotExA ? 0 : k == kgpu::kSlotAff ? 1 : k == kgpu::kSlotAnti ? 2 : -1;
    if (kind < 0) continue;
    if (m == max_maps) return fail(c, KGPU_E_INVAL, "more histograms than max_maps");
    const int64_t D = pl.slot_key[s] >= 0 ? c->key_n_values[(size_t)pl.slot_key[s]] : 0;
    if (D > max_values) return fail(c, KGPU_E_INVAL, "a topology key has more values than max_values");
    kinds[m] = kind;
    keys[m] = pl.slot_key[s];
    for (int64_t v = 0; v < max_values; ++v)
      counts[(size_t)m * max_values + v] = v < D ? sc[(size_t)(pl.slot_off[s] + v)] : 0;
    ++m;
  }
  *n_maps = m;
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_debug_broken_linear(kgpu_ctx* c, const kgpu_shape_point* points, int32_t n_points, const int64_t* p,
                             int32_t n, int64_t* out) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !points || !p || !out || n_points <= 0 || n_points > 16 || n <= 0) return KGPU_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  fail_point();
  int64_t* d = nullptr;
  HIP_OK(c, hipMalloc(&d, sizeof(int64_t) * 2 * (size_t)n));
  int rc = KGPU_OK;
  if (hipMemcpyAsync(d, p, sizeof(int64_t) * (size_t)n, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      kgpu::launch_debug_broken_linear(points, n_points, d, d + n, n, c->stream) ||
      hipMemcpyAsync(out, d + n, sizeof(int64_t) * (size_t)n, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    rc = fail(c, KGPU_E_DEVICE, "broken-linear probe failed");
  (void)hipFree(d);
  return rc;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_get_filter(kgpu_ctx* c, uint32_t* words) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !words) return KGPU_E_INVAL;
  if (!c->last_diag) return fail(c, KGPU_E_STATE, "no kgpu_schedule_one cycle to report");
  HIP_OK(c, hipMemcpy(words, c->st.status, sizeof(uint32_t) * (size_t)c->st.N, hipMemcpyDeviceToHost));
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_get_filter_all(kgpu_ctx* c, uint32_t* words) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !words) return KGPU_E_INVAL;
  if (!c->last_diag || !c->last_run_all)
    return fail(c, KGPU_E_STATE, "no kgpu_schedule_one cycle under KGPU_OPT_RUN_ALL_FILTERS to report");
  const size_t nf = (size_t)c->cfg.n_filters, N = (size_t)c->st.N;
  if (nf * N) HIP_OK(c, hipMemcpy(words, c->st.status_all, sizeof(uint32_t) * nf * N, hipMemcpyDeviceToHost));
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_get_scores(kgpu_ctx* c, int32_t plugin, int64_t* raw, int64_t* normalized) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || plugin < 0 || plugin >= KGPU_NUM_SCORES) return KGPU_E_INVAL;
  if (!c->last_diag) return fail(c, KGPU_E_STATE, "no kgpu_schedule_one cycle to report");
  const size_t N = (size_t)c->st.N;
  if (raw) HIP_OK(c, hipMemcpy(raw, c->st.diag_raw + plugin * N, sizeof(int64_t) * N, hipMemcpyDeviceToHost));
  if (normalized)
    HIP_OK(c, hipMemcpy(normalized, c->st.diag_norm + plugin * N, sizeof(int64_t) * N, hipMemcpyDeviceToHost));
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_filter_reasons(kgpu_ctx* c, const kgpu_reason_args* a, char* buf, int64_t len, int64_t* bytes) try {
  if (!a || len < 0 || (a->n_taints > 0 && !a->taints) || a->n_taints < 0) return KGPU_E_INVAL;
  if (bytes) *bytes = 0;
  const uint32_t pos = a->word & 0xFFu;
  if (pos == 0 || a->word == KGPU_FS_NOT_EVALUATED) return 0;  // feasible / never examined: no status
  const int32_t nf = c ? c->cfg.n_filters : a->n_filters;
  const int32_t* fl = c ? c->cfg.filters : a->filters;
  if (!fl || (int32_t)pos > nf) return c ? fail(c, KGPU_E_INVAL, "status word names no filter of the profile") : KGPU_E_INVAL;
  kgpu::ScalarRead read;
  if (c) {
    read = [c, a](int32_t col, int64_t* alloc, int64_t* used) {
      if (!c->uploaded || a->node < 0 || a->node >= c->st.N || col < 0 || col >= c->st.S) return false;
      const size_t at = (size_t)col * (size_t)c->st.N + (size_t)a->node;
      return hipStreamSynchronize(c->stream) == hipSuccess &&
             hipMemcpy(alloc, c->st.alloc_scalar + at, 8, hipMemcpyDeviceToHost) == hipSuccess &&
             hipMemcpy(used, c->st.req_scalar + at, 8, hipMemcpyDeviceToHost) == hipSuccess;
    };
  }
  std::vector<std::string> rs;
  const int rc = kgpu::filter_reasons(fl[pos - 1], a->word, *a, read, &rs);
  if (rc != KGPU_OK) return c ? fail(c, rc, "status word cannot be formatted from these arguments") : rc;
  const int64_t need = kgpu::pack_reasons(rs, buf, len);
  if (bytes) *bytes = need;
  if (need > len) return KGPU_E_CAPACITY;
  return (int)rs.size();
} catch (...) {
  return on_exception(c, false);
}

int kgpu_read_nodes(kgpu_ctx* c, int64_t* req_cpu, int64_t* req_mem, int64_t* req_eph, int64_t* nz_cpu,
                    int64_t* nz_mem, int32_t* num_pods) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !c->uploaded) return KGPU_E_INVAL;
  SYNC_OK(c);
  const size_t N = (size_t)c->st.N;
  if (req_cpu) HIP_OK(c, hipMemcpy(req_cpu, c->st.req_cpu, 8 * N, hipMemcpyDeviceToHost));
  if (req_mem) HIP_OK(c, hipMemcpy(req_mem, c->st.req_mem, 8 * N, hipMemcpyDeviceToHost));
  if (req_eph) HIP_OK(c, hipMemcpy(req_eph, c->st.req_eph, 8 * N, hipMemcpyDeviceToHost));
  if (nz_cpu) HIP_OK(c, hipMemcpy(nz_cpu, c->st.nz_cpu, 8 * N, hipMemcpyDeviceToHost));
  if (nz_mem) HIP_OK(c, hipMemcpy(nz_mem, c->st.nz_mem, 8 * N, hipMemcpyDeviceToHost));
  if (num_pods) HIP_OK(c, hipMemcpy(num_pods, c->st.num_pods, 4 * N, hipMemcpyDeviceToHost));
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_forget_pod(kgpu_ctx* c, int32_t slot) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c) return KGPU_E_INVAL;
  if (!c->uploaded) return fail(c, KGPU_E_STATE, "no snapshot uploaded");
  if (slot < 0 || slot >= (int32_t)c->recs.size() || !c->recs[(size_t)slot].active)
    return fail(c, KGPU_E_INVAL, "no such pod slot");
  kgpu_ctx::PodRec& a = c->recs[(size_t)slot];
  if (!a.has_res)
    return fail(c, KGPU_E_UNSUPPORTED, "snapshot pod: remove it with a REMOVE_POD delta carrying the pod");
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  // NodeInfo.RemovePod (types.go:484-533) as one k_delta op over the stored resource record
  const int local = a.node - c->st.node_base;
  int rc = KGPU_OK;
  if (a.node >= 0 && local >= 0 && local < c->st.N) {
    kgpu_pod_query q = a.q;
    q.scalars = kgpu_range{0, (int32_t)a.sc.size()};
    q.ports = kgpu_range{0, (int32_t)a.ports.size()};
    DeltaBuild db;
    for (int32_t r : node_rows(c, local)) pod_op(c, db, kgpu::kDRemovePod, r, 0, slot);
    rc = launch_ops(c, db, &q, 1, nullptr, 0, nullptr, 0, nullptr, 0, a.sc.data(), (int)a.sc.size(), a.ports.data(),
                    (int)a.ports.size());
  }
  if (rc) {
    c->uploaded = false;
    return rc;
  }
  a.active = false;
  c->pod_rows[(size_t)slot].flags &= ~KGPU_PF_ACTIVE;
  pod_row_dirty(c, slot);
  if (a.has_uid) c->uid_slot.erase(a.uid);
  return KGPU_OK;
} catch (...) {
  return on_exception(c, true);
}

int kgpu_next_slot(const kgpu_ctx* c) { return c ? (int)std::min<size_t>(c->recs.size(), INT32_MAX) : -1; }

int kgpu_adopt_pod(kgpu_ctx* c, int32_t slot, int64_t uid) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c) return KGPU_E_INVAL;
  if (!c->uploaded) return fail(c, KGPU_E_STATE, "no snapshot uploaded");
  if (slot < 0 || slot >= (int32_t)c->recs.size() || !c->recs[(size_t)slot].active || !c->recs[(size_t)slot].has_res)
    return fail(c, KGPU_E_INVAL, "no pod assumed by kgpu_schedule_* at this slot");
  kgpu_ctx::PodRec& a = c->recs[(size_t)slot];
  if (a.has_uid && a.uid == uid) return KGPU_OK;
  auto it = c->uid_slot.find(uid);
  if (it != c->uid_slot.end()) return fail(c, KGPU_E_STATE, "the pod uid is already on a node");
  if (a.has_uid) c->uid_slot.erase(a.uid);
  a.uid = uid;
  a.has_uid = true;
  c->uid_slot.emplace(uid, slot);
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_prepare_pods(kgpu_ctx* c, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || n < 0 || (n > 0 && !qs)) return KGPU_E_INVAL;
  if (!c->uploaded) return fail(c, KGPU_E_STATE, "no snapshot uploaded");
  if (!topo_profile(c) || n == 0) return KGPU_OK;
  std::vector<kgpu::QPlan> plans;
  std::vector<int32_t> aux;
  std::vector<kgpu::TTerm> aux_terms;
  int64_t scratch = 0;
  kgpu_pools empty{};
  int rc = build_plans(c, qs, n, pools ? pools : &empty, plans, aux, aux_terms, &scratch);
  if (rc == KGPU_E_UNSUPPORTED) return KGPU_OK;  // such a pod's own cycle reports it
  if (rc) return rc;
  // the device scratch their plans need, allocated now rather than on a cycle
  if ((rc = ensure_grow(c, c->scratch, sizeof(int64_t) * (size_t)std::max<int64_t>(scratch, 1)))) return rc;
  c->st.scratch = static_cast<int64_t*>(c->scratch.p);
  return sync_classes(c);
} catch (...) {
  return on_exception(c, false);
}

int kgpu_apply_delta(kgpu_ctx* c, const kgpu_delta_batch* b, int64_t generation, int32_t* slots) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !b) return KGPU_E_INVAL;
  if (!c->uploaded) return fail(c, KGPU_E_STATE, "no snapshot uploaded");
  if (b->n_deltas < 0 || b->n_pods < 0 || b->n_rows < 0 || b->n_order < 0 || (b->n_deltas && !b->deltas) ||
      (b->n_pods && !b->pods) || (b->n_rows && !b->rows) || (b->n_order && !b->order))
    return fail(c, KGPU_E_INVAL, "malformed delta batch");
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  SYNC_OK(c);
  int rc = apply_delta(c, b, slots);
  if (!rc && c->comm) rc = sync_prefer_union(c);  // every rank applies the same batch
  if (rc) {
    // a half-applied batch leaves the mirror unlike any cache state
    c->uploaded = false;
    return rc;
  }
  c->generation = generation;
  return KGPU_OK;
} catch (...) {
  return on_exception(c, true);
}

// ---- node sharding over xGMI: the persistent kernel's granule exchange through peer stores
// Geometry every rank shares: the persistent layout of the largest shard.
static int xgmi_geometry(kgpu_ctx* c, int32_t nranks) {
  const int64_t nmax = ((int64_t)c->st.n_total + nranks - 1) / nranks;
  const int maxg = std::max(1, std::min(std::min(c->n_cus, 256), kgpu::kXgmiMaxGT / nranks));
  c->xg_geo = kgpu::batch_geometry((int)nmax, maxg, &c->xg_per, &c->xg_groups, c->batch_geo_first);
  c->xg_GT = nranks * c->xg_groups;
  return c->xg_geo;
}

int kgpu_xgmi_handle(kgpu_ctx* c, int32_t nranks, uint8_t handle[64]) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !handle || nranks < 2 || nranks > kgpu::kMaxRanks) return KGPU_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  if (!c->uploaded) return fail(c, KGPU_E_STATE, "upload this rank's shard before kgpu_xgmi_handle");
  int64_t maxs = 0;  // the granule key's score field is 20 bits wide in the ring layout
  for (int i = 0; i < c->cfg.n_scores; ++i) maxs += 100 * std::max<int64_t>(c->cfg.score_weights[i], 1);
  if (maxs + 1 >= (1 << 20)) return fail(c, KGPU_E_UNSUPPORTED, "score weights too large for the xGMI granule key");
  if (xgmi_geometry(c, nranks) < 0) return fail(c, KGPU_E_CAPACITY, "shard too large for the persistent kernel");
  const size_t cells = (size_t)kgpu::kXgmiRing * (size_t)c->xg_GT;
  for (void* q : c->xg_open)
    if (q) (void)hipIpcCloseMemHandle(q);
  c->xg_open.clear();
  if (c->xg_box.p) HIP_OK(c, hipFree(c->xg_box.p));
  c->xg_box = DevBuf{};
  // [granule ring | feasible-count ring | topology TX ring | init-reduction mailbox]
  auto up256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
  c->xg_tx_off = up256(cells * (sizeof(uint64_t) + sizeof(int32_t)));
  c->xg_init_off = up256(c->xg_tx_off + sizeof(uint64_t) * (size_t)kgpu::kTXRing * (size_t)kgpu::tx_row_words(nranks));
  const size_t box = c->xg_init_off + sizeof(int32_t) * 2 * (size_t)nranks * kgpu::kXInitCap +
                     sizeof(uint64_t) * 2 * (size_t)nranks;
  HIP_OK(c, hipMalloc(&c->xg_box.p, box));
  c->xg_box.bytes = box;
  // zeroed before any peer can learn the handle: no lap of the ring reads as valid
  HIP_OK(c, hipMemset(c->xg_box.p, 0, c->xg_box.bytes));
  HIP_OK(c, hipDeviceSynchronize());
  hipIpcMemHandle_t h;
  HIP_OK(c, hipIpcGetMemHandle(&h, c->xg_box.p));
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle exceeds the ABI's 64 bytes");
  std::memset(handle, 0, 64);
  std::memcpy(handle, &h, sizeof(h));
  c->xg_nranks = 0;  // not usable until kgpu_xgmi_init
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_xgmi_init(kgpu_ctx* c, int32_t nranks, int32_t rank, const uint8_t* handles) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !handles || nranks < 2 || nranks > kgpu::kMaxRanks || rank < 0 || rank >= nranks) return KGPU_E_INVAL;
  c->tc.valid = false;
  if (hipSetDevice(c->device) != hipSuccess) return KGPU_E_DEVICE;
  if (!c->xg_box.p || c->xg_GT != nranks * c->xg_groups)
    return fail(c, KGPU_E_STATE, "kgpu_xgmi_handle(nranks) must precede kgpu_xgmi_init");
  const size_t cells = (size_t)kgpu::kXgmiRing * (size_t)c->xg_GT;
  std::vector<void*> gr((size_t)nranks), fe((size_t)nranks), tx((size_t)nranks), xi((size_t)nranks);
  for (int r = 0; r < nranks; ++r) {
    void* base = nullptr;
    if (r == rank) {
      base = c->xg_box.p;
    } else {
      hipIpcMemHandle_t h;
      std::memcpy(&h, handles + 64 * (size_t)r, sizeof(h));
      HIP_OK(c, hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess));
      c->xg_open.push_back(base);
      // the peer's ring lives on its GPU: this device must reach it over the fabric
      hipPointerAttribute_t at{};
      HIP_OK(c, hipPointerGetAttributes(&at, base));
      if (at.device != c->device && at.device >= 0) {
        int can = 0;
        HIP_OK(c, hipDeviceCanAccessPeer(&can, c->device, at.device));
        if (!can) return fail(c, KGPU_E_UNSUPPORTED, "no peer access to a rank's GPU: per-pod RCCL exchange only");
        const hipError_t pe = hipDeviceEnablePeerAccess(at.device, 0);
        if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled)
          return fail(c, KGPU_E_UNSUPPORTED, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(pe));
        (void)hipGetLastError();
      }
    }
    gr[(size_t)r] = base;
    fe[(size_t)r] = static_cast<uint64_t*>(base) + cells;
    tx[(size_t)r] = static_cast<char*>(base) + c->xg_tx_off;
    xi[(size_t)r] = static_cast<char*>(base) + c->xg_init_off;
  }
  // device array: granule bases | feasible-count bases | TX ring bases | init mailbox bases
  std::vector<void*> arr(gr);
  arr.insert(arr.end(), fe.begin(), fe.end());
  arr.insert(arr.end(), tx.begin(), tx.end());
  arr.insert(arr.end(), xi.begin(), xi.end());
  int rc = ensure(c, c->xg_arr, sizeof(void*) * arr.size());
  if (rc) return rc;
  HIP_OK(c, hipMemcpy(c->xg_arr.p, arr.data(), sizeof(void*) * arr.size(), hipMemcpyHostToDevice));
  c->xg_nranks = nranks;
  c->xg_rank = rank;
  c->xg_seq = 0;
  c->xt_seq = 0;
  c->xr_seq = 0;
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_comm_unique_id(uint8_t id[128]) try {
  if (!id) return KGPU_E_INVAL;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  if (!rccl().ok) return KGPU_E_UNSUPPORTED;  // librccl could not be loaded
  ncclUniqueId u;
  if (rccl().GetUniqueId(&u) != ncclSuccess) return KGPU_E_DEVICE;
  std::memcpy(id, &u, 128);
  return KGPU_OK;
} catch (...) {
  return on_exception(nullptr, false);
}

int kgpu_comm_init(kgpu_ctx* c, int32_t nranks, int32_t rank, const uint8_t id[128]) try {
  if (c && !c->pipe_q.empty())
    return fail(c, KGPU_E_STATE, "pipelined batches in flight: complete them with kgpu_schedule_batch_wait first");
  if (c && c->unsettled) {  // a short cycle returned on its completion word: the stream first
    const int rs_ = settle(c);
    if (rs_) return rs_;
  }
  if (!c || !id) return KGPU_E_INVAL;
  c->tc.valid = false;
  if (nranks < 1 || nranks > kgpu::kMaxRanks || rank < 0 || rank >= nranks)
    return fail(c, KGPU_E_INVAL, "nranks must be in [1, 64] and 0 <= rank < nranks");
  if (c->comm) return fail(c, KGPU_E_STATE, "communicator already initialized");
  if (!c->uploaded) return fail(c, KGPU_E_STATE, "upload this rank's shard of the snapshot first");
  HIP_OK(c, hipSetDevice(c->device));
  ncclUniqueId u;
  std::memcpy(&u, id, 128);
  ncclComm_t comm = nullptr;
  if (!rccl().ok) return fail(c, KGPU_E_UNSUPPORTED, "librccl could not be loaded");
  const ncclResult_t r = rccl().CommInitRank(&comm, nranks, u, rank);
  if (r != ncclSuccess) return fail(c, KGPU_E_DEVICE, std::string("ncclCommInitRank: ") + rccl().GetErrorString(r));
  const size_t bytes = sizeof(BlkKey) + sizeof(BlkStat) + 2 * kgpu::kMaxRanks * (sizeof(BlkKey) + sizeof(BlkStat));
  int rc;
  if ((rc = ensure(c, c->shard, bytes))) {
    (void)rccl().CommDestroy(comm);
    return rc;
  }
  HIP_OK(c, hipMemset(c->shard.p, 0, bytes));
  char* b = static_cast<char*>(c->shard.p);
  c->st.shard_send_key = reinterpret_cast<BlkKey*>(b);
  c->st.shard_send_stat = reinterpret_cast<BlkStat*>(b + sizeof(BlkKey));
  c->st.shard_keys = reinterpret_cast<BlkKey*>(b + sizeof(BlkKey) + sizeof(BlkStat));
  c->st.shard_stats = reinterpret_cast<BlkStat*>(c->st.shard_keys + 2 * kgpu::kMaxRanks);
  c->st.nranks = nranks;
  c->comm = comm;
  c->nranks = nranks;
  c->rank = rank;
  if ((rc = sync_prefer_union(c))) return rc;
  if (nranks > 1 && c->xgmi) {
    // persistent runs exchange their granules through peer stores into every rank's mailbox; the
    // IPC handles travel over RCCL, and every rank takes the path only if every rank could map
    // every peer (the decision is an all-reduce MIN)
    std::vector<uint8_t> mine(64, 0), all((size_t)64 * nranks, 0);
    int ok = kgpu_xgmi_handle(c, nranks, mine.data()) == KGPU_OK ? 1 : 0;
    DevBuf tmp;
    if ((rc = ensure(c, tmp, 64 + 64 * (size_t)nranks + 64))) return rc;
    uint8_t* d = static_cast<uint8_t*>(tmp.p);
    HIP_OK(c, hipMemcpy(d, mine.data(), 64, hipMemcpyHostToDevice));
    ncclResult_t nr = rccl().AllGather(d, d + 64, 64, ncclUint8, comm, c->stream);
    if (nr == ncclSuccess) SYNC_OK(c);
    if (nr == ncclSuccess) HIP_OK(c, hipMemcpy(all.data(), d + 64, 64 * (size_t)nranks, hipMemcpyDeviceToHost));
    if (nr != ncclSuccess) ok = 0;
    if (ok && kgpu_xgmi_init(c, nranks, rank, all.data()) != KGPU_OK) ok = 0;
    int32_t* flag = reinterpret_cast<int32_t*>(d + 64 + 64 * (size_t)nranks);
    HIP_OK(c, hipMemcpy(flag, &ok, sizeof(int32_t), hipMemcpyHostToDevice));
    nr = rccl().AllReduce(flag, flag, 1, ncclInt32, ncclMin, comm, c->stream);
    if (nr == ncclSuccess) SYNC_OK(c);
    int32_t all_ok = 0;
    if (nr == ncclSuccess) HIP_OK(c, hipMemcpy(&all_ok, flag, sizeof(int32_t), hipMemcpyDeviceToHost));
    (void)hipFree(tmp.p);
    if (!all_ok) c->xg_nranks = 0;  // per-pod RCCL exchange only
    c->err.clear();
  }
  return KGPU_OK;
} catch (...) {
  return on_exception(c, false);
}

int kgpu_xgmi_active(const kgpu_ctx* c) { return c && c->xg_nranks > 1 && c->xgmi ? 1 : 0; }

int kgpu_comm_info(const kgpu_ctx* c, int32_t out[4]) try {
  if (!c || !out) return KGPU_E_INVAL;
  out[0] = out[1] = out[2] = out[3] = 0;
  if (c->comm) {
    int n = 0, r = 0;
    if (rccl().CommCount && rccl().CommCount(c->comm, &n) == ncclSuccess) out[0] = n;
    if (rccl().CommUserRank && rccl().CommUserRank(c->comm, &r) == ncclSuccess) out[1] = r;
  }
  if (c->xg_nranks > 1 && c->xgmi) {
    out[2] = c->xg_nranks;
    int32_t mapped = 0;
    for (void* p : c->xg_open) mapped += p != nullptr;
    out[3] = mapped;
  }
  return KGPU_OK;
} catch (...) {
  return on_exception(nullptr, false);
}

int kgpu_debug_fail_alloc(int32_t countdown) {
  g_fail_alloc.store(countdown > 0 ? countdown : 0, std::memory_order_relaxed);
  return KGPU_OK;
}

}  // extern "C"
