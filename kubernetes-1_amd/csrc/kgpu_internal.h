// Internal layout shared by the host runtime (kgpu_api.cpp) and the CDNA4 kernels
// (kgpu_kernels.hip).  Not part of the ABI.
#pragma once
#include <stdint.h>

#include "../../include/kgpu.h"

namespace kgpu {

constexpr int kBlock = 64;         // threads per node-evaluation workgroup: one wave64
constexpr int kMaxBlocks = 1024;   // cap so that the fused winner resolution stays cheap
constexpr int kSelAnd = 0, kSelNothing = 1, kSelEmpty = 2;
constexpr uint64_t kMask40 = (1ull << 40) - 1;

// Per-workgroup partial of the node-evaluation kernel for one pod.
struct BlkStat {
  int32_t feasible;     // feasible nodes in the block
  int32_t max_taint;    // max raw TaintToleration score over feasible nodes
  int32_t max_na;       // max raw NodeAffinity score over feasible nodes
  int32_t pad;
};
struct BlkKey {
  uint64_t key;         // packed (score << 40 | rank40), 0 = no feasible node
  int32_t idx;          // local node index of the key
  int32_t feasible;
};

struct DevPools {
  const kgpu_req* reqs;
  const int32_t* ints;
  const uint64_t* words;
  const kgpu_node_term* node_terms;
  const kgpu_pref_term* pref_terms;
  const kgpu_spread* spreads;
  const kgpu_pod_term* pod_terms;
  const kgpu_scalar_req* scalars;
  const kgpu_port* ports;
};

// Everything a kernel needs, passed by value (well under the 4 KiB kernel-argument limit).
struct DevState {
  // ---- geometry
  int32_t N;            // local nodes
  int32_t node_base;    // global index of local node 0
  int32_t n_total;      // global node count
  int32_t S, K, TW, PS; // scalar columns, node label keys, taint words, port slots
  int32_t n_zones;
  // ---- node SoA (Snapshot.List() order)
  int64_t *alloc_cpu, *alloc_mem, *alloc_eph;
  int32_t* alloc_pods;
  int64_t *req_cpu, *req_mem, *req_eph, *nz_cpu, *nz_mem;
  int32_t* num_pods;
  int64_t *alloc_scalar, *req_scalar;   // [S][N]
  uint8_t* unsched;
  int32_t* label_val;                   // [K][N]
  int32_t* key_n_values;
  int32_t* value_off;
  int64_t* value_int;
  uint8_t* value_int_ok;
  int32_t* key_empty_value;
  uint64_t *taint_nosched, *taint_prefer; // [TW][N]
  int32_t* port_count;
  kgpu_port* ports;                     // [PS][N]
  int32_t *image_off, *image_id;
  int64_t* image_score;
  int32_t *avoid_off, *avoid_id;
  int32_t* zone_id;
  // ---- queries of the current batch
  const kgpu_pod_query* queries;
  DevPools qp;
  // ---- profile
  int32_t n_filters;
  int32_t filters[KGPU_NUM_FILTERS];
  int32_t n_scores;
  int32_t scores[KGPU_NUM_SCORES];
  int64_t weights[KGPU_NUM_SCORES];     // by profile position
  int64_t w_of[KGPU_NUM_SCORES];        // by plugin id, 0 = plugin not in the profile
  int32_t n_least, n_most;
  kgpu_resource_weight least[8], most[8];
  int64_t least_wsum, most_wsum;
  int32_t tie_mode;
  int32_t pad0;
  uint64_t seed;
  int32_t any_prefer_taint;             // some node carries a PreferNoSchedule taint
  int32_t pad1;
  // ---- work buffers
  uint32_t* status;                     // [N] filter status word (diagnostics / two-pass)
  int32_t* raw_taint;                   // [N]
  int32_t* raw_na;                      // [N]
  int64_t* partial;                     // [N] weighted sum of the non-normalized plugins
  BlkStat* sbuf;                        // [2][kMaxBlocks]
  BlkKey* kbuf;                         // [2][kMaxBlocks]
  kgpu_result* results;                 // [batch capacity]
  int64_t* diag_raw;                    // [KGPU_NUM_SCORES][N] or null
  int64_t* diag_norm;                   // [KGPU_NUM_SCORES][N] or null
};

// Per-launch parameters.
struct PodArgs {
  int32_t pod;          // query index in the batch (-1: resolve only)
  int32_t prev;         // pod whose winner is resolved (and assumed) at kernel start, -1 none
  int32_t prev_blocks;  // number of BlkKey partials of `prev`
  int32_t prev_parity;
  int32_t parity;       // buffer half for this pod's partials
  int32_t norm;         // 1: this pod needs the normalize pass (keys come from k_final)
  int32_t assume;       // apply NodeInfo.AddPod for resolved winners
  int32_t diag;         // write per-plugin raw/normalized scores
  int64_t seq;          // tie-break sequence number of `pod`
};

// Persistent batch launch: a run of `count` pods (queries first..first+count-1) in one kernel.
struct BatchArgs {
  int32_t first;        // first query index of the run
  int32_t count;        // pods in the run
  int32_t per;          // nodes owned by one workgroup
  int32_t assume;
  int64_t seq0;         // tie-break sequence number of query `first`
  uint64_t* gran;       // [count][groups] granules, zeroed before the launch
  int32_t* feas;        // [count][groups] feasible count of each published variant
  int32_t* abort;       // raised (1) by a workgroup that lost co-residency; zeroed before the launch
  int64_t* trace;       // null, or [count + 1][16] s_memrealtime stamps, 8 per traced workgroup
                        // (0 and last): iteration start, evaluated, previous pod resolved,
                        // granule published, iteration end
};

// Host-side launchers (kgpu_kernels.hip).
// The DevState lives in device memory (one copy per batch): kernel arguments stay at 40 bytes,
// so no launch pulls a kilobyte of kernarg segment through the host-coherent path.
int launch_eval(const DevState* st, const PodArgs& a, int blocks, int spec, void* stream);
// Kernel instantiation for a profile: 0 = generic list-walking kernel, else a straight-line one.
int select_spec(const int32_t* filters, int nf, const int32_t* scores, int ns, bool def_res);
int launch_final(const DevState* st, const PodArgs& a, int blocks, int stat_blocks, void* stream);
int launch_resolve(const DevState* st, int N, const PodArgs& a, void* stream);
int eval_blocks(int N);
// Geometry index (workgroup size x rows per lane) and grid of the persistent kernel, -1 when N
// does not fit in max_groups workgroups.
int batch_geometry(int N, int max_groups, int* per, int* groups);
int launch_batch(const DevState* st, const BatchArgs& a, int groups, int kidx, int spec, void* stream);

}  // namespace kgpu
