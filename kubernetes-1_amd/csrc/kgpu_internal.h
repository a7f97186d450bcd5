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
constexpr int kMaxRanks = 64;      // node shards (one per GPU) combined per pod

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

// ---------------------------------------------------------------- topology plugins
// PodTopologySpread / InterPodAffinity / DefaultPodTopologySpread run on device-resident
// per-node match counts instead of re-walking every existing pod per incoming pod:
//   mcnt[c][n]  = existing pods on node n matching pod class c (namespace set + label selector(s),
//                 optionally excluding terminating pods) -- one class per distinct spread
//                 selector / incoming pod term / DefaultPodTopologySpread selector;
//   tcnt[t][n]  = existing pods on node n carrying term class t (kind, weight, topology key,
//                 namespaces, selector) -- the existing pods' (anti-)affinity terms.
// The host interns classes by content (kgpu_api.cpp), initializes new columns on the device from
// the pod table (k_class_init), and every assume increments the columns of the classes the pod
// matches and of the term classes it owns.  Per incoming pod the domain histograms
// (topologyPair -> count) are rebuilt from these columns in one pass over the nodes.
constexpr int kMaxSpread = 4;   // spread constraints per kind (DoNotSchedule / ScheduleAnyway)
constexpr int kMaxIpa = 4;      // required (anti-)affinity terms per kind
constexpr int kMaxPref = 8;     // preferred terms (affinity + anti-affinity)
constexpr int kMaxSlots = 24;   // domain histograms per pod

// A pod class item: pod in `ns` (int32 ids in the class pool) and matching `sel` (class pool reqs).
struct ClassItem {
  kgpu_range ns;
  kgpu_selector sel;
};
struct ClassRec {
  int32_t item0, n_items;  // ANDed items (podMatchesAllAffinityTerms uses several)
  int32_t excl_terminating;
  int32_t pad;
};
struct TermClassRec {
  int32_t kind, weight, topo_key, pad;
  ClassItem item;
};

struct TSpread {
  int32_t cls, key, rslot, cslot;        // class, node label key, registration / count histogram slots
  int32_t max_skew, self_match, is_hostname, first_of_key;
};
struct TTerm {
  int32_t cls, key, slot, weight;        // class (or term class), node label key, histogram slot, weight
};

// Per-query plan built by the host at batch start (not part of the ABI).
struct QPlan {
  int32_t topo;              // 1: the pod takes the topology pipeline
  int32_t n_hard, n_soft;
  int32_t dpts_cls;          // -1: no DefaultPodTopologySpread counts (empty selector), -2: pod has TSC
  TSpread hard[kMaxSpread];
  TSpread soft[kMaxSpread];
  int32_t n_aff, conj_cls, n_anti, n_pref;
  int32_t self_all;          // podMatchesAllAffinityTerms(pod, RequiredAffinityTerms)
  int32_t pad0;
  TTerm aff[kMaxIpa];
  TTerm anti[kMaxIpa];
  TTerm pref[kMaxPref];
  kgpu_range ex;             // TTerm aux pool: existing term classes matching this pod
  int32_t n_ex_anti;         // the first n_ex_anti of ex are required anti-affinity (EXA slots)
  int32_t n_slots;
  kgpu_range assume_cls;     // int aux pool: classes this pod matches (mcnt increments on assume)
  kgpu_range own_tcls;       // int aux pool: term classes this pod owns (tcnt increments on assume)
  int32_t slot_key[kMaxSlots];
  int32_t slot_kind[kMaxSlots];
  int64_t slot_off[kMaxSlots];  // int64 offsets into the pod's scratch
  int64_t scratch_len;       // int64 words (header + zone sums + slots)
};
enum SlotKind { kSlotPReg = 0, kSlotPCnt, kSlotSReg, kSlotSCnt, kSlotExA, kSlotAff, kSlotAnti, kSlotTopo };

// Scratch header of one topology pod (zeroed before its first kernel).
struct TopoHdr {
  int64_t pmin[kMaxSpread];   // critical-path minimum per hard constraint
  int64_t ssize[kMaxSpread];  // topology size per soft constraint (first constraint of its key)
  int64_t pts_min, pts_max, ipa_min, ipa_max, dpts_max;
  int32_t pany, aff_any, ex_any, topo_any;
  int32_t feas_nonign, have_zones, done1, done2;
  int32_t pmin_set, pad[3];
};
constexpr int kHdrWords = (int)(sizeof(TopoHdr) / 8);

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
  int32_t n_rtcr, n_shape;               // RequestedToCapacityRatio
  kgpu_resource_weight rtcr[8];
  kgpu_shape_point shape[16];
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
  // ---- topology plugins
  const QPlan* plans;                   // [batch] per-query plans (null: no topology state)
  const int32_t* aux;                   // int aux pool of the plans
  const TTerm* aux_terms;               // TTerm aux pool of the plans
  int32_t* mcnt;                        // [Ccap][N]
  int32_t* tcnt;                        // [TCcap][N]
  const ClassRec* classes;
  const ClassItem* class_items;
  const TermClassRec* tclasses;
  const kgpu_req* creqs;                // class pool
  const int32_t* cints;
  int32_t* key_empty;                   // == key_empty_value
  double* log_table;                    // [n_total + 3] math.Log(x) for x = 0..n_total+2
  int64_t* scratch;                     // per-pod topology scratch
  int64_t* raw_pts;                     // [N] (INT64_MIN = ignored node)
  int64_t* raw_ipa;                     // [N]
  int64_t* raw_dpts;                    // [N]
  int32_t hard_pod_affinity_weight;
  int32_t pad2;
  // pod table (existing + assumed pods) for class initialization
  int32_t* pod_node;                    // [Pcap] global node index
  int32_t* pod_ns;
  uint32_t* pod_flags;
  int32_t* pod_lab;                     // [PKcap][Pcap]
  int32_t Pcap, PKcap;
  // ---- node sharding (null / 0 when unsharded).  Per pod every rank packs its shard's winner
  // (BlkKey with a GLOBAL node index) and its normalize maxima (BlkStat) into shard_send; an RCCL
  // all-gather fills shard_keys / shard_stats [2 parities][kMaxRanks], which the next launch
  // resolves exactly like the per-workgroup partials of an unsharded launch.
  BlkKey* shard_send_key;
  BlkStat* shard_send_stat;
  BlkKey* shard_keys;
  BlkStat* shard_stats;
  int32_t nranks;
  // ---- percentageOfNodesToScore (generic_scheduler.go:379-399,424-495): to_find =
  // numFeasibleNodesToFind(n_total); cut_state[0] = nextStartNodeIndex, cut_state[1] = the last cut
  // pod's EvaluatedNodes (len(filtered) + len(statuses)).  cut_state is null when to_find == N.
  int32_t to_find;
  int32_t* cut_state;
  int32_t* port_overflow;               // set by assume / delta when a node's host-port slots run out
  // ---- nominated pods (kgpu_set_nominated): pass-1 status word per node (0: pass 1 succeeded or the
  // node has no nominated pods); k_eval / k_topo_filter report it instead of their own verdict.
  // Null when the nominator is empty.
  const uint32_t* nom_status;
  // zeroed word: k_final's last workgroup ticket when it resolves its own pod (PodArgs.resolve_self)
  int32_t* ticket;
  // ---- runAllFilters (framework.go:90,494; KGPU_OPT_RUN_ALL_FILTERS): a diagnostic cycle runs every
  // filter plugin on every node, status[n] becomes PluginToStatus.Merge's word (the first failing
  // plugin's position and detail, the merged code) and status_all[i][n] the i-th plugin's own word
  uint32_t* status_all;                 // [KGPU_NUM_FILTERS][N]
  int32_t run_all;
  int32_t pad3;
};
// Filter status word of a node the cycle never examined (findNodesThatPassFilters stopped before
// it), or of the feasible node whose discovery cancelled the search: not in `filtered` and not in
// the statuses map.
constexpr uint32_t kStatusNotEvaluated = 0xFFu;

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
  int32_t cut;          // 1: numFeasibleNodesToFind < N -- k_cut trims the feasible set (R2)
  int32_t zero_diag;    // 1: k_eval zeroes every node's diag rows itself (no memset launches)
  int32_t resolve_self; // 1: k_final's last workgroup resolves and assumes `pod` (no k_resolve launch)
  int32_t q_inline;     // 1: `pod`'s query is `q` below (a one-pod cycle: no query upload)
  int64_t seq;          // tie-break sequence number of `pod`
  int32_t* done_out;    // null, or (resolve_self) the pinned host word the resolving workgroup sets to 0 once
                        // every store of the cycle is written back: the host returns on it without waiting
                        // for the stream's completion signal (~8 us later, profiles/r05_host_trace.txt)
  kgpu_pod_query q;
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
  int32_t* abort;       // zeroed before the launch; OR-ed by a workgroup whose spin gave up: 2 (kAbortClean)
                        // before the run resolved any pod -- no device state changed, the call may be
                        // issued again -- else 1
  int64_t* trace;        // null, or [count + 1][16] s_memrealtime stamps, 8 per traced workgroup
                        // (0 and last): iteration start, evaluated, previous pod resolved,
                        // granule published, iteration end
  int32_t abort_at;     // KGPU_OPT_ABORT_AT test hook: workgroup 0 raises the abort word at this
                        // iteration (-1: never)
  int32_t skip_release_at;  // KGPU_OPT_SKIP_RELEASE_AT test hook: at this iteration the candidate lane
                            // stages its row but never releases the hand-off, so the next pod's LDS
                            // wait times out (-1: never)
  int32_t hold;         // KGPU_OPT_HOLD_GROUP test hook: this workgroup leaves at once (an ordinary launch
                        // whose workgroup never became resident; -1: none)
  int32_t pad_h;
  // pipelined batches (kgpu_schedule_batch_submit): k_batch_fixup also writes every record into pinned host
  // memory (res_out), copies the run's abort word there (abort_out), and zeroes the other pipeline slot's
  // granule area for the batch after next (zero_buf, zero_n16 16-byte words); all null / 0 otherwise
  kgpu_result* res_out;
  int32_t* abort_out;
  uint64_t* zero_buf;
  int64_t zero_n16;
  // Node sharding over xGMI (kgpu_xgmi_init): every workgroup of every rank publishes its granule
  // and feasible count into every rank's mailbox ring; each rank polls its own.  Unsharded:
  // nranks 1, pgran[0] = gran, pfeas[0] = feas, GT = groups, R = 0 (rows are this launch's pods,
  // zeroed before it).  With R > 0, pod i sits on ring row (xseq0 + i) % R and its granules carry
  // the ring lap (xseq0 + i) / R mod 8 in bits 60-62, so rows of an earlier lap never read as
  // valid and no rank has to clear another's mailbox.
  uint64_t* const* pgran;  // [nranks] granule ring bases (this rank's own at [rank] == gran)
  int32_t* const* pfeas;   // [nranks] feasible-count ring bases
  int32_t nranks, rank;
  int32_t GT;              // granules per pod row: nranks * groups
  int32_t R;               // ring rows, 0 = linear rows
  int64_t xseq0;
};
// abort word codes (OR-ed): a spin gave up before the run resolved its first pod (nothing on the device
// changed) / after it
constexpr int32_t kAbortDirty = 1, kAbortClean = 2;
constexpr int kXgmiRing = 4096;      // mailbox ring rows (a persistent run holds at most half)
constexpr int kXgmiMaxGT = 1024;     // granules per row the poll sweeps (16 per lane)

// ---------------------------------------------------------------- persistent topology kernel
// k_tbatch schedules a run of PodTopologySpread / InterPodAffinity / DefaultPodTopologySpread pods
// inside ONE launch.  Every topologyPair -> count map those plugins build per cycle is a
// pod-independent DOMAIN HISTOGRAM of a match-count column: H[col][key][v] = sum over the nodes
// whose label `key` has value v of col[n] (col = a pod class of mcnt or a term class of tcnt;
// bin D = nodes without the key), optionally restricted to the nodes a pod's NodeAffinity admits
// (PodTopologySpread's ScheduleAnyway counts).  Histograms over keys with few values live in LDS,
// one replica per workgroup, and every workgroup applies the same +1 deltas after each winner;
// keys whose every value sits on at most one node (hostname-like) need no histogram: the owner
// lane reads the node's own column.  Per pod: one pass over the register-resident node rows
// (filters + raw scores), one granule round for the normalize statistics, one for selectHost.
constexpr int kTMaxSoftWords = 8;   // shared ScheduleAnyway key: <= 256 domains (OR-ed bitmask)
constexpr int kTMaxZones = 32;      // DefaultPodTopologySpread zone sums carried in the stats round
constexpr int kTLdsBudget = 144 * 1024;

struct THist {
  int32_t col_kind;  // 0: mcnt pod class, 1: tcnt term class
  int32_t col;
  int32_t key;       // node label key
  int32_t sig;       // -1: all nodes; else eligibility signature (TSig) the counted nodes must pass
  int32_t D;         // distinct values of key (bins 0..D-1, bin D = key missing)
  int32_t off;       // first LDS bin, -1: node-unique key (lookups read the node's own column)
};
struct TSig {
  int32_t rep;       // query index whose nodeSelector / required NodeAffinity defines the signature
  int32_t n_keys;
  int32_t keys[kMaxSpread];
  int32_t elig_word; // first uint32 word of this signature's node bitmap in TBatchArgs::elig
  int32_t pad;
};
struct TReg {        // registered topology pairs of (signature, key): D-bit mask in LDS
  int32_t sig, key, D, word;
};
struct TLook {       // one lookup H[col][key][label(key, n)]: LDS bins at `off`, or (off < 0, node-unique
                     // key) the node's own column col of mcnt (col_kind 0) / tcnt (1)
  int32_t key, weight, off, D;
  int32_t col_kind, col, pad0, pad1;
};
// A per-pod lookup table over the values of one key, built in LDS before the pod's node pass
// (int64 entries at `off`): kind 0 = TpPairToMatchNum of a DoNotSchedule key (sum over the
// constraints on the key, 0 for unregistered pairs; `reg` = TReg), 1 = existing pods' required
// anti-affinity counts of the key, 2 = InterPodAffinity topologyScore[key][*].
struct TTab {
  int32_t kind, key, D, off;
  int32_t reg, empty_v;
  kgpu_range terms;  // TLook aux (shared-key histograms only)
};
struct THard {
  int32_t key, max_skew, self_match, tab;  // tab: index of the key's kind-0 table in the pod's tabs
  int32_t pt_off, pad0;                    // that table's first entry
};
struct TDelta {      // one histogram a pod increments when assumed
  int32_t hist, off, D, key;
  int32_t sig, pad0, pad1, pad2;
};
struct TPlan {
  int32_t n_hard, hard_sig;
  THard hard[kMaxSpread];
  int32_t n_soft;     // 0 or 1
  int32_t soft_mode;  // 0 shared key (LDS histogram, topoSize = registered domains),
                      // 1 kubernetes.io/hostname (count = the node's own column, topoSize = nodes),
                      // 2 node-unique key (own column if the node is eligible, topoSize = nodes)
  int32_t soft_off, soft_col, soft_key, soft_max_skew, soft_sig, soft_words;
  int32_t n_aff, self_all;
  TLook aff[kMaxIpa];
  int32_t n_anti, dpts_cls;
  TLook anti[kMaxIpa];
  int32_t aff_hist[kMaxIpa];  // THist index of each affinity term (TOT: the map is non-empty)
  kgpu_range tabs;    // TTab aux
  int32_t pt_words, n_exa_tabs;  // int64 words of the pod's tables; order: kind 0, kind 2, then the
                                 // n_exa_tabs kind-1 tables
  kgpu_range exa_u;   // TLook aux: required anti-affinity terms of existing pods on node-unique keys
  kgpu_range score_u; // TLook aux: InterPodAffinity score terms on node-unique keys
  kgpu_range deltas;  // TDelta aux: histograms this pod increments when assumed
  kgpu_range assume_cls, own_tcls;  // int aux: mcnt / tcnt columns this pod increments
  int32_t need_ipa;
  int32_t aff_sig;    // TSig of PodMatchesNodeSelectorAndAffinityTerms alone: the NodeAffinity filter
};
// statistics slots of the normalize round (values are 63-bit encoded, see k_tbatch)
enum TStat { kTFeas = 0, kTMaxT, kTMaxNA, kTNonIgn, kTAdjMin, kTAdjMax, kTIpaMin, kTIpaMax, kTDptsMax, kTZoned, kTFixed };
constexpr int kTMaxTabs = 16;  // per-pod lookup tables
struct TBatchArgs {
  int32_t first, count;   // query range of the run
  int32_t per;            // nodes owned by one workgroup
  int32_t assume;
  int64_t seq0;
  const TPlan* plans;     // distinct plans of the run
  const int32_t* plan_of; // [count] plan of each pod
  const int32_t* aux;
  const TLook* looks;
  const TTab* tabs;
  const TDelta* deltas;
  const THist* hists;
  int32_t n_hists, n_sigs, n_regs;
  int32_t lds_bins;       // LDS histogram bins
  int32_t reg_words;
  int32_t R;              // stats slots per pod (kTFixed + soft words + zones)
  int32_t soft_words, zones;
  const TSig* sigs;
  const TReg* regs;
  int32_t* hist_init;     // [lds_bins] zeroed, filled by k_tbatch_init
  int32_t* tot_init;      // [n_hists]
  uint32_t* reg_init;     // [reg_words]
  int32_t* sig_any;       // [n_sigs]
  uint32_t* elig;         // [n_sigs][ceil(N/32)]
  uint64_t* gran;         // per pod: [R][groups] statistics granules, then [groups] key granules; zeroed
  int32_t* abort;
  int32_t* done;          // null, or a zeroed counter of workgroups that left the pod loop ...
  int32_t* abort_out;     // ... and the pinned host word the last of them copies the abort word into
                          // (a short cycle reads it after its stream synchronize: no read-back copy)
  int32_t lds_bytes;
  int32_t def_res;        // Least/Most over {cpu: 1, memory: 1}
  int32_t pt_words;       // largest per-pod table area of the run (int64 words)
  int32_t n_keys;         // node label keys the run's deltas read (winner's labels staged in LDS)
  // byte offsets of the LDS regions (histogram bins start at 0)
  int32_t o_reg, o_tot, o_sany, o_stat, o_smask, o_zsum, o_misc, o_pt, o_lab;
  int32_t lab_keys;       // node label keys cached in LDS per workgroup ([lab_keys][per] value ids)
  int32_t wlab;           // 1: every node's values of the n_keys keys in LDS at o_wlab ([n_keys][N]): the assume
                          // phase reads the winner's labels there instead of a dependent global load
  int32_t o_wlab;
  int32_t abort_at;       // KGPU_OPT_ABORT_AT test hook (-1: never), as in BatchArgs
  int32_t diag;           // kgpu_schedule_one: status word and per-plugin raw / normalized scores of every
                          // node (the run is one pod; every lane zeroes its nodes' diagnostic rows first)
  int32_t ahead;          // evaluate the next pod's non-topology half during the exchanges (KGPU_OPT_TOPO_AHEAD)
  int32_t writeback;      // workgroup 0 stores its final histogram bins and totals back into hist_init /
                          // tot_init: the next run with the same tables starts from them without a
                          // k_tbatch_init pass (kgpu_api.cpp TCache)
  int32_t zero_n16;       // the other resident-state buffer: its first zero_n16 16-byte words are zeroed by
                          // the grid at kernel entry, so the next miss starts from zeros without a memset
  int32_t hold;           // KGPU_OPT_HOLD_GROUP test hook, as in BatchArgs
  int32_t poll_sleep;     // 1: a short sleep between statistics sweeps (KGPU_OPT_TBATCH_POLL_SLEEP)
  int32_t trace_mode;     // KGPU_OPT_PHASE_TRACE value: 2 moves stamps 1 / 2 into the normalize phase
  struct alignas(16) Z16 { uint64_t lo, hi; };
  Z16* zero_buf;
  int64_t* trace;        // null, or [count + 1][16] s_memrealtime stamps (KGPU_OPT_PHASE_TRACE): per pod
                          // and traced workgroup (0, last): start, PreFilter minima, rows evaluated,
                          // stats published, stats resolved, key published, winner resolved, end
  int64_t* trace_wg;      // null, or [count][groups][8] stamps of EVERY workgroup (thread 0): pod start,
                          // rows done (wave 0), statistics published, key published, every wave's
                          // statistics reduced (barrier), statistics received, winner received
  // ---- node sharding over xGMI (the XG instantiation; kgpu_xgmi_init).  Each rank runs the local
  // protocol above over its own shard, then one record per rank crosses the ranks through the
  // topology mailbox ring (TX row, below): its combined statistics (published by workgroup 0) and its
  // best key with the winning node's label values and signature bits (published by the rank's local
  // winner, info before key).  Every workgroup of every rank combines the nranks records itself.
  // Pod i sits on ring row (xseq0 + i) % kTXRing; records carry the lap in bits 60-62.
  uint64_t* const* ptx;   // [nranks] TX ring bases (this rank's own at [rank])
  int32_t nranks, rank;
  int64_t xseq0;
};

// TX row of the topology mailbox ring, in u64 words: stats [nranks][kTXRCap] | keys [nranks] |
// info [nranks][kTXInfo / 2] (int32: the winner's value of each of the first 64 node label keys, then
// two words of signature bits).  Stats records are biased by kTXBias into bits 0-59.
constexpr int kTXRing = 8;
constexpr int kTXRCap = 64;          // >= kTFixed + kTMaxSoftWords + kTMaxZones
constexpr int kTXInfo = 68;          // int32 per info record (64 label values + 2 signature words + pad)
constexpr int64_t kTXBias = 1ll << 58;
constexpr int64_t tx_row_words(int nranks) { return (int64_t)nranks * (kTXRCap + 1 + kTXInfo / 2); }
// Cross-rank reduction of a run's histogram initialization (k_xput / k_xflag / k_xsum): words
// [0, n_sum) are summed over the ranks, [n_sum, n_sum + n_or) OR-ed.  Per rank the init mailbox holds
// [2 parities][nranks][kXInitCap] int32 partials, then [2][nranks] u64 arrival flags (sequence numbers).
constexpr int kXInitCap = 40960;
struct XReduce {
  int32_t* const* pinit;  // [nranks] init mailbox bases (own at [rank])
  int32_t nranks, rank, parity, pad;
  uint64_t seq;           // identical on every rank: the flag value of this reduction
  int32_t* buf;           // local partials in, reduced values out
  int32_t n_sum, n_or;
  int32_t* abort;
};
int launch_xreduce(const XReduce& x, void* stream);

// ---------------------------------------------------------------- nominated pods / preemption
// One pod added to (nominated, pass 1) or removed from (potential victim) a node, resolved against
// the pod being scheduled on the host (kgpu_api.cpp build_effect).  Its requests and host ports
// come from its record (PreemptArgs::v_recs / n_recs [item]).
struct PEff {
  int32_t item;
  uint32_t pts_mask;   // bit i: PodTopologySpread updateWithPod counts it for DoNotSchedule constraint i
                       // (same namespace, selector matches; filtering.go:123-143)
  uint32_t anti_mask;  // bit i: matches the pod's required anti-affinity term i (filtering.go:133-148)
  int32_t aff_all;     // matches all of the pod's required affinity terms (filtering.go:115-129)
  kgpu_range exa;      // aux ints: topology keys of its own required anti-affinity terms that match the pod
  int32_t prio;
  int32_t pad;
  int64_t start;
  uint64_t pdb_mask;
};
struct PreemptArgs {
  int32_t pod;              // query index of the pod being scheduled
  int32_t preempt;          // 1: selectVictimsOnNode, 0: nominated pass 1 only (writes nom_status)
  const int32_t* v_off;     // [N+1] victims of local node n: veff[v_off[n] .. v_off[n+1]), MoreImportantPod order
  const PEff* veff;
  const int32_t* n_off;     // [N+1] nominated pods added in pass 1 (priority >= the pod's, other UID)
  const PEff* neff;
  const kgpu_pod_query* v_recs;   // victim records and their pools (kgpu_preempt_args::pods)
  const kgpu_scalar_req* v_scalars;
  const kgpu_port* v_ports;
  const kgpu_pod_query* n_recs;   // nominated pod records and their pools (kgpu_set_nominated)
  const kgpu_scalar_req* n_scalars;
  const kgpu_port* n_ports;
  const int32_t* aux;
  int32_t n_pdbs;
  int32_t pad;
  const int32_t* pdb_allowed;
  uint8_t* vstate;          // [victims] 0 removed, 1 kept, 2 evicted
  int32_t* order;           // [victims] reprieve order (positions), per node range
  kgpu_node_victims* out;   // [N]
  int32_t* out_victims;     // [victims]
  int64_t* prep;            // k_vict_prep: per DoNotSchedule constraint {min, argmin, second min}, then the
                            // number of non-zero affinity-map entries (len(topologyToMatchedAffinityTerms))
  uint32_t* nom_status;     // [N] pass-1 status words (nominated pass)
};
constexpr int kPrepWords = 3 * kMaxSpread + 1;
int launch_vict_prep(const DevState* st, const PreemptArgs* a, void* stream);
int launch_victims(const DevState* st, const PreemptArgs* a, int N, void* stream);

// Host-side launchers (kgpu_kernels.hip).
// The DevState lives in device memory (one copy per batch): kernel arguments stay at 40 bytes,
// so no launch pulls a kilobyte of kernarg segment through the host-coherent path.
int launch_eval(const DevState* st, const PodArgs& a, int blocks, int spec, void* stream);
// Kernel instantiation for a profile: 0 = generic list-walking kernel, else a straight-line one.
int select_spec(const int32_t* filters, int nf, const int32_t* scores, int ns, bool def_res);
int launch_final(const DevState* st, const PodArgs& a, int blocks, int stat_blocks, void* stream);
// findNodesThatPassFilters' stopping rule over the evaluated status words: keep the first
// to_find feasible nodes from nextStartNodeIndex on (rotated order), mark the rest
// kStatusNotEvaluated, advance nextStartNodeIndex, write the kept set's normalize stats into
// sbuf[parity] (slot 0; slots 1..blocks-1 zeroed).  One workgroup.
int launch_cut(const DevState* st, const PodArgs& a, int blocks, int n_filters, void* stream);
int launch_resolve(const DevState* st, int N, const PodArgs& a, void* stream);
int eval_blocks(int N);
// Node sharding: reduce this shard's `blocks` partials of buffer half `parity` to one record in
// shard_send_key (what = 0, global node index) or shard_send_stat (what = 1).
int launch_shard_pack(const DevState* st, int parity, int blocks, int what, void* stream);
// Geometry index (B row threads x K slots per lane, plus one communication wave) and grid of the
// persistent kernel: *per = B*K - 1 nodes per workgroup (the last slot of the last lane is the
// variant-B spare), -1 when N does not fit in max_groups workgroups.
// first: the smallest geometry index considered (KGPU_OPT_BATCH_GEO; 0 = all)
int batch_geometry(int N, int max_groups, int* per, int* groups, int first = 0);
// helper: config (b)'s profile on the one-row-wave geometry takes the helper-wave instantiation (HB)
int launch_batch(const DevState* st, const BatchArgs& a, int groups, int kidx, int spec, bool coop, bool helper,
                 void* stream);
// Topology pipeline for one pod (PodArgs.pod): domain histograms, critical-path minima, filters,
// scores, normalize + argmax, resolve + assume.  next_scratch: words of the next topology pod's
// scratch to zero in the resolve launch (0 none).
// fused = one cooperative launch with grid barriers between the phases, else six launches (the
// default: measured faster).  A pod with a.cut (percentageOfNodesToScore < 100) always
// takes the separate launches, with k_cut + k_topo_reg between the filter and score phases.
// bar: the fused kernel's grid-barrier counter (grows monotonically); bar_base: its value before
// this launch.  A fused launch adds topo_barriers(min_values) * blocks arrivals.
int launch_topo(const DevState* st, PodArgs a, int blocks, int64_t min_values, int64_t next_scratch,
                bool fused, unsigned long long* bar, unsigned long long bar_base, int n_filters, void* stream,
                const PreemptArgs* nom = nullptr, int N = 0);
inline int topo_barriers(int64_t min_values) { return min_values > 0 ? 5 : 4; }
// Initialize mcnt columns [c0, c0 + nc) from the pod table (n_pods rows).
int launch_class_init(const DevState* st, int c0, int nc, int n_pods, void* stream);
int launch_debug_broken_linear(const kgpu_shape_point* pts, int n_pts, const int64_t* p, int64_t* out, int n,
                               void* stream);
int launch_topo_phase(const DevState* st, const PodArgs& a, int phase, int blocks, int64_t extra, void* stream);
// Persistent topology run: signature bitmaps + pair registrations and histogram
// initialization from the match-count columns (k_tbatch_init), then k_tbatch.  kidx: geometry.
// first: the smallest geometry index considered (KGPU_OPT_TBATCH_GEO)
int tbatch_geometry(int N, int max_groups, int* per, int* groups, int first);
// The launch-argument layouts as the kernel translation unit saw them: a library linked from a host
// object and a kernel object of different revisions refuses to start (kgpu_create).
constexpr int64_t layout_sig_of() {
  return (int64_t)sizeof(TBatchArgs) * 1000003 + (int64_t)sizeof(BatchArgs) * 10007 + (int64_t)sizeof(DevState) * 101 +
         (int64_t)sizeof(PodArgs) + (int64_t)sizeof(TPlan) * 7919;
}
int64_t kernel_layout_sig();
// k_tbatch_init over the local nodes (a.per * groups >= N); then, on a node-sharded
// engine, launch_xreduce over the init region; then launch_tbatch (xg: the XG instantiation).
int launch_tbatch_init(const DevState* st, const TBatchArgs& a, int groups, void* stream);
int launch_tbatch(const DevState* st, const TBatchArgs& a, int groups, int geo, int spec, bool xg, bool coop,
                  void* stream);

// ---------------------------------------------------------------- delta stream (kgpu_apply_delta)
enum DeltaKind { kDAddPod = 0, kDRemovePod = 1, kDSetNode = 2 };
// One NodeInfo change on a local row, applied in order by k_delta.
struct DeltaOp {
  int32_t kind;        // DeltaKind
  int32_t node;        // local node row
  int32_t item;        // pod (query) index / node row index
  int32_t slot;        // pod-table slot written for an added / removed pod (-1: table not resident)
  kgpu_range cls;      // aux ints: pod classes whose mcnt column moves by +-1
  kgpu_range tcls;     // aux ints: term classes (the pod's own terms) whose tcnt column moves by +-1
};
struct DeltaArgs {
  const DeltaOp* ops;            // grouped by node, each group in batch order
  const int32_t* group_off;      // [n_groups + 1] op ranges, one workgroup per node
  int32_t n_ops;
  int32_t n_groups;
  const kgpu_pod_query* pods;
  const kgpu_node_row* rows;
  const int32_t* ints;           // pools of pods / rows
  const uint64_t* words;
  const kgpu_scalar_req* scalars;
  const kgpu_port* ports;
  const int32_t* aux;
};
int launch_delta(const DevState* st, const DeltaArgs& a, void* stream);

// Column gather for a node-list rebuild: dst[c][i] = src[c][from[i]] (0 when from[i] < 0).
struct RemapCol {
  const void* src;
  void* dst;
  int32_t elem;        // bytes per element: 1, 4, 8 or 16
  int32_t ncols;
};
int launch_remap(const RemapCol* cols, int n_cols, const int32_t* from, int old_n, int new_n, void* stream);

}  // namespace kgpu
