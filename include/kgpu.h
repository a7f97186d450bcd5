/*
 * kgpu.h -- C ABI of libkgpu.so, the MI355X-native node-evaluation engine behind the
 * kube-scheduler framework's PreFilter/Filter/PreScore/Score/NormalizeScore/Reserve plugin
 * interfaces (reference: pkg/scheduler/framework/v1alpha1/interface.go:208-394).
 *
 * One entry point replaces one reference interface (see INTEGRATION.md for the cgo binding):
 *
 *   kgpu_create / kgpu_destroy      framework.PluginFactory (framework/v1alpha1/registry.go:28) +
 *                                   NewFramework weights/args (framework/v1alpha1/framework.go:205-298)
 *   kgpu_upload_snapshot            cache.UpdateSnapshot -> Snapshot.List() order
 *                                   (internal/cache/cache.go:202-301, node_tree.go:147-170)
 *   kgpu_schedule_one               genericScheduler.Schedule (core/generic_scheduler.go:146-209):
 *                                   RunPreFilterPlugins + findNodesThatPassFilters (:403-495) +
 *                                   prioritizeNodes (:622-716) + selectHost (:217-238) [+ assume]
 *   kgpu_schedule_batch             scheduleOne loop (scheduler.go:509-593) with on-device assume
 *                                   (cache.AssumePod cache.go:338 -> NodeInfo.AddPod types.go:456)
 *   kgpu_get_filter                 per-node PluginToStatus.Merge code (framework.go:477-502)
 *   kgpu_get_filter_all             runAllFilters: every plugin's status per node (framework.go:484-499)
 *   kgpu_get_scores                 PluginToNodeScores (framework.go:579-656), raw and normalized
 *   kgpu_forget_pod                 cache.ForgetPod (cache.go:383-410) -> NodeInfo.RemovePod (types.go:484)
 *   kgpu_apply_delta                the NodeInfo side of the informer / cache event stream between two
 *                                   UpdateSnapshot calls (cache.go:202-301, 338-523, 581-647):
 *                                   NodeInfo.AddPod / RemovePod (types.go:456-533) by pod UID,
 *                                   NodeInfo.SetNode (types.go:587-600), and the Snapshot.List()
 *                                   rebuild after a node add / remove (cache.go:278-301)
 *   kgpu_set_nominated              framework.PodNominator (internal/queue/scheduling_queue.go) for the
 *                                   two-pass filter of podPassesFiltersOnNode (generic_scheduler.go:526-615)
 *   kgpu_select_victims             selectNodesForPreemption / selectVictimsOnNode /
 *                                   pickOneNodeForPreemption (generic_scheduler.go:718-1012)
 *   kgpu_comm_*                     node sharding over RCCL/xGMI (no reference counterpart: the
 *                                   reference parallelises over 16 goroutines only,
 *                                   internal/parallelize/parallelism.go:26-43)
 *
 * Conventions: every call returns KGPU_OK (0) or a negative KGPU_E_* code; no exception crosses
 * the ABI; all buffers are caller-owned host memory; calls on one context are serialized by the
 * caller.  Node indices are positions in Snapshot.List().  All identifiers for strings (label
 * keys/values, namespaces, taints, images, controller UIDs) are dictionary ids assigned by the
 * caller's compile step (kubernetes-1_amd/kgpu/compile.py, or the Go shim).
 */
#ifndef KGPU_H
#define KGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KGPU_ABI_VERSION 3

/* ---- return codes */
#define KGPU_OK 0
#define KGPU_E_INVAL (-1)
#define KGPU_E_NOMEM (-2)
#define KGPU_E_DEVICE (-3)
#define KGPU_E_CAPACITY (-4)
#define KGPU_E_STATE (-5)
#define KGPU_E_UNSUPPORTED (-6)

/* ---- framework.Code (interface.go:51-75) */
#define KGPU_CODE_SUCCESS 0
#define KGPU_CODE_ERROR 1
#define KGPU_CODE_UNSCHEDULABLE 2
#define KGPU_CODE_UNRESOLVABLE 3

/* ---- filter plugins (default profile order: algorithmprovider/registry.go:92-109) */
#define KGPU_F_NODE_UNSCHEDULABLE 0
#define KGPU_F_NODE_RESOURCES_FIT 1
#define KGPU_F_NODE_NAME 2
#define KGPU_F_NODE_PORTS 3
#define KGPU_F_NODE_AFFINITY 4
#define KGPU_F_TAINT_TOLERATION 5
#define KGPU_F_POD_TOPOLOGY_SPREAD 6
#define KGPU_F_INTER_POD_AFFINITY 7
#define KGPU_NUM_FILTERS 8

/* ---- score plugins (default weights: algorithmprovider/registry.go:119-133) */
#define KGPU_S_BALANCED_ALLOCATION 0
#define KGPU_S_IMAGE_LOCALITY 1
#define KGPU_S_INTER_POD_AFFINITY 2
#define KGPU_S_LEAST_ALLOCATED 3
#define KGPU_S_NODE_AFFINITY 4
#define KGPU_S_NODE_PREFER_AVOID_PODS 5
#define KGPU_S_POD_TOPOLOGY_SPREAD 6
#define KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD 7
#define KGPU_S_TAINT_TOLERATION 8
#define KGPU_S_MOST_ALLOCATED 9
/* not in the default provider; enabled by a profile */
#define KGPU_S_REQUESTED_TO_CAPACITY_RATIO 10  /* noderesources/requested_to_capacity_ratio.go:124-170 */
#define KGPU_S_RESOURCE_LIMITS 11              /* noderesources/resource_limits.go:104-160 (NodeResourceLimits) */
#define KGPU_NUM_SCORES 12

/* ---- per-node filter status word (kgpu_get_filter):
 *   bits 0-7   index+1 in the profile's filter order of the first failing filter (0 = feasible)
 *   bits 8-9   framework.Code of that failure
 *   bits 16-31 detail: NodeResourcesFit insufficiency mask (bit0 pods, bit1 cpu, bit2 memory,
 *              bit3 ephemeral-storage, bit4+s scalar request s); InterPodAffinity rule
 *              (1 affinity, 2 anti-affinity, 3 existing pods' anti-affinity) */
#define KGPU_FS_FEASIBLE 0u
/* percentageOfNodesToScore < 100: a node findNodesThatPassFilters never examined, or the feasible
 * node whose discovery cancelled the search (generic_scheduler.go:451-471): in neither `filtered`
 * nor the statuses map */
#define KGPU_FS_NOT_EVALUATED 0xFFu

/* ---- selector requirement operators (labels/selector.go:198-242) */
#define KGPU_OP_IN 0
#define KGPU_OP_NOTIN 1
#define KGPU_OP_EXISTS 2
#define KGPU_OP_DNE 3
#define KGPU_OP_GT 4
#define KGPU_OP_LT 5

/* ---- selector kinds */
#define KGPU_SEL_AND 0     /* AND of requirements; zero requirements = Everything */
#define KGPU_SEL_NOTHING 1 /* labels.Nothing() */
#define KGPU_SEL_EMPTY 2   /* DefaultSelector found nothing: Selector.Empty() (counts are 0) */

/* ---- pod term kinds (existing pods' terms) */
#define KGPU_TERM_REQ_AFF 0
#define KGPU_TERM_REQ_ANTI 1
#define KGPU_TERM_PREF_AFF 2
#define KGPU_TERM_PREF_ANTI 3

/* ---- existing-pod flags */
#define KGPU_PF_TERMINATING 1u   /* DeletionTimestamp != nil */
#define KGPU_PF_WITH_AFFINITY 2u /* in NodeInfo.PodsWithAffinity (types.go:472-475) */
#define KGPU_PF_ACTIVE 4u        /* slot holds a pod (forgotten pods are deactivated) */

/* ---- pod query flags */
#define KGPU_Q_TOLERATES_UNSCHEDULABLE 1u  /* node_unschedulable.go:56-59 */
#define KGPU_Q_FIT_ALL_ZERO 2u             /* fit.go:212-217 podRequest all zero */
#define KGPU_Q_HAS_TSC 4u                  /* len(TopologySpreadConstraints) != 0 */
#define KGPU_Q_HAS_POD_AFFINITY 8u         /* affinity.PodAffinity != nil */
#define KGPU_Q_HAS_POD_ANTI 16u            /* affinity.PodAntiAffinity != nil */
#define KGPU_Q_SELF_MATCH_ALL_AFF 32u      /* podMatchesAllAffinityTerms(pod, RequiredAffinityTerms) */
#define KGPU_Q_TERMINATING 64u
#define KGPU_Q_REQ_NODE_AFFINITY 128u      /* RequiredDuringScheduling != nil: terms apply */
#define KGPU_Q_SCORE_ERROR 256u            /* a Score plugin returns Error (invalid preferred term):
                                              the cycle fails whenever scoring runs */
#define KGPU_Q_NO_KNOWN_IMAGE 512u         /* no container image is on any node: ImageLocality is 0 */

typedef struct kgpu_range {
  int32_t begin;
  int32_t count;
} kgpu_range;

/* One label requirement.  `key` is a key id in the selector's key space (node label keys for
 * node selectors, pod label keys for label selectors); -1 = a key no object carries.  `vals`
 * indexes the int32 value pool (value ids of that key; values no object carries are dropped).
 * `imm` is the Gt/Lt operand (strconv.ParseInt of the requirement value). */
typedef struct kgpu_req {
  int32_t key;
  int32_t op;
  kgpu_range vals;
  int64_t imm;
} kgpu_req;

typedef struct kgpu_selector {
  int32_t kind; /* KGPU_SEL_* */
  int32_t pad;
  kgpu_range reqs;
} kgpu_selector;

/* A required node-affinity term (NodeSelectorTerm, helpers.go:317-346): matchExpressions ANDed
 * with one optional metadata.name matchFields requirement.  A term that matches nothing (empty,
 * or an invalid requirement) has never_match = 1. */
typedef struct kgpu_node_term {
  kgpu_range reqs;      /* node label requirements */
  int32_t field_op;     /* -1 none, KGPU_OP_IN, KGPU_OP_NOTIN on metadata.name */
  int32_t field_node;   /* node index named by the field requirement, -1 = no such node */
  int32_t never_match;
  int32_t pad;
} kgpu_node_term;

/* A preferred node-affinity term (node_affinity.go:80-99). */
typedef struct kgpu_pref_term {
  int32_t weight;
  int32_t pad;
  kgpu_selector sel;    /* node label key space */
} kgpu_pref_term;

/* A topology spread constraint (podtopologyspread/common.go:34-39). */
typedef struct kgpu_spread {
  int32_t max_skew;
  int32_t key;          /* node label key id of TopologyKey, -1 = no node has it */
  int32_t is_hostname;  /* TopologyKey == kubernetes.io/hostname (scoring.go:83,105,196) */
  int32_t self_match;   /* selector matches the pod's own labels */
  kgpu_selector sel;    /* pod label key space */
} kgpu_spread;

/* An inter-pod (anti-)affinity term (framework/v1alpha1/types.go:79-90). */
typedef struct kgpu_pod_term {
  int32_t weight;
  int32_t topo_key;     /* node label key id, -1 = no node has it */
  kgpu_range ns;        /* namespace ids (int32 pool) */
  kgpu_selector sel;    /* pod label key space */
} kgpu_pod_term;

/* An existing pod's term (the owner pod's PodInfo terms). */
typedef struct kgpu_term {
  int32_t pod;          /* owner existing-pod index */
  int32_t kind;         /* KGPU_TERM_* */
  kgpu_pod_term t;
} kgpu_term;

/* A scalar (extended / hugepages / attachable) resource request. */
typedef struct kgpu_scalar_req {
  int32_t col;          /* scalar column, -1 = resource no node advertises (allocatable 0) */
  int32_t check;        /* 1 = NodeResourcesFit checks it; 0 = ignoredResources (fit.go:248-253)
                           or an entry that only carries a scorer request */
  int64_t value;        /* Fit request (computePodResourceRequest) == assume delta */
  int64_t score_value;  /* scorer request (GetNonzeroRequestForResource, resource_allocation.go:118) */
} kgpu_scalar_req;

/* A wanted host port (containerPort.HostPort > 0 only; types.go:728-731). */
typedef struct kgpu_port {
  int32_t ip;           /* ip id; id 0 is "0.0.0.0" */
  int32_t proto;        /* protocol id (0 TCP, 1 UDP, 2 SCTP) */
  int32_t port;
  int32_t pad;
} kgpu_port;

/* One pod to schedule, compiled on the host from the v1.Pod (PreFilter-time work). */
typedef struct kgpu_pod_query {
  int32_t ns;                 /* namespace id */
  uint32_t flags;             /* KGPU_Q_* */
  int64_t req[3];             /* Fit: milliCPU, memory, ephemeral (fit.go:112-129) */
  int64_t nz[2];              /* NonZeroRequested delta: milliCPU, memory (types.go:524-555) */
  int64_t score_req[3];       /* scorer pod request cpu/mem/eph (resource_allocation.go:118-142) */
  kgpu_range scalars;         /* kgpu_scalar_req pool */
  int32_t node_name;          /* spec.nodeName: -1 none, -2 names no node, >= 0 node index */
  int32_t n_containers;       /* ImageLocality maxThreshold */
  kgpu_range ports;           /* kgpu_port pool */
  kgpu_range tol_nosched;     /* u64 word pool: taint ids tolerated (NoSchedule/NoExecute) */
  kgpu_range tol_prefer;      /* u64 word pool: PreferNoSchedule taint ids tolerated */
  kgpu_range node_selector;   /* kgpu_req pool (node keys), ANDed; nodeSelector map */
  kgpu_range req_terms;       /* kgpu_node_term pool (ORed) -- only with KGPU_Q_REQ_NODE_AFFINITY */
  kgpu_range pref_terms;      /* kgpu_pref_term pool */
  kgpu_range images;          /* int32 pool: image id per container (-1 unknown) */
  int32_t avoid_id;           /* controller id (RC/RS controllerRef), -1 none */
  int32_t pad0;
  kgpu_range pts_hard;        /* kgpu_spread pool (DoNotSchedule) */
  kgpu_range pts_soft;        /* kgpu_spread pool (ScheduleAnyway) */
  kgpu_selector dpts;         /* DefaultSelector (helper/spread.go:29-72) */
  kgpu_range ipa_req_aff;     /* kgpu_pod_term pool */
  kgpu_range ipa_req_anti;
  kgpu_range ipa_pref_aff;
  kgpu_range ipa_pref_anti;
  kgpu_range labels;          /* int32 pool: (pod key id, value id) pairs */
  int64_t limits[2];          /* NodeResourceLimits: milliCPU, memory limits (resource_limits.go:145-156) */
  int32_t priority;           /* podutil.GetPodPriority (spec.priority, 0 when unset) */
  int32_t pad1;
  int64_t uid;                /* caller id of the pod's types.UID (addNominatedPods skips the pod itself) */
} kgpu_pod_query;

/* Variable-length parts referenced by queries (or by snapshot terms). */
typedef struct kgpu_pools {
  const kgpu_req* reqs;            int32_t n_reqs;
  const int32_t* ints;             int32_t n_ints;       /* value ids, ns ids, image ids, label pairs */
  const uint64_t* words;           int32_t n_words;      /* toleration masks */
  const kgpu_node_term* node_terms; int32_t n_node_terms;
  const kgpu_pref_term* pref_terms; int32_t n_pref_terms;
  const kgpu_spread* spreads;      int32_t n_spreads;
  const kgpu_pod_term* pod_terms;  int32_t n_pod_terms;
  const kgpu_scalar_req* scalars;  int32_t n_scalars;
  const kgpu_port* ports;          int32_t n_ports;
} kgpu_pools;

/* Resource ids for scorer weights: 0 cpu, 1 memory, 2 ephemeral-storage, 3+s scalar column s. */
typedef struct kgpu_resource_weight {
  int32_t resource;
  int32_t weight;
} kgpu_resource_weight;

/* One point of RequestedToCapacityRatioArgs.Shape; score already scaled to MaxNodeScore
 * (UtilizationShapePoint.Score x MaxNodeScore / MaxCustomPriorityScore, requested_to_capacity_ratio.go:54-58). */
typedef struct kgpu_shape_point {
  int64_t utilization;
  int64_t score;
} kgpu_shape_point;

typedef struct kgpu_config {
  int32_t abi_version;
  int32_t device;                           /* HIP device ordinal */
  int32_t n_filters;
  int32_t filters[KGPU_NUM_FILTERS];        /* enabled filters in profile order */
  int32_t n_scores;
  int32_t scores[KGPU_NUM_SCORES];          /* enabled score plugins */
  int64_t score_weights[KGPU_NUM_SCORES];   /* parallel to scores[] (0 -> 1, framework.go:262-265) */
  int32_t n_least;
  kgpu_resource_weight least[8];            /* NodeResourcesLeastAllocatedArgs.Resources */
  int32_t n_most;
  kgpu_resource_weight most[8];             /* NodeResourcesMostAllocatedArgs.Resources */
  int32_t hard_pod_affinity_weight;         /* InterPodAffinityArgs (v1beta1/defaults.go:165-167) */
  int32_t percentage_of_nodes_to_score;     /* 0 = adaptive (the reference default), 1-100; 100 in every
                                               BASELINE config.  < 100: numFeasibleNodesToFind +
                                               nextStartNodeIndex (generic_scheduler.go:379-495) */
  int32_t tie_break_mode;                   /* 0 hashed rank, 1 first maximum in snapshot order */
  int32_t pad0;
  uint64_t seed;                            /* tie-break seed */
  int32_t node_capacity;                    /* device rows to reserve (>= n_nodes) */
  int32_t pod_capacity;                     /* existing-pod rows to reserve incl. assumed pods */
  int32_t term_capacity;                    /* existing-term rows to reserve */
  int32_t pad1;
  int32_t n_rtcr;                           /* RequestedToCapacityRatioArgs.Resources (weight 0 -> 1) */
  int32_t n_shape;                          /* RequestedToCapacityRatioArgs.Shape points, ascending */
  kgpu_resource_weight rtcr[8];
  kgpu_shape_point shape[16];
} kgpu_config;

/* Snapshot in Snapshot.List() order (the local shard of it when sharded). */
typedef struct kgpu_snapshot {
  int32_t n_nodes;             /* nodes in this shard */
  int32_t node_base;           /* global index of local node 0 */
  int32_t n_total_nodes;       /* global node count (ImageLocality uses len(NodeInfos().List())) */
  int32_t pad0;
  const int64_t *alloc_cpu, *alloc_mem, *alloc_eph;
  const int32_t* alloc_pods;
  const int64_t *req_cpu, *req_mem, *req_eph;
  const int64_t *nz_cpu, *nz_mem;
  const int32_t* num_pods;
  int32_t n_scalar;            /* scalar resource columns */
  int32_t pad1;
  const int64_t* alloc_scalar; /* [n_scalar][n_nodes] */
  const int64_t* req_scalar;   /* [n_scalar][n_nodes] */
  const uint8_t* unschedulable;
  /* node labels */
  int32_t n_label_keys;
  int32_t pad2;
  const int32_t* label_val;     /* [n_label_keys][n_nodes]: value id, -1 = absent */
  const int32_t* key_n_values;  /* [n_label_keys] distinct values (domains) per key */
  const int32_t* value_off;     /* [n_label_keys+1] offsets into value_int/value_int_ok */
  const int64_t* value_int;     /* strconv.ParseInt of each value (Gt/Lt) */
  const uint8_t* value_int_ok;
  const int32_t* key_empty_value; /* [n_label_keys] value id of "" (-1 none) */
  /* taints: dictionary bitsets */
  int32_t taint_words;
  int32_t pad3;
  const uint64_t* taint_nosched; /* [taint_words][n_nodes] NoSchedule|NoExecute taint ids */
  const uint64_t* taint_prefer;  /* [taint_words][n_nodes] PreferNoSchedule taint ids */
  /* host ports in use: fixed slots per node */
  int32_t port_slots;
  int32_t pad4;
  const int32_t* port_count;    /* [n_nodes] */
  const kgpu_port* ports;       /* [port_slots][n_nodes] */
  /* ImageLocality: CSR sorted by image id; score = scaledImageScore (image_locality.go:110-113) */
  const int32_t* image_off;     /* [n_nodes+1] */
  const int32_t* image_id;
  const int64_t* image_score;
  /* NodePreferAvoidPods: CSR of avoided controller ids */
  const int32_t* avoid_off;     /* [n_nodes+1] */
  const int32_t* avoid_id;
  /* GetZoneKey (pkg/util/node/node.go:148-174) id, -1 = no zone */
  const int32_t* zone_id;
  int32_t n_zones;
  /* existing pods (all nodes, not only this shard: PTS/IPA count across the cluster) */
  int32_t n_pods;
  const int32_t* pod_node;      /* global node index */
  const int32_t* pod_ns;
  const uint32_t* pod_flags;    /* KGPU_PF_* */
  int32_t n_pod_label_keys;
  int32_t n_terms;
  const int32_t* pod_label_val; /* [n_pod_label_keys][n_pods] value id, -1 absent */
  const kgpu_term* terms;       /* existing pods' affinity terms */
  kgpu_pools pools;             /* pools referenced by terms */
  const int64_t* pod_uid;       /* [n_pods] caller id of each pod's types.UID (kgpu_apply_delta); NULL:
                                   the snapshot pods cannot be addressed by deltas */
  const uint8_t* key_unique;    /* [n_label_keys] 1: no value of the key labels two nodes of the WHOLE
                                   cluster (every shard of Snapshot.List()): hostname-like keys, whose
                                   topology counts are a node's own.  NULL: derived from this snapshot's
                                   nodes -- exact unsharded; a node-sharded engine then treats every key
                                   as shared (ADVICE/DESIGN: sharded topology runs need the caller's view) */
} kgpu_snapshot;

typedef struct kgpu_result {
  int32_t node;        /* chosen node (global index), -1 = FitError (no feasible node) */
  int32_t feasible;    /* ScheduleResult.FeasibleNodes */
  int32_t evaluated;   /* ScheduleResult.EvaluatedNodes = len(filtered) + len(statuses) */
  int32_t scored;      /* 0 when prioritizeNodes was skipped (generic_scheduler.go:184-191) */
  int64_t score;       /* total weighted score of the chosen node */
} kgpu_result;

typedef struct kgpu_stats {
  int64_t pods;            /* pods processed */
  int64_t scheduled;       /* pods placed */
  double device_ms;        /* device time of the batch (HIP events) */
  double eval_kernel_ms;   /* summed duration of node-evaluation launches */
  int64_t eval_launches;
} kgpu_stats;

typedef struct kgpu_ctx kgpu_ctx;

int kgpu_abi_version(void);
/* sizeof of each ABI struct, in declaration order (kgpu_range ... kgpu_stats), for binding checks. */
int kgpu_struct_sizes(int32_t* out, int32_t n);
int kgpu_create(const kgpu_config* cfg, kgpu_ctx** out);
int kgpu_destroy(kgpu_ctx* ctx);
const char* kgpu_last_error(const kgpu_ctx* ctx);

int kgpu_upload_snapshot(kgpu_ctx* ctx, const kgpu_snapshot* snap, int64_t generation);
int64_t kgpu_generation(const kgpu_ctx* ctx);

/* One scheduling cycle.  assume != 0 applies NodeInfo.AddPod for the chosen node on the device
 * (Reserve -> assume); the pod then becomes existing pod `*assumed_slot` (may be NULL). */
int kgpu_schedule_one(kgpu_ctx* ctx, const kgpu_pod_query* q, const kgpu_pools* pools, int64_t pod_seq,
                      int32_t assume, kgpu_result* res, int32_t* assumed_slot);

/* The scheduleOne loop over n pods in queue order, each placement assumed before the next pod
 * is evaluated.  Pod i uses tie-break sequence number first_seq + i. */
int kgpu_schedule_batch(kgpu_ctx* ctx, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools,
                        int64_t first_seq, kgpu_result* results, kgpu_stats* stats);

/* Pipelined batches: the scheduleOne loop over consecutive batches, each batch's host work (the caller's
 * compile, staging, the launch) overlapped with the previous batch's device run.  _submit stages and
 * launches a batch and returns; `results` and `stats` must stay valid until the batch is completed by
 * _wait, which completes the OLDEST batch in flight and returns its status.  Two batches are kept in
 * flight (a third submit first completes the oldest).  A batch the pipeline does not carry (topology
 * pods, normalize pods, host ports, nominated pods, node sharding, percentageOfNodesToScore < 100,
 * short batches) runs synchronously inside _submit after the batches in flight; its _wait returns its
 * status.  Every other call on the context fails with KGPU_E_STATE while batches are in flight.
 * kgpu_pipelined returns the number of batches submitted and not yet waited for.
 * A pipelined batch is never re-issued: if one of its persistent workgroups starts late (the ordinary
 * launch of KGPU_OPT_COOPERATIVE 0 under transient contention), its _wait fails with KGPU_E_DEVICE and
 * the mirror must be uploaded again, even when the abort was clean (a later batch may already be queued
 * behind it).  Callers that cannot afford a re-upload set KGPU_OPT_COOPERATIVE to 1. */
int kgpu_schedule_batch_submit(kgpu_ctx* ctx, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools,
                               int64_t first_seq, kgpu_result* results, kgpu_stats* stats);
int kgpu_schedule_batch_wait(kgpu_ctx* ctx);
int kgpu_pipelined(const kgpu_ctx* ctx);

/* Diagnostics for the last kgpu_schedule_one: per-node filter status words, and per-node raw /
 * normalized (unweighted) scores of one score plugin over the feasible nodes (others: 0). */
int kgpu_get_filter(kgpu_ctx* ctx, uint32_t* status_words);
/* KGPU_OPT_RUN_ALL_FILTERS: the last kgpu_schedule_one cycle's per-plugin status words,
 * [n_filters][N] in profile filter order -- row i holds filter i's word for every node (0: it passed),
 * each word in kgpu_get_filter's format with its own position; PluginToStatus {plugin: Status} of a
 * node is the non-zero words of its column, and kgpu_filter_reasons formats each of them.
 * Replaces framework.go:484-499's statuses map under runAllFilters.  KGPU_E_STATE when the last cycle
 * did not run with the option. */
int kgpu_get_filter_all(kgpu_ctx* ctx, uint32_t* status_words);
int kgpu_get_scores(kgpu_ctx* ctx, int32_t plugin, int64_t* raw, int64_t* normalized);

/* ---- Filter status reasons (kgpu_filter_reasons).  A node taint as the caller's NodeInfo holds it. */
typedef struct kgpu_taint_ref {
  const char* key;
  const char* value;
  const char* effect;   /* v1.TaintEffect: "NoSchedule", "PreferNoSchedule", "NoExecute" */
  int32_t id;           /* taint dictionary id (the bit of the query's toleration masks) */
  int32_t pad;
} kgpu_taint_ref;

typedef struct kgpu_reason_args {
  const kgpu_pod_query* q;          /* the pod the word was computed for, and its pools */
  const kgpu_pools* pools;
  int32_t node;                     /* local node index of the word (Snapshot.List() position) */
  uint32_t word;                    /* that node's status word (kgpu_get_filter) */
  const kgpu_taint_ref* taints;     /* the node's Spec.Taints, in spec order */
  int32_t n_taints;
  int32_t n_filters;                /* ctx == NULL only: the profile's filter order (KGPU_F_*) */
  const int32_t* filters;
  const char* const* scalar_names;  /* resource name of each of q's scalar requests, in q->scalars order */
} kgpu_reason_args;

/* The reasons of a failed node's Filter status (framework.Status.Reasons()), formatted exactly as the
 * failing plugin formats them: they become the FitError's per-node reasons and the pod's
 * FailedScheduling event (replaces the plugins' NewStatus calls: node_unschedulable.go:61-63,
 * node_name.go:50-52, node_ports.go:107-109, node_affinity.go:58-60, taint_toleration.go:59-71 with
 * apis/core/v1/helper/helpers.go:448-471, noderesources/fit.go:159-176,194-267,
 * podtopologyspread/filtering.go:297-324, interpodaffinity/filtering.go:372-396).
 * Writes the reasons into buf as consecutive NUL-terminated strings and returns how many there are
 * (0 for a feasible or unevaluated word); *bytes = the bytes they need.  KGPU_E_CAPACITY when that
 * exceeds len (buf untouched).  ctx may be NULL (pure formatting: args.filters gives the profile's
 * order); with a ctx, a pod with more than 12 scalar requests reads the node's scalar columns. */
int kgpu_filter_reasons(kgpu_ctx* ctx, const kgpu_reason_args* args, char* buf, int64_t len, int64_t* bytes);
/* Diagnostics (parity against the reference's PodTopologySpread state tables,
 * podtopologyspread/filtering_test.go:543 and scoring_test.go:38): the state the device builds for one
 * pod, for its constraint `constraint` (0-based, in kgpu_pod_query.pts_hard / pts_soft order), per
 * value id v of the constraint's key (key_n_values[key] entries):
 *   kind 0, PreFilter (calPreFilterState, filtering.go:198-273): registered[v] = the pair is a
 *           TpPairToMatchNum key (an eligible node carries it), counts[v] = TpPairToMatchNum; *scalar =
 *           criticalPaths[0].MatchNum (MaxInt32 when no pair is registered);
 *   kind 1, PreScore over the nodes the profile's filters pass (initPreScoreState, scoring.go:59-169):
 *           registered[v] = the pair is a TopologyPairToPodCounts key, counts[v] its count; *scalar = the
 *           topology size behind topologyNormalizingWeight (-1: not the key's first constraint).
 * Unsharded engines only. */
int kgpu_debug_pts_state(kgpu_ctx* ctx, const kgpu_pod_query* q, const kgpu_pools* pools, int32_t kind,
                         int32_t constraint, uint8_t* registered, int64_t* counts, int64_t* scalar);

/* Mirror coherence: ForgetPod / RemovePod of an existing pod slot (cache.go:383-410). */
int kgpu_forget_pod(kgpu_ctx* ctx, int32_t pod_slot);

/* Batch-ahead (a caller that runs kgpu_schedule_batch with assume for the pods its queue pops next,
 * then serves the per-pod cycles from the results): the slot the next pod assumed by
 * kgpu_schedule_* will get (slots are consecutive in batch order, placed pods only), and adoption --
 * when the scheduler's own cache.AssumePod (cache.go:338-361) lands the pod on the node the device
 * already assumed it on, the pod's UID is registered for that slot, so later deltas (REMOVE_POD by
 * UID) address it and no ADD_POD is sent for it.  A speculative assume that is not adopted is undone
 * with kgpu_forget_pod. */
int kgpu_next_slot(const kgpu_ctx* ctx);
int kgpu_adopt_pod(kgpu_ctx* ctx, int32_t pod_slot, int64_t uid);

/* Register ahead of need the pod classes of pods the caller expects to schedule (the queue's pending pods,
 * the templates of its workloads): the label-selector classes and term classes their topology plugins
 * count (PodTopologySpread constraints, DefaultPodTopologySpread selectors, InterPodAffinity terms) are
 * interned and their per-node count columns initialized now -- one launch over the pod table -- instead of
 * on the cycle of the first pod that needs them.  Changes no placement: a class is a function of the
 * cluster's pods, kept current by every assume, forget and delta from then on.  Pods whose plans the engine
 * does not support are skipped (their own cycle reports it).  No-op outside a topology profile. */
int kgpu_prepare_pods(kgpu_ctx* ctx, const kgpu_pod_query* qs, int32_t n, const kgpu_pools* pools);

/* ---- delta stream (kgpu_apply_delta).  The caller keeps the scheduler cache's bookkeeping
 * (podStates / assumedPods / nodeTree, cache.go) and sends the NodeInfo changes it implies; the
 * engine applies them to the device mirror in one launch and de-duplicates pods by UID. */
#define KGPU_D_ADD_POD 1     /* NodeInfo.AddPod (types.go:456-480) on `node`: item = the pod (query).
                                AssumePod, AddPod of a new or expired pod, the add half of UpdatePod or
                                of a confirmed pod bound elsewhere.  E_STATE if `uid` is already on a node. */
#define KGPU_D_REMOVE_POD 2  /* NodeInfo.RemovePod (types.go:484-533): item = the pod being removed (its
                                requests are subtracted, as RemovePod recomputes them from the object);
                                E_STATE if `uid` is not on `node`.  ForgetPod, RemovePod, the remove half
                                of UpdatePod. */
#define KGPU_D_SET_NODE 3    /* NodeInfo.SetNode (types.go:587-600) with the node's list position
                                unchanged: item = node row.  cache.UpdateNode; a zone change does not
                                move the node until the next list rebuild (cache.go:278-301). */

typedef struct kgpu_delta {
  int32_t op;         /* KGPU_D_* */
  int32_t node;       /* global node index in Snapshot.List() after this batch's reorder */
  int64_t uid;        /* pod ops: the caller's id for the pod's types.UID */
  int32_t item;       /* pod ops: index into kgpu_delta_batch.pods; SET_NODE: into .rows */
  int32_t pad;
} kgpu_delta;

/* A node's own attributes (everything NodeInfo derives from the v1.Node, not from its pods). */
typedef struct kgpu_node_row {
  int64_t alloc_cpu, alloc_mem, alloc_eph;
  int32_t alloc_pods;
  int32_t unschedulable;
  int32_t zone_id;            /* GetZoneKey id, -1 none (may exceed n_zones: the count grows) */
  int32_t pad;
  kgpu_range labels;          /* int32 pool: (node label key id, value id) pairs; other keys absent */
  kgpu_range taints;          /* u64 word pool: taint_words NoSchedule|NoExecute words, then
                                 taint_words PreferNoSchedule words (empty range: no taints) */
  kgpu_range alloc_scalar;    /* u64 word pool: n_scalar int64 allocatable values (empty: all 0) */
} kgpu_node_row;

typedef struct kgpu_delta_batch {
  int32_t n_deltas;
  int32_t n_pods;
  const kgpu_delta* deltas;          /* applied in order, after the reorder below */
  const kgpu_pod_query* pods;        /* pod records referenced by pod deltas */
  int32_t n_rows;
  int32_t n_order;                   /* 0: the node list is unchanged */
  const kgpu_node_row* rows;         /* rows referenced by SET_NODE deltas (and new nodes) */
  /* Node add / remove: the new Snapshot.List() (nodeTree.next() x numNodes, cache.go:278-301) as,
   * per new position, the old index or -1 - r for a node with no old row (its attributes come from
   * a SET_NODE delta on it in this batch; it starts with no pods).  Pods of dropped nodes leave the
   * device (cache.RemoveNode drops the NodeInfo, cache.go:626-640). */
  const int32_t* order;
  /* label dictionary growth (new values of existing keys); NULL: unchanged.  Same layout as
   * kgpu_snapshot: key_n_values[K], value_off[K+1], value_int / value_int_ok[value_off[K]],
   * key_empty_value[K]. */
  const int32_t* key_n_values;
  const int32_t* value_off;
  const int64_t* value_int;
  const uint8_t* value_int_ok;
  const int32_t* key_empty_value;
  /* ImageLocality / NodePreferAvoidPods CSR over the (new) node list; NULL: unchanged.  Required
   * with a reorder (scaledImageScore depends on len(NodeInfos().List()), image_locality.go:110). */
  const int32_t* image_off;
  const int32_t* image_id;
  const int64_t* image_score;
  const int32_t* avoid_off;
  const int32_t* avoid_id;
  int32_t n_zones;                   /* zone ids in use (0: unchanged) */
  int32_t pad;
  kgpu_pools pools;                  /* pools of `pods` and `rows` */
  const uint8_t* key_unique;         /* [n_label_keys] as kgpu_snapshot.key_unique after this batch; NULL:
                                        the caller's flags are unchanged */
} kgpu_delta_batch;

/* Apply one batch of cache deltas to the device mirror and stamp it with `generation`
 * (Snapshot.generation, cache.go:248-251).  slots (may be NULL) receives, per delta, the pod-table
 * slot the pod occupies after an ADD_POD (-1 otherwise).  On any error the mirror is marked invalid
 * (KGPU_E_STATE on later cycles) and the snapshot must be uploaded again. */
int kgpu_apply_delta(kgpu_ctx* ctx, const kgpu_delta_batch* batch, int64_t generation, int32_t* slots);

/* Read back node rows (requested / nonzero / pod count) for coherence checks. */
int kgpu_read_nodes(kgpu_ctx* ctx, int64_t* req_cpu, int64_t* req_mem, int64_t* req_eph, int64_t* nz_cpu,
                    int64_t* nz_mem, int32_t* num_pods);

/* Options.  KGPU_OPT_KERNEL_TIMING (1): bracket every node-evaluation launch with HIP events and
 * report their summed duration in kgpu_stats.eval_kernel_ms (adds per-launch overhead: use in a
 * separate measurement pass).  KGPU_OPT_PERSISTENT (2): schedule runs of pods whose normalize
 * maxima are constant inside one persistent launch, node rows register-resident (default 1);
 * 0 = one evaluation launch per pod. */
#define KGPU_OPT_KERNEL_TIMING 1
#define KGPU_OPT_PERSISTENT 2
/* KGPU_OPT_PERSIST_GROUPS (3): cap on the persistent kernel's workgroups (0 = one per CU); a
 * lower cap gives each lane more node rows (tests use it to cover every rows-per-lane variant). */
#define KGPU_OPT_PERSIST_GROUPS 3
/* KGPU_OPT_PHASE_TRACE (4): record per-pod phase timestamps of the persistent kernel (diagnostics;
 * read with kgpu_read_phase_trace).  2: the topology kernel's stamps 1 and 2 mark the end of its
 * normalize + key pass and of the workgroup argmax instead of PreFilter and the rows; 3: the end of its
 * per-pod record loads + accumulator reset and of its lookup tables (PreFilter split). */
#define KGPU_OPT_PHASE_TRACE 4
/* KGPU_OPT_TOPO_FUSED (5): 1 = run a topology pod's six phases (histograms, critical-path minima,
 * filters, scores, normalize + argmax, resolve + assume) in one cooperative launch with grid
 * barriers; 0 (default) = one launch per phase, which measured faster on MI355X. */
#define KGPU_OPT_TOPO_FUSED 5
/* KGPU_OPT_TOPO_PERSISTENT (6): 1 (default) = runs of PodTopologySpread / InterPodAffinity /
 * DefaultPodTopologySpread pods go through one persistent launch with device-resident domain
 * histograms; 0 = one topology pipeline per pod. */
#define KGPU_OPT_TOPO_PERSISTENT 6
/* KGPU_OPT_ABORT_AT (7): test hook -- the persistent run holding batch query `value` raises its
 * abort word there, as a workgroup that lost co-residency would (-1, the default: never).  The
 * batch then fails with KGPU_E_DEVICE and the engine refuses cycles until the next upload. */
#define KGPU_OPT_ABORT_AT 7
/* KGPU_OPT_XGMI (8): 1 (default) = on a node-sharded engine, persistent runs exchange their per-pod
 * granules through peer stores into every rank's mailbox ring over xGMI (kgpu_xgmi_*); 0 = the
 * per-pod RCCL all-gather for every pod. */
#define KGPU_OPT_XGMI 8
/* KGPU_OPT_SKIP_RELEASE_AT (9): test hook -- in the persistent run holding batch query `value`, the
 * workgroups' candidate rows are staged for the next pod but the LDS hand-off is never released, so
 * the next pod's wait on it times out (the path a lost LDS release would take): the batch fails with
 * KGPU_E_DEVICE and the mirror is invalidated (-1, the default: never). */
#define KGPU_OPT_SKIP_RELEASE_AT 9
/* KGPU_OPT_COOPERATIVE (10): 0 (default) = the persistent kernels go out as ordinary launches of a grid
 * the engine sized to be co-resident (at most one workgroup per CU: an LDS reservation above half a CU,
 * and an occupancy query per kernel instantiation at its first launch); 1 = every persistent launch goes
 * through hipLaunchCooperativeKernel (+15-19 us of host time per launch, MI355X_MICROARCH.md coop-launch).
 * A workgroup that does not start on time makes the others' spins time out: when that happens before the
 * run resolved its first pod, nothing on the device changed, and a call whose only state-changing launch
 * was that run is issued again once with a cooperative launch (kgpu_debug_counters out[0]); any later
 * abort fails the call with KGPU_E_DEVICE and invalidates the mirror. */
#define KGPU_OPT_COOPERATIVE 10
/* KGPU_OPT_BATCH_GEO (11): the smallest k_batch geometry considered (index into the geometry table
 * of kgpu_kernels.hip: 0 = 64 row threads, 1 = 128, 2 = 192, 3 = 448, 4 = 960, 5 = 512 x 4 rows per
 * lane); the first one whose workgroups fit the GPU is used.  Default 0. */
#define KGPU_OPT_BATCH_GEO 11
/* KGPU_OPT_ARENA_BYTES (12): bytes a short cycle (kgpu_schedule_one, batches of up to 64 pods) may
 * stage beside its DevState and queries for its single host-to-device copy (changed pools, topology
 * plans, a one-pod persistent topology run's tables and zeroed words); items beyond it take copies of
 * their own.  0 = no staging beyond DevState and queries.  Default and maximum 1 MiB. */
#define KGPU_OPT_ARENA_BYTES 12
/* KGPU_OPT_TOPO_RESIDENT (13): 1 (default) = a persistent topology run starts from the histograms,
 * pair registrations and eligibility bitmaps the previous run with the same tables left on the device
 * (it writes its final bins back) when nothing else changed the mirror in between, instead of
 * recomputing them in an init pass over every node; 0 = always recompute. */
#define KGPU_OPT_TOPO_RESIDENT 13
/* KGPU_OPT_BATCH_HELPER (14): 1 (default) = the persistent batch kernel of the NodeResourcesFit +
 * BalancedAllocation + LeastAllocated profile on its one-row-wave geometry runs a helper wave that
 * evaluates LeastAllocated and the tie-break ranks beside the row wave; 0 = the row wave alone. */
#define KGPU_OPT_BATCH_HELPER 14
/* KGPU_OPT_TOPO_AHEAD (15): 1 (default) = the persistent topology kernel evaluates the next pod's
 * filters and scores outside PodTopologySpread / InterPodAffinity while the current pod's statistics
 * and key travel; 0 = every pod's rows are evaluated after the previous pod's assume. */
#define KGPU_OPT_TOPO_AHEAD 15
/* KGPU_OPT_TBATCH_GEO (16): the smallest persistent topology kernel geometry considered (0 = 256
 * threads x 1 row per lane, 1 = 512 x 1, 2 = 512 x 2); the first whose workgroups fit the GPU is used.
 * Default 1 (256 x 1 measured equal at 5k nodes, with twice the exchange traffic). */
#define KGPU_OPT_TBATCH_GEO 16
/* KGPU_OPT_HOLD_GROUP (17): test hook -- on an ordinary (non-cooperative) persistent launch, workgroup
 * `value` leaves at once, as a workgroup that never became resident (-1, the default: none). */
#define KGPU_OPT_HOLD_GROUP 17
/* KGPU_OPT_TBATCH_WLAB (18): 1 (default) = a persistent topology batch run keeps every node's label values
 * of the delta keys in LDS when they fit, so the assume phase reads the winner's labels there; 0 = a global
 * load per pod (A/B switch). */
#define KGPU_OPT_TBATCH_WLAB 18
/* 19: unused (KGPU_OPT_TBATCH_OWN in round 5, removed after its A/B: DESIGN.md 4.4) */
/* KGPU_OPT_RUN_ALL_FILTERS (20): the framework's runAllFilters (framework.go:90,155-160,484-499; set from
 * the legacy Policy's AlwaysCheckAllPredicates, factory.go:107,278-281).  1 = a kgpu_schedule_one cycle
 * runs every filter plugin on every node: kgpu_get_filter's word becomes PluginToStatus.Merge's
 * (interface.go:162-191: UnschedulableAndUnresolvable over Unschedulable; the position and detail bits
 * stay the first failing plugin's) and kgpu_get_filter_all returns each plugin's own word; preemption's
 * nodesWherePreemptionMightHelp reads the merged code.  Placements do not change.  Default 0. */
#define KGPU_OPT_RUN_ALL_FILTERS 20
/* KGPU_OPT_TBATCH_POLL_SLEEP (21): 1 (default) = the persistent topology kernel's statistics polls sleep
 * briefly between sweeps; 0 = back to back (A/B switch). */
#define KGPU_OPT_TBATCH_POLL_SLEEP 21
/* 22: unused (a register cache of table records in round 5, removed after its A/B) */
/* KGPU_OPT_ZEROCOPY_POOLS (23): 1 (default) = a kgpu_schedule_one cycle whose only kernel is k_eval reads
 * the pod's query pools from pinned host memory (no copy on the stream); 0 = they ride in the cycle's
 * copy (A/B switch). */
#define KGPU_OPT_ZEROCOPY_POOLS 23
int kgpu_set_option(kgpu_ctx* ctx, int32_t option, int64_t value);
/* Engine counters: out[0] = calls issued again with a cooperative launch after a persistent run's
 * workgroups were not all resident before its first pod (KGPU_OPT_COOPERATIVE); out[1] = persistent
 * launches; out[2] = cooperative persistent launches; out[3] = k_class_init launches (pod classes met
 * for the first time, kgpu_prepare_pods); out[4] = whole pod-table uploads (the table is otherwise sent
 * incrementally).  Returns how many counters exist. */
int kgpu_debug_counters(const kgpu_ctx* ctx, int64_t* out, int32_t n);
/* Diagnostics of KGPU_OPT_TOPO_RESIDENT: out[0] = persistent topology runs that started from the
 * resident state, out[1] = runs that recomputed it. */
int kgpu_debug_topo_resident(const kgpu_ctx* ctx, int64_t out[2]);
/* Phase stamps of the last persistent run (100 MHz s_memrealtime ticks), 16 per pipeline
 * iteration (pods + 1): workgroup 0's {start, evaluated, previous pod resolved, published, end, 0,
 * 0, 0}, then the last workgroup's.  Returns the number of iterations written (<= max_iters). */
int kgpu_read_phase_trace(kgpu_ctx* ctx, int64_t* out, int32_t max_iters);

/* ---- nominated pods and preemption.
 *
 * kgpu_set_nominated replaces the engine's copy of the scheduling queue's nominator
 * (framework.PodNominator / nominatedPodMap, internal/queue/scheduling_queue.go): pods that preempted
 * and wait for their victims to leave, by nominated node, in nomination order.  While it is
 * non-empty every cycle filters a node carrying nominated pods of equal or higher priority (and
 * another UID) twice, as podPassesFiltersOnNode does (core/generic_scheduler.go:526-615): once with
 * those pods added to the NodeInfo and to the PodTopologySpread / InterPodAffinity PreFilter state
 * (their AddPod extensions), once without; the node fits only if both pass.  kgpu_schedule_batch
 * then runs its pods one cycle at a time and drops each placed pod from the nominator, as
 * scheduler.assume does (scheduler.go:448).  n = 0 clears it.  `pods` / `pools`: the nominated
 * pods' records (compiled like queries). */
typedef struct kgpu_nominated {
  int32_t node;         /* global node index of NominatedNodeName */
  int32_t item;         /* index into the pod records */
} kgpu_nominated;
int kgpu_set_nominated(kgpu_ctx* ctx, const kgpu_nominated* noms, int32_t n, const kgpu_pod_query* pods,
                       const kgpu_pools* pools);

/* selectNodesForPreemption + pickOneNodeForPreemption (generic_scheduler.go:718-1012) for a pod
 * whose cycle ended in a FitError.  The candidate nodes are those whose filter status is not
 * UnschedulableAndUnresolvable (nodesWherePreemptionMightHelp, :1014-1028); on each, every
 * potential victim is removed (NodeInfo.RemovePod + the RemovePod extensions), the pod is filtered
 * (two passes when pods are nominated there), and the victims are reprieved one at a time,
 * PodDisruptionBudget-violating ones first, each group in MoreImportantPod order
 * (util/utils.go:76-83).  One device thread per node. */
typedef struct kgpu_victim {
  int32_t node;         /* global node index the pod runs on */
  int32_t slot;         /* its pod-table slot (snapshot pod index, or the slot an assume / ADD_POD gave it) */
  int32_t item;         /* its record in `pods` (requests and host ports are subtracted as RemovePod does;
                           priority from the record) */
  int32_t pad;
  int64_t start_time;   /* GetPodStartTime in any monotone unit; pods without status.startTime: the caller's now */
  uint64_t pdb_mask;    /* bit j: PodDisruptionBudget j selects the pod (same namespace, non-empty selector
                           matching its labels, and the pod has labels: filterPodsWithPDBViolation, :878-919) */
} kgpu_victim;
typedef struct kgpu_preempt_args {
  int32_t n_victims;          /* potential victims over all nodes: pods with priority < the preemptor's, in
                                 NodeInfo.Pods order per node (ties of MoreImportantPod keep that order) */
  int32_t n_pdbs;             /* <= 64 */
  const kgpu_victim* victims;
  const int32_t* pdb_allowed; /* [n_pdbs] Status.DisruptionsAllowed */
  const kgpu_pod_query* pods; /* victim records; their pools are the preemptor's `pools` */
} kgpu_preempt_args;
typedef struct kgpu_node_victims {
  int32_t fits;               /* 1: the node is in nodeNameToVictims */
  int32_t n_victims;          /* victims to evict */
  int32_t num_pdb_violations;
  int32_t first;              /* victims_out[first .. first + n_victims): indices into args.victims, in
                                 Victims.Pods order */
} kgpu_node_victims;
/* nodes_out: [n_nodes of this engine]; victims_out: [n_victims]; *chosen: the node
 * pickOneNodeForPreemption returns (global index, -1: none), ties broken by Snapshot.List() order. */
int kgpu_select_victims(kgpu_ctx* ctx, const kgpu_pod_query* q, const kgpu_pools* pools,
                        const kgpu_preempt_args* args, kgpu_node_victims* nodes_out, int32_t* victims_out,
                        int32_t* chosen);

/* Node sharding across GPUs (one process per GPU).  kgpu_comm_unique_id fills 128 bytes on rank
 * 0; the caller broadcasts them; every rank calls kgpu_comm_init with its shard's snapshot
 * already uploaded (node_base / n_total_nodes set). */
int kgpu_comm_unique_id(uint8_t id[128]);
/* With nranks > 1 and KGPU_OPT_XGMI on, kgpu_comm_init also sets up the xGMI mailboxes (the IPC
 * handles travel over RCCL); kgpu_xgmi_active reports whether every rank could map every peer. */
int kgpu_comm_init(kgpu_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t id[128]);
int kgpu_xgmi_active(const kgpu_ctx* ctx);
/* What a sharded engine's exchange actually holds: out[0] = ranks in its RCCL communicator
 * (ncclCommCount; 0 before kgpu_comm_init), out[1] = this rank in it (ncclCommUserRank), out[2] =
 * ranks on the xGMI mailbox path (0 when it is not active), out[3] = peer rings this rank mapped. */
int kgpu_comm_info(const kgpu_ctx* ctx, int32_t out[4]);
/* The mailbox exchange without RCCL (the caller moves the handles, e.g. over its own transport):
 * kgpu_xgmi_handle allocates and zeroes this rank's ring for `nranks` ranks and returns its 64-byte
 * IPC handle; after every rank has its handle, kgpu_xgmi_init(handles = nranks x 64 bytes in rank
 * order) maps the peers.  Every rank must then issue the same schedule calls.  Pods that need a
 * per-pod exchange outside a persistent run (normalize / topology pods) still need kgpu_comm_init. */
int kgpu_xgmi_handle(kgpu_ctx* ctx, int32_t nranks, uint8_t handle[64]);
int kgpu_xgmi_init(kgpu_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t* handles);

/* Test hook (fault injection): the countdown-th host allocation point reached from now on, in any
 * context, throws std::bad_alloc as operator new would (0 = off).  Points: context creation, snapshot
 * upload, the batch / cycle staging, the topology plans, the delta stream.  The entry point that
 * reaches it returns KGPU_E_NOMEM with last_error set -- the exception barrier every extern "C" entry
 * carries -- and a state-changing entry (upload / schedule / delta / forget) also invalidates the
 * device mirror (KGPU_E_STATE until the next kgpu_upload_snapshot). */
int kgpu_debug_fail_alloc(int32_t countdown);

/* Diagnostic: the per-workgroup phase stamps of the last traced persistent topology run
 * (KGPU_OPT_PHASE_TRACE): [pods][groups][8] s_memrealtime ticks (pod start, rows done, statistics
 * published, key published, statistics reduced over the workgroup, statistics received, winner
 * received, unused); *groups = the run's workgroups.  Returns the words copied. */
int kgpu_debug_wg_trace(kgpu_ctx* ctx, int64_t* out, int64_t max_words, int32_t* groups);

/* Diagnostic: the InterPodAffinity PreFilter state the device builds for one pod on the current
 * snapshot (preFilterState, pkg/scheduler/framework/plugins/interpodaffinity/filtering.go:166-271;
 * replaces getPreFilterState in filtering_test.go:1697 TestPreFilterStateAddRemovePod and :2045
 * TestGetTPMapMatchingIncomingAffinityAntiAffinity).  One histogram per (map, topology key):
 * kinds[m] = 0 topologyToMatchedExistingAntiAffinityTerms, 1 topologyToMatchedAffinityTerms,
 * 2 topologyToMatchedAntiAffinityTerms; keys[m] = node label key id; counts[m * max_values + v] =
 * the pair (key, value v)'s count.  *n_maps = histograms written.  Unsharded engines only. */
int kgpu_debug_ipa_state(kgpu_ctx* ctx, const kgpu_pod_query* q, const kgpu_pools* pools, int32_t max_maps,
                         int32_t max_values, int32_t* kinds, int32_t* keys, int64_t* counts, int32_t* n_maps);

/* Diagnostic: the device's broken-linear shape function (the one RequestedToCapacityRatio scores
 * with) evaluated at n utilizations over n_points ascending points taken as given (unscaled).
 * Replaces buildBrokenLinearFunction's direct use in requested_to_capacity_ratio_test.go:119
 * (pkg/scheduler/framework/plugins/noderesources/requested_to_capacity_ratio.go:150-170). */
int kgpu_debug_broken_linear(kgpu_ctx* ctx, const kgpu_shape_point* points, int32_t n_points, const int64_t* p,
                             int32_t n, int64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* KGPU_H */
