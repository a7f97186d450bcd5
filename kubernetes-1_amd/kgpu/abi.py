"""numpy / ctypes mirrors of the structs in include/kgpu.h (checked against kgpu_struct_sizes)."""
import ctypes as C

import numpy as np

ABI_VERSION = 3
OK, E_INVAL, E_NOMEM, E_DEVICE, E_CAPACITY, E_STATE, E_UNSUPPORTED = 0, -1, -2, -3, -4, -5, -6
ERRNAMES = {0: "OK", -1: "KGPU_E_INVAL", -2: "KGPU_E_NOMEM", -3: "KGPU_E_DEVICE", -4: "KGPU_E_CAPACITY",
            -5: "KGPU_E_STATE", -6: "KGPU_E_UNSUPPORTED"}

OPT_KERNEL_TIMING, OPT_PERSISTENT, OPT_PERSIST_GROUPS, OPT_PHASE_TRACE, OPT_TOPO_FUSED = 1, 2, 3, 4, 5
OPT_TOPO_PERSISTENT = 6
OPT_ABORT_AT = 7
OPT_XGMI = 8
OPT_SKIP_RELEASE_AT = 9
OPT_COOPERATIVE = 10
OPT_BATCH_GEO = 11
OPT_ARENA_BYTES = 12
OPT_TOPO_RESIDENT = 13
OPT_BATCH_HELPER = 14
OPT_TOPO_AHEAD = 15
OPT_TBATCH_GEO = 16
OPT_HOLD_GROUP = 17
OPT_TBATCH_WLAB = 18
OPT_RUN_ALL_FILTERS = 20
OPT_TBATCH_POLL_SLEEP = 21
OPT_ZEROCOPY_POOLS = 23
CODE_SUCCESS, CODE_ERROR, CODE_UNSCHEDULABLE, CODE_UNRESOLVABLE = 0, 1, 2, 3
STATUS_NOT_EVALUATED = 0xFF  # KGPU_FS_NOT_EVALUATED: percentageOfNodesToScore stopped before the node

F_NODE_UNSCHEDULABLE, F_FIT, F_NODE_NAME, F_NODE_PORTS, F_NODE_AFFINITY, F_TAINT, F_PTS, F_IPA = range(8)
NUM_FILTERS = 8
FILTER_IDS = {"NodeUnschedulable": 0, "NodeResourcesFit": 1, "NodeName": 2, "NodePorts": 3, "NodeAffinity": 4,
              "TaintToleration": 5, "PodTopologySpread": 6, "InterPodAffinity": 7}
FILTER_NAMES = {v: k for k, v in FILTER_IDS.items()}

(S_BALANCED, S_IMAGE, S_IPA, S_LEAST, S_NODE_AFFINITY, S_NPAP, S_PTS, S_DPTS, S_TAINT, S_MOST, S_RTCR,
 S_LIMITS) = range(12)
NUM_SCORES = 12
SCORE_IDS = {"NodeResourcesBalancedAllocation": 0, "ImageLocality": 1, "InterPodAffinity": 2,
             "NodeResourcesLeastAllocated": 3, "NodeAffinity": 4, "NodePreferAvoidPods": 5,
             "PodTopologySpread": 6, "DefaultPodTopologySpread": 7, "TaintToleration": 8,
             "NodeResourcesMostAllocated": 9, "RequestedToCapacityRatio": 10, "NodeResourceLimits": 11}
SCORE_NAMES = {v: k for k, v in SCORE_IDS.items()}

OP_IN, OP_NOTIN, OP_EXISTS, OP_DNE, OP_GT, OP_LT = range(6)
SEL_AND, SEL_NOTHING = 0, 1
TERM_REQ_AFF, TERM_REQ_ANTI, TERM_PREF_AFF, TERM_PREF_ANTI = range(4)
PF_TERMINATING, PF_WITH_AFFINITY, PF_ACTIVE = 1, 2, 4
(Q_TOLERATES_UNSCHED, Q_FIT_ALL_ZERO, Q_HAS_TSC, Q_HAS_POD_AFFINITY, Q_HAS_POD_ANTI, Q_SELF_MATCH_ALL_AFF,
 Q_TERMINATING, Q_REQ_NODE_AFFINITY, Q_SCORE_ERROR) = (1, 2, 4, 8, 16, 32, 64, 128, 256)
Q_NO_KNOWN_IMAGE = 512

RANGE = np.dtype([("begin", "<i4"), ("count", "<i4")], align=True)
REQ = np.dtype([("key", "<i4"), ("op", "<i4"), ("vals", RANGE), ("imm", "<i8")], align=True)
SELECTOR = np.dtype([("kind", "<i4"), ("pad", "<i4"), ("reqs", RANGE)], align=True)
NODE_TERM = np.dtype([("reqs", RANGE), ("field_op", "<i4"), ("field_node", "<i4"), ("never_match", "<i4"),
                      ("pad", "<i4")], align=True)
PREF_TERM = np.dtype([("weight", "<i4"), ("pad", "<i4"), ("sel", SELECTOR)], align=True)
SPREAD = np.dtype([("max_skew", "<i4"), ("key", "<i4"), ("is_hostname", "<i4"), ("self_match", "<i4"),
                   ("sel", SELECTOR)], align=True)
POD_TERM = np.dtype([("weight", "<i4"), ("topo_key", "<i4"), ("ns", RANGE), ("sel", SELECTOR)], align=True)
TERM = np.dtype([("pod", "<i4"), ("kind", "<i4"), ("t", POD_TERM)], align=True)
SCALAR_REQ = np.dtype([("col", "<i4"), ("check", "<i4"), ("value", "<i8"), ("score_value", "<i8")], align=True)
PORT = np.dtype([("ip", "<i4"), ("proto", "<i4"), ("port", "<i4"), ("pad", "<i4")], align=True)
QUERY = np.dtype([
    ("ns", "<i4"), ("flags", "<u4"), ("req", "<i8", (3,)), ("nz", "<i8", (2,)), ("score_req", "<i8", (3,)),
    ("scalars", RANGE), ("node_name", "<i4"), ("n_containers", "<i4"), ("ports", RANGE),
    ("tol_nosched", RANGE), ("tol_prefer", RANGE), ("node_selector", RANGE), ("req_terms", RANGE),
    ("pref_terms", RANGE), ("images", RANGE), ("avoid_id", "<i4"), ("pad0", "<i4"), ("pts_hard", RANGE),
    ("pts_soft", RANGE), ("dpts", SELECTOR), ("ipa_req_aff", RANGE), ("ipa_req_anti", RANGE),
    ("ipa_pref_aff", RANGE), ("ipa_pref_anti", RANGE), ("labels", RANGE), ("limits", "<i8", (2,)),
    ("priority", "<i4"), ("pad1", "<i4"), ("uid", "<i8")], align=True)
RESULT = np.dtype([("node", "<i4"), ("feasible", "<i4"), ("evaluated", "<i4"), ("scored", "<i4"),
                   ("score", "<i8")], align=True)

vp = C.c_void_p


class ResourceWeight(C.Structure):
    _fields_ = [("resource", C.c_int32), ("weight", C.c_int32)]


class ShapePoint(C.Structure):
    _fields_ = [("utilization", C.c_int64), ("score", C.c_int64)]


class Config(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("device", C.c_int32), ("n_filters", C.c_int32),
                ("filters", C.c_int32 * NUM_FILTERS), ("n_scores", C.c_int32), ("scores", C.c_int32 * NUM_SCORES),
                ("score_weights", C.c_int64 * NUM_SCORES), ("n_least", C.c_int32), ("least", ResourceWeight * 8),
                ("n_most", C.c_int32), ("most", ResourceWeight * 8), ("hard_pod_affinity_weight", C.c_int32),
                ("percentage_of_nodes_to_score", C.c_int32), ("tie_break_mode", C.c_int32), ("pad0", C.c_int32),
                ("seed", C.c_uint64), ("node_capacity", C.c_int32), ("pod_capacity", C.c_int32),
                ("term_capacity", C.c_int32), ("pad1", C.c_int32), ("n_rtcr", C.c_int32), ("n_shape", C.c_int32),
                ("rtcr", ResourceWeight * 8), ("shape", ShapePoint * 16)]


class Pools(C.Structure):
    _fields_ = [("reqs", vp), ("n_reqs", C.c_int32), ("ints", vp), ("n_ints", C.c_int32), ("words", vp),
                ("n_words", C.c_int32), ("node_terms", vp), ("n_node_terms", C.c_int32), ("pref_terms", vp),
                ("n_pref_terms", C.c_int32), ("spreads", vp), ("n_spreads", C.c_int32), ("pod_terms", vp),
                ("n_pod_terms", C.c_int32), ("scalars", vp), ("n_scalars", C.c_int32), ("ports", vp),
                ("n_ports", C.c_int32)]


class Snapshot(C.Structure):
    _fields_ = [("n_nodes", C.c_int32), ("node_base", C.c_int32), ("n_total_nodes", C.c_int32),
                ("pad0", C.c_int32),
                ("alloc_cpu", vp), ("alloc_mem", vp), ("alloc_eph", vp), ("alloc_pods", vp),
                ("req_cpu", vp), ("req_mem", vp), ("req_eph", vp), ("nz_cpu", vp), ("nz_mem", vp),
                ("num_pods", vp), ("n_scalar", C.c_int32), ("pad1", C.c_int32), ("alloc_scalar", vp),
                ("req_scalar", vp), ("unschedulable", vp), ("n_label_keys", C.c_int32), ("pad2", C.c_int32),
                ("label_val", vp), ("key_n_values", vp), ("value_off", vp), ("value_int", vp),
                ("value_int_ok", vp), ("key_empty_value", vp), ("taint_words", C.c_int32), ("pad3", C.c_int32),
                ("taint_nosched", vp), ("taint_prefer", vp), ("port_slots", C.c_int32), ("pad4", C.c_int32),
                ("port_count", vp), ("ports", vp), ("image_off", vp), ("image_id", vp), ("image_score", vp),
                ("avoid_off", vp), ("avoid_id", vp), ("zone_id", vp), ("n_zones", C.c_int32),
                ("n_pods", C.c_int32), ("pod_node", vp), ("pod_ns", vp), ("pod_flags", vp),
                ("n_pod_label_keys", C.c_int32), ("n_terms", C.c_int32), ("pod_label_val", vp), ("terms", vp),
                ("pools", Pools), ("pod_uid", vp), ("key_unique", vp)]


D_ADD_POD, D_REMOVE_POD, D_SET_NODE = 1, 2, 3
DELTA = np.dtype([("op", "<i4"), ("node", "<i4"), ("uid", "<i8"), ("item", "<i4"), ("pad", "<i4")], align=True)
NODE_ROW = np.dtype([("alloc_cpu", "<i8"), ("alloc_mem", "<i8"), ("alloc_eph", "<i8"), ("alloc_pods", "<i4"),
                     ("unschedulable", "<i4"), ("zone_id", "<i4"), ("pad", "<i4"), ("labels", RANGE),
                     ("taints", RANGE), ("alloc_scalar", RANGE)], align=True)


class DeltaBatch(C.Structure):
    _fields_ = [("n_deltas", C.c_int32), ("n_pods", C.c_int32), ("deltas", vp), ("pods", vp),
                ("n_rows", C.c_int32), ("n_order", C.c_int32), ("rows", vp), ("order", vp),
                ("key_n_values", vp), ("value_off", vp), ("value_int", vp), ("value_int_ok", vp),
                ("key_empty_value", vp), ("image_off", vp), ("image_id", vp), ("image_score", vp),
                ("avoid_off", vp), ("avoid_id", vp), ("n_zones", C.c_int32), ("pad", C.c_int32),
                ("pools", Pools), ("key_unique", vp)]


class Stats(C.Structure):
    _fields_ = [("pods", C.c_int64), ("scheduled", C.c_int64), ("device_ms", C.c_double),
                ("eval_kernel_ms", C.c_double), ("eval_launches", C.c_int64)]


NOMINATED = np.dtype([("node", "<i4"), ("item", "<i4")], align=True)
VICTIM = np.dtype([("node", "<i4"), ("slot", "<i4"), ("item", "<i4"), ("pad", "<i4"), ("start_time", "<i8"),
                   ("pdb_mask", "<u8")], align=True)
NODE_VICTIMS = np.dtype([("fits", "<i4"), ("n_victims", "<i4"), ("num_pdb_violations", "<i4"), ("first", "<i4")],
                        align=True)


class PreemptArgs(C.Structure):
    _fields_ = [("n_victims", C.c_int32), ("n_pdbs", C.c_int32), ("victims", vp), ("pdb_allowed", vp), ("pods", vp)]


class TaintRef(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_char_p), ("effect", C.c_char_p), ("id", C.c_int32),
                ("pad", C.c_int32)]


class ReasonArgs(C.Structure):
    _fields_ = [("q", vp), ("pools", C.POINTER(Pools)), ("node", C.c_int32), ("word", C.c_uint32),
                ("taints", C.POINTER(TaintRef)), ("n_taints", C.c_int32), ("n_filters", C.c_int32),
                ("filters", C.POINTER(C.c_int32)), ("scalar_names", C.POINTER(C.c_char_p))]


# declaration order of kgpu_struct_sizes
STRUCT_SIZES = [("kgpu_range", RANGE.itemsize), ("kgpu_req", REQ.itemsize), ("kgpu_selector", SELECTOR.itemsize),
                ("kgpu_node_term", NODE_TERM.itemsize), ("kgpu_pref_term", PREF_TERM.itemsize),
                ("kgpu_spread", SPREAD.itemsize), ("kgpu_pod_term", POD_TERM.itemsize),
                ("kgpu_term", TERM.itemsize), ("kgpu_scalar_req", SCALAR_REQ.itemsize),
                ("kgpu_port", PORT.itemsize), ("kgpu_pod_query", QUERY.itemsize),
                ("kgpu_pools", C.sizeof(Pools)), ("kgpu_resource_weight", C.sizeof(ResourceWeight)),
                ("kgpu_config", C.sizeof(Config)), ("kgpu_snapshot", C.sizeof(Snapshot)),
                ("kgpu_result", RESULT.itemsize), ("kgpu_stats", C.sizeof(Stats)), ("kgpu_delta", DELTA.itemsize),
                ("kgpu_node_row", NODE_ROW.itemsize), ("kgpu_delta_batch", C.sizeof(DeltaBatch)),
                ("kgpu_shape_point", C.sizeof(ShapePoint)), ("kgpu_nominated", NOMINATED.itemsize),
                ("kgpu_victim", VICTIM.itemsize), ("kgpu_preempt_args", C.sizeof(PreemptArgs)),
                ("kgpu_node_victims", NODE_VICTIMS.itemsize), ("kgpu_taint_ref", C.sizeof(TaintRef)),
                ("kgpu_reason_args", C.sizeof(ReasonArgs))]


def ptr(a):
    """Data pointer of a numpy array (None for None / empty)."""
    if a is None:
        return None
    return a.ctypes.data if a.size else None
