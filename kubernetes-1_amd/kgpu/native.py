"""ctypes binding of libkgpu.so (include/kgpu.h).  The product path: no fallback.

If the shared library is missing or fails to load, every entry point raises -- there is no CPU
path behind this module.
"""
import ctypes as C
import os

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
# KGPU_LIB_PATH: an alternative build of the same library (kernel experiments side by side)
LIB_PATH = os.environ.get("KGPU_LIB_PATH") or os.path.join(_HERE, "libkgpu.so")
_lib = None

EXPORTS = ["kgpu_abi_version", "kgpu_struct_sizes", "kgpu_create", "kgpu_destroy", "kgpu_last_error",
           "kgpu_upload_snapshot", "kgpu_generation", "kgpu_schedule_one", "kgpu_schedule_batch",
           "kgpu_get_filter", "kgpu_get_filter_all", "kgpu_get_scores", "kgpu_forget_pod", "kgpu_read_nodes", "kgpu_set_option",
           "kgpu_read_phase_trace", "kgpu_comm_unique_id", "kgpu_comm_init", "kgpu_apply_delta",
           "kgpu_set_nominated", "kgpu_select_victims", "kgpu_xgmi_handle", "kgpu_xgmi_init", "kgpu_xgmi_active",
           "kgpu_comm_info",
           "kgpu_debug_fail_alloc", "kgpu_debug_pts_state", "kgpu_debug_ipa_state", "kgpu_debug_broken_linear",
           "kgpu_debug_wg_trace", "kgpu_debug_topo_resident",
           "kgpu_next_slot", "kgpu_adopt_pod", "kgpu_prepare_pods", "kgpu_filter_reasons", "kgpu_debug_counters",
           "kgpu_schedule_batch_submit", "kgpu_schedule_batch_wait", "kgpu_pipelined"]


class KgpuError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__("%s: %s" % (abi.ERRNAMES.get(code, code), msg))
        self.code = code


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise KgpuError(abi.E_STATE, "libkgpu.so not built (run __graft_entry__.build()): %s" % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    L.kgpu_abi_version.restype = C.c_int
    L.kgpu_struct_sizes.argtypes = [vp, i32]
    L.kgpu_create.argtypes = [C.POINTER(abi.Config), C.POINTER(vp)]
    L.kgpu_destroy.argtypes = [vp]
    L.kgpu_last_error.argtypes = [vp]
    L.kgpu_last_error.restype = C.c_char_p
    L.kgpu_upload_snapshot.argtypes = [vp, C.POINTER(abi.Snapshot), i64]
    L.kgpu_generation.argtypes = [vp]
    L.kgpu_generation.restype = i64
    L.kgpu_schedule_one.argtypes = [vp, vp, C.POINTER(abi.Pools), i64, i32, vp, C.POINTER(i32)]
    L.kgpu_schedule_batch.argtypes = [vp, vp, i32, C.POINTER(abi.Pools), i64, vp, C.POINTER(abi.Stats)]
    L.kgpu_get_filter.argtypes = [vp, vp]
    L.kgpu_get_filter_all.argtypes = [vp, vp]
    L.kgpu_get_scores.argtypes = [vp, i32, vp, vp]
    L.kgpu_forget_pod.argtypes = [vp, i32]
    L.kgpu_read_nodes.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.kgpu_set_option.argtypes = [vp, i32, i64]
    L.kgpu_read_phase_trace.argtypes = [vp, vp, i32]
    L.kgpu_comm_unique_id.argtypes = [vp]
    L.kgpu_comm_init.argtypes = [vp, i32, i32, vp]
    L.kgpu_apply_delta.argtypes = [vp, C.POINTER(abi.DeltaBatch), i64, vp]
    L.kgpu_set_nominated.argtypes = [vp, vp, i32, vp, C.POINTER(abi.Pools)]
    L.kgpu_xgmi_handle.argtypes = [vp, i32, vp]
    L.kgpu_xgmi_init.argtypes = [vp, i32, i32, vp]
    L.kgpu_xgmi_active.argtypes = [vp]
    L.kgpu_comm_info.argtypes = [vp, vp]
    L.kgpu_debug_fail_alloc.argtypes = [i32]
    L.kgpu_debug_pts_state.argtypes = [vp, vp, C.POINTER(abi.Pools), i32, i32, vp, vp, C.POINTER(i64)]
    L.kgpu_debug_ipa_state.argtypes = [vp, vp, C.POINTER(abi.Pools), i32, i32, vp, vp, vp, C.POINTER(i32)]
    L.kgpu_debug_broken_linear.argtypes = [vp, vp, i32, vp, i32, vp]
    L.kgpu_debug_wg_trace.argtypes = [vp, vp, i64, C.POINTER(i32)]
    L.kgpu_debug_topo_resident.argtypes = [vp, vp]
    L.kgpu_next_slot.argtypes = [vp]
    L.kgpu_adopt_pod.argtypes = [vp, i32, i64]
    L.kgpu_prepare_pods.argtypes = [vp, vp, i32, vp]
    L.kgpu_select_victims.argtypes = [vp, vp, C.POINTER(abi.Pools), C.POINTER(abi.PreemptArgs), vp, vp,
                                      C.POINTER(i32)]
    L.kgpu_debug_counters.argtypes = [vp, vp, i32]
    L.kgpu_schedule_batch_submit.argtypes = [vp, vp, i32, C.POINTER(abi.Pools), i64, vp, vp]
    L.kgpu_schedule_batch_wait.argtypes = [vp]
    L.kgpu_pipelined.argtypes = [vp]
    L.kgpu_filter_reasons.argtypes = [vp, C.POINTER(abi.ReasonArgs), vp, i64, C.POINTER(i64)]
    if L.kgpu_abi_version() != abi.ABI_VERSION:
        raise KgpuError(abi.E_STATE, "ABI version mismatch")
    _lib = L
    check_layout(L)
    return L


def check_layout(L=None):
    L = L or lib()
    out = np.zeros(64, np.int32)
    m = L.kgpu_struct_sizes(out.ctypes.data, 64)
    got = [int(x) for x in out[:m]]
    want = [s for _, s in abi.STRUCT_SIZES]
    if got != want:
        bad = [(n, w, g) for (n, w), g in zip(abi.STRUCT_SIZES, got) if w != g]
        raise KgpuError(abi.E_STATE, "struct layout mismatch (python, C): %r" % bad)
    return True


class Engine:
    """One libkgpu context: a profile on one GPU holding one device-resident snapshot."""

    def __init__(self, config):
        L = lib()
        self._cfg = config
        h = C.c_void_p()
        rc = L.kgpu_create(C.byref(config), C.byref(h))
        if rc != 0:
            raise KgpuError(rc, "kgpu_create failed")
        self.h = h
        self._keep = None

    def _check(self, rc):
        if rc != 0:
            msg = lib().kgpu_last_error(self.h)
            raise KgpuError(rc, msg.decode() if msg else "")

    def close(self):
        if getattr(self, "h", None):
            lib().kgpu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, snap, arrays, generation=0):
        self._keep = (snap, arrays)  # the library copies, but keep buffers alive across the call
        self._check(lib().kgpu_upload_snapshot(self.h, C.byref(snap), generation))

    def set_option(self, opt, value):
        self._check(lib().kgpu_set_option(self.h, opt, value))

    def schedule_batch(self, queries, pools, first_seq=0, stats=None):
        q = np.ascontiguousarray(queries, dtype=abi.QUERY)
        res = np.zeros(len(q), abi.RESULT)
        st = stats if stats is not None else abi.Stats()
        self._check(lib().kgpu_schedule_batch(self.h, q.ctypes.data, len(q), C.byref(pools), first_seq,
                                              res.ctypes.data, C.byref(st)))
        return res, st

    def schedule_batch_submit(self, queries, pools, first_seq=0, stats=None):
        """kgpu_schedule_batch_submit: stage and launch a batch, return at once; schedule_batch_wait
        completes the oldest batch in flight and returns its (results, stats).  The arrays handed to the
        library stay referenced here until then."""
        q = np.ascontiguousarray(queries, dtype=abi.QUERY)
        res = np.zeros(len(q), abi.RESULT)
        if not hasattr(self, "_inflight"):
            self._inflight = []
        self._inflight.append((q, res, stats, pools))
        rc = lib().kgpu_schedule_batch_submit(self.h, q.ctypes.data, len(q), C.byref(pools), first_seq, res.ctypes.data,
                                              C.byref(stats) if stats is not None else None)
        if rc != 0:
            self._inflight.pop()
            self._check(rc)

    def schedule_batch_wait(self):
        q, res, stats, pools = self._inflight.pop(0)
        self._check(lib().kgpu_schedule_batch_wait(self.h))
        return res, stats

    def pipelined(self):
        return int(lib().kgpu_pipelined(self.h))

    def schedule_one(self, query, pools, seq=0, assume=True):
        # the per-cycle call: a record taken from a query array (np.void) is copied as bytes into a buffer
        # whose address is known (an array's .ctypes.data costs microseconds per access); libkgpu copies
        # the query before it returns, so the buffer is reused
        one = self.__dict__.get("_one")
        if one is None:
            q1 = np.zeros(1, abi.QUERY)
            slot = C.c_int32(-1)
            one = self._one = (q1, q1.ctypes.data, slot, C.byref(slot))
        q1, qp, slot, slotp = one
        if isinstance(query, np.void) and query.dtype == abi.QUERY:
            C.memmove(qp, query.tobytes(), abi.QUERY.itemsize)
        else:
            q = np.ascontiguousarray(np.atleast_1d(query), dtype=abi.QUERY)
            C.memmove(qp, q.ctypes.data, abi.QUERY.itemsize)
        res = np.zeros(1, abi.RESULT)
        slot.value = -1
        self._check(lib().kgpu_schedule_one(self.h, qp, C.byref(pools), seq, 1 if assume else 0,
                                            res.ctypes.data, slotp))
        return res[0], slot.value

    def filter_words(self, n):
        out = np.zeros(n, np.uint32)
        self._check(lib().kgpu_get_filter(self.h, out.ctypes.data))
        return out

    def filter_words_all(self, n_filters, n):
        """KGPU_OPT_RUN_ALL_FILTERS: the last cycle's per-plugin words, [n_filters][n]."""
        out = np.zeros((n_filters, n), np.uint32)
        self._check(lib().kgpu_get_filter_all(self.h, out.ctypes.data))
        return out

    def scores(self, plugin, n):
        raw = np.zeros(n, np.int64)
        norm = np.zeros(n, np.int64)
        self._check(lib().kgpu_get_scores(self.h, plugin, raw.ctypes.data, norm.ctypes.data))
        return raw, norm

    def read_nodes(self, n):
        cols = [np.zeros(n, np.int64) for _ in range(5)] + [np.zeros(n, np.int32)]
        self._check(lib().kgpu_read_nodes(self.h, *[c.ctypes.data for c in cols]))
        return dict(zip(["req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods"], cols))

    def phase_trace(self, max_iters):
        """[iterations][2][8] s_memrealtime stamps (workgroup 0, last workgroup) of the last
        persistent run: start, evaluated, previous pod resolved, published, end."""
        out = np.zeros((max_iters, 16), np.int64)
        n = lib().kgpu_read_phase_trace(self.h, out.ctypes.data, max_iters)
        if n < 0:
            self._check(n)
        return out[:n].reshape(n, 2, 8)

    def forget(self, slot):
        self._check(lib().kgpu_forget_pod(self.h, slot))

    def apply_delta(self, batch, generation, n_deltas, keep=()):
        """kgpu_apply_delta: `batch` is an abi.DeltaBatch whose arrays `keep` holds alive.
        Returns the pod-table slot of every delta (-1 for non-ADD_POD)."""
        slots = np.full(max(n_deltas, 1), -1, np.int32)
        self._check(lib().kgpu_apply_delta(self.h, C.byref(batch), generation, slots.ctypes.data))
        return slots[:n_deltas]

    def set_nominated(self, noms, pods, pools):
        """kgpu_set_nominated: noms = abi.NOMINATED records (global node, record index), pods = their
        abi.QUERY records compiled against `pools` (copied by the engine).  Empty clears it."""
        n = np.ascontiguousarray(noms, abi.NOMINATED)
        q = np.ascontiguousarray(pods, abi.QUERY)
        self._check(lib().kgpu_set_nominated(self.h, n.ctypes.data if len(n) else None, len(n),
                                             q.ctypes.data if len(q) else None, C.byref(pools)))

    def select_victims(self, query, pools, victims, pods, pdb_allowed, n_nodes):
        """kgpu_select_victims: returns (per-node NODE_VICTIMS records, victim index array, chosen global
        node or -1).  victims: abi.VICTIM records; pods: their abi.QUERY records (same pools as query)."""
        q = np.ascontiguousarray(np.asarray(query, abi.QUERY).reshape(1))
        v = np.ascontiguousarray(victims, abi.VICTIM)
        pr = np.ascontiguousarray(pods, abi.QUERY)
        pa = np.ascontiguousarray(pdb_allowed, np.int32)
        args = abi.PreemptArgs(len(v), len(pa), v.ctypes.data if len(v) else None,
                               pa.ctypes.data if len(pa) else None, pr.ctypes.data if len(pr) else None)
        out = np.zeros(max(n_nodes, 1), abi.NODE_VICTIMS)
        vout = np.full(max(len(v), 1), -1, np.int32)
        chosen = C.c_int32(-1)
        self._check(lib().kgpu_select_victims(self.h, q.ctypes.data, C.byref(pools), C.byref(args), out.ctypes.data,
                                              vout.ctypes.data, C.byref(chosen)))
        return out[:n_nodes], vout[:len(v)], int(chosen.value)

    def xgmi_handle(self, nranks):
        """kgpu_xgmi_handle: this rank's 64-byte mailbox IPC handle (the shard must be uploaded)."""
        buf = (C.c_uint8 * 64)()
        self._check(lib().kgpu_xgmi_handle(self.h, nranks, buf))
        return bytes(buf)

    def xgmi_init(self, nranks, rank, handles):
        """kgpu_xgmi_init: handles = every rank's 64 bytes, in rank order."""
        b = bytes(handles)
        buf = (C.c_uint8 * len(b)).from_buffer_copy(b)
        self._check(lib().kgpu_xgmi_init(self.h, nranks, rank, buf))

    def pts_state(self, query, pools, kind, constraint, n_values):
        """kgpu_debug_pts_state: (registered[n_values] bool, counts[n_values] int64, scalar) of one pod's
        PodTopologySpread PreFilter (kind 0) or PreScore (kind 1) state on the device."""
        q = np.ascontiguousarray(np.asarray(query, abi.QUERY).reshape(1))
        reg = np.zeros(max(n_values, 1), np.uint8)
        cnt = np.zeros(max(n_values, 1), np.int64)
        out = C.c_int64(0)
        self._check(lib().kgpu_debug_pts_state(self.h, q.ctypes.data, C.byref(pools), kind, constraint,
                                                reg.ctypes.data, cnt.ctypes.data, C.byref(out)))
        return reg[:n_values].astype(bool), cnt[:n_values], int(out.value)

    def ipa_state(self, query, pools, max_values, max_maps=32):
        """kgpu_debug_ipa_state: [(kind, key id, counts[max_values] int64)] of one pod's InterPodAffinity
        PreFilter maps on the device (kind 0 existing anti-affinity, 1 affinity, 2 anti-affinity)."""
        q = np.ascontiguousarray(np.asarray(query, abi.QUERY).reshape(1))
        kinds = np.zeros(max_maps, np.int32)
        keys = np.zeros(max_maps, np.int32)
        cnt = np.zeros((max_maps, max(max_values, 1)), np.int64)
        n = C.c_int32(0)
        self._check(lib().kgpu_debug_ipa_state(self.h, q.ctypes.data, C.byref(pools), max_maps, max(max_values, 1),
                                                kinds.ctypes.data, keys.ctypes.data, cnt.ctypes.data, C.byref(n)))
        return [(int(kinds[m]), int(keys[m]), cnt[m, :max_values]) for m in range(n.value)]

    def next_slot(self):
        """kgpu_next_slot: the slot the next pod assumed by kgpu_schedule_* gets."""
        return int(lib().kgpu_next_slot(self.h))

    def prepare_pods(self, queries, pools):
        """kgpu_prepare_pods: intern the topology classes of pods expected soon and count their columns now."""
        q = np.ascontiguousarray(np.atleast_1d(queries), dtype=abi.QUERY)
        self._check(lib().kgpu_prepare_pods(self.h, q.ctypes.data, len(q), C.byref(pools)))

    def adopt_pod(self, slot, uid):
        """kgpu_adopt_pod: register the UID of a pod the device assumed in a batch (batch-ahead)."""
        self._check(lib().kgpu_adopt_pod(self.h, int(slot), int(uid)))

    def wg_trace(self, pods):
        """kgpu_debug_wg_trace: [pods][groups][8] per-workgroup stamps of the last traced k_tbatch run."""
        g = C.c_int32(0)
        probe = np.zeros(1, np.int64)
        lib().kgpu_debug_wg_trace(self.h, probe.ctypes.data, 0, C.byref(g))  # the run's workgroup count
        out = np.zeros(max(pods * g.value * 8, 1), np.int64)
        n = lib().kgpu_debug_wg_trace(self.h, out.ctypes.data, len(out), C.byref(g))
        return out[:n].reshape(-1, g.value, 8) if g.value else out[:0].reshape(0, 0, 8)

    def topo_resident(self):
        """kgpu_debug_topo_resident: (runs that started from the resident topology state, runs that
        recomputed it)."""
        out = np.zeros(2, np.int64)
        self._check(lib().kgpu_debug_topo_resident(self.h, out.ctypes.data))
        return int(out[0]), int(out[1])

    def counters(self):
        """kgpu_debug_counters: {coop_retries, persistent_launches, coop_launches, class_inits,
        pod_table_full_uploads}."""
        out = np.zeros(8, np.int64)
        n = lib().kgpu_debug_counters(self.h, out.ctypes.data, len(out))
        if n < 0:
            self._check(n)
        return dict(zip(["coop_retries", "persistent_launches", "coop_launches", "class_inits", "pod_table_full_uploads"],
                        [int(x) for x in out[:n]]))

    def broken_linear(self, points, utilizations):
        """kgpu_debug_broken_linear: the device's broken-linear shape function (the one
        RequestedToCapacityRatio scores with) over `points` [(utilization, score)], unscaled."""
        pts = (abi.ShapePoint * len(points))()
        for i, (u, sc) in enumerate(points):
            pts[i].utilization, pts[i].score = int(u), int(sc)
        p = np.ascontiguousarray(utilizations, np.int64)
        out = np.zeros(len(p), np.int64)
        self._check(lib().kgpu_debug_broken_linear(self.h, pts, len(points), p.ctypes.data, len(p), out.ctypes.data))
        return [int(x) for x in out]

    def xgmi_active(self):
        return bool(lib().kgpu_xgmi_active(self.h))

    def comm_info(self):
        """kgpu_comm_info: {rccl_nranks, rccl_rank, xgmi_nranks, xgmi_peers_mapped} as the library sees them."""
        out = np.zeros(4, np.int32)
        self._check(lib().kgpu_comm_info(self.h, out.ctypes.data))
        return {"rccl_nranks": int(out[0]), "rccl_rank": int(out[1]), "xgmi_nranks": int(out[2]),
                "xgmi_peers_mapped": int(out[3])}

    def comm_init(self, nranks, rank, uid):
        """Join the node-sharding communicator (RCCL): this engine holds one contiguous shard of the
        snapshot; every rank must then issue the same schedule calls with the same queries."""
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        self._check(lib().kgpu_comm_init(self.h, nranks, rank, buf))


def comm_unique_id():
    """128-byte RCCL unique id (rank 0 creates it, the caller broadcasts it)."""
    buf = (C.c_uint8 * 128)()
    rc = lib().kgpu_comm_unique_id(buf)
    if rc != 0:
        raise KgpuError(rc, "kgpu_comm_unique_id failed")
    return bytes(buf)


def filter_reasons(handle, query, pools, node, word, taints, scalar_names, filters=None):
    """kgpu_filter_reasons: the failing plugin's reasons for one node's status word, formatted by the
    library.  handle: an engine context, or None with `filters` (the profile's KGPU_F_* order) for
    pure formatting.  taints: the node's Spec.Taints as [(key, value, effect, dictionary id)] in spec
    order; scalar_names: the resource name of each of the query's scalar requests, in order."""
    q = np.ascontiguousarray(np.asarray(query, abi.QUERY).reshape(1))
    tr = (abi.TaintRef * max(len(taints), 1))()
    keep = []
    for i, (k, v, e, tid) in enumerate(taints):
        b = [x.encode() for x in (k, v, e)]
        keep.append(b)
        tr[i].key, tr[i].value, tr[i].effect, tr[i].id = b[0], b[1], b[2], int(tid)
    names = (C.c_char_p * max(len(scalar_names), 1))(*[n.encode() for n in scalar_names])
    fl = (C.c_int32 * max(len(filters or ()), 1))(*(filters or ()))
    a = abi.ReasonArgs(q.ctypes.data, C.pointer(pools), int(node), int(word) & 0xFFFFFFFF, tr, len(taints),
                       len(filters or ()), fl, names)
    need = C.c_int64(0)
    buf = C.create_string_buffer(512)
    L = lib()
    n = L.kgpu_filter_reasons(handle, C.byref(a), buf, len(buf), C.byref(need))
    if n == abi.E_CAPACITY:
        buf = C.create_string_buffer(need.value)
        n = L.kgpu_filter_reasons(handle, C.byref(a), buf, len(buf), C.byref(need))
    if n < 0:
        msg = L.kgpu_last_error(handle) if handle else b""
        raise KgpuError(n, (msg or b"kgpu_filter_reasons").decode())
    return [x.decode() for x in buf.raw[:need.value].split(b"\0")[:n]]


def debug_fail_alloc(countdown):
    """Test hook: the countdown-th host allocation point from now on throws std::bad_alloc inside
    the library (0: off); the entry point that reaches it must return KGPU_E_NOMEM."""
    lib().kgpu_debug_fail_alloc(int(countdown))


def shard_range(n_nodes, world, rank):
    """Contiguous shard of Snapshot.List() owned by `rank`: (node_base, count)."""
    base = rank * n_nodes // world
    return base, (rank + 1) * n_nodes // world - base
