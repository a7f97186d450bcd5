"""Compile k8s-v1-shaped objects into the engine's dictionary-encoded SoA inputs (include/kgpu.h).

The compile itself is libkgpu's (include/kgpu_compile.h, csrc/kgpu_compile.cpp): the one implementation
of the PreFilter-time string work that the Go shim calls too.  This module marshals dicts into its
descriptors (cdesc.py), holds the handles, and copies the results into numpy arrays:

  Compiler           kgpu_compiler: the cluster dictionaries of one upload epoch (label keys / values,
                     namespaces, taints, images, controller UIDs become dense ids)
  Pools              kgpu_pool_set: the records kgpu_range fields point into, interned by content
  compile_pod        kgpu_compile_pod -> kgpu_pod_query
  compile_snapshot   kgpu_compile_snapshot -> kgpu_snapshot columns (existing pods folded in)
  node_row / key_meta / node_lists   the delta stream's records (kgpu_apply_delta)

What stays host-side here is lister work the Go shim gets from the reference's own helpers:
helper.DefaultSelector (default_selector below, helper/spread.go:29-72) and the PodDisruptionBudget
selector check of preemption (label_selector_matches).
"""
import ctypes as C

import numpy as np

from . import abi
from . import api
from . import cdesc

HOSTNAME = api.LABEL_HOSTNAME

class StrDict:
    __slots__ = ("ids", "items")

    def __init__(self):
        self.ids, self.items = {}, []

    def add(self, s):
        i = self.ids.get(s)
        if i is None:
            i = self.ids[s] = len(self.items)
            self.items.append(s)
        return i

    def get(self, s):
        return self.ids.get(s, -1)

    def __len__(self):
        return len(self.items)


class KeySpace:
    """Label keys, each with its own dense value dictionary (values are topology domains)."""

    def __init__(self):
        self.keys = StrDict()
        self.vals = []

    def add(self, k, v):
        ki = self.keys.add(k)
        if ki == len(self.vals):
            self.vals.append(StrDict())
        return ki, self.vals[ki].add(v)

    def key(self, k):
        return self.keys.get(k)

    def add_key(self, k):
        ki = self.keys.add(k)
        if ki == len(self.vals):
            self.vals.append(StrDict())
        return ki

    def val(self, ki, v):
        return -1 if ki < 0 else self.vals[ki].get(v)


class CompileError(Exception):
    pass


class NeedsUpload(Exception):
    """A cluster change the device columns cannot absorb as a delta: upload the snapshot again."""


_POOL_FIELDS = (("reqs", abi.REQ), ("ints", np.dtype("<i4")), ("words", np.dtype("<u8")),
                ("node_terms", abi.NODE_TERM), ("pref_terms", abi.PREF_TERM), ("spreads", abi.SPREAD),
                ("pod_terms", abi.POD_TERM), ("scalars", abi.SCALAR_REQ), ("ports", abi.PORT))


def _copy(ptr, dtype, count, shape=None):
    """A numpy copy of `count` records at a C pointer (owned by the compiler)."""
    dtype = np.dtype(dtype)
    if not count:
        out = np.zeros(0, dtype)
    else:
        buf = (C.c_char * (dtype.itemsize * int(count))).from_address(ptr)
        out = np.frombuffer(buf, dtype).copy()
    return out.reshape(shape) if shape is not None else out


def pools_numpy(view):
    """Numpy copies of a kgpu_pools view's records, by pool name."""
    return {f: _copy(getattr(view, f), dt, getattr(view, "n_" + f)) for f, dt in _POOL_FIELDS}


def pools_struct(P):
    """An abi.Pools pointing at the numpy arrays P (the struct keeps them alive)."""
    c = abi.Pools()
    for k, a in P.items():
        setattr(c, k, abi.ptr(a))
        setattr(c, "n_" + k, len(a))
    c._keep = P
    return c


class Pools:
    """A kgpu_pool_set: growable pools referenced by kgpu_range fields, interned by content (pods compiled
    from one template, a Deployment's replicas, share every record)."""

    def __init__(self):
        self._L = cdesc.lib()
        h = C.c_void_p()
        rc = self._L.kgpu_pools_create(C.byref(h))
        if rc != 0:
            raise MemoryError("kgpu_pools_create failed")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self._L.kgpu_pools_destroy(h)
            self.h = None

    def view(self):
        v = abi.Pools()
        self._L.kgpu_pools_view(self.h, C.byref(v))
        return v

    def scalar_name(self, i):
        s = cdesc.Str()
        if self._L.kgpu_pools_scalar_name(self.h, int(i), C.byref(s)) != 0:
            raise IndexError(i)
        return C.string_at(s.p, s.n).decode() if s.n else ""

    def finalize(self):
        """(abi.Pools over numpy copies of the records, {pool name: numpy array})."""
        P = pools_numpy(self.view())
        return pools_struct(P), P

def label_selector_matches(ps, labels):
    """Host-side evaluation of a LabelSelector against a label map (used for self-matches)."""
    if ps is None:
        return False
    ml = ps.get("matchLabels") or {}
    for k, v in ml.items():
        if labels.get(k) != v:
            return False
    for e in ps.get("matchExpressions") or []:
        k, op, vals = e.get("key", ""), e.get("operator"), e.get("values") or []
        if op == "In" and not (k in labels and labels[k] in vals):
            return False
        if op == "NotIn" and (k in labels and labels[k] in vals):
            return False
        if op == "Exists" and k not in labels:
            return False
        if op == "DoesNotExist" and k in labels:
            return False
    return True


def set_selector_matches(sel_map, labels):
    return all(labels.get(k) == v for k, v in sel_map.items())


class Profile:
    """KubeSchedulerProfile plugin set + plugin args (apis/config/types.go:115-239)."""

    DEFAULT_FILTERS = ["NodeUnschedulable", "NodeResourcesFit", "NodeName", "NodePorts", "NodeAffinity",
                       "TaintToleration", "PodTopologySpread", "InterPodAffinity"]
    DEFAULT_SCORES = [("NodeResourcesBalancedAllocation", 1), ("ImageLocality", 1), ("InterPodAffinity", 1),
                      ("NodeResourcesLeastAllocated", 1), ("NodeAffinity", 1), ("NodePreferAvoidPods", 10000),
                      ("PodTopologySpread", 2), ("DefaultPodTopologySpread", 1), ("TaintToleration", 1)]

    def __init__(self, filters=None, scores=None, least_resources=(("cpu", 1), ("memory", 1)),
                 most_resources=(("cpu", 1), ("memory", 1)), hard_pod_affinity_weight=1, ignored_resources=(),
                 pts_default_constraints=(), percentage_of_nodes_to_score=100, tie_break_mode=0, seed=0x7B,
                 rtcr_resources=(("cpu", 1), ("memory", 1)), rtcr_shape=((0, 10), (100, 0)), run_all_filters=False):
        """rtcr_*: RequestedToCapacityRatioArgs (apis/config/types_pluginargs.go): Resources as
        (name, weight), Shape as (utilization, score 0-10).  run_all_filters: the framework's
        runAllFilters (framework.go:90,155-160; the legacy Policy's AlwaysCheckAllPredicates,
        factory.go:278-281)."""
        self.run_all_filters = bool(run_all_filters)
        self.filters = list(self.DEFAULT_FILTERS if filters is None else filters)
        self.scores = [tuple(s) for s in (self.DEFAULT_SCORES if scores is None else scores)]
        self.least_resources = [tuple(r) for r in least_resources]
        self.most_resources = [tuple(r) for r in most_resources]
        self.hard_pod_affinity_weight = hard_pod_affinity_weight
        self.ignored_resources = set(ignored_resources)
        self.pts_default_constraints = list(pts_default_constraints)
        self.percentage_of_nodes_to_score = percentage_of_nodes_to_score
        self.tie_break_mode = tie_break_mode
        self.seed = seed
        self.rtcr_resources = [tuple(r) for r in rtcr_resources]
        self.rtcr_shape = [tuple(p) for p in rtcr_shape]
        for _, rl in (("least", self.least_resources), ("most", self.most_resources)):
            for n, w in rl:
                if w <= 0:
                    raise ValueError("resource Weight of %s should be a positive value, got %d" % (n, w))
                if w > 100:
                    raise ValueError("resource Weight of %s should be less than 100, got %d" % (n, w))

    @staticmethod
    def cluster_autoscaler(**kw):
        scores = [("NodeResourcesMostAllocated" if n == "NodeResourcesLeastAllocated" else n, w)
                  for n, w in Profile.DEFAULT_SCORES]
        return Profile(scores=scores, **kw)

    def has_score(self, name):
        return any(n == name for n, _ in self.scores)


class Cluster:
    """Objects that DefaultSelector lists (helper/spread.go): services, RCs, RSs, StatefulSets."""

    def __init__(self, services=(), rcs=(), rss=(), sss=()):
        self.services, self.rcs, self.rss, self.sss = list(services), list(rcs), list(rss), list(sss)


def default_selector(pod, cluster):
    """helper.DefaultSelector (helper/spread.go:29-72) -> LabelSelector dict or None (empty)."""
    ns = api.ns_of(pod)
    pl = api.labels_of(pod)
    label_set = {}
    for s in cluster.services:
        if api.ns_of(s) != ns:
            continue
        sel = api.spec(s).get("selector")
        if sel is None:
            continue
        if set_selector_matches(sel, pl):
            label_set.update(sel)
    exprs = []
    if pl:
        for rc in cluster.rcs:
            if api.ns_of(rc) != ns:
                continue
            sel = api.spec(rc).get("selector") or {}
            if not sel or not set_selector_matches(sel, pl):
                continue
            label_set.update(sel)
        for lst in (cluster.rss, cluster.sss):
            found, failed = [], False
            for o in lst:
                if api.ns_of(o) != ns:
                    continue
                ps = api.spec(o).get("selector")
                try:
                    if ps is not None:
                        for e in ps.get("matchExpressions") or []:
                            if e.get("operator") not in ("In", "NotIn", "Exists", "DoesNotExist"):
                                raise CompileError("bad op")
                except CompileError:
                    failed = True
                    break
                if ps is None or (not (ps.get("matchLabels") or {}) and not (ps.get("matchExpressions") or [])):
                    continue  # Nothing / Everything selectors are skipped (Empty() or no match)
                if not label_selector_matches(ps, pl):
                    continue
                found.append(ps)
            if not failed:
                for ps in found:
                    for k, v in sorted((ps.get("matchLabels") or {}).items()):
                        exprs.append({"key": k, "operator": "In", "values": [v]})
                    exprs.extend(ps.get("matchExpressions") or [])
    if not label_set and not exprs:
        return None
    return {"matchLabels": dict(label_set), "matchExpressions": exprs}


# ----------------------------------------------------------------- the compiler
class CDict:
    """One of the compiler's dictionaries (kgpu_dict_*): ids in first-seen order.  Taints are (key, value,
    effect) tuples and controllers (kind, uid) tuples, the others strings."""

    def __init__(self, comp, d, key=0):
        self.comp, self.d, self.key = comp, d, key
        self.parts = 3 if d == cdesc.DICT_TAINT else (2 if d == cdesc.DICT_CONTROLLER else 1)

    def _parts(self, x):
        xs = tuple(x) if self.parts > 1 else (x,)
        return (cdesc.Str * len(xs))(*[cdesc.s_(p if p is not None else "") for p in xs]), len(xs)

    def add(self, x):
        arr, n = self._parts(x)
        i = self.comp._L.kgpu_dict_add(self.comp._cc, self.d, self.key, arr, n)
        if i < 0:
            raise ValueError("kgpu_dict_add(%d): %d %s" % (self.d, i, self.comp._err()))
        return i

    def get(self, x):
        arr, n = self._parts(x)
        return self.comp._L.kgpu_dict_get(self.comp._cc, self.d, self.key, arr, n)

    def add_many(self, xs):
        """Single-part items in order, in one call (a columnar generator's million hostnames)."""
        bs = [x.encode() for x in xs]
        off = np.zeros(len(bs) + 1, np.int64)
        np.cumsum([len(b) for b in bs], out=off[1:])
        rc = self.comp._L.kgpu_dict_add_many(self.comp._cc, self.d, self.key, b"".join(bs), off.ctypes.data,
                                             len(bs), None)
        if rc != 0:
            raise ValueError("kgpu_dict_add_many: %d %s" % (rc, self.comp._err()))

    def __len__(self):
        return max(0, self.comp._L.kgpu_dict_size(self.comp._cc, self.d, self.key))

    def item(self, i):
        L = self.comp._L
        n = L.kgpu_dict_item(self.comp._cc, self.d, self.key, i, None, 0)
        buf = C.create_string_buffer(max(1, n))
        L.kgpu_dict_item(self.comp._cc, self.d, self.key, i, buf, n)
        s = buf.raw[:n].decode()
        return tuple(s.split("\0")) if self.parts > 1 else s

    @property
    def items(self):
        return [self.item(i) for i in range(len(self))]

    @property
    def ids(self):
        return {x: i for i, x in enumerate(self.items)}


class CKeySpace:
    """Label keys, each with its own value dictionary (values are topology domains)."""

    class _Vals:
        def __init__(self, ks):
            self.ks = ks

        def __getitem__(self, k):
            if k < 0 or k >= len(self):
                raise IndexError(k)
            return CDict(self.ks.comp, self.ks.vald, k)

        def __len__(self):
            return len(self.ks.keys)

        def __iter__(self):
            return (self[k] for k in range(len(self)))

    def __init__(self, comp, keyd, vald):
        self.comp, self.vald = comp, vald
        self.keys = CDict(comp, keyd)
        self.vals = CKeySpace._Vals(self)

    def add_key(self, k):
        return self.keys.add(k)

    def add(self, k, v):
        ki = self.keys.add(k)
        return ki, CDict(self.comp, self.vald, ki).add(v)

    def key(self, k):
        return self.keys.get(k)

    def val(self, ki, v):
        return -1 if ki < 0 else CDict(self.comp, self.vald, ki).get(v)


_SNAP_1D = (("alloc_cpu", "<i8"), ("alloc_mem", "<i8"), ("alloc_eph", "<i8"), ("alloc_pods", "<i4"),
            ("req_cpu", "<i8"), ("req_mem", "<i8"), ("req_eph", "<i8"), ("nz_cpu", "<i8"), ("nz_mem", "<i8"),
            ("num_pods", "<i4"), ("unschedulable", "u1"), ("zone_id", "<i4"), ("port_count", "<i4"))


class Compiler:
    """A kgpu_compiler: the cluster dictionaries of one upload epoch, and the compile of pods, snapshots and
    delta records against them (csrc/kgpu_compile.cpp)."""

    def __init__(self, profile, cluster=None):
        self.profile = profile
        self.cluster = cluster or Cluster()
        self._L = cdesc.lib()
        p, keep = cdesc.profile_desc(profile)
        h = C.c_void_p()
        rc = self._L.kgpu_compiler_create(C.byref(p), C.byref(h))
        if rc != 0:
            raise MemoryError("kgpu_compiler_create failed")
        self._cc = h
        self.nkeys = CKeySpace(self, cdesc.DICT_NODE_KEY, cdesc.DICT_NODE_VALUE)
        self.pkeys = CKeySpace(self, cdesc.DICT_POD_KEY, cdesc.DICT_POD_VALUE)
        for attr, d in (("ns", cdesc.DICT_NAMESPACE), ("taints", cdesc.DICT_TAINT), ("scalars", cdesc.DICT_SCALAR),
                        ("images", cdesc.DICT_IMAGE), ("controllers", cdesc.DICT_CONTROLLER),
                        ("uids", cdesc.DICT_UID), ("ips", cdesc.DICT_IP), ("protos", cdesc.DICT_PROTOCOL),
                        ("zones", cdesc.DICT_ZONE)):
            setattr(self, attr, CDict(self, d))
        self.order = []
        self.node_index = {}

    def __del__(self):
        h = getattr(self, "_cc", None)
        if h is not None and h.value:
            self._L.kgpu_compiler_destroy(h)
            self._cc = None

    def _err(self):
        m = self._L.kgpu_compiler_last_error(self._cc)
        return m.decode() if m else ""

    @property
    def dims(self):
        d = np.zeros(3, np.int32)
        self._L.kgpu_compiler_dims(self._cc, d.ctypes.data)
        return {"S": int(d[0]), "K": int(d[1]), "TW": int(d[2])}

    def set_order(self, names, first_wins=True):
        """The node list node names resolve against (Snapshot.List() order)."""
        names = list(names)
        bs = [n.encode() for n in names]
        off = np.zeros(len(bs) + 1, np.int64)
        np.cumsum([len(b) for b in bs], out=off[1:])
        rc = self._L.kgpu_compiler_set_order(self._cc, b"".join(bs), off.ctypes.data, len(bs), 1 if first_wins else 0)
        if rc != 0:
            raise ValueError(self._err())
        self.order = names
        idx = {}
        if first_wins:
            for i, nm in enumerate(names):
                idx.setdefault(nm, i)
        else:
            idx = {nm: i for i, nm in enumerate(names)}
        self.node_index = idx

    # -------------------------------------------------- dictionaries
    def register_node(self, n):
        cdesc.clear_cache()
        d = cdesc.node_desc(n)
        self._L.kgpu_compiler_register_node(self._cc, C.byref(d))

    def register_pod(self, p):
        cdesc.clear_cache()
        d = cdesc.pod_desc(p)
        self._L.kgpu_compiler_register_pod(self._cc, C.byref(d))

    def register(self, nodes, existing=(), pods=()):
        for n in nodes:
            self.register_node(n)
        for p in list(existing) + list(pods):
            self.register_pod(p)
        self.ns.add("")

    # -------------------------------------------------- snapshot
    def compile_snapshot(self, nodes, existing=(), shard=None, ordered=None, uid_of=None):
        """nodes: insertion order; returns (kgpu_snapshot ctypes struct, arrays dict, node names in
        Snapshot.List() order).  shard=(base, count) keeps only that slice of node rows.
        ordered: the node objects already in Snapshot.List() order (a cache mirror's nodeTree pass);
        uid_of(pod) -> int64: fills kgpu_snapshot.pod_uid so that deltas can address the pods."""
        cdesc.clear_cache()
        ordered = api.snapshot_order(nodes) if ordered is None else list(ordered)
        names = [api.name_of(n) for n in ordered]
        self.order, self.node_index = names, {nm: i for i, nm in enumerate(names)}
        nd = [cdesc.node_desc(n) for n in ordered]
        ex = list(existing)
        ed = [cdesc.pod_desc(p) for p in ex]
        uids = None
        if uid_of is not None:
            uids = np.array([uid_of(p) if (api.spec(p).get("nodeName", "") or "") in self.node_index else 0
                             for p in ex], np.int64)
        out = abi.Snapshot()
        base, cnt = (0, -1) if shard is None else shard
        rc = self._L.kgpu_compile_snapshot(self._cc, cdesc._arr(cdesc.NodeDesc, nd), len(nd),
                                           cdesc._arr(cdesc.PodDesc, ed), len(ed),
                                           uids.ctypes.data if uids is not None and len(uids) else None,
                                           base, cnt, C.byref(out))
        if rc != 0:
            raise CompileError(self._err())
        return self._take_snapshot(out, uids is not None)

    def snapshot_from_columns(self, A, shard=None):
        """The snapshot of node columns a columnar generator filled against the current dictionaries
        (A: alloc_*, unschedulable, label_val, taint_nosched / taint_prefer, zone_id, alloc_scalar in the
        order set by set_order), no existing pods (kgpu_compile_snapshot_columns)."""
        cols = abi.Snapshot()
        N = len(self.order)
        cols.n_nodes, cols.n_total_nodes = N, N
        keep = {}
        for f in ("alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "unschedulable", "zone_id", "alloc_scalar",
                  "label_val", "taint_nosched", "taint_prefer"):
            keep[f] = np.ascontiguousarray(A[f])
            setattr(cols, f, abi.ptr(keep[f]))
        cols.n_scalar = A["alloc_scalar"].shape[0]
        cols.n_label_keys = A["label_val"].shape[0]
        cols.taint_words = A["taint_nosched"].shape[0]
        out = abi.Snapshot()
        base, cnt = (0, -1) if shard is None else shard
        rc = self._L.kgpu_compile_snapshot_columns(self._cc, C.byref(cols), None, 0, None, base, cnt, C.byref(out))
        if rc != 0:
            raise CompileError(self._err())
        return self._take_snapshot(out, False)

    def empty_columns(self, N):
        """The node columns of an N-node snapshot against the current dictionaries, zeroed (for
        snapshot_from_columns)."""
        A = {}
        for f in ("alloc_cpu", "alloc_mem", "alloc_eph"):
            A[f] = np.zeros(N, np.int64)
        A["alloc_pods"] = np.zeros(N, np.int32)
        A["alloc_scalar"] = np.zeros((len(self.scalars), N), np.int64)
        A["unschedulable"] = np.zeros(N, np.uint8)
        A["label_val"] = np.full((len(self.nkeys.keys), N), -1, np.int32)
        TW = max(1, (len(self.taints) + 63) // 64)
        A["taint_nosched"] = np.zeros((TW, N), np.uint64)
        A["taint_prefer"] = np.zeros((TW, N), np.uint64)
        A["zone_id"] = np.full(N, -1, np.int32)
        return A

    def _take_snapshot(self, s, with_uids):
        """Numpy copies of the compiler's kgpu_snapshot arrays and an abi.Snapshot over them."""
        n, S, K, TW = s.n_nodes, s.n_scalar, s.n_label_keys, s.taint_words
        A = {}
        for f, dt in _SNAP_1D:
            A[f] = _copy(getattr(s, f), dt, n)
        A["alloc_scalar"] = _copy(s.alloc_scalar, "<i8", S * n, (S, n))
        A["req_scalar"] = _copy(s.req_scalar, "<i8", S * n, (S, n))
        A["label_val"] = _copy(s.label_val, "<i4", K * n, (K, n))
        A["key_n_values"] = _copy(s.key_n_values, "<i4", K)
        A["value_off"] = _copy(s.value_off, "<i4", K + 1)
        nv = int(A["value_off"][-1])
        A["value_int"] = _copy(s.value_int, "<i8", nv)
        A["value_int_ok"] = _copy(s.value_int_ok, "u1", nv)
        A["key_empty_value"] = _copy(s.key_empty_value, "<i4", K)
        A["key_unique"] = _copy(s.key_unique, "u1", K)
        A["taint_nosched"] = _copy(s.taint_nosched, "<u8", TW * n, (TW, n))
        A["taint_prefer"] = _copy(s.taint_prefer, "<u8", TW * n, (TW, n))
        A["port_slots"] = s.port_slots
        A["ports"] = _copy(s.ports, abi.PORT, s.port_slots * n, (s.port_slots, n))
        A["image_off"] = _copy(s.image_off, "<i4", n + 1)
        A["image_id"] = _copy(s.image_id, "<i4", int(A["image_off"][-1]))
        A["image_score"] = _copy(s.image_score, "<i8", int(A["image_off"][-1]))
        A["avoid_off"] = _copy(s.avoid_off, "<i4", n + 1)
        A["avoid_id"] = _copy(s.avoid_id, "<i4", int(A["avoid_off"][-1]))
        P, PK = s.n_pods, s.n_pod_label_keys
        A["pod_node"] = _copy(s.pod_node, "<i4", P)
        A["pod_ns"] = _copy(s.pod_ns, "<i4", P)
        A["pod_flags"] = _copy(s.pod_flags, "<u4", P)
        A["pod_label_val"] = _copy(s.pod_label_val, "<i4", PK * P, (PK, P))
        A["terms"] = _copy(s.terms, abi.TERM, s.n_terms)
        A["pod_uid"] = _copy(s.pod_uid, "<i8", P) if with_uids else None
        snap = abi.Snapshot()
        for f in ("n_nodes", "node_base", "n_total_nodes", "n_scalar", "n_label_keys", "taint_words", "port_slots",
                  "n_zones", "n_pods", "n_pod_label_keys", "n_terms"):
            setattr(snap, f, getattr(s, f))
        for f, a in A.items():
            if isinstance(a, np.ndarray):
                setattr(snap, f, abi.ptr(a))
        A["_pools_np"] = pools_numpy(s.pools)
        snap.pools = pools_struct(A["_pools_np"])
        A["_snap"] = snap
        return snap, A, self.order

    # -------------------------------------------------- node rows for deltas (kgpu_node_row)
    def node_row(self, n, pools):
        """kgpu_node_row of a v1.Node against the dictionaries of the last upload.  Raises NeedsUpload when
        the node brings a label key, taint word or scalar resource the device columns have no room for;
        new values of known keys grow the dictionaries (key_meta)."""
        cdesc.clear_cache()
        r = np.zeros((), abi.NODE_ROW)
        d = cdesc.node_desc(n)
        rc = self._L.kgpu_compile_node_row(self._cc, pools.h, C.byref(d), r.ctypes.data)
        if rc == abi.E_CAPACITY:
            raise NeedsUpload(self._err())
        if rc != 0:
            raise CompileError(self._err())
        return r

    def key_meta(self):
        """key_n_values / value_off / value_int / value_int_ok / key_empty_value of the node keys."""
        m = cdesc.KeyMeta()
        rc = self._L.kgpu_compiler_key_meta(self._cc, C.byref(m))
        if rc != 0:
            raise CompileError(self._err())
        K = m.n_keys
        return {"key_n_values": _copy(m.key_n_values, "<i4", K), "value_off": _copy(m.value_off, "<i4", K + 1),
                "value_int": _copy(m.value_int, "<i8", m.n_values),
                "value_int_ok": _copy(m.value_int_ok, "u1", m.n_values),
                "key_empty_value": _copy(m.key_empty_value, "<i4", K)}

    def node_lists(self, ordered, all_nodes=None):
        """ImageLocality scaledImageScore CSR (image_locality.go:100-113: NumNodes of the image over the
        cache's nodes, spread over len(NodeInfos().List())) and the NodePreferAvoidPods CSR, in list
        order."""
        cdesc.clear_cache()
        ordered = list(ordered)
        al = ordered if all_nodes is None else list(all_nodes)
        od = [cdesc.node_desc(n) for n in ordered]
        ad = od if all_nodes is None else [cdesc.node_desc(n) for n in al]
        out = cdesc.NodeLists()
        rc = self._L.kgpu_compile_node_lists(self._cc, cdesc._arr(cdesc.NodeDesc, od), len(od),
                                             cdesc._arr(cdesc.NodeDesc, ad), len(ad), C.byref(out))
        if rc != 0:
            raise CompileError(self._err())
        n = out.n_nodes
        return {"image_off": _copy(out.image_off, "<i4", n + 1), "image_id": _copy(out.image_id, "<i4", out.n_images),
                "image_score": _copy(out.image_score, "<i8", out.n_images),
                "avoid_off": _copy(out.avoid_off, "<i4", n + 1), "avoid_id": _copy(out.avoid_id, "<i4", out.n_avoid)}

    # -------------------------------------------------- pod queries
    def pod_desc(self, pod):
        """kgpu_pod_desc of a pod, with its DefaultSelector from this compiler's cluster listers."""
        return cdesc.pod_desc(pod, default_selector(pod, self.cluster))

    def compile_pod(self, pod, pools):
        cdesc.clear_cache()
        q = np.zeros((), abi.QUERY)
        d = self.pod_desc(pod)
        rc = self._L.kgpu_compile_pod(self._cc, pools.h, C.byref(d), q.ctypes.data)
        if rc != 0:
            raise CompileError(self._err())
        return q

    def compile_pods(self, pods, pools):
        """kgpu_compile_pods over `pods` in one call: (queries, {index: error message})."""
        cdesc.clear_cache()
        pods = list(pods)
        q = np.zeros(len(pods), abi.QUERY)
        if not pods:
            return q, {}
        descs = cdesc._arr(cdesc.PodDesc, [self.pod_desc(p) for p in pods])
        status = np.zeros(len(pods), np.int32)
        rc = self._L.kgpu_compile_pods(self._cc, pools.h, descs, len(pods), q.ctypes.data, status.ctypes.data)
        if rc < 0:
            raise CompileError(self._err())
        errors = {}
        if rc:
            # the messages: compile the failed pods again one at a time (the batch keeps the last only)
            for i in np.nonzero(status)[0]:
                try:
                    self.compile_pod(pods[int(i)], pools)
                except CompileError as e:
                    errors[int(i)] = str(e)
        return q, errors

    def scalar_names(self, pod):
        """The resource name of each scalar request compile_pod writes for `pod`, in query order (what
        kgpu_filter_reasons quotes in "Insufficient <name>")."""
        pools = Pools()
        q = self.compile_pod(pod, pools)
        b, c = int(q["scalars"]["begin"]), int(q["scalars"]["count"])
        return [pools.scalar_name(b + i) for i in range(c)]

    # -------------------------------------------------- config
    def config(self, device=0, node_capacity=0, pod_capacity=0, term_capacity=0):
        prof = self.profile
        c = abi.Config()
        c.abi_version = abi.ABI_VERSION
        c.device = device
        fl = [abi.FILTER_IDS[f] for f in prof.filters if f in abi.FILTER_IDS]
        c.n_filters = len(fl)
        for i, f in enumerate(fl):
            c.filters[i] = f
        c.n_scores = len(prof.scores)
        for i, (n, w) in enumerate(prof.scores):
            c.scores[i] = abi.SCORE_IDS[n]
            c.score_weights[i] = w or 1
        for attr, lst in (("least", prof.least_resources), ("most", prof.most_resources),
                          ("rtcr", prof.rtcr_resources)):
            merged = {}
            for r, w in lst:
                merged[r] = w
            setattr(c, "n_" + attr, len(merged))
            arr = getattr(c, attr)
            for i, (r, w) in enumerate(merged.items()):
                rid = {"cpu": 0, "memory": 1, "ephemeral-storage": 2}.get(r)
                if rid is None:
                    rid = 3 + self.scalars.get(r) if api.is_scalar(r) else -1
                arr[i].resource, arr[i].weight = rid, w
        # Shape scores scale by MaxNodeScore / MaxCustomPriorityScore (requested_to_capacity_ratio.go:54-58)
        c.n_shape = len(prof.rtcr_shape)
        for i, (u, sc) in enumerate(prof.rtcr_shape):
            c.shape[i].utilization, c.shape[i].score = u, sc * (100 // 10)
        c.hard_pod_affinity_weight = prof.hard_pod_affinity_weight
        c.percentage_of_nodes_to_score = prof.percentage_of_nodes_to_score
        c.tie_break_mode = prof.tie_break_mode
        c.seed = prof.seed
        c.node_capacity, c.pod_capacity, c.term_capacity = node_capacity, pod_capacity, term_capacity
        return c
