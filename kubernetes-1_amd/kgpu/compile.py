"""Compile k8s-v1-shaped objects into the engine's dictionary-encoded SoA inputs (include/kgpu.h).

This is the host half of PreFilter: everything that is per-pod or per-object string work happens
here once (label keys/values, namespaces, taints, images and controller UIDs become dense ids;
selectors become requirement programs; tolerations become bit masks over the cluster's taint
dictionary), so that the device only ever compares integers.

Semantics follow the reference files cited at each step; the device and the C restatement
consume exactly these arrays.
"""
import numpy as np

from . import abi
from . import api

HOSTNAME = api.LABEL_HOSTNAME
_PROTO = {"TCP": 0, "UDP": 1, "SCTP": 2}


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


class Pools:
    """Growable pools referenced by kgpu_range fields.

    Ranges are interned by content: pods compiled from one template (a Deployment's replicas)
    share every record, so the device reads one cache-hot copy instead of a fresh line per pod."""

    def __init__(self):
        self.reqs, self.ints, self.words = [], [], []
        self.node_terms, self.pref_terms, self.spreads, self.pod_terms = [], [], [], []
        self.scalars, self.ports = [], []
        self._cache = {}
        self._np = None

    def _rng(self, lst, items):
        items = list(items)
        if not items:
            return (0, 0)
        key = (id(lst), tuple(items))
        r = self._cache.get(key)
        if r is None:
            r = self._cache[key] = (len(lst), len(items))
            lst.extend(items)
        return r

    def truncate(self, lst, n):
        """Drop records appended after position n (a compile step that failed half-way)."""
        del lst[n:]
        for k in [k for k, v in self._cache.items() if k[0] == id(lst) and v[0] + v[1] > n]:
            del self._cache[k]

    def ints_range(self, xs):
        return self._rng(self.ints, [int(x) for x in xs])

    def words_range(self, ws):
        return self._rng(self.words, [int(w) for w in ws])

    def finalize(self):
        P = {}
        P["reqs"] = np.array(self.reqs, dtype=abi.REQ) if self.reqs else np.zeros(0, abi.REQ)
        P["ints"] = np.array(self.ints, dtype=np.int32)
        P["words"] = np.array(self.words, dtype=np.uint64)
        P["node_terms"] = np.array(self.node_terms, dtype=abi.NODE_TERM) if self.node_terms else np.zeros(0, abi.NODE_TERM)
        P["pref_terms"] = np.array(self.pref_terms, dtype=abi.PREF_TERM) if self.pref_terms else np.zeros(0, abi.PREF_TERM)
        P["spreads"] = np.array(self.spreads, dtype=abi.SPREAD) if self.spreads else np.zeros(0, abi.SPREAD)
        P["pod_terms"] = np.array(self.pod_terms, dtype=abi.POD_TERM) if self.pod_terms else np.zeros(0, abi.POD_TERM)
        P["scalars"] = np.array(self.scalars, dtype=abi.SCALAR_REQ) if self.scalars else np.zeros(0, abi.SCALAR_REQ)
        P["ports"] = np.array(self.ports, dtype=abi.PORT) if self.ports else np.zeros(0, abi.PORT)
        self._np = P
        c = abi.Pools()
        for k, a in P.items():
            setattr(c, k, abi.ptr(a))
            setattr(c, "n_" + k, len(a))
        c._keep = P  # the struct holds raw pointers: the arrays live as long as it does
        return c, P


# ----------------------------------------------------------------- selector compilation
_LSEL = {"In": abi.OP_IN, "NotIn": abi.OP_NOTIN, "Exists": abi.OP_EXISTS, "DoesNotExist": abi.OP_DNE}
_NSEL = dict(_LSEL, Gt=abi.OP_GT, Lt=abi.OP_LT)


def _validate_req(key, op, vals):
    """labels.NewRequirement validation (selector.go:140-190); raises CompileError."""
    if not api.qualified_name_ok(key):
        raise CompileError("invalid label key %r" % key)
    if op in (abi.OP_IN, abi.OP_NOTIN) and len(vals) == 0:
        raise CompileError("values set can't be empty")
    if op in (abi.OP_EXISTS, abi.OP_DNE) and len(vals) != 0:
        raise CompileError("values set must be empty")
    if op in (abi.OP_GT, abi.OP_LT):
        if len(vals) != 1 or api.parse_int64(vals[0]) is None:
            raise CompileError("Gt/Lt needs one integer value")
    for v in vals:
        if not api.label_value_ok(v):
            raise CompileError("invalid label value %r" % v)


def _req_rec(ks, pools, key, op, vals, register=False):
    """register: pod label selectors add their key and values to the pod key space, so that a pod
    compiled later with that label gets the ids the selector already holds (node selectors run
    against the fixed node set of the snapshot and drop unknown values instead)."""
    if register:
        ki = ks.add_key(key)
        for v in vals if op in (abi.OP_IN, abi.OP_NOTIN) else ():
            ks.add(key, v)
    else:
        ki = ks.key(key)
    vids = []
    if op in (abi.OP_IN, abi.OP_NOTIN) and ki >= 0:
        vids = sorted({ks.val(ki, v) for v in vals} - {-1})
    imm = api.parse_int64(vals[0]) if op in (abi.OP_GT, abi.OP_LT) else 0
    return (ki, op, pools.ints_range(vids), imm)


def compile_label_selector(ks, pools, ps):
    """metav1.LabelSelectorAsSelector (apis/meta/v1/helpers.go:34-70) -> kgpu_selector tuple."""
    if ps is None:
        return (abi.SEL_NOTHING, 0, (0, 0))
    ml = ps.get("matchLabels") or {}
    me = ps.get("matchExpressions") or []
    recs = []
    for k in sorted(ml):
        _validate_req(k, abi.OP_IN, [ml[k]])
        recs.append(_req_rec(ks, pools, k, abi.OP_IN, [ml[k]], register=True))
    for e in me:
        op = _LSEL.get(e.get("operator"))
        if op is None:
            raise CompileError("invalid pod selector operator %r" % e.get("operator"))
        vals = list(e.get("values") or [])
        _validate_req(e.get("key", ""), op, vals)
        recs.append(_req_rec(ks, pools, e.get("key", ""), op, vals, register=True))
    return (abi.SEL_AND, 0, pools._rng(pools.reqs, recs))


def compile_node_reqs(ks, pools, nsm, validate=True):
    """NodeSelectorRequirementsAsSelector (helpers.go:237-267) body; returns a reqs range."""
    recs = []
    for e in nsm:
        op = _NSEL.get(e.get("operator"))
        if op is None:
            raise CompileError("invalid node selector operator %r" % e.get("operator"))
        vals = list(e.get("values") or [])
        if validate:
            _validate_req(e.get("key", ""), op, vals)
        recs.append(_req_rec(ks, pools, e.get("key", ""), op, vals))
    return pools._rng(pools.reqs, recs)


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


# ----------------------------------------------------------------- taints / tolerations
def _tolerates(t, key, value, effect):
    """v1.Toleration.ToleratesTaint (staging/src/k8s.io/api/core/v1/toleration.go:37-56)."""
    te = t.get("effect", "") or ""
    if te and te != effect:
        return False
    tk = t.get("key", "") or ""
    if tk and tk != key:
        return False
    op = t.get("operator", "") or ""
    if op in ("", "Equal"):
        return (t.get("value", "") or "") == value
    return op == "Exists"


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
                            if e.get("operator") not in _LSEL:
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
class Compiler:
    def __init__(self, profile, cluster=None):
        self.profile = profile
        self.cluster = cluster or Cluster()
        self.nkeys = KeySpace()       # node label keys / values
        self.pkeys = KeySpace()       # pod label keys / values
        self.ns = StrDict()
        self.taints = StrDict()       # (key, value, effect)
        self.scalars = StrDict()
        self.images = StrDict()
        self.controllers = StrDict()  # (kind, uid)
        self.uids = StrDict()         # pod UIDs (kgpu_pod_query.uid = id + 1; 0: none)
        self.ips = StrDict()
        self.ips.add("0.0.0.0")
        self.protos = StrDict()
        for p in ("TCP", "UDP", "SCTP"):
            self.protos.add(p)
        self.zones = StrDict()
        self.node_index = {}
        self.order = []
        for r, _ in list(profile.least_resources) + list(profile.most_resources) + list(profile.rtcr_resources):
            if r not in ("cpu", "memory", "ephemeral-storage"):
                self.scalars.add(r)

    # -------------------------------------------------- dictionaries
    def register_node(self, n):
        for k, v in api.labels_of(n).items():
            self.nkeys.add(k, v)
        for t in api.spec(n).get("taints") or []:
            self.taints.add((t.get("key", "") or "", t.get("value", "") or "", t.get("effect", "") or ""))
        for r in ((n.get("status") or {}).get("allocatable") or {}):
            if api.is_scalar(r):
                self.scalars.add(r)
        for im in (n.get("status") or {}).get("images") or []:
            for nm in im.get("names") or []:
                self.images.add(nm)
        for a in api.avoid_pods(n):
            self.controllers.add(a)
        z = api.zone_key(n)
        if z:
            self.zones.add(z)

    def register_pod(self, p):
        for k, v in api.labels_of(p).items():
            self.pkeys.add(k, v)
        self.ns.add(api.ns_of(p))
        for c in api.containers(p) + api.init_containers(p):
            for r in api.requests_of(c):
                if api.is_scalar(r):
                    self.scalars.add(r)
        oh = api.spec(p).get("overhead") or {}
        for r in oh:
            if api.is_scalar(r):
                self.scalars.add(r)
        for c in api.containers(p):
            for pt in c.get("ports") or []:
                if int(pt.get("hostPort", 0) or 0) > 0:
                    self.ips.add(pt.get("hostIP", "") or "0.0.0.0")
                    self.protos.add(pt.get("protocol", "") or "TCP")

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
        ordered = api.snapshot_order(nodes) if ordered is None else list(ordered)
        self.order = [api.name_of(n) for n in ordered]
        self.node_index = {nm: i for i, nm in enumerate(self.order)}
        N = len(ordered)
        A = self.empty_columns(N)
        img_lists, avoid_lists = [], []
        name_to_nodes = {}
        for n in ordered:
            for im in (n.get("status") or {}).get("images") or []:
                for nm in im.get("names") or []:
                    name_to_nodes.setdefault(nm, set()).add(api.name_of(n))
        for i, n in enumerate(ordered):
            al = (n.get("status") or {}).get("allocatable") or {}
            cpu = mem = eph = pods = 0
            for r, q in al.items():
                if r == "cpu":
                    cpu += api.q_milli(q)
                elif r == "memory":
                    mem += api.q_value(q)
                elif r == "pods":
                    pods += api.q_value(q)
                elif r == "ephemeral-storage":
                    eph += api.q_value(q)
                elif api.is_scalar(r):
                    A["alloc_scalar"][self.scalars.get(r), i] += api.q_value(q)
            A["alloc_cpu"][i], A["alloc_mem"][i], A["alloc_eph"][i], A["alloc_pods"][i] = cpu, mem, eph, pods
            A["unschedulable"][i] = 1 if api.spec(n).get("unschedulable") else 0
            for k, v in api.labels_of(n).items():
                ki = self.nkeys.key(k)
                A["label_val"][ki, i] = self.nkeys.val(ki, v)
            for t in api.spec(n).get("taints") or []:
                key = (t.get("key", "") or "", t.get("value", "") or "", t.get("effect", "") or "")
                tid = self.taints.get(key)
                w, b = divmod(tid, 64)
                if key[2] in ("NoSchedule", "NoExecute"):
                    A["taint_nosched"][w, i] |= np.uint64(1 << b)
                elif key[2] == "PreferNoSchedule":
                    A["taint_prefer"][w, i] |= np.uint64(1 << b)
            z = api.zone_key(n)
            A["zone_id"][i] = self.zones.get(z) if z else -1
            ims = {}
            for im in (n.get("status") or {}).get("images") or []:
                for nm in im.get("names") or []:
                    spread = float(len(name_to_nodes[nm])) / float(N)
                    ims[self.images.get(nm)] = int(float(int(im.get("sizeBytes", 0))) * spread)
            img_lists.append(sorted(ims.items()))
            av = set()
            for a in api.avoid_pods(n):
                av.add(self.controllers.get(a))
            avoid_lists.append(sorted(av))
        return self.finish_snapshot(A, img_lists, avoid_lists, existing, shard, uid_of)

    def empty_columns(self, N):
        """The node columns of an N-node snapshot against the current dictionaries, zeroed."""
        A = {}
        for f in ("alloc_cpu", "alloc_mem", "alloc_eph", "req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem"):
            A[f] = np.zeros(N, np.int64)
        A["alloc_pods"] = np.zeros(N, np.int32)
        A["num_pods"] = np.zeros(N, np.int32)
        S = len(self.scalars)
        A["alloc_scalar"] = np.zeros((S, N), np.int64)
        A["req_scalar"] = np.zeros((S, N), np.int64)
        A["unschedulable"] = np.zeros(N, np.uint8)
        A["label_val"] = np.full((len(self.nkeys.keys), N), -1, np.int32)
        TW = max(1, (len(self.taints) + 63) // 64)
        A["taint_nosched"] = np.zeros((TW, N), np.uint64)
        A["taint_prefer"] = np.zeros((TW, N), np.uint64)
        A["zone_id"] = np.full(N, -1, np.int32)
        return A

    def finish_snapshot(self, A, img_lists, avoid_lists, existing=(), shard=None, uid_of=None):
        """Everything after the per-node columns: existing pods, label-value metadata, the image /
        avoid CSRs, the shard slice and the kgpu_snapshot struct.  self.order / self.node_index
        hold Snapshot.List(); A holds empty_columns(N) filled in that order."""
        N = len(self.order)
        base, cnt = (0, N) if shard is None else shard
        S = len(self.scalars)
        K = len(self.nkeys.keys)
        TW = max(1, (len(self.taints) + 63) // 64)
        # existing pods -> node rows + pod table
        A.update(self._compile_existing(existing, A, uid_of))
        # label value metadata
        A["key_n_values"] = np.array([len(d) for d in self.nkeys.vals], np.int32) if K else np.zeros(0, np.int32)
        off = [0]
        ints, oks = [], []
        empty = []
        for ki in range(K):
            d = self.nkeys.vals[ki]
            for v in d.items:
                iv = api.parse_int64(v)
                ints.append(0 if iv is None else iv)
                oks.append(0 if iv is None else 1)
            off.append(len(ints))
            empty.append(d.get(""))
        A["value_off"] = np.array(off, np.int32)
        A["value_int"] = np.array(ints, np.int64)
        A["value_int_ok"] = np.array(oks, np.uint8)
        A["key_empty_value"] = np.array(empty, np.int32)
        A["key_unique"] = self.key_unique(A["label_val"])
        # images / avoid CSR
        A["image_off"], A["image_id"], A["image_score"] = self._csr(img_lists, True)
        A["avoid_off"], A["avoid_id"], _ = self._csr([[(a, 0) for a in lst] for lst in avoid_lists], False)
        # shard slice
        if shard is not None:
            A = self._slice(A, base, cnt)
        snap = abi.Snapshot()
        snap.n_nodes, snap.node_base, snap.n_total_nodes = cnt, base, N
        for f in ("alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "req_cpu", "req_mem", "req_eph", "nz_cpu",
                  "nz_mem", "num_pods", "alloc_scalar", "req_scalar", "unschedulable", "label_val", "key_n_values",
                  "value_off", "value_int", "value_int_ok", "key_empty_value", "taint_nosched", "taint_prefer",
                  "port_count", "ports", "image_off", "image_id", "image_score", "avoid_off", "avoid_id",
                  "zone_id", "pod_node", "pod_ns", "pod_flags", "pod_label_val", "terms", "pod_uid", "key_unique"):
            if A.get(f) is None:
                continue
            A[f] = np.ascontiguousarray(A[f])
            setattr(snap, f, abi.ptr(A[f]))
        self.dims = {"S": S, "K": K, "TW": TW}  # device column counts fixed by this upload
        snap.n_scalar = S
        snap.n_label_keys = K
        snap.taint_words = TW
        snap.port_slots = A["port_slots"]
        snap.n_zones = len(self.zones)
        snap.n_pods = len(A["pod_node"])
        snap.n_pod_label_keys = A["pod_label_val"].shape[0]  # keys registered later have no snapshot pod
        snap.n_terms = len(A["terms"])
        snap.pools, A["_pools_np"] = A["_pools"].finalize()
        A["_snap"] = snap
        return snap, A, self.order

    @staticmethod
    def key_unique(label_val):
        """kgpu_snapshot.key_unique over the WHOLE list (before any shard slice): per node label key,
        1 when no value labels two nodes -- the engine's hostname-like keys, whose counts a sharded
        topology run reads from the node's own column."""
        K = label_val.shape[0]
        out = np.zeros(K, np.uint8)
        for k in range(K):
            v = label_val[k][label_val[k] >= 0]
            out[k] = 1 if len(np.unique(v)) == len(v) else 0
        return out

    @staticmethod
    def _csr(lists, with_val):
        off = np.zeros(len(lists) + 1, np.int32)
        ids, vals = [], []
        for i, lst in enumerate(lists):
            off[i + 1] = off[i] + len(lst)
            for a, v in lst:
                ids.append(a)
                vals.append(v)
        return off, np.array(ids, np.int32), np.array(vals, np.int64)

    @staticmethod
    def _slice(A, base, cnt):
        out = dict(A)
        for f in ("alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "req_cpu", "req_mem", "req_eph", "nz_cpu",
                  "nz_mem", "num_pods", "unschedulable", "zone_id", "port_count"):
            out[f] = A[f][base:base + cnt]
        for f in ("alloc_scalar", "req_scalar", "label_val", "taint_nosched", "taint_prefer", "ports"):
            out[f] = A[f][:, base:base + cnt]
        for fo, fi, fv in (("image_off", "image_id", "image_score"), ("avoid_off", "avoid_id", None)):
            off = A[fo]
            lo, hi = off[base], off[base + cnt]
            out[fo] = off[base:base + cnt + 1] - lo
            out[fi] = A[fi][lo:hi]
            if fv:
                out[fv] = A[fv][lo:hi]
        return out

    def _compile_existing(self, existing, A, uid_of=None):
        N = len(self.order)
        pools = Pools()
        pod_node, pod_ns, pod_flags, pod_uid = [], [], [], []
        PK = len(self.pkeys.keys)
        plab = []
        terms = []
        used_ports = [[] for _ in range(N)]
        for p in existing:
            nn = api.spec(p).get("nodeName", "") or ""
            ni = self.node_index.get(nn)
            if ni is None:
                continue  # NewSnapshot keeps such pods on node-less NodeInfos: never scheduled onto
            res = api.PodResources(p)
            A["req_cpu"][ni] += res.cpu
            A["req_mem"][ni] += res.mem
            A["req_eph"][ni] += res.eph
            for r, v in res.scalars.items():
                A["req_scalar"][self.scalars.get(r), ni] += v
            A["nz_cpu"][ni] += res.nz_cpu
            A["nz_mem"][ni] += res.nz_mem
            A["num_pods"][ni] += 1
            for c in api.containers(p):
                for pt in c.get("ports") or []:
                    port = int(pt.get("hostPort", 0) or 0)
                    if port > 0:
                        used_ports[ni].append((self.ips.get(pt.get("hostIP", "") or "0.0.0.0"),
                                               self.protos.get(pt.get("protocol", "") or "TCP"), port))
            slot = len(pod_node)
            pod_node.append(ni)
            if uid_of is not None:
                pod_uid.append(uid_of(p))
            pod_ns.append(self.ns.get(api.ns_of(p)))
            fl = abi.PF_ACTIVE
            if api.meta(p).get("deletionTimestamp") is not None:
                fl |= abi.PF_TERMINATING
            a = api.spec(p).get("affinity")
            if a is not None and (a.get("podAffinity") is not None or a.get("podAntiAffinity") is not None):
                fl |= abi.PF_WITH_AFFINITY
            pod_flags.append(fl)
            row = [-1] * PK
            for k, v in api.labels_of(p).items():
                ki = self.pkeys.key(k)
                row[ki] = self.pkeys.val(ki, v)
            plab.append(row)
            for kind, t in self.pod_terms(p, pools):
                terms.append((slot, kind, t))
        P = len(pod_node)
        slots = max([len(u) for u in used_ports] + [1])
        port_count = np.array([len(u) for u in used_ports], np.int32)
        ports = np.zeros((slots, N), abi.PORT)
        for i, u in enumerate(used_ports):
            for s, (ip, pr, port) in enumerate(sorted(set(u))):
                ports[s, i] = (ip, pr, port, 0)
            port_count[i] = len(set(u))
        out = {"pod_node": np.array(pod_node, np.int32), "pod_ns": np.array(pod_ns, np.int32),
               "pod_flags": np.array(pod_flags, np.uint32),
               "pod_label_val": (np.array(plab, np.int32).T.copy() if P and PK else np.zeros((PK, P), np.int32)),
               "terms": np.array(terms, dtype=abi.TERM) if terms else np.zeros(0, abi.TERM),
               "port_count": port_count, "ports": ports, "port_slots": slots, "_pools": pools,
               "pod_uid": np.array(pod_uid, np.int64) if uid_of is not None else None}
        return out

    # -------------------------------------------------- node rows for deltas (kgpu_node_row)
    def node_row(self, n, pools):
        """kgpu_node_row of a v1.Node against the dictionaries of the last upload.  Raises
        NeedsUpload when the node brings a label key, taint word or scalar resource the device
        columns have no room for; new values of known keys grow the dictionaries (key_meta)."""
        dims = self.dims
        r = np.zeros((), abi.NODE_ROW)
        al = (n.get("status") or {}).get("allocatable") or {}
        cpu = mem = eph = pods = 0
        sc = [0] * dims["S"]
        for res, q in al.items():
            if res == "cpu":
                cpu += api.q_milli(q)
            elif res == "memory":
                mem += api.q_value(q)
            elif res == "pods":
                pods += api.q_value(q)
            elif res == "ephemeral-storage":
                eph += api.q_value(q)
            elif api.is_scalar(res):
                col = self.scalars.add(res)
                if col >= dims["S"]:
                    raise NeedsUpload("new scalar resource %r" % res)
                sc[col] += api.q_value(q)
        r["alloc_cpu"], r["alloc_mem"], r["alloc_eph"], r["alloc_pods"] = cpu, mem, eph, pods
        r["unschedulable"] = 1 if api.spec(n).get("unschedulable") else 0
        z = api.zone_key(n)
        r["zone_id"] = self.zones.add(z) if z else -1
        pairs = []
        for k, v in sorted(api.labels_of(n).items()):
            ki = self.nkeys.key(k)
            if ki < 0 or ki >= dims["K"]:
                raise NeedsUpload("new node label key %r" % k)
            pairs += [ki, self.nkeys.add(k, v)[1]]
        r["labels"] = pools.ints_range(pairs)
        TW = dims["TW"]
        words = [0] * (2 * TW)
        for t in api.spec(n).get("taints") or []:
            key = (t.get("key", "") or "", t.get("value", "") or "", t.get("effect", "") or "")
            tid = self.taints.add(key)
            w, b = divmod(tid, 64)
            if w >= TW:
                raise NeedsUpload("taint dictionary outgrew %d words" % TW)
            if key[2] in ("NoSchedule", "NoExecute"):
                words[w] |= 1 << b
            elif key[2] == "PreferNoSchedule":
                words[TW + w] |= 1 << b
        r["taints"] = pools.words_range(words) if any(words) else (0, 0)
        r["alloc_scalar"] = pools.words_range([v & 0xFFFFFFFFFFFFFFFF for v in sc]) if any(sc) else (0, 0)
        for im in (n.get("status") or {}).get("images") or []:
            for nm in im.get("names") or []:
                self.images.add(nm)
        for a in api.avoid_pods(n):
            self.controllers.add(a)
        return r

    def key_meta(self):
        """key_n_values / value_off / value_int / value_int_ok / key_empty_value of the node keys."""
        K = self.dims["K"]
        off, ints, oks, empty = [0], [], [], []
        for ki in range(K):
            d = self.nkeys.vals[ki]
            for v in d.items:
                iv = api.parse_int64(v)
                ints.append(0 if iv is None else iv)
                oks.append(0 if iv is None else 1)
            off.append(len(ints))
            empty.append(d.get(""))
        return {"key_n_values": np.array([len(self.nkeys.vals[k]) for k in range(K)], np.int32),
                "value_off": np.array(off, np.int32), "value_int": np.array(ints, np.int64),
                "value_int_ok": np.array(oks, np.uint8), "key_empty_value": np.array(empty, np.int32)}

    def node_lists(self, ordered, all_nodes=None):
        """ImageLocality scaledImageScore CSR (image_locality.go:100-113: NumNodes of the image over
        the cache's nodes, spread over len(NodeInfos().List())) and the NodePreferAvoidPods CSR, in
        list order."""
        N = len(ordered)
        name_to_nodes = {}
        for n in (ordered if all_nodes is None else all_nodes):
            for im in (n.get("status") or {}).get("images") or []:
                for nm in im.get("names") or []:
                    name_to_nodes.setdefault(nm, set()).add(api.name_of(n))
        img_lists, avoid_lists = [], []
        for n in ordered:
            ims = {}
            for im in (n.get("status") or {}).get("images") or []:
                for nm in im.get("names") or []:
                    spread = float(len(name_to_nodes[nm])) / float(N)
                    ims[self.images.add(nm)] = int(float(int(im.get("sizeBytes", 0))) * spread)
            img_lists.append(sorted(ims.items()))
            avoid_lists.append(sorted({self.controllers.add(a) for a in api.avoid_pods(n)}))
        out = {}
        out["image_off"], out["image_id"], out["image_score"] = self._csr(img_lists, True)
        out["avoid_off"], out["avoid_id"], _ = self._csr([[(a, 0) for a in lst] for lst in avoid_lists], False)
        return out

    # -------------------------------------------------- pod terms (framework/v1alpha1/types.go:92-160)
    def _pod_term(self, pod, term, pools, weight=0):
        ns = term.get("namespaces") or []
        names = ns if ns else [api.ns_of(pod)]
        sel = compile_label_selector(self.pkeys, pools, term.get("labelSelector"))
        nsr = pools.ints_range([self.ns.add(x) for x in sorted(set(names))])
        tk = term.get("topologyKey", "") or ""
        return (weight, self.nkeys.key(tk), nsr, sel)

    def _terms(self, pod, v1terms, pools, weighted):
        """getAffinityTerms / getWeightedAffinityTerms: any selector error drops the whole list."""
        if not v1terms:
            return []
        out = []
        save = (len(pools.reqs), len(pools.ints))
        try:
            for t in v1terms:
                if weighted:
                    out.append(self._pod_term(pod, t.get("podAffinityTerm") or {}, pools, int(t.get("weight", 0))))
                else:
                    out.append(self._pod_term(pod, t, pools))
        except CompileError:
            pools.truncate(pools.reqs, save[0])
            pools.truncate(pools.ints, save[1])
            return []
        return out

    def pod_terms(self, pod, pools):
        a = api.spec(pod).get("affinity")
        out = []
        if a is None:
            return out
        pa, paa = a.get("podAffinity"), a.get("podAntiAffinity")
        if pa is not None:
            for t in self._terms(pod, pa.get("requiredDuringSchedulingIgnoredDuringExecution"), pools, False):
                out.append((abi.TERM_REQ_AFF, t))
        if paa is not None:
            for t in self._terms(pod, paa.get("requiredDuringSchedulingIgnoredDuringExecution"), pools, False):
                out.append((abi.TERM_REQ_ANTI, t))
        if pa is not None:
            for t in self._terms(pod, pa.get("preferredDuringSchedulingIgnoredDuringExecution"), pools, True):
                out.append((abi.TERM_PREF_AFF, t))
        if paa is not None:
            for t in self._terms(pod, paa.get("preferredDuringSchedulingIgnoredDuringExecution"), pools, True):
                out.append((abi.TERM_PREF_ANTI, t))
        return out

    # -------------------------------------------------- pod query
    def _scalar_requests(self, res, pod):
        """[(resource name, kgpu_scalar_req)] of a pod in query order: its scalar requests (Fit checks
        them unless ignored, fit.go:247-264), then the scorers' scalar resources it does not request."""
        prof = self.profile
        out = []
        seen = set()
        for r, v in res.scalars.items():
            check = 0 if (api.is_extended(r) and r in prof.ignored_resources) else 1
            out.append((r, (self.scalars.get(r), check, v, api.PodResources._score(res, r, pod))))
            seen.add(r)
        for r, _ in list(prof.least_resources) + list(prof.most_resources):
            if r not in ("cpu", "memory", "ephemeral-storage") and r not in seen and api.is_scalar(r):
                out.append((r, (self.scalars.get(r), 0, 0, api.PodResources._score(res, r, pod))))
                seen.add(r)
        return out

    def scalar_names(self, pod):
        """The resource name of each scalar request compile_pod writes for `pod`, in query order (what
        kgpu_filter_reasons quotes in "Insufficient <name>")."""
        return [r for r, _ in self._scalar_requests(api.PodResources(pod), pod)]

    def compile_pod(self, pod, pools):
        q = np.zeros((), abi.QUERY)
        prof = self.profile
        flags = 0
        res = api.PodResources(pod)
        q["ns"] = self.ns.add(api.ns_of(pod))
        q["req"] = (res.cpu, res.mem, res.eph)
        q["nz"] = (res.nz_cpu, res.nz_mem)
        q["score_req"] = (res.score["cpu"], res.score["memory"], res.score["ephemeral-storage"])
        if res.fit_all_zero:
            flags |= abi.Q_FIT_ALL_ZERO
        sc = [rec for _, rec in self._scalar_requests(res, pod)]
        q["scalars"] = pools._rng(pools.scalars, sc)
        nn = api.spec(pod).get("nodeName", "") or ""
        q["node_name"] = -1 if nn == "" else self.node_index.get(nn, -2)
        q["n_containers"] = len(api.containers(pod))
        want = []
        for c in api.containers(pod):
            for pt in c.get("ports") or []:
                port = int(pt.get("hostPort", 0) or 0)
                if port > 0:
                    want.append((self.ips.add(pt.get("hostIP", "") or "0.0.0.0"),
                                 self.protos.add(pt.get("protocol", "") or "TCP"), port, 0))
        q["ports"] = pools._rng(pools.ports, want)
        tols = api.spec(pod).get("tolerations") or []
        TW = max(1, (len(self.taints) + 63) // 64)
        m_ns = [0] * TW
        m_pr = [0] * TW
        prefer_tols = [t for t in tols if not t.get("effect") or t.get("effect") == "PreferNoSchedule"]
        for tid, (k, v, e) in enumerate(self.taints.items):
            w, b = divmod(tid, 64)
            if e in ("NoSchedule", "NoExecute") and any(_tolerates(t, k, v, e) for t in tols):
                m_ns[w] |= 1 << b
            if e == "PreferNoSchedule" and any(_tolerates(t, k, v, e) for t in prefer_tols):
                m_pr[w] |= 1 << b
        q["tol_nosched"] = pools.words_range(m_ns)
        q["tol_prefer"] = pools.words_range(m_pr)
        if any(_tolerates(t, "node.kubernetes.io/unschedulable", "", "NoSchedule") for t in tols):
            flags |= abi.Q_TOLERATES_UNSCHED
        # nodeSelector map (labels.SelectorFromSet: no validation, helper/node_affinity.go:30-36)
        nsel = api.spec(pod).get("nodeSelector") or {}
        q["node_selector"] = compile_node_reqs(self.nkeys, pools, [{"key": k, "operator": "In", "values": [v]}
                                                                   for k, v in sorted(nsel.items())],
                                               validate=False)
        aff = api.spec(pod).get("affinity")
        na = aff.get("nodeAffinity") if aff is not None else None
        if na is not None and na.get("requiredDuringSchedulingIgnoredDuringExecution") is not None:
            flags |= abi.Q_REQ_NODE_AFFINITY
            terms = (na["requiredDuringSchedulingIgnoredDuringExecution"].get("nodeSelectorTerms")) or []
            recs = [self._node_term(t, pools) for t in terms]
            q["req_terms"] = pools._rng(pools.node_terms, recs)
        prefs = []
        if na is not None and na.get("preferredDuringSchedulingIgnoredDuringExecution") is not None:
            for t in na["preferredDuringSchedulingIgnoredDuringExecution"]:
                w = int(t.get("weight", 0))
                if w == 0:
                    continue
                me = ((t.get("preference") or {}).get("matchExpressions")) or []
                if not me:
                    prefs.append((w, 0, (abi.SEL_NOTHING, 0, (0, 0))))
                    continue
                try:
                    r = compile_node_reqs(self.nkeys, pools, me)
                except CompileError:
                    flags |= abi.Q_SCORE_ERROR
                    continue
                prefs.append((w, 0, (abi.SEL_AND, 0, r)))
        q["pref_terms"] = pools._rng(pools.pref_terms, prefs)
        imgs = [self.images.get(api.normalized_image_name(c.get("image", "") or "")) for c in api.containers(pod)]
        q["images"] = pools.ints_range(imgs)
        if all(i < 0 for i in imgs):
            flags |= abi.Q_NO_KNOWN_IMAGE  # image_locality.go:53-79: sumScores 0 -> score 0
        ref = api.controller_ref(pod)
        q["avoid_id"] = -1
        if ref is not None and ref.get("kind") in ("ReplicationController", "ReplicaSet"):
            q["avoid_id"] = self.controllers.get((ref.get("kind"), ref.get("uid")))
        # PodTopologySpread (common.go:44-99)
        tsc = api.spec(pod).get("topologySpreadConstraints") or []
        if tsc:
            flags |= abi.Q_HAS_TSC
        q["pts_hard"] = self._spreads(pod, tsc, "DoNotSchedule", pools)
        q["pts_soft"] = self._spreads(pod, tsc, "ScheduleAnyway", pools)
        # DefaultPodTopologySpread selector (default_pod_topology_spread.go:191-205)
        ds = default_selector(pod, self.cluster)
        q["dpts"] = (abi.SEL_AND, 0, (0, 0)) if ds is None else compile_label_selector(self.pkeys, pools, ds)
        if ds is None:
            q["dpts"]["kind"] = 2  # empty selector: countMatchingPods returns 0 (Empty())
        # InterPodAffinity (types.go:92-160)
        if aff is not None:
            if aff.get("podAffinity") is not None:
                flags |= abi.Q_HAS_POD_AFFINITY
            if aff.get("podAntiAffinity") is not None:
                flags |= abi.Q_HAS_POD_ANTI
        byk = {abi.TERM_REQ_AFF: [], abi.TERM_REQ_ANTI: [], abi.TERM_PREF_AFF: [], abi.TERM_PREF_ANTI: []}
        for kind, t in self.pod_terms(pod, pools):
            byk[kind].append(t)
        q["ipa_req_aff"] = pools._rng(pools.pod_terms, byk[abi.TERM_REQ_AFF])
        q["ipa_req_anti"] = pools._rng(pools.pod_terms, byk[abi.TERM_REQ_ANTI])
        q["ipa_pref_aff"] = pools._rng(pools.pod_terms, byk[abi.TERM_PREF_AFF])
        q["ipa_pref_anti"] = pools._rng(pools.pod_terms, byk[abi.TERM_PREF_ANTI])
        if byk[abi.TERM_REQ_AFF] and self._self_match_all(pod):
            flags |= abi.Q_SELF_MATCH_ALL_AFF
        pairs = []
        for k, v in sorted(api.labels_of(pod).items()):
            ki, vi = self.pkeys.add(k, v)
            pairs += [ki, vi]
        q["labels"] = pools.ints_range(pairs)
        if api.meta(pod).get("deletionTimestamp") is not None:
            flags |= abi.Q_TERMINATING
        q["flags"] = flags
        q["limits"] = api.pod_limits(pod)
        pr = api.spec(pod).get("priority")
        q["priority"] = 0 if pr is None else int(pr)  # podutil.GetPodPriority
        q["uid"] = 1 + self.uids.add(api.meta(pod).get("uid", "") or "%s/%s" % (api.ns_of(pod), api.name_of(pod)))
        return q

    def _self_match_all(self, pod):
        a = api.spec(pod).get("affinity") or {}
        terms = ((a.get("podAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution")) or []
        pl = api.labels_of(pod)
        for t in terms:
            ns = t.get("namespaces") or [api.ns_of(pod)]
            if api.ns_of(pod) not in ns or not label_selector_matches(t.get("labelSelector"), pl):
                return False
        return True

    def _node_term(self, t, pools):
        """One NodeSelectorTerm (helpers.go:317-346) -> kgpu_node_term tuple."""
        me = t.get("matchExpressions") or []
        mf = t.get("matchFields") or []
        never = (0, 0), -1, -1, 1, 0
        if not me and not mf:
            return never
        reqs = (0, 0)
        if me:
            try:
                reqs = compile_node_reqs(self.nkeys, pools, me)
            except CompileError:
                return never
        fop, fnode = -1, -1
        if mf:
            ins, notins = set(), set()
            for e in mf:
                op, vals = e.get("operator"), e.get("values") or []
                if op not in ("In", "NotIn") or len(vals) != 1:
                    return never
                key = e.get("key", "")
                if key != "metadata.name":
                    got = ""  # fields.Set{"metadata.name": ...}.Get(other) == ""
                    if (op == "In") != (got == vals[0]):
                        return never
                    continue
                (ins if op == "In" else notins).add(vals[0])
            if len(ins) > 1 or (ins & notins):
                return never
            if ins:
                fop, fnode = abi.OP_IN, self.node_index.get(next(iter(ins)), -1)
            elif notins:
                idx = [self.node_index[x] for x in notins if x in self.node_index]
                if len(idx) > 1:
                    raise CompileError("more than one metadata.name NotIn requirement in a term")
                if idx:
                    fop, fnode = abi.OP_NOTIN, idx[0]
            if me == [] and fop == -1:
                fop, fnode = abi.OP_NOTIN, -1  # fields only, all satisfied: matches every node
        return reqs, fop, fnode, 0, 0

    def _spreads(self, pod, tsc, action, pools):
        pl = api.labels_of(pod)
        cons = []
        if tsc:
            for c in tsc:
                if c.get("whenUnsatisfiable") == action:
                    cons.append((int(c.get("maxSkew", 0)), c.get("topologyKey", ""), c.get("labelSelector")))
        else:
            dflt = [c for c in self.profile.pts_default_constraints if c.get("whenUnsatisfiable") == action]
            if dflt:
                ds = default_selector(pod, self.cluster)
                if ds is not None:
                    cons = [(int(c.get("maxSkew", 0)), c.get("topologyKey", ""), ds) for c in dflt]
        recs = []
        for ms, key, ps in cons:
            sel = compile_label_selector(self.pkeys, pools, ps)
            recs.append((ms, self.nkeys.key(key), 1 if key == HOSTNAME else 0,
                         1 if label_selector_matches(ps, pl) else 0, sel))
        return pools._rng(pools.spreads, recs)

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
