"""ctypes binding of the compiler's C ABI (include/kgpu_compile.h) and the marshalling of k8s-v1-shaped
dicts into its descriptors.

Marshalling only: every semantic step of the compile (requests and their non-zero defaults, toleration
masks, selector programs, node terms, topology spread constraints, affinity terms, node columns) runs in
libkgpu's kgpu_compile.cpp, the same code the Go shim calls.  Here a dict becomes a descriptor: strings,
lists in object order, and quantities evaluated to (Value(), MilliValue()) exactly
(api.q_value / api.q_milli, resource/quantity.go:695-716).
"""
import ctypes as C
import os

from . import abi
from . import api

vp, i32, i64, u32 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32


class Str(C.Structure):
    _fields_ = [("p", C.c_char_p), ("n", i64)]


class KV(C.Structure):
    _fields_ = [("key", Str), ("value", Str)]


class Quantity(C.Structure):
    _fields_ = [("name", Str), ("value", i64), ("milli", i64)]


class Expr(C.Structure):
    _fields_ = [("key", Str), ("op", Str), ("values", C.POINTER(Str)), ("n_values", i32), ("pad", i32)]


class LabelSelector(C.Structure):
    _fields_ = [("present", i32), ("n_match_labels", i32), ("match_labels", C.POINTER(KV)),
                ("exprs", C.POINTER(Expr)), ("n_exprs", i32), ("pad", i32)]


class NodeTerm(C.Structure):
    _fields_ = [("exprs", C.POINTER(Expr)), ("fields", C.POINTER(Expr)), ("n_exprs", i32), ("n_fields", i32)]


class PrefNodeTerm(C.Structure):
    _fields_ = [("weight", i32), ("pad", i32), ("preference", NodeTerm)]


class PodTerm(C.Structure):
    _fields_ = [("weight", i32), ("n_namespaces", i32), ("namespaces", C.POINTER(Str)), ("topology_key", Str),
                ("selector", LabelSelector)]


class Toleration(C.Structure):
    _fields_ = [("key", Str), ("op", Str), ("value", Str), ("effect", Str)]


class Spread(C.Structure):
    _fields_ = [("max_skew", i32), ("pad", i32), ("topology_key", Str), ("when_unsatisfiable", Str),
                ("selector", LabelSelector)]


class Port(C.Structure):
    _fields_ = [("host_port", i32), ("pad", i32), ("host_ip", Str), ("protocol", Str)]


class Container(C.Structure):
    _fields_ = [("image", Str), ("requests", C.POINTER(Quantity)), ("limits", C.POINTER(Quantity)),
                ("ports", C.POINTER(Port)), ("n_requests", i32), ("n_limits", i32), ("n_ports", i32), ("pad", i32)]


PD_AFFINITY, PD_NODE_AFFINITY, PD_NODE_REQUIRED, PD_POD_AFFINITY, PD_POD_ANTI = 1, 2, 4, 8, 16
PD_TERMINATING, PD_PRIORITY, PD_CONTROLLER, PD_DEFAULT_SELECTOR = 32, 64, 128, 256


class PodDesc(C.Structure):
    _fields_ = [("name", Str), ("ns", Str), ("uid", Str), ("node_name", Str), ("flags", u32), ("priority", i32),
                ("labels", C.POINTER(KV)), ("containers", C.POINTER(Container)),
                ("init_containers", C.POINTER(Container)), ("overhead", C.POINTER(Quantity)),
                ("tolerations", C.POINTER(Toleration)), ("node_selector", C.POINTER(KV)),
                ("required_terms", C.POINTER(NodeTerm)), ("preferred_terms", C.POINTER(PrefNodeTerm)),
                ("affinity_required", C.POINTER(PodTerm)), ("affinity_preferred", C.POINTER(PodTerm)),
                ("anti_required", C.POINTER(PodTerm)), ("anti_preferred", C.POINTER(PodTerm)),
                ("spreads", C.POINTER(Spread)),
                ("n_labels", i32), ("n_containers", i32), ("n_init_containers", i32), ("n_overhead", i32),
                ("n_tolerations", i32), ("n_node_selector", i32), ("n_required_terms", i32),
                ("n_preferred_terms", i32), ("n_affinity_required", i32), ("n_affinity_preferred", i32),
                ("n_anti_required", i32), ("n_anti_preferred", i32), ("n_spreads", i32), ("pad", i32),
                ("controller_kind", Str), ("controller_uid", Str), ("default_selector", LabelSelector)]


class Taint(C.Structure):
    _fields_ = [("key", Str), ("value", Str), ("effect", Str)]


class Image(C.Structure):
    _fields_ = [("names", C.POINTER(Str)), ("n_names", i32), ("pad", i32), ("size_bytes", i64)]


class Avoid(C.Structure):
    _fields_ = [("kind", Str), ("uid", Str)]


class NodeDesc(C.Structure):
    _fields_ = [("name", Str), ("labels", C.POINTER(KV)), ("taints", C.POINTER(Taint)),
                ("allocatable", C.POINTER(Quantity)), ("images", C.POINTER(Image)), ("avoid", C.POINTER(Avoid)),
                ("n_labels", i32), ("n_taints", i32), ("n_allocatable", i32), ("n_images", i32), ("n_avoid", i32),
                ("unschedulable", i32)]


class DefaultSpread(C.Structure):
    _fields_ = [("max_skew", i32), ("pad", i32), ("topology_key", Str), ("when_unsatisfiable", Str)]


class CompileProfile(C.Structure):
    _fields_ = [("column_resources", C.POINTER(Str)), ("n_column_resources", i32), ("n_score_resources", i32),
                ("ignored_resources", C.POINTER(Str)), ("n_ignored_resources", i32), ("n_default_spreads", i32),
                ("default_spreads", C.POINTER(DefaultSpread))]


class KeyMeta(C.Structure):
    _fields_ = [("n_keys", i32), ("n_values", i32), ("key_n_values", vp), ("value_off", vp), ("value_int", vp),
                ("value_int_ok", vp), ("key_empty_value", vp)]


class NodeLists(C.Structure):
    _fields_ = [("n_nodes", i32), ("n_images", i32), ("n_avoid", i32), ("pad", i32), ("image_off", vp),
                ("image_id", vp), ("image_score", vp), ("avoid_off", vp), ("avoid_id", vp)]


STRUCT_SIZES = [(n, C.sizeof(t)) for n, t in (
    ("kgpu_str", Str), ("kgpu_kv", KV), ("kgpu_quantity", Quantity), ("kgpu_expr_desc", Expr),
    ("kgpu_label_selector_desc", LabelSelector), ("kgpu_node_term_desc", NodeTerm),
    ("kgpu_pref_node_term_desc", PrefNodeTerm), ("kgpu_pod_term_desc", PodTerm), ("kgpu_toleration_desc", Toleration),
    ("kgpu_spread_desc", Spread), ("kgpu_port_desc", Port), ("kgpu_container_desc", Container),
    ("kgpu_pod_desc", PodDesc), ("kgpu_taint_desc", Taint), ("kgpu_image_desc", Image), ("kgpu_avoid_desc", Avoid),
    ("kgpu_node_desc", NodeDesc), ("kgpu_default_spread", DefaultSpread), ("kgpu_compile_profile", CompileProfile),
    ("kgpu_key_meta", KeyMeta), ("kgpu_node_lists", NodeLists))]

(DICT_NODE_KEY, DICT_NODE_VALUE, DICT_POD_KEY, DICT_POD_VALUE, DICT_NAMESPACE, DICT_TAINT, DICT_SCALAR, DICT_IMAGE,
 DICT_CONTROLLER, DICT_UID, DICT_IP, DICT_PROTOCOL, DICT_ZONE) = range(13)

EXPORTS = ["kgpu_compile_struct_sizes", "kgpu_compiler_create", "kgpu_compiler_destroy", "kgpu_compiler_last_error",
           "kgpu_dict_add", "kgpu_dict_get", "kgpu_dict_size", "kgpu_dict_item", "kgpu_dict_add_many",
           "kgpu_compiler_register_node", "kgpu_compiler_register_pod", "kgpu_compiler_set_order",
           "kgpu_compiler_dims", "kgpu_pools_create", "kgpu_pools_destroy", "kgpu_pools_view",
           "kgpu_pools_scalar_name", "kgpu_compile_pod", "kgpu_compile_pods", "kgpu_compile_snapshot",
           "kgpu_compile_snapshot_columns", "kgpu_compile_node_row", "kgpu_compiler_key_meta",
           "kgpu_compile_node_lists"]

_lib = None


def lib():
    """libkgpu.so's compiler entries (KGPU_COMPILE_LIB: a stand-alone build of kgpu_compile.cpp, e.g. the
    sanitizer build of tests/test_sanitizers.py)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("KGPU_COMPILE_LIB")
    if path:
        L = C.CDLL(path)
    else:
        from . import native
        L = native.lib()
    P = C.POINTER
    L.kgpu_compile_struct_sizes.argtypes = [vp, i32]
    L.kgpu_compiler_create.argtypes = [P(CompileProfile), P(vp)]
    L.kgpu_compiler_destroy.argtypes = [vp]
    L.kgpu_compiler_last_error.argtypes = [vp]
    L.kgpu_compiler_last_error.restype = C.c_char_p
    L.kgpu_dict_add.argtypes = [vp, i32, i32, P(Str), i32]
    L.kgpu_dict_add.restype = i32
    L.kgpu_dict_get.argtypes = [vp, i32, i32, P(Str), i32]
    L.kgpu_dict_get.restype = i32
    L.kgpu_dict_size.argtypes = [vp, i32, i32]
    L.kgpu_dict_size.restype = i32
    L.kgpu_dict_item.argtypes = [vp, i32, i32, i32, vp, i64]
    L.kgpu_dict_item.restype = i64
    L.kgpu_dict_add_many.argtypes = [vp, i32, i32, C.c_char_p, vp, i32, vp]
    L.kgpu_compiler_register_node.argtypes = [vp, P(NodeDesc)]
    L.kgpu_compiler_register_pod.argtypes = [vp, P(PodDesc)]
    L.kgpu_compiler_set_order.argtypes = [vp, C.c_char_p, vp, i32, i32]
    L.kgpu_compiler_dims.argtypes = [vp, vp]
    L.kgpu_pools_create.argtypes = [P(vp)]
    L.kgpu_pools_destroy.argtypes = [vp]
    L.kgpu_pools_view.argtypes = [vp, P(abi.Pools)]
    L.kgpu_pools_scalar_name.argtypes = [vp, i32, P(Str)]
    L.kgpu_compile_pod.argtypes = [vp, vp, P(PodDesc), vp]
    L.kgpu_compile_pods.argtypes = [vp, vp, P(PodDesc), i32, vp, vp]
    L.kgpu_compile_snapshot.argtypes = [vp, P(NodeDesc), i32, P(PodDesc), i32, vp, i32, i32, P(abi.Snapshot)]
    L.kgpu_compile_snapshot_columns.argtypes = [vp, P(abi.Snapshot), P(PodDesc), i32, vp, i32, i32,
                                                P(abi.Snapshot)]
    L.kgpu_compile_node_row.argtypes = [vp, vp, P(NodeDesc), vp]
    L.kgpu_compiler_key_meta.argtypes = [vp, P(KeyMeta)]
    L.kgpu_compile_node_lists.argtypes = [vp, P(NodeDesc), i32, P(NodeDesc), i32, P(NodeLists)]
    out = (i32 * 64)()
    m = L.kgpu_compile_struct_sizes(out, 64)
    got = [int(out[i]) for i in range(m)]
    want = [s for _, s in STRUCT_SIZES]
    if got != want:
        bad = [(n, w, g) for (n, w), g in zip(STRUCT_SIZES, got) if w != g]
        raise RuntimeError("compiler descriptor layout mismatch (python, C): %r" % (bad,))
    _lib = L
    return L


# ------------------------------------------------------------------ marshalling
_STR = {}


def s_(x):
    """A kgpu_str of a Python string (cached: the bytes stay alive while the cache holds them)."""
    r = _STR.get(x)
    if r is None:
        b = (x if isinstance(x, str) else str(x)).encode()
        r = _STR[x] = Str(b, len(b))
    return r


def clear_cache():
    """Called between compile calls only: the C side copies every string it keeps."""
    if len(_STR) > 200000:
        _STR.clear()


def _arr(T, items):
    return (T * len(items))(*items) if items else None


def strs(xs):
    return _arr(Str, [s_(x) for x in xs])


_Q = {}


def quantity(name, q):
    key = (name, q)
    r = _Q.get(key)
    if r is None:
        r = Quantity(s_(name), api.q_value(q), api.q_milli(q))
        if len(_Q) < 100000:
            _Q[key] = r
    return r


def resource_list(rl):
    return [quantity(r, q) for r, q in (rl or {}).items()]


def kvs(m):
    return [KV(s_(k), s_(v)) for k, v in (m or {}).items()]


def _ne(v):
    return "" if v is None else v


def expr(e):
    vals = list(e.get("values") or [])
    return Expr(s_(_ne(e.get("key", ""))), s_(_ne(e.get("operator"))), strs(vals), len(vals), 0)


def label_selector(ps):
    if ps is None:
        return LabelSelector()
    ml = kvs(ps.get("matchLabels"))
    ex = [expr(e) for e in ps.get("matchExpressions") or []]
    return LabelSelector(1, len(ml), _arr(KV, ml), _arr(Expr, ex), len(ex), 0)


def node_term(t):
    me = [expr(e) for e in (t or {}).get("matchExpressions") or []]
    mf = [expr(e) for e in (t or {}).get("matchFields") or []]
    return NodeTerm(_arr(Expr, me), _arr(Expr, mf), len(me), len(mf))


def pod_term(t, weight=0):
    ns = list(t.get("namespaces") or [])
    return PodTerm(weight, len(ns), strs(ns), s_(t.get("topologyKey", "") or ""), label_selector(t.get("labelSelector")))


def _containers(cs):
    out = []
    for c in cs:
        res = c.get("resources") or {}
        req = resource_list(res.get("requests"))
        lim = resource_list(res.get("limits"))
        ports = [Port(int(pt.get("hostPort", 0) or 0), 0, s_(pt.get("hostIP", "") or ""),
                      s_(pt.get("protocol", "") or "")) for pt in c.get("ports") or []]
        out.append(Container(s_(c.get("image", "") or ""), _arr(Quantity, req), _arr(Quantity, lim),
                             _arr(Port, ports), len(req), len(lim), len(ports), 0))
    return out


def pod_desc(pod, default_selector=None):
    """kgpu_pod_desc of a v1.Pod dict; default_selector: helper.DefaultSelector's LabelSelector dict (None:
    Empty())."""
    md, sp = api.meta(pod), api.spec(pod)
    d = PodDesc()
    d.name, d.ns = s_(md.get("name", "") or ""), s_(md.get("namespace", "") or "")
    d.uid, d.node_name = s_(md.get("uid", "") or ""), s_(sp.get("nodeName", "") or "")
    flags = 0
    lab = kvs(md.get("labels"))
    d.labels, d.n_labels = _arr(KV, lab), len(lab)
    cs = _containers(sp.get("containers") or [])
    d.containers, d.n_containers = _arr(Container, cs), len(cs)
    ics = _containers(sp.get("initContainers") or [])
    d.init_containers, d.n_init_containers = _arr(Container, ics), len(ics)
    oh = sp.get("overhead")
    if oh is not None:
        ql = resource_list(oh)
        d.overhead, d.n_overhead = _arr(Quantity, ql), len(ql)
    tols = [Toleration(s_(t.get("key", "") or ""), s_(t.get("operator", "") or ""), s_(t.get("value", "") or ""),
                       s_(t.get("effect", "") or "")) for t in sp.get("tolerations") or []]
    d.tolerations, d.n_tolerations = _arr(Toleration, tols), len(tols)
    ns = kvs(sp.get("nodeSelector"))
    d.node_selector, d.n_node_selector = _arr(KV, ns), len(ns)
    a = sp.get("affinity")
    if a is not None:
        flags |= PD_AFFINITY
        na = a.get("nodeAffinity")
        if na is not None:
            flags |= PD_NODE_AFFINITY
            req = na.get("requiredDuringSchedulingIgnoredDuringExecution")
            if req is not None:
                flags |= PD_NODE_REQUIRED
                ts = [node_term(t) for t in req.get("nodeSelectorTerms") or []]
                d.required_terms, d.n_required_terms = _arr(NodeTerm, ts), len(ts)
            pts = [PrefNodeTerm(int(t.get("weight", 0)), 0, node_term(t.get("preference") or {}))
                   for t in na.get("preferredDuringSchedulingIgnoredDuringExecution") or []]
            d.preferred_terms, d.n_preferred_terms = _arr(PrefNodeTerm, pts), len(pts)
        for key, flag, rq, pf in (("podAffinity", PD_POD_AFFINITY, "affinity_required", "affinity_preferred"),
                                  ("podAntiAffinity", PD_POD_ANTI, "anti_required", "anti_preferred")):
            pa = a.get(key)
            if pa is None:
                continue
            flags |= flag
            r = [pod_term(t) for t in pa.get("requiredDuringSchedulingIgnoredDuringExecution") or []]
            w = [pod_term(t.get("podAffinityTerm") or {}, int(t.get("weight", 0)))
                 for t in pa.get("preferredDuringSchedulingIgnoredDuringExecution") or []]
            setattr(d, rq, _arr(PodTerm, r))
            setattr(d, "n_" + rq, len(r))
            setattr(d, pf, _arr(PodTerm, w))
            setattr(d, "n_" + pf, len(w))
    tsc = [Spread(int(c.get("maxSkew", 0)), 0, s_(_ne(c.get("topologyKey", ""))),
                  s_(_ne(c.get("whenUnsatisfiable", ""))), label_selector(c.get("labelSelector")))
           for c in sp.get("topologySpreadConstraints") or []]
    d.spreads, d.n_spreads = _arr(Spread, tsc), len(tsc)
    if md.get("deletionTimestamp") is not None:
        flags |= PD_TERMINATING
    pr = sp.get("priority")
    if pr is not None:
        flags |= PD_PRIORITY
        d.priority = int(pr)
    ref = api.controller_ref(pod)
    if ref is not None:
        flags |= PD_CONTROLLER
        d.controller_kind, d.controller_uid = s_(ref.get("kind") or ""), s_(ref.get("uid") or "")
    if default_selector is not None:
        flags |= PD_DEFAULT_SELECTOR
        d.default_selector = label_selector(default_selector)
    d.flags = flags
    return d


def node_desc(n):
    """kgpu_node_desc of a v1.Node dict (the preferAvoidPods annotation decoded by api.avoid_pods)."""
    md, sp, st = api.meta(n), api.spec(n), n.get("status") or {}
    d = NodeDesc()
    d.name = s_(md.get("name", "") or "")
    lab = kvs(md.get("labels"))
    d.labels, d.n_labels = _arr(KV, lab), len(lab)
    ts = [Taint(s_(t.get("key", "") or ""), s_(t.get("value", "") or ""), s_(t.get("effect", "") or ""))
          for t in sp.get("taints") or []]
    d.taints, d.n_taints = _arr(Taint, ts), len(ts)
    al = resource_list(st.get("allocatable"))
    d.allocatable, d.n_allocatable = _arr(Quantity, al), len(al)
    ims = []
    for im in st.get("images") or []:
        names = list(im.get("names") or [])
        ims.append(Image(strs(names), len(names), 0, int(im.get("sizeBytes", 0))))
    d.images, d.n_images = _arr(Image, ims), len(ims)
    av = [Avoid(s_(k or ""), s_(u or "")) for k, u in api.avoid_pods(n)]
    d.avoid, d.n_avoid = _arr(Avoid, av), len(av)
    d.unschedulable = 1 if sp.get("unschedulable") else 0
    return d


def profile_desc(profile):
    """kgpu_compile_profile of a compile.Profile; returns (struct, keepalive)."""
    score = [r for r, _ in list(profile.least_resources) + list(profile.most_resources)]
    cols = score + [r for r, _ in profile.rtcr_resources]
    ign = sorted(profile.ignored_resources)
    dflt = [DefaultSpread(int(c.get("maxSkew", 0)), 0, s_(c.get("topologyKey", "") or ""),
                          s_(c.get("whenUnsatisfiable", "") or "")) for c in profile.pts_default_constraints]
    keep = (strs(cols), strs(ign), _arr(DefaultSpread, dflt))
    p = CompileProfile(keep[0], len(cols), len(score), keep[1], len(ign), len(dflt), keep[2])
    return p, keep
