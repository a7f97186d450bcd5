"""ORACLE (test infrastructure only) -- restatement of the in-tree scheduler plugins
on the hot path, operating on k8s-v1-shaped dicts.

Each plugin follows the cited reference file; names and control flow mirror the Go code so
that a reader can check them side by side.  All int64 arithmetic is exact Python ints
(Go int64 does not overflow for any in-range input); float64 islands are Python floats
(IEEE double, no FMA contraction) evaluated in the reference's operation order.
"""
import json
import math

from . import labels as L
from . import nodeinfo as NI
from .golog import go_log

MAX_NODE_SCORE = 100
MIN_NODE_SCORE = 0

SUCCESS, ERROR, UNSCHEDULABLE, UNRESOLVABLE = 0, 1, 2, 3


class Status:
    __slots__ = ("code", "reasons")

    def __init__(self, code, *reasons):
        self.code, self.reasons = code, list(reasons)

    def __repr__(self):
        return "Status(%d, %r)" % (self.code, self.reasons)


def is_success(s):
    return s is None or s.code == SUCCESS


def code_of(s):
    return SUCCESS if s is None else s.code


def _spec(p):
    return p.get("spec") or {}


def tolerations(pod):
    return _spec(pod).get("tolerations") or []


def taints(node):
    return _spec(node).get("taints") or []


def toleration_tolerates_taint(t, taint):
    """staging/src/k8s.io/api/core/v1/toleration.go:37-56."""
    eff = t.get("effect", "") or ""
    if eff and eff != taint.get("effect", ""):
        return False
    key = t.get("key", "") or ""
    if key and key != taint.get("key", ""):
        return False
    op = t.get("operator", "") or ""
    if op in ("", "Equal"):
        return (t.get("value", "") or "") == (taint.get("value", "") or "")
    if op == "Exists":
        return True
    return False


def tolerations_tolerate_taint(tols, taint):
    return any(toleration_tolerates_taint(t, taint) for t in tols)


def pod_matches_node_selector_and_affinity_terms(pod, node):
    """plugins/helper/node_affinity.go:28-78."""
    nl = NI.labels_of(node)
    ns = _spec(pod).get("nodeSelector") or {}
    if len(ns) > 0:
        if not L.selector_from_set(ns).matches(nl):
            return False
    aff = _spec(pod).get("affinity")
    if aff is not None and aff.get("nodeAffinity") is not None:
        na = aff["nodeAffinity"]
        req = na.get("requiredDuringSchedulingIgnoredDuringExecution")
        if req is None:
            return True
        terms = req.get("nodeSelectorTerms") or []
        return L.match_node_selector_terms(terms, nl, {"metadata.name": NI.name(node)})
    return True


# ============================================================ NodeUnschedulable
class NodeUnschedulable:
    """nodeunschedulable/node_unschedulable.go:51-65."""
    name = "NodeUnschedulable"

    def filter(self, state, pod, ni):
        if ni is None or ni.node is None:
            return Status(UNRESOLVABLE, "node(s) had unknown conditions")
        tol = tolerations_tolerate_taint(tolerations(pod), {"key": "node.kubernetes.io/unschedulable",
                                                            "effect": "NoSchedule"})
        if (_spec(ni.node).get("unschedulable") or False) and not tol:
            return Status(UNRESOLVABLE, "node(s) were unschedulable")
        return None


# ============================================================ NodeName
class NodeName:
    """nodename/node_name.go:46-59."""
    name = "NodeName"

    def filter(self, state, pod, ni):
        nn = _spec(pod).get("nodeName", "") or ""
        if not (len(nn) == 0 or nn == NI.name(ni.node)):
            return Status(UNRESOLVABLE, "node(s) didn't match the requested hostname")
        return None


# ============================================================ NodePorts
class NodePorts:
    """nodeports/node_ports.go:60-129."""
    name = "NodePorts"

    def prefilter(self, state, pod):
        state["NodePorts"] = NI.pod_ports(pod)
        return None

    def filter(self, state, pod, ni):
        want = state.get("NodePorts")
        if want is None:
            return Status(ERROR, "error reading prefilter state")
        for cp in want:
            if ni.ports_conflict(cp.get("hostIP", ""), cp.get("protocol", ""), int(cp.get("hostPort", 0) or 0)):
                return Status(UNSCHEDULABLE, "node(s) didn't have free ports for the requested pod ports")
        return None


# ============================================================ NodeResourcesFit
class Fit:
    """noderesources/fit.go:112-267."""
    name = "NodeResourcesFit"

    def __init__(self, ignored_resources=()):
        self.ignored = set(ignored_resources or ())

    def prefilter(self, state, pod):
        state["PreFilterNodeResourcesFit"] = NI.compute_pod_resource_request(pod)
        return None

    def insufficient(self, req, ni):
        out = []
        if len(ni.pods) + 1 > ni.allocatable.allowed_pods:
            out.append("Too many pods")
        if req.milli_cpu == 0 and req.memory == 0 and req.eph == 0 and len(req.scalars or {}) == 0:
            return out
        if ni.allocatable.milli_cpu < req.milli_cpu + ni.requested.milli_cpu:
            out.append("Insufficient cpu")
        if ni.allocatable.memory < req.memory + ni.requested.memory:
            out.append("Insufficient memory")
        if ni.allocatable.eph < req.eph + ni.requested.eph:
            out.append("Insufficient ephemeral-storage")
        for rname, rq in (req.scalars or {}).items():
            if NI.is_extended(rname) and rname in self.ignored:
                continue
            if ni.allocatable.scalar(rname) < rq + ni.requested.scalar(rname):
                out.append("Insufficient %s" % rname)
        return out

    def filter(self, state, pod, ni):
        req = state.get("PreFilterNodeResourcesFit")
        if req is None:
            return Status(ERROR, "error reading prefilter state")
        ins = self.insufficient(req, ni)
        if ins:
            return Status(UNSCHEDULABLE, *ins)
        return None


# ============================================================ resource scorers
def _pod_score_request(pod, resource):
    """resource_allocation.go:118-142 calculatePodResourceRequest."""
    v = 0
    for c in NI.containers(pod):
        v += NI.nonzero_request(resource, ((c.get("resources") or {}).get("requests")) or {})
    for ic in NI.init_containers(pod):
        v = max(v, NI.nonzero_request(resource, ((ic.get("resources") or {}).get("requests")) or {}))
    oh = _spec(pod).get("overhead")
    if oh is not None and resource in oh:
        from .quantity import value
        v += value(oh[resource])
    return v


def _alloc_request(ni, pod, resource):
    """resource_allocation.go:92-113 calculateResourceAllocatableRequest."""
    pr = _pod_score_request(pod, resource)
    if resource == "cpu":
        return ni.allocatable.milli_cpu, ni.non_zero.milli_cpu + pr
    if resource == "memory":
        return ni.allocatable.memory, ni.non_zero.memory + pr
    if resource == "ephemeral-storage":
        return ni.allocatable.eph, ni.requested.eph + pr
    if NI.is_scalar_resource_name(resource):
        return ni.allocatable.scalar(resource), ni.requested.scalar(resource) + pr
    return 0, 0


def go_div(a, b):
    """Go int64 division truncates toward zero."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def validate_resource_weights(resources):
    """apis/config/validation ValidateNodeResources{Least,Most}AllocatedArgs."""
    for r in resources:
        w = r[1]
        if w <= 0:
            raise ValueError("resource Weight of %s should be a positive value, got %d" % (r[0], w))
        if w > MAX_NODE_SCORE:
            raise ValueError("resource Weight of %s should be less than 100, got %d" % (r[0], w))


class _ResourceScorer:
    def __init__(self, handle, resources):
        self.handle = handle
        validate_resource_weights(resources)
        self.weights = {}
        for name, w in resources:  # Go map: duplicate names collapse to the last weight
            self.weights[name] = w

    def score(self, state, pod, node_name):
        ni = self.handle.snapshot.get(node_name)
        node_score = weight_sum = 0
        for res, w in self.weights.items():
            alloc, req = _alloc_request(ni, pod, res)
            node_score += self.resource_score(req, alloc) * w
            weight_sum += w
        return go_div(node_score, weight_sum), None


class LeastAllocated(_ResourceScorer):
    """noderesources/least_allocated.go:47-117."""
    name = "NodeResourcesLeastAllocated"

    @staticmethod
    def resource_score(requested, capacity):
        if capacity == 0 or requested > capacity:
            return 0
        return go_div((capacity - requested) * MAX_NODE_SCORE, capacity)


class MostAllocated(_ResourceScorer):
    """noderesources/most_allocated.go:47-117."""
    name = "NodeResourcesMostAllocated"

    @staticmethod
    def resource_score(requested, capacity):
        if capacity == 0 or requested > capacity:
            return 0
        return go_div(requested * MAX_NODE_SCORE, capacity)


def go_round(x):
    """math.Round: half away from zero."""
    f = math.floor(abs(x) + 0.5)
    return int(f if x >= 0 else -f)


class RequestedToCapacityRatio:
    """noderesources/requested_to_capacity_ratio.go:42-170.  shape: (utilization, score 0-10)."""
    name = "RequestedToCapacityRatio"

    def __init__(self, handle, shape, resources):
        self.handle = handle
        # score scaled to MaxNodeScore / MaxCustomPriorityScore (:54-58)
        self.shape = [(int(u), int(sc) * (MAX_NODE_SCORE // 10)) for u, sc in shape]
        self.weights = {}
        for name, w in resources:          # :61-67: weight 0 -> 1, duplicate names: last wins
            self.weights[name] = w if w != 0 else 1

    def broken_linear(self, p):           # :150-170
        sh = self.shape
        for i in range(len(sh)):
            if p <= sh[i][0]:
                if i == 0:
                    return sh[0][1]
                return sh[i - 1][1] + go_div((sh[i][1] - sh[i - 1][1]) * (p - sh[i - 1][0]), sh[i][0] - sh[i - 1][0])
        return sh[-1][1]

    def resource_score(self, requested, capacity):  # :127-133
        if capacity == 0 or requested > capacity:
            return self.broken_linear(100)
        return self.broken_linear(100 - go_div((capacity - requested) * 100, capacity))

    def score(self, state, pod, node_name):
        ni = self.handle.snapshot.get(node_name)
        node_score = weight_sum = 0
        for res, w in self.weights.items():
            alloc, req = _alloc_request(ni, pod, res)
            rs = self.resource_score(req, alloc)
            if rs > 0:
                node_score += rs * w
                weight_sum += w
        if weight_sum == 0:
            return 0, None
        return go_round(float(node_score) / float(weight_sum)), None


def resource_limits(pod):
    """getResourceLimits (resource_limits.go:145-156): milliCPU, memory."""
    from .quantity import milli_value, value
    cpu = mem = 0
    for c in NI.containers(pod):
        lim = (c.get("resources") or {}).get("limits") or {}
        if "cpu" in lim:
            cpu += milli_value(lim["cpu"])
        if "memory" in lim:
            mem += value(lim["memory"])
    for c in NI.init_containers(pod):
        lim = (c.get("resources") or {}).get("limits") or {}
        if "cpu" in lim:
            cpu = max(cpu, milli_value(lim["cpu"]))
        if "memory" in lim:
            mem = max(mem, value(lim["memory"]))
    return cpu, mem


class ResourceLimits:
    """noderesources/resource_limits.go:30-160 (NodeResourceLimits)."""
    name = "NodeResourceLimits"

    def __init__(self, handle):
        self.handle = handle

    def prescore(self, state, pod, nodes):
        if len(nodes) == 0:
            return None
        state["PreScoreNodeResourceLimits"] = resource_limits(pod)
        return None

    def score(self, state, pod, node_name):
        ni = self.handle.snapshot.get(node_name)
        lim = state.get("PreScoreNodeResourceLimits")
        if lim is None:
            return 0, Status(ERROR, 'Error reading "PreScoreNodeResourceLimits" from cycleState')

        def compute(limit, allocatable):
            return 1 if (limit != 0 and allocatable != 0 and limit <= allocatable) else 0
        c = compute(lim[0], ni.allocatable.milli_cpu)
        m = compute(lim[1], ni.allocatable.memory)
        return (1 if (c == 1 or m == 1) else 0), None


def _fraction(req, cap):
    if cap == 0:
        return 1.0
    return float(req) / float(cap)


class BalancedAllocation:
    """noderesources/balanced_allocation.go:49-120 (BalanceAttachedNodeVolumes off)."""
    name = "NodeResourcesBalancedAllocation"

    def __init__(self, handle):
        self.handle = handle

    def score(self, state, pod, node_name):
        ni = self.handle.snapshot.get(node_name)
        ca, cr = _alloc_request(ni, pod, "cpu")
        ma, mr = _alloc_request(ni, pod, "memory")
        cpu_f = _fraction(cr, ca)
        mem_f = _fraction(mr, ma)
        if cpu_f >= 1 or mem_f >= 1:
            return 0, None
        diff = abs(cpu_f - mem_f)
        return int((1 - diff) * float(MAX_NODE_SCORE)), None


def default_normalize_score(max_priority, reverse, scores):
    """plugins/helper/normalize_score.go:26-54."""
    max_count = 0
    for s in scores:
        if s[1] > max_count:
            max_count = s[1]
    if max_count == 0:
        if reverse:
            for s in scores:
                s[1] = max_priority
        return None
    for s in scores:
        v = go_div(max_priority * s[1], max_count)
        if reverse:
            v = max_priority - v
        s[1] = v
    return None


# ============================================================ TaintToleration
class TaintToleration:
    """tainttoleration/taint_toleration.go:54-157."""
    name = "TaintToleration"

    def __init__(self, handle):
        self.handle = handle

    def filter(self, state, pod, ni):
        if ni is None or ni.node is None:
            return Status(ERROR, "invalid nodeInfo")
        tols = tolerations(pod)
        for t in taints(ni.node):
            if t.get("effect") not in ("NoSchedule", "NoExecute"):
                continue
            if not tolerations_tolerate_taint(tols, t):
                return Status(UNRESOLVABLE, "node(s) had taint {%s: %s}, that the pod didn't tolerate"
                              % (t.get("key", ""), t.get("value", "")))
        return None

    def prescore(self, state, pod, nodes):
        if len(nodes) == 0:
            return None
        state["PreScoreTaintToleration"] = [t for t in tolerations(pod)
                                            if not t.get("effect") or t.get("effect") == "PreferNoSchedule"]
        return None

    def score(self, state, pod, node_name):
        ni = self.handle.snapshot.get(node_name)
        tols = state.get("PreScoreTaintToleration")
        if tols is None:
            return 0, Status(ERROR, "error reading prescore state")
        n = 0
        for t in taints(ni.node):
            if t.get("effect") != "PreferNoSchedule":
                continue
            if not tolerations_tolerate_taint(tols, t):
                n += 1
        return n, None

    def normalize(self, state, pod, scores):
        return default_normalize_score(MAX_NODE_SCORE, True, scores)


# ============================================================ NodeAffinity
class NodeAffinity:
    """nodeaffinity/node_affinity.go:53-108."""
    name = "NodeAffinity"

    def __init__(self, handle):
        self.handle = handle

    def filter(self, state, pod, ni):
        if ni.node is None:
            return Status(ERROR, "node not found")
        if not pod_matches_node_selector_and_affinity_terms(pod, ni.node):
            return Status(UNRESOLVABLE, "node(s) didn't match node selector")
        return None

    def score(self, state, pod, node_name):
        ni = self.handle.snapshot.get(node_name)
        aff = _spec(pod).get("affinity")
        count = 0
        if aff is not None and aff.get("nodeAffinity") is not None:
            pref = aff["nodeAffinity"].get("preferredDuringSchedulingIgnoredDuringExecution")
            if pref is not None:
                for t in pref:
                    w = int(t.get("weight", 0))
                    if w == 0:
                        continue
                    try:
                        sel = L.node_selector_requirements_as_selector(
                            ((t.get("preference") or {}).get("matchExpressions")) or [])
                    except L.SelectorError as e:
                        return 0, Status(ERROR, str(e))
                    if sel.matches(NI.labels_of(ni.node)):
                        count += w
        return count, None

    def normalize(self, state, pod, scores):
        return default_normalize_score(MAX_NODE_SCORE, False, scores)


# ============================================================ ImageLocality
MB = 1024 * 1024
MIN_THRESHOLD = 23 * MB
MAX_CONTAINER_THRESHOLD = 1000 * MB


def normalized_image_name(n):
    if n.rfind(":") <= n.rfind("/"):
        n = n + ":latest"
    return n


class ImageLocality:
    """imagelocality/image_locality.go:53-125."""
    name = "ImageLocality"

    def __init__(self, handle):
        self.handle = handle

    def score(self, state, pod, node_name):
        ni = self.handle.snapshot.get(node_name)
        total = self.handle.snapshot.num_nodes_listed()
        s = 0
        cs = NI.containers(pod)
        for c in cs:
            st = ni.image_states.get(normalized_image_name(c.get("image", "") or ""))
            if st is not None:
                size, num = st
                spread = float(num) / float(total)
                s += int(float(size) * spread)
        max_t = MAX_CONTAINER_THRESHOLD * len(cs)
        if s < MIN_THRESHOLD:
            s = MIN_THRESHOLD
        elif s > max_t:
            s = max_t
        return go_div(MAX_NODE_SCORE * (s - MIN_THRESHOLD), (max_t - MIN_THRESHOLD)), None


# ============================================================ NodePreferAvoidPods
def controller_ref(pod):
    for o in ((pod.get("metadata") or {}).get("ownerReferences")) or []:
        if o.get("controller"):
            return o
    return None


class NodePreferAvoidPods:
    """nodepreferavoidpods/node_prefer_avoid_pods.go:47-82.

    The node annotation scheduler.alpha.kubernetes.io/preferAvoidPods (JSON, as in the reference)
    is decoded by _avoids; the already-decoded shorthand node.metadata.annotations["preferAvoidPods"]
    = [{"kind": ..., "uid": ...}] is accepted beside it.
    """
    name = "NodePreferAvoidPods"

    def __init__(self, handle):
        self.handle = handle

    def score(self, state, pod, node_name):
        ni = self.handle.snapshot.get(node_name)
        ref = controller_ref(pod)
        if ref is not None and ref.get("kind") not in ("ReplicationController", "ReplicaSet"):
            ref = None
        if ref is None:
            return MAX_NODE_SCORE, None
        for kind, uid in _avoids(ni.node):
            if kind == ref.get("kind") and uid == ref.get("uid"):
                return 0, None
        return MAX_NODE_SCORE, None


def _json_field(d, key):
    # encoding/json: exact field name first, then a case-insensitive match
    if not isinstance(d, dict):
        return None
    if key in d:
        return d[key]
    return next((v for k, v in d.items() if k.lower() == key.lower()), None)


def _avoids(node):
    """v1helper.GetAvoidPodsFromNodeAnnotations (pkg/apis/core/v1/helper/helpers.go:500-509); a
    decode error reads as no entries (node_prefer_avoid_pods.go:68-72), entries without a
    podController are skipped (:73-78)."""
    ann = (node.get("metadata") or {}).get("annotations") or {}
    out = []
    raw = ann.get("scheduler.alpha.kubernetes.io/preferAvoidPods") or ""
    if raw:
        try:
            entries = _json_field(json.loads(raw), "preferAvoidPods") or []
            for a in entries:
                pc = _json_field(_json_field(a, "podSignature"), "podController")
                if pc is not None:
                    out.append((_json_field(pc, "kind") or "", _json_field(pc, "uid") or ""))
        except (ValueError, TypeError, AttributeError):
            out = []
    out += [(a.get("kind"), a.get("uid")) for a in ann.get("preferAvoidPods") or []]
    return out


# ============================================================ DefaultSelector (helper/spread.go:29-72)
def default_selector(pod, handle):
    ns = NI.namespace(pod)
    plabels = NI.labels_of(pod)
    label_set = {}
    for svc in handle.services:
        if NI.namespace(svc) != ns:
            continue
        sel = (svc.get("spec") or {}).get("selector")
        if sel is None:
            continue
        if L.selector_from_set(sel).matches(plabels):
            label_set.update(sel)
    if len(plabels) > 0:
        for rc in handle.rcs:
            if NI.namespace(rc) != ns:
                continue
            s = L.selector_from_set((rc.get("spec") or {}).get("selector") or {})
            if s.empty() or not s.matches(plabels):
                continue
            label_set.update((rc.get("spec") or {}).get("selector") or {})
    reqs = []
    if len(label_set) != 0:
        reqs = list(L.selector_from_set(label_set).reqs)
    for lst in (handle.rss, handle.sss):
        if len(plabels) == 0:
            continue  # Get{Pod}ReplicaSets/StatefulSets error out on label-less pods
        found, failed = [], False
        for obj in lst:
            if NI.namespace(obj) != ns:
                continue
            try:
                s = L.label_selector_as_selector((obj.get("spec") or {}).get("selector"))
            except L.SelectorError:
                failed = True  # the lister returns an error: none of its objects are used
                break
            if s.empty() or not s.matches(plabels):
                continue
            found.extend(s.reqs)
        if not failed:
            reqs.extend(found)
    return L.Selector(reqs)


# ============================================================ PodTopologySpread
def filter_tsc(constraints, action):
    out = []
    for c in constraints or []:
        if c.get("whenUnsatisfiable") == action:
            sel = L.label_selector_as_selector(c.get("labelSelector"))
            out.append((int(c.get("maxSkew", 0)), c.get("topologyKey", ""), sel))
    return out


def node_labels_match_spread(nl, constraints):
    return all(c[1] in nl for c in constraints)


def count_pods_match_selector(pod_infos, sel, ns):
    n = 0
    for pi in pod_infos:
        p = pi.pod
        if (p.get("metadata") or {}).get("deletionTimestamp") is not None or NI.namespace(p) != ns:
            continue
        if sel.matches(NI.labels_of(p)):
            n += 1
    return n


class CriticalPaths:
    """podtopologyspread/filtering.go:82-121."""

    def __init__(self):
        self.p = [["", 2 ** 31 - 1], ["", 2 ** 31 - 1]]

    def update(self, tpval, num):
        p = self.p
        i = -1
        if tpval == p[0][0]:
            i = 0
        elif tpval == p[1][0]:
            i = 1
        if i >= 0:
            p[i][1] = num
            if p[0][1] > p[1][1]:
                p[0], p[1] = p[1], p[0]
        else:
            if num < p[0][1]:
                p[1] = list(p[0])
                p[0] = [tpval, num]
            elif num < p[1][1]:
                p[1] = [tpval, num]


class PodTopologySpread:
    """podtopologyspread/{common,filtering,scoring}.go."""
    name = "PodTopologySpread"

    def __init__(self, handle, default_constraints=()):
        self.handle = handle
        self.default_constraints = list(default_constraints or [])

    def _constraints(self, pod, action):
        tsc = _spec(pod).get("topologySpreadConstraints") or []
        if len(tsc) > 0:
            return filter_tsc(tsc, action)
        cs = filter_tsc(self.default_constraints, action)
        if not cs:
            return []
        sel = default_selector(pod, self.handle)
        if sel.empty():
            return []
        return [(c[0], c[1], sel) for c in cs]

    # ---- filtering.go:146-273
    def prefilter(self, state, pod):
        try:
            cons = self._constraints(pod, "DoNotSchedule")
        except L.SelectorError as e:
            return Status(ERROR, str(e))
        if not cons:
            state["PreFilterPodTopologySpread"] = {"constraints": [], "pairs": {}, "paths": {}}
            return None
        pairs = {}
        for ni in self.handle.snapshot.list:
            node = ni.node
            if not pod_matches_node_selector_and_affinity_terms(pod, node):
                continue
            nl = NI.labels_of(node)
            if not node_labels_match_spread(nl, cons):
                continue
            for c in cons:
                pairs[(c[1], nl[c[1]])] = 0
        ns = NI.namespace(pod)
        for ni in self.handle.snapshot.list:
            nl = NI.labels_of(ni.node)
            for c in cons:
                pair = (c[1], nl.get(c[1], ""))
                if pair not in pairs:
                    continue
                pairs[pair] += count_pods_match_selector(ni.pods, c[2], ns)
        paths = {}
        for c in cons:
            paths[c[1]] = CriticalPaths()
        # map iteration order is random in Go; any order yields the same paths[0].MatchNum
        # unless a topology value is the empty string (see DESIGN.md determinism notes).
        for (k, v), n in sorted(pairs.items()):
            paths[k].update(v, n)
        state["PreFilterPodTopologySpread"] = {"constraints": cons, "pairs": pairs, "paths": paths}
        return None

    # ---- filtering.go:123-143, 161-180 (AddPod / RemovePod, used by the nominated-pod pass)
    def update_with_pod(self, state, updated_pod, preemptor, node, delta):
        s = state.get("PreFilterPodTopologySpread")
        if s is None or NI.namespace(updated_pod) != NI.namespace(preemptor) or node is None:
            return
        nl = NI.labels_of(node)
        if not node_labels_match_spread(nl, s["constraints"]):
            return
        plabels = NI.labels_of(updated_pod)
        for _, key, sel in s["constraints"]:
            if not sel.matches(plabels):
                continue
            pair = (key, nl[key])
            # *s.TpPairToMatchNum[pair] += delta: the reference dereferences a nil entry (panics) for a
            # pair no eligible node registered; only reachable on a node NodeAffinity rejects -- 0 here
            s["pairs"][pair] = s["pairs"].get(pair, 0) + delta
            s["paths"][key].update(nl[key], s["pairs"][pair])

    def add_pod(self, state, pod, pod_to_add, ni):
        self.update_with_pod(state, pod_to_add, pod, ni.node, 1)

    def remove_pod(self, state, pod, pod_to_remove, ni):
        self.update_with_pod(state, pod_to_remove, pod, ni.node, -1)

    def filter(self, state, pod, ni):
        s = state.get("PreFilterPodTopologySpread")
        if s is None:
            return Status(ERROR, "error reading prefilter state")
        if len(s["pairs"]) == 0 or len(s["constraints"]) == 0:
            return None
        nl = NI.labels_of(ni.node)
        plabels = NI.labels_of(pod)
        for max_skew, key, sel in s["constraints"]:
            if key not in nl:
                return Status(UNSCHEDULABLE, "node(s) didn't match pod topology spread constraints")
            self_match = 1 if sel.matches(plabels) else 0
            paths = s["paths"].get(key)
            if paths is None:
                continue
            min_match = paths.p[0][1]
            match = s["pairs"].get((key, nl[key]), 0)
            if match + self_match - min_match > max_skew:
                return Status(UNSCHEDULABLE, "node(s) didn't match pod topology spread constraints")
        return None

    # ---- scoring.go:59-257
    def prescore(self, state, pod, filtered):
        all_nodes = self.handle.snapshot.list
        if len(filtered) == 0 or len(all_nodes) == 0:
            return None
        try:
            cons = self._constraints(pod, "ScheduleAnyway")
        except L.SelectorError as e:
            return Status(ERROR, "error when calculating preScoreState: %s" % e)
        st = {"constraints": cons, "ignored": set(), "counts": {}, "weights": []}
        if cons:
            topo_size = [0] * len(cons)
            for node in filtered:
                nl = NI.labels_of(node)
                if not node_labels_match_spread(nl, cons):
                    st["ignored"].add(NI.name(node))
                    continue
                for i, c in enumerate(cons):
                    if c[1] == NI.LABEL_HOSTNAME:
                        continue
                    pair = (c[1], nl[c[1]])
                    if pair not in st["counts"]:
                        st["counts"][pair] = 0
                        topo_size[i] += 1
            for i, c in enumerate(cons):
                sz = topo_size[i]
                if c[1] == NI.LABEL_HOSTNAME:
                    sz = len(filtered) - len(st["ignored"])
                st["weights"].append(go_log(float(sz + 2)))
            ns = NI.namespace(pod)
            for ni in all_nodes:
                node = ni.node
                nl = NI.labels_of(node)
                if not pod_matches_node_selector_and_affinity_terms(pod, node) or \
                        not node_labels_match_spread(nl, cons):
                    continue
                for c in cons:
                    pair = (c[1], nl[c[1]])
                    if pair not in st["counts"]:
                        continue
                    st["counts"][pair] += count_pods_match_selector(ni.pods, c[2], ns)
        state["PreScorePodTopologySpread"] = st
        return None

    def score(self, state, pod, node_name):
        ni = self.handle.snapshot.get(node_name)
        s = state.get("PreScorePodTopologySpread")
        if s is None:
            return 0, Status(ERROR, "error reading prescore state")
        if node_name in s["ignored"]:
            return 0, None
        nl = NI.labels_of(ni.node)
        score = 0.0
        ns = NI.namespace(pod)
        for i, (max_skew, key, sel) in enumerate(s["constraints"]):
            if key in nl:
                if key == NI.LABEL_HOSTNAME:
                    cnt = count_pods_match_selector(ni.pods, sel, ns)
                else:
                    cnt = s["counts"][(key, nl[key])]
                if cnt < max_skew:
                    cnt = max_skew - 1
                score += float(cnt) * s["weights"][i]
        return int(score), None

    def normalize(self, state, pod, scores):
        s = state.get("PreScorePodTopologySpread")
        if s is None:
            return Status(ERROR, "error reading prescore state")
        min_s, max_s = 2 ** 63 - 1, 0
        for sc in scores:
            if sc[0] in s["ignored"]:
                continue
            min_s = min(min_s, sc[1])
            max_s = max(max_s, sc[1])
        for sc in scores:
            if sc[0] in s["ignored"]:
                sc[1] = 0
                continue
            if max_s == 0:
                sc[1] = MAX_NODE_SCORE
                continue
            sc[1] = go_div(MAX_NODE_SCORE * (max_s + min_s - sc[1]), max_s)
        return None


# ============================================================ DefaultPodTopologySpread
ZONE_WEIGHTING = 2.0 / 3.0


class DefaultPodTopologySpread:
    """defaultpodtopologyspread/default_pod_topology_spread.go:75-213."""
    name = "DefaultPodTopologySpread"

    def __init__(self, handle):
        self.handle = handle

    @staticmethod
    def _skip(pod):
        return len(_spec(pod).get("topologySpreadConstraints") or []) != 0

    def prescore(self, state, pod, nodes):
        state["PreScoreDefaultPodTopologySpread"] = default_selector(pod, self.handle)
        return None

    def score(self, state, pod, node_name):
        if self._skip(pod):
            return 0, None
        sel = state.get("PreScoreDefaultPodTopologySpread")
        if sel is None:
            return 0, Status(ERROR, "error reading prescore state")
        ni = self.handle.snapshot.get(node_name)
        if len(ni.pods) == 0 or sel.empty():
            return 0, None
        ns = NI.namespace(pod)
        n = 0
        for pi in ni.pods:
            p = pi.pod
            if ns == NI.namespace(p) and (p.get("metadata") or {}).get("deletionTimestamp") is None:
                if sel.matches(NI.labels_of(p)):
                    n += 1
        return n, None

    def normalize(self, state, pod, scores):
        if self._skip(pod):
            return None
        counts_by_zone = {}
        max_zone = 0
        max_node = 0
        for sc in scores:
            if sc[1] > max_node:
                max_node = sc[1]
            z = NI.get_zone_key(self.handle.snapshot.get(sc[0]).node)
            if z == "":
                continue
            counts_by_zone[z] = counts_by_zone.get(z, 0) + sc[1]
        for z, v in counts_by_zone.items():
            if v > max_zone:
                max_zone = v
        have_zones = len(counts_by_zone) != 0
        fmax_node = float(max_node)
        fmax_zone = float(max_zone)
        M = float(MAX_NODE_SCORE)
        for sc in scores:
            f = M
            if max_node > 0:
                f = M * (float(max_node - sc[1]) / fmax_node)
            if have_zones:
                z = NI.get_zone_key(self.handle.snapshot.get(sc[0]).node)
                if z != "":
                    zs = M
                    if max_zone > 0:
                        zs = M * (float(max_zone - counts_by_zone[z]) / fmax_zone)
                    f = (f * (1.0 - ZONE_WEIGHTING)) + (ZONE_WEIGHTING * zs)
            sc[1] = int(f)
        return None


# ============================================================ InterPodAffinity
def pod_matches_term_ns_selector(pod, namespaces, sel):
    """util/topologies.go:40-49."""
    if NI.namespace(pod) not in namespaces:
        return False
    return sel.matches(NI.labels_of(pod))


def pod_matches_all_affinity_terms(pod, terms):
    if len(terms) == 0:
        return False
    for t in terms:
        if not pod_matches_term_ns_selector(pod, t.namespaces, t.selector):
            return False
    return True


def _update_with_affinity_terms(m, target_pod, target_node, terms, value):
    if pod_matches_all_affinity_terms(target_pod, terms):
        nl = NI.labels_of(target_node)
        for t in terms:
            if t.topology_key in nl:
                pair = (t.topology_key, nl[t.topology_key])
                m[pair] = m.get(pair, 0) + value
                if m[pair] == 0:
                    del m[pair]


def _update_with_anti_affinity_terms(m, target_pod, target_node, terms, value):
    nl = NI.labels_of(target_node)
    for a in terms:
        if pod_matches_term_ns_selector(target_pod, a.namespaces, a.selector):
            if a.topology_key in nl:
                pair = (a.topology_key, nl[a.topology_key])
                m[pair] = m.get(pair, 0) + value
                if m[pair] == 0:
                    del m[pair]


class InterPodAffinity:
    """interpodaffinity/{filtering,scoring}.go."""
    name = "InterPodAffinity"

    def __init__(self, handle, hard_pod_affinity_weight=1):
        self.handle = handle
        self.hard_weight = hard_pod_affinity_weight

    # ---- filtering.go:166-271
    def prefilter(self, state, pod):
        snap = self.handle.snapshot
        pi = NI.PodInfo(pod)
        existing_anti = {}
        for ni in snap.have_pods_with_affinity():
            for ep in ni.pods_with_affinity:
                _update_with_anti_affinity_terms(existing_anti, pod, ni.node, ep.req_anti, 1)
        aff, anti = {}, {}
        if len(pi.req_aff) != 0 or len(pi.req_anti) != 0:
            for ni in snap.list:
                for ep in ni.pods:
                    _update_with_affinity_terms(aff, ep.pod, ni.node, pi.req_aff, 1)
                    _update_with_anti_affinity_terms(anti, ep.pod, ni.node, pi.req_anti, 1)
        state["PreFilterInterPodAffinity"] = {"existing_anti": existing_anti, "aff": aff, "anti": anti,
                                              "pi": pi}
        return None

    # ---- filtering.go:75-90 updateWithPod, :277-296 AddPod / RemovePod (nominated pods, preemption)
    def update_with_pod(self, state, updated_pod, node, mult):
        s = state.get("PreFilterInterPodAffinity")
        if s is None:
            return
        upi = NI.PodInfo(updated_pod)
        _update_with_anti_affinity_terms(s["existing_anti"], s["pi"].pod, node, upi.req_anti, mult)
        _update_with_affinity_terms(s["aff"], updated_pod, node, s["pi"].req_aff, mult)
        _update_with_anti_affinity_terms(s["anti"], updated_pod, node, s["pi"].req_anti, mult)

    def add_pod(self, state, pod, pod_to_add, ni):
        self.update_with_pod(state, pod_to_add, ni.node, 1)

    def remove_pod(self, state, pod, pod_to_remove, ni):
        self.update_with_pod(state, pod_to_remove, ni.node, -1)

    def filter(self, state, pod, ni):
        if ni.node is None:
            return Status(ERROR, "node not found")
        s = state.get("PreFilterInterPodAffinity")
        if s is None:
            return Status(ERROR, "error reading prefilter state")
        nl = NI.labels_of(ni.node)
        pi = s["pi"]
        # satisfyPodAffinity
        pods_exist = True
        ok = True
        for t in pi.req_aff:
            if t.topology_key in nl:
                if s["aff"].get((t.topology_key, nl[t.topology_key]), 0) <= 0:
                    pods_exist = False
            else:
                ok = False
                break
        if ok and not pods_exist:
            ok = len(s["aff"]) == 0 and pod_matches_all_affinity_terms(pod, pi.req_aff)
        if not ok:
            return Status(UNRESOLVABLE, "node(s) didn't match pod affinity/anti-affinity",
                          "node(s) didn't match pod affinity rules")
        for t in pi.req_anti:
            if t.topology_key in nl:
                if s["anti"].get((t.topology_key, nl[t.topology_key]), 0) > 0:
                    return Status(UNSCHEDULABLE, "node(s) didn't match pod affinity/anti-affinity",
                                  "node(s) didn't match pod anti-affinity rules")
        if len(s["existing_anti"]) > 0:
            for k, v in nl.items():
                if s["existing_anti"].get((k, v), 0) > 0:
                    return Status(UNSCHEDULABLE, "node(s) didn't match pod affinity/anti-affinity",
                                  "node(s) didn't satisfy existing pods anti-affinity rules")
        return None

    # ---- scoring.go:47-272
    @staticmethod
    def _process_term(m, term, weight, pod_to_check, fixed_node, mult):
        nl = NI.labels_of(fixed_node)
        if len(nl) == 0:
            return
        match = pod_matches_term_ns_selector(pod_to_check, term.namespaces, term.selector)
        if match and term.topology_key in nl:
            d = m.setdefault(term.topology_key, {})
            v = nl[term.topology_key]
            d[v] = d.get(v, 0) + weight * mult

    def prescore(self, state, pod, nodes):
        if len(nodes) == 0:
            return None
        a = _spec(pod).get("affinity")
        has_aff = a is not None and a.get("podAffinity") is not None
        has_anti = a is not None and a.get("podAntiAffinity") is not None
        snap = self.handle.snapshot
        all_nodes = snap.list if (has_aff or has_anti) else snap.have_pods_with_affinity()
        pi = NI.PodInfo(pod)
        topo = {}
        for ni in all_nodes:
            pods = ni.pods if (has_aff or has_anti) else ni.pods_with_affinity
            for ep in pods:
                for t in pi.pref_aff:
                    self._process_term(topo, t, t.weight, ep.pod, ni.node, 1)
                for t in pi.pref_anti:
                    self._process_term(topo, t, t.weight, ep.pod, ni.node, -1)
                if self.hard_weight > 0:
                    for t in ep.req_aff:
                        self._process_term(topo, t, self.hard_weight, pod, ni.node, 1)
                for t in ep.pref_aff:
                    self._process_term(topo, t, t.weight, pod, ni.node, 1)
                for t in ep.pref_anti:
                    self._process_term(topo, t, t.weight, pod, ni.node, -1)
        state["PreScoreInterPodAffinity"] = topo
        return None

    def score(self, state, pod, node_name):
        ni = self.handle.snapshot.get(node_name)
        topo = state.get("PreScoreInterPodAffinity")
        if topo is None:
            return 0, Status(ERROR, "error reading prescore state")
        nl = NI.labels_of(ni.node)
        s = 0
        for k, vals in topo.items():
            if k in nl:
                s += vals.get(nl[k], 0)
        return s, None

    def normalize(self, state, pod, scores):
        topo = state.get("PreScoreInterPodAffinity")
        if topo is None:
            return Status(ERROR, "error reading prescore state")
        if len(topo) == 0:
            return None
        mx = mn = 0
        for sc in scores:
            mx = max(mx, sc[1])
            mn = min(mn, sc[1])
        diff = mx - mn
        for sc in scores:
            f = 0.0
            if diff > 0:
                f = float(MAX_NODE_SCORE) * (float(sc[1] - mn) / float(diff))
            sc[1] = int(f)
        return None
