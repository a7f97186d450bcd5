"""Fixture builders with the vocabulary of the reference's test wrappers
(pkg/scheduler/testing/wrappers.go: MakePod / MakeNode / MakeLabelSelector), producing the
k8s-v1-shaped dicts the golden fixtures hold.  Used only to transcribe test tables."""
import copy

HOSTNAME = "kubernetes.io/hostname"
ZONE_BETA = "failure-domain.beta.kubernetes.io/zone"
DO_NOT_SCHEDULE, SCHEDULE_ANYWAY = "DoNotSchedule", "ScheduleAnyway"
# PodAffinityKind (wrappers.go:241-258)
NIL, REQ, PREF, REQ_PREF = 0, 1, 2, 3
ANTI_REQ, ANTI_PREF, ANTI_REQ_PREF = 4, 5, 6


class LS:
    """MakeLabelSelector (wrappers.go:72-133)."""

    def __init__(self):
        self.d = {}

    def label(self, k, v):
        self.d.setdefault("matchLabels", {})[k] = v
        return self

    def _expr(self, k, op, vals=None):
        e = {"key": k, "operator": op}
        if vals is not None:
            e["values"] = list(vals)
        self.d.setdefault("matchExpressions", []).append(e)
        return self

    def in_(self, k, vals):
        return self._expr(k, "In", vals)

    def not_in(self, k, vals):
        return self._expr(k, "NotIn", vals)

    def exists(self, k):
        return self._expr(k, "Exists")

    def not_exist(self, k):
        return self._expr(k, "DoesNotExist")

    def obj(self):
        return copy.deepcopy(self.d)


class P:
    """MakePod (wrappers.go:136-358)."""

    def __init__(self):
        self.m = {"name": "", "namespace": ""}
        self.s = {}

    def name(self, s):
        self.m["name"] = s
        return self

    def uid(self, s):
        self.m["uid"] = s
        return self

    def namespace(self, s):
        self.m["namespace"] = s
        return self

    def container(self, image):
        cs = self.s.setdefault("containers", [])
        cs.append({"name": "con%d" % len(cs), "image": image})
        return self

    def terminating(self):
        self.m["deletionTimestamp"] = "2020-01-01T00:00:00Z"
        return self

    def node(self, s):
        self.s["nodeName"] = s
        return self

    def node_selector(self, m):
        self.s["nodeSelector"] = dict(m)
        return self

    def _na(self, op, key, vals):
        a = self.s.setdefault("affinity", {}).setdefault("nodeAffinity", {})
        a["requiredDuringSchedulingIgnoredDuringExecution"] = {
            "nodeSelectorTerms": [{"matchExpressions": [{"key": key, "operator": op, "values": list(vals)}]}]}
        return self

    def node_affinity_in(self, key, vals):
        return self._na("In", key, vals)

    def node_affinity_not_in(self, key, vals):
        return self._na("NotIn", key, vals)

    def _pa(self, field, label_key, topo, kind, anti):
        if kind == NIL:
            return self
        a = self.s.setdefault("affinity", {}).setdefault(field, {})
        term = {"labelSelector": LS().exists(label_key).obj(), "topologyKey": topo}
        req = kind in ((ANTI_REQ, ANTI_REQ_PREF) if anti else (REQ, REQ_PREF))
        pref = kind in ((ANTI_PREF, ANTI_REQ_PREF) if anti else (PREF, REQ_PREF))
        if req:
            a.setdefault("requiredDuringSchedulingIgnoredDuringExecution", []).append(copy.deepcopy(term))
        if pref:
            a.setdefault("preferredDuringSchedulingIgnoredDuringExecution", []).append(
                {"weight": 1, "podAffinityTerm": copy.deepcopy(term)})
        return self

    def pod_affinity_exists(self, label_key, topo, kind):
        return self._pa("podAffinity", label_key, topo, kind, False)

    def pod_anti_affinity_exists(self, label_key, topo, kind):
        return self._pa("podAntiAffinity", label_key, topo, kind, True)

    def spread(self, max_skew, key, mode, selector):
        c = {"maxSkew": max_skew, "topologyKey": key, "whenUnsatisfiable": mode}
        if selector is not None:
            c["labelSelector"] = selector
        self.s.setdefault("topologySpreadConstraints", []).append(c)
        return self

    def label(self, k, v):
        self.m.setdefault("labels", {})[k] = v
        return self

    def labels(self, d):
        self.m["labels"] = dict(d)
        return self

    def affinity(self, a):
        self.s["affinity"] = copy.deepcopy(a)
        return self

    def obj(self):
        return {"metadata": copy.deepcopy(self.m), "spec": copy.deepcopy(self.s)}


class N:
    """MakeNode (wrappers.go:361-392)."""

    def __init__(self):
        self.m = {"name": ""}

    def name(self, s):
        self.m["name"] = s
        return self

    def label(self, k, v):
        self.m.setdefault("labels", {})[k] = v
        return self

    def labels(self, d):
        self.m["labels"] = dict(d)
        return self

    def obj(self):
        return {"metadata": copy.deepcopy(self.m), "spec": {}, "status": {"allocatable": {}}}


def pods_on(prefix_node_counts, ns=None, labels=(("foo", ""),)):
    """Shorthand for the tables' runs of st.MakePod().Name("p-a1").Node("node-a").Label("foo", "")."""
    out = []
    for name, node_name in prefix_node_counts:
        p = P().name(name).node(node_name)
        if ns:
            p.namespace(ns)
        for k, v in labels:
            p.label(k, v)
        out.append(p.obj())
    return out
