"""ORACLE (test infrastructure only) -- NodeInfo / PodInfo / Snapshot restatement.

Follows:
  pkg/scheduler/framework/v1alpha1/types.go:70-160   PodInfo, AffinityTerm, NewPodInfo
  pkg/scheduler/framework/v1alpha1/types.go:171-209  NodeInfo
  pkg/scheduler/framework/v1alpha1/types.go:262-385  Resource Add / SetMaxResource
  pkg/scheduler/framework/v1alpha1/types.go:456-620  AddPod / RemovePod / calculateResource / ports
  pkg/scheduler/framework/v1alpha1/types.go:677-765  HostPortInfo
  pkg/scheduler/util/non_zero.go:36-80               GetNonzeroRequestForResource
  pkg/scheduler/internal/cache/node_tree.go:31-170   zone round-robin snapshot order
  pkg/scheduler/internal/cache/snapshot.go:49-125    NewSnapshot, image states
  pkg/util/node/node.go:148-174                       GetZoneKey
  pkg/apis/core/v1/helper/helpers.go:33-143          resource-name classes
"""
from . import quantity as Q
from . import labels as L

DEFAULT_MILLI_CPU = 100
DEFAULT_MEMORY = 200 * 1024 * 1024

LABEL_HOSTNAME = "kubernetes.io/hostname"
LABEL_ZONE = "failure-domain.beta.kubernetes.io/zone"
LABEL_REGION = "failure-domain.beta.kubernetes.io/region"
LABEL_ZONE_STABLE = "topology.kubernetes.io/zone"
LABEL_REGION_STABLE = "topology.kubernetes.io/region"


# ---------------------------------------------------------------- resource names
def is_prefixed_native(name):
    return "kubernetes.io/" in name


def is_native(name):
    return "/" not in name or is_prefixed_native(name)


def is_extended(name):
    if is_native(name) or name.startswith("requests."):
        return False
    return L.is_qualified_name("requests." + name)


def is_scalar_resource_name(name):
    return (is_extended(name) or name.startswith("hugepages-") or is_prefixed_native(name)
            or name.startswith("attachable-volumes-"))


class Resource:
    __slots__ = ("milli_cpu", "memory", "eph", "allowed_pods", "scalars")

    def __init__(self):
        self.milli_cpu = 0
        self.memory = 0
        self.eph = 0
        self.allowed_pods = 0
        self.scalars = None  # lazily allocated map, like Go

    def add(self, rl):
        for name, q in (rl or {}).items():
            if name == "cpu":
                self.milli_cpu += Q.milli_value(q)
            elif name == "memory":
                self.memory += Q.value(q)
            elif name == "pods":
                self.allowed_pods += Q.value(q)
            elif name == "ephemeral-storage":
                self.eph += Q.value(q)  # LocalStorageCapacityIsolation = true
            elif is_scalar_resource_name(name):
                self.add_scalar(name, Q.value(q))

    def add_scalar(self, name, v):
        if self.scalars is None:
            self.scalars = {}
        self.scalars[name] = self.scalars.get(name, 0) + v

    def set_max(self, rl):
        for name, q in (rl or {}).items():
            if name == "memory":
                self.memory = max(self.memory, Q.value(q))
            elif name == "cpu":
                self.milli_cpu = max(self.milli_cpu, Q.milli_value(q))
            elif name == "ephemeral-storage":
                self.eph = max(self.eph, Q.value(q))
            elif is_scalar_resource_name(name):
                v = Q.value(q)
                if v > (self.scalars or {}).get(name, 0):
                    if self.scalars is None:
                        self.scalars = {}
                    self.scalars[name] = v

    def scalar(self, name):
        return (self.scalars or {}).get(name, 0)


def nonzero_request(resource, requests):
    """util.GetNonzeroRequestForResource (non_zero.go:50-80)."""
    requests = requests or {}
    if resource == "cpu":
        if "cpu" not in requests:
            return DEFAULT_MILLI_CPU
        return Q.milli_value(requests["cpu"])
    if resource == "memory":
        if "memory" not in requests:
            return DEFAULT_MEMORY
        return Q.value(requests["memory"])
    if resource == "ephemeral-storage":
        if "ephemeral-storage" not in requests:
            return 0
        return Q.value(requests["ephemeral-storage"])
    if is_scalar_resource_name(resource):
        if resource not in requests:
            return 0
        return Q.value(requests[resource])
    return 0


def _spec(pod):
    return pod.get("spec") or {}


def _meta(obj):
    return obj.get("metadata") or {}


def containers(pod):
    return _spec(pod).get("containers") or []


def init_containers(pod):
    return _spec(pod).get("initContainers") or []


def _requests(c):
    return ((c.get("resources") or {}).get("requests")) or {}


def calculate_resource(pod):
    """types.go calculateResource: (Resource, non0CPU, non0Mem)."""
    res = Resource()
    n0c = n0m = 0
    for c in containers(pod):
        res.add(_requests(c))
        n0c += nonzero_request("cpu", _requests(c))
        n0m += nonzero_request("memory", _requests(c))
    for ic in init_containers(pod):
        res.set_max(_requests(ic))
        n0c = max(n0c, nonzero_request("cpu", _requests(ic)))
        n0m = max(n0m, nonzero_request("memory", _requests(ic)))
    oh = _spec(pod).get("overhead")
    if oh is not None:
        res.add(oh)
        if "cpu" in oh:
            n0c += Q.milli_value(oh["cpu"])
        if "memory" in oh:
            n0m += Q.value(oh["memory"])
    return res, n0c, n0m


def compute_pod_resource_request(pod):
    """noderesources/fit.go:112-129 computePodResourceRequest."""
    r = Resource()
    for c in containers(pod):
        r.add(_requests(c))
    for ic in init_containers(pod):
        r.set_max(_requests(ic))
    oh = _spec(pod).get("overhead")
    if oh is not None:
        r.add(oh)
    return r


# ---------------------------------------------------------------- pod info
class AffinityTerm:
    __slots__ = ("namespaces", "selector", "topology_key", "weight")

    def __init__(self, namespaces, selector, topology_key, weight=0):
        self.namespaces, self.selector, self.topology_key, self.weight = namespaces, selector, topology_key, weight


def _new_affinity_term(pod, term):
    ns = term.get("namespaces") or []
    namespaces = set(ns) if ns else {namespace(pod)}
    try:
        sel = L.label_selector_as_selector(term.get("labelSelector"))
    except L.SelectorError:
        return None
    return AffinityTerm(namespaces, sel, term.get("topologyKey", ""))


def _get_affinity_terms(pod, v1terms):
    if v1terms is None:
        return None
    out = []
    for t in v1terms:
        at = _new_affinity_term(pod, t)
        if at is None:
            return None
        out.append(at)
    return out


def _get_weighted_terms(pod, v1terms):
    if v1terms is None:
        return None
    out = []
    for wt in v1terms:
        at = _new_affinity_term(pod, wt.get("podAffinityTerm") or {})
        if at is None:
            return None
        at.weight = int(wt.get("weight", 0))
        out.append(at)
    return out


def affinity(pod):
    return _spec(pod).get("affinity")


def pod_affinity_terms(pod):
    """util.GetPodAffinityTerms (utils.go:86-99)."""
    a = affinity(pod)
    if a is not None and a.get("podAffinity") is not None:
        t = a["podAffinity"].get("requiredDuringSchedulingIgnoredDuringExecution") or []
        if len(t) != 0:
            return t
    return None


def pod_anti_affinity_terms(pod):
    a = affinity(pod)
    if a is not None and a.get("podAntiAffinity") is not None:
        t = a["podAntiAffinity"].get("requiredDuringSchedulingIgnoredDuringExecution") or []
        if len(t) != 0:
            return t
    return None


class PodInfo:
    __slots__ = ("pod", "req_aff", "req_anti", "pref_aff", "pref_anti")

    def __init__(self, pod):
        self.pod = pod
        pref_a = pref_anti = None
        a = affinity(pod)
        if a is not None:
            if a.get("podAffinity") is not None:
                pref_a = a["podAffinity"].get("preferredDuringSchedulingIgnoredDuringExecution")
            if a.get("podAntiAffinity") is not None:
                pref_anti = a["podAntiAffinity"].get("preferredDuringSchedulingIgnoredDuringExecution")
        self.req_aff = _get_affinity_terms(pod, pod_affinity_terms(pod)) or []
        self.req_anti = _get_affinity_terms(pod, pod_anti_affinity_terms(pod)) or []
        self.pref_aff = _get_weighted_terms(pod, pref_a) or []
        self.pref_anti = _get_weighted_terms(pod, pref_anti) or []


def namespace(obj):
    return _meta(obj).get("namespace", "") or ""


def name(obj):
    return _meta(obj).get("name", "") or ""


def labels_of(obj):
    return _meta(obj).get("labels") or {}


def pod_key(pod):
    m = _meta(pod)
    uid = m.get("uid")
    if uid:
        return uid
    return "%s/%s" % (m.get("namespace", ""), m.get("name", ""))


def has_pod_affinity_fields(pod):
    a = affinity(pod)
    return a is not None and (a.get("podAffinity") is not None or a.get("podAntiAffinity") is not None)


def pod_ports(pod):
    out = []
    for c in containers(pod):
        for p in c.get("ports") or []:
            out.append(p)
    return out


# ---------------------------------------------------------------- node info
def sanitize(ip, proto):
    return (ip or "0.0.0.0"), (proto or "TCP")


class NodeInfo:
    def __init__(self, node=None):
        self.node = None
        self.pods = []
        self.pods_with_affinity = []
        self.used_ports = {}
        self.requested = Resource()
        self.non_zero = Resource()
        self.allocatable = Resource()
        self.image_states = {}
        if node is not None:
            self.set_node(node)

    def set_node(self, node):
        self.node = node
        self.allocatable = Resource()
        self.allocatable.add((node.get("status") or {}).get("allocatable") or {})

    def add_pod(self, pod):
        pi = PodInfo(pod)
        res, n0c, n0m = calculate_resource(pod)
        self.requested.milli_cpu += res.milli_cpu
        self.requested.memory += res.memory
        self.requested.eph += res.eph
        for k, v in (res.scalars or {}).items():
            self.requested.add_scalar(k, v)
        self.non_zero.milli_cpu += n0c
        self.non_zero.memory += n0m
        self.pods.append(pi)
        if has_pod_affinity_fields(pod):
            self.pods_with_affinity.append(pi)
        for p in pod_ports(pod):
            port = int(p.get("hostPort", 0) or 0)
            if port <= 0:
                continue
            ip, proto = sanitize(p.get("hostIP", ""), p.get("protocol", ""))
            self.used_ports.setdefault(ip, set()).add((proto, port))

    def remove_pod(self, pod):
        k1 = pod_key(pod)
        for i, pi in enumerate(self.pods_with_affinity):
            if pod_key(pi.pod) == k1:
                self.pods_with_affinity[i] = self.pods_with_affinity[-1]
                self.pods_with_affinity.pop()
                break
        for i, pi in enumerate(self.pods):
            if pod_key(pi.pod) == k1:
                self.pods[i] = self.pods[-1]
                self.pods.pop()
                res, n0c, n0m = calculate_resource(pod)
                self.requested.milli_cpu -= res.milli_cpu
                self.requested.memory -= res.memory
                self.requested.eph -= res.eph
                for k, v in (res.scalars or {}).items():
                    self.requested.add_scalar(k, -v)
                self.non_zero.milli_cpu -= n0c
                self.non_zero.memory -= n0m
                for p in pod_ports(pod):
                    port = int(p.get("hostPort", 0) or 0)
                    if port <= 0:
                        continue
                    ip, proto = sanitize(p.get("hostIP", ""), p.get("protocol", ""))
                    m = self.used_ports.get(ip)
                    if m is not None:
                        m.discard((proto, port))
                        if not m:
                            del self.used_ports[ip]
                return
        raise KeyError("no corresponding pod %s" % name(pod))

    def ports_conflict(self, ip, proto, port):
        """HostPortInfo.CheckConflict (types.go:726-756)."""
        if port <= 0:
            return False
        ip, proto = sanitize(ip, proto)
        pp = (proto, port)
        if ip == "0.0.0.0":
            return any(pp in m for m in self.used_ports.values())
        for key in ("0.0.0.0", ip):
            if pp in self.used_ports.get(key, ()):
                return True
        return False


def get_zone_key(node):
    lab = labels_of(node) if node is not None else None
    if not lab:
        return ""
    zone = lab.get(LABEL_ZONE, lab.get(LABEL_ZONE_STABLE, ""))
    if LABEL_ZONE in lab:
        zone = lab[LABEL_ZONE]
    region = lab[LABEL_REGION] if LABEL_REGION in lab else lab.get(LABEL_REGION_STABLE, "")
    if region == "" and zone == "":
        return ""
    return region + ":\x00:" + zone


class NodeTreeRef:
    """node_tree.go:31-196 step by step: tree map + zones list + zoneIndex + per-array lastIndex."""

    def __init__(self, nodes=()):
        self.tree = {}
        self.zones = []
        self.zone_index = 0
        self.num_nodes = 0
        for n in nodes or ():
            self.add_node(n)

    def add_node(self, n):                          # node_tree.go:69-86
        zone = get_zone_key(n)
        na = self.tree.get(zone)
        if na is not None:
            if name(n) in na["nodes"]:
                return
            na["nodes"].append(name(n))
        else:
            self.zones.append(zone)
            self.tree[zone] = {"nodes": [name(n)], "last": 0}
        self.num_nodes += 1

    def remove_node(self, n):                       # node_tree.go:88-108; returns the error or None
        zone = get_zone_key(n)
        na = self.tree.get(zone)
        if na is not None:
            for i, nm in enumerate(na["nodes"]):
                if nm == name(n):
                    del na["nodes"][i]
                    if not na["nodes"]:
                        del self.tree[zone]
                        self.zones.remove(zone)
                    self.num_nodes -= 1
                    return None
        return "node %r in group %r was not found" % (name(n), zone)

    def update_node(self, old, new):                # node_tree.go:120-132
        old_zone = get_zone_key(old) if old is not None else ""
        if old_zone == get_zone_key(new):
            return
        self.remove_node(old)
        self.add_node(new)

    def next(self):                                 # node_tree.go:144-170
        if not self.zones:
            return ""
        num_exhausted = 0
        while True:
            if self.zone_index >= len(self.zones):
                self.zone_index = 0
            na = self.tree[self.zones[self.zone_index]]
            self.zone_index += 1
            if na["last"] >= len(na["nodes"]):
                num_exhausted += 1
                if num_exhausted >= len(self.zones):
                    for a in self.tree.values():
                        a["last"] = 0
                    self.zone_index = 0
                continue
            na["last"] += 1
            return na["nodes"][na["last"] - 1]


def node_tree_order(nodes):
    """nodeTree: zone groups in first-insertion order, then round-robin (node_tree.go:147-170)."""
    zones, tree = [], {}
    for n in nodes:
        z = get_zone_key(n)
        if z not in tree:
            zones.append(z)
            tree[z] = []
        if name(n) not in tree[z]:
            tree[z].append(name(n))
    out = []
    idx = {z: 0 for z in zones}
    total = sum(len(v) for v in tree.values())
    zi = 0
    while len(out) < total:
        z = zones[zi % len(zones)]
        zi += 1
        if idx[z] < len(tree[z]):
            out.append(tree[z][idx[z]])
            idx[z] += 1
    return out


class Snapshot:
    """Cache snapshot: NodeInfos in Snapshot.List() order (zone round robin of add order)."""

    def __init__(self, nodes, pods=(), order="tree", image_nodes=None):
        """image_nodes: the nodes whose images count toward ImageStateSummary.NumNodes -- the
        scheduler cache's nodes (cache.go:658-700), which a Snapshot.List() built by UpdateSnapshot
        may not all hold (node_tree.go:147-170); default: `nodes`."""
        by_name = {}
        for n in nodes:
            by_name[name(n)] = NodeInfo(n)
        self.phantoms = 0
        for p in pods:
            nn = _spec(p).get("nodeName", "") or ""
            if nn in by_name:
                by_name[nn].add_pod(p)
            else:
                self.phantoms += 1  # NewSnapshot creates NodeInfos without a node; they never fit
        names = node_tree_order(nodes) if order == "tree" else [name(n) for n in nodes]
        self.list = [by_name[x] for x in names]
        self.map = by_name
        # image states (snapshot.go:92-125)
        exist = {}
        for n in (nodes if image_nodes is None else image_nodes):
            for im in (n.get("status") or {}).get("images") or []:
                for nm in im.get("names") or []:
                    exist.setdefault(nm, set()).add(name(n))
        for n in nodes:
            st = {}
            for im in (n.get("status") or {}).get("images") or []:
                for nm in im.get("names") or []:
                    st[nm] = (int(im.get("sizeBytes", 0)), len(exist.get(nm, ())))
            by_name[name(n)].image_states = st
        self._phantom_names = set()
        for p in pods:
            nn = _spec(p).get("nodeName", "") or ""
            if nn not in by_name:
                self._phantom_names.add(nn)

    def num_nodes_listed(self):
        """len(NodeInfos().List()) -- includes node-less NodeInfos created by NewSnapshot."""
        return len(self.list) + len(self._phantom_names)

    def get(self, n):
        return self.map[n]

    def have_pods_with_affinity(self):
        return [ni for ni in self.list if ni.pods_with_affinity]
