"""Host-side view of v1 objects (k8s-v1-shaped dicts) as the Go plugin sees them.

This is the part of the cgo shim's job that turns API objects into engine inputs: resource
quantities (staging/.../api/resource/quantity.go:695-716), resource-name classes
(pkg/apis/core/v1/helper/helpers.go:33-143), pod request arithmetic
(framework/v1alpha1/types.go:262-385,524-555; noderesources/fit.go:112-129;
noderesources/resource_allocation.go:118-142; util/non_zero.go:36-80), label validation
(apimachinery/pkg/util/validation) and GetZoneKey (pkg/util/node/node.go:148-174).
"""
from fractions import Fraction
import re

DEFAULT_MILLI_CPU = 100
DEFAULT_MEMORY = 200 * 1024 * 1024
LABEL_HOSTNAME = "kubernetes.io/hostname"
_ZONE, _REGION = "failure-domain.beta.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/region"
_ZONE_S, _REGION_S = "topology.kubernetes.io/zone", "topology.kubernetes.io/region"

_SUFFIX = {"Ki": 1 << 10, "Mi": 1 << 20, "Gi": 1 << 30, "Ti": 1 << 40, "Pi": 1 << 50, "Ei": 1 << 60,
           "n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": 1,
           "k": 10 ** 3, "M": 10 ** 6, "G": 10 ** 9, "T": 10 ** 12, "P": 10 ** 15, "E": 10 ** 18}
_QRE = re.compile(r"^([+-]?)(\d*)(?:\.(\d*))?([a-zA-Z]*|[eE][+-]?\d+)$")
_qcache = {}


def quantity(q):
    """Exact value of a resource.Quantity string."""
    if isinstance(q, int):
        return Fraction(q)
    v = _qcache.get(q)
    if v is not None:
        return v
    m = _QRE.match(str(q).strip())
    if not m or (not m.group(2) and not m.group(3)):
        raise ValueError("invalid quantity %r" % (q,))
    sign, whole, frac, suf = m.groups()
    x = Fraction(int(whole or "0"))
    if frac:
        x += Fraction(int(frac), 10 ** len(frac))
    if sign == "-":
        x = -x
    if suf in _SUFFIX:
        x *= _SUFFIX[suf]
    elif suf[:1] in "eE":
        x *= Fraction(10) ** int(suf[1:])
    else:
        raise ValueError("invalid quantity suffix %r" % (q,))
    _qcache[q] = x
    return x


def _ceil_away(x):
    if x.denominator == 1:
        return int(x.numerator)
    f = x.numerator // x.denominator
    return f + 1 if x > 0 else f


def q_value(q):
    return _ceil_away(quantity(q))


def q_milli(q):
    return _ceil_away(quantity(q) * 1000)


_NAME_RE = re.compile(r"^[A-Za-z0-9]([-A-Za-z0-9_.]*[A-Za-z0-9])?$")
_DNS_RE = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$")


def qualified_name_ok(v):
    parts = v.split("/")
    if len(parts) > 2:
        return False
    if len(parts) == 2:
        if not parts[0] or len(parts[0]) > 253 or not _DNS_RE.match(parts[0]):
            return False
    name = parts[-1]
    return 0 < len(name) <= 63 and bool(_NAME_RE.match(name))


def label_value_ok(v):
    return v == "" or (len(v) <= 63 and bool(_NAME_RE.match(v)))


def parse_int64(s):
    if not isinstance(s, str) or not re.match(r"^[+-]?\d+$", s):
        return None
    v = int(s)
    return v if -(1 << 63) <= v < (1 << 63) else None


def is_extended(name):
    if "/" not in name or "kubernetes.io/" in name or name.startswith("requests."):
        return False
    return qualified_name_ok("requests." + name)


def is_scalar(name):
    return (is_extended(name) or name.startswith("hugepages-") or "kubernetes.io/" in name
            or name.startswith("attachable-volumes-"))


def meta(o):
    return o.get("metadata") or {}


def spec(o):
    return o.get("spec") or {}


def name_of(o):
    return meta(o).get("name", "") or ""


def ns_of(o):
    return meta(o).get("namespace", "") or ""


def labels_of(o):
    return meta(o).get("labels") or {}


def containers(p):
    return spec(p).get("containers") or []


def init_containers(p):
    return spec(p).get("initContainers") or []


def requests_of(c):
    return ((c.get("resources") or {}).get("requests")) or {}


class PodResources:
    """Everything the engine needs from a pod's resource requests."""
    __slots__ = ("cpu", "mem", "eph", "scalars", "nz_cpu", "nz_mem", "score", "fit_all_zero")

    def __init__(self, pod):
        cpu = mem = eph = 0
        sc = {}
        for c in containers(pod):
            cpu, mem, eph = self._add(c, cpu, mem, eph, sc)
        for ic in init_containers(pod):
            r = requests_of(ic)
            for k, q in r.items():
                if k == "cpu":
                    cpu = max(cpu, q_milli(q))
                elif k == "memory":
                    mem = max(mem, q_value(q))
                elif k == "ephemeral-storage":
                    eph = max(eph, q_value(q))
                elif is_scalar(k):
                    v = q_value(q)
                    if v > sc.get(k, 0):
                        sc[k] = v
        oh = spec(pod).get("overhead")
        if oh is not None:
            cpu, mem, eph = self._add({"resources": {"requests": oh}}, cpu, mem, eph, sc)
        self.cpu, self.mem, self.eph, self.scalars = cpu, mem, eph, sc
        self.fit_all_zero = cpu == 0 and mem == 0 and eph == 0 and len(sc) == 0
        # NonZeroRequested delta (types.go calculateResource: overhead cpu as MilliValue) and the
        # scorer request (resource_allocation.go calculatePodResourceRequest: overhead Value()).
        self.nz_cpu, self.nz_mem = nz_deltas(pod)
        self.score = {r: self._score(r, pod) for r in ("cpu", "memory", "ephemeral-storage")}

    @staticmethod
    def _add(c, cpu, mem, eph, sc):
        for k, q in requests_of(c).items():
            if k == "cpu":
                cpu += q_milli(q)
            elif k == "memory":
                mem += q_value(q)
            elif k == "ephemeral-storage":
                eph += q_value(q)
            elif k != "pods" and is_scalar(k):
                sc[k] = sc.get(k, 0) + q_value(q)
        return cpu, mem, eph

    @staticmethod
    def nonzero(resource, req):
        if resource == "cpu":
            return q_milli(req["cpu"]) if "cpu" in req else DEFAULT_MILLI_CPU
        if resource == "memory":
            return q_value(req["memory"]) if "memory" in req else DEFAULT_MEMORY
        if resource == "ephemeral-storage" or is_scalar(resource):
            return q_value(req[resource]) if resource in req else 0
        return 0

    def _score(self, resource, pod):
        v = 0
        for c in containers(pod):
            v += self.nonzero(resource, requests_of(c))
        for ic in init_containers(pod):
            v = max(v, self.nonzero(resource, requests_of(ic)))
        oh = spec(pod).get("overhead")
        if oh is not None and resource in oh:
            # the scorer adds Quantity.Value() for every resource, cpu included
            # (resource_allocation.go:137-139); calculateResource uses MilliValue for cpu.
            v += q_value(oh[resource])
        return v

    def score_value(self, resource, pod):
        return self._score(resource, pod)


def nz_deltas(pod):
    """types.go calculateResource non0CPU / non0Mem (overhead cpu as MilliValue)."""
    n0c = n0m = 0
    for c in containers(pod):
        r = requests_of(c)
        n0c += PodResources.nonzero("cpu", r)
        n0m += PodResources.nonzero("memory", r)
    for ic in init_containers(pod):
        r = requests_of(ic)
        n0c = max(n0c, PodResources.nonzero("cpu", r))
        n0m = max(n0m, PodResources.nonzero("memory", r))
    oh = spec(pod).get("overhead")
    if oh is not None:
        if "cpu" in oh:
            n0c += q_milli(oh["cpu"])
        if "memory" in oh:
            n0m += q_value(oh["memory"])
    return n0c, n0m


def zone_key(node):
    lab = labels_of(node)
    if not lab:
        return ""
    zone = lab[_ZONE] if _ZONE in lab else lab.get(_ZONE_S, "")
    region = lab[_REGION] if _REGION in lab else lab.get(_REGION_S, "")
    if region == "" and zone == "":
        return ""
    return region + ":\x00:" + zone


class NodeTree:
    """The scheduler cache's nodeTree (internal/cache/node_tree.go:31-196).

    Zones (GetZoneKey) in first-insertion order, each an array of node names with a cursor.  The
    cursors and the zone index persist across snapshots: Snapshot.List() after a node event is the
    next numNodes outputs of next() (cache.go:278-301), which need not restart at zone 0."""

    def __init__(self, nodes=()):
        self.zones = []      # zone keys, first-insertion order
        self.arrays = {}     # zone -> [names, cursor, set(names)] (the set: O(1) membership)
        self.zone_index = 0
        self.num_nodes = 0
        for n in nodes:
            self.add_node(n)

    def add_node(self, n):
        z, nm = zone_key(n), name_of(n)
        arr = self.arrays.get(z)
        if arr is None:
            self.zones.append(z)
            self.arrays[z] = [[nm], 0, {nm}]
        elif nm in arr[2]:
            return                          # node_tree.go:72-77: already present, no change
        else:
            arr[0].append(nm)
            arr[2].add(nm)
        self.num_nodes += 1

    def remove_node(self, n):
        """Returns False when the node is not in its zone's array (node_tree.go:106-107)."""
        z, nm = zone_key(n), name_of(n)
        arr = self.arrays.get(z)
        if arr is None or nm not in arr[2]:
            return False
        arr[0].remove(nm)
        arr[2].discard(nm)
        if not arr[0]:
            del self.arrays[z]
            self.zones.remove(z)
        self.num_nodes -= 1
        return True

    def update_node(self, old, new):
        if old is not None and zone_key(old) == zone_key(new):
            return
        if old is None and zone_key(new) == "":
            return
        if old is not None:
            self.remove_node(old)
        self.add_node(new)

    def _reset(self):
        for arr in self.arrays.values():
            arr[1] = 0
        self.zone_index = 0

    def next(self):
        if not self.zones:
            return ""
        exhausted = 0
        while True:
            if self.zone_index >= len(self.zones):
                self.zone_index = 0
            arr = self.arrays[self.zones[self.zone_index]]
            self.zone_index += 1
            if arr[1] < len(arr[0]):
                arr[1] += 1
                return arr[0][arr[1] - 1]
            exhausted += 1
            if exhausted >= len(self.zones):
                self._reset()

    def list(self):
        """One Snapshot.List() pass: numNodes calls of next()."""
        return [self.next() for _ in range(self.num_nodes)]

    def tree(self):
        return {z: list(self.arrays[z][0]) for z in self.zones}


def snapshot_order(nodes):
    """Snapshot.List() order of a freshly built cache: node objects in nodeTree order."""
    by_name = {}
    for n in nodes:
        by_name.setdefault(name_of(n), n)
    return [by_name[nm] for nm in NodeTree(nodes).list()]


def normalized_image_name(n):
    if n.rfind(":") <= n.rfind("/"):
        n = n + ":latest"
    return n


def controller_ref(pod):
    for o in meta(pod).get("ownerReferences") or []:
        if o.get("controller"):
            return o
    return None


PREFER_AVOID_PODS_ANNOTATION = "scheduler.alpha.kubernetes.io/preferAvoidPods"


def _ci(d, key):
    """encoding/json matches struct field names case-insensitively."""
    if not isinstance(d, dict):
        return None
    if key in d:
        return d[key]
    for k, v in d.items():
        if k.lower() == key.lower():
            return v
    return None


def avoid_pods(node):
    """(kind, uid) of every preferAvoidPods entry with a podController.

    pkg/apis/core/v1/helper/helpers.go:500-509 GetAvoidPodsFromNodeAnnotations decodes the JSON
    annotation; node_prefer_avoid_pods.go:68-72 treats a decode error as "no entries".  The
    already-decoded shorthand annotations["preferAvoidPods"] = [{"kind", "uid"}] is accepted too."""
    ann = meta(node).get("annotations") or {}
    out = []
    raw = ann.get(PREFER_AVOID_PODS_ANNOTATION)
    if isinstance(raw, str) and raw != "":
        import json
        try:
            doc = json.loads(raw)
            for a in _ci(doc, "preferAvoidPods") or []:
                pc = _ci(_ci(a, "podSignature"), "podController")
                if pc is not None:
                    out.append((_ci(pc, "kind") or "", _ci(pc, "uid") or ""))
        except (ValueError, TypeError, AttributeError):
            return []
    for a in ann.get("preferAvoidPods") or []:
        out.append((a.get("kind"), a.get("uid")))
    return out


def pod_limits(pod):
    """getResourceLimits (resource_limits.go:145-156): containers' limits added, init containers'
    taken as a max (Resource.Add / SetMaxResource, types.go:262-323); milliCPU and memory."""
    cpu = mem = 0
    for c in containers(pod):
        lim = (c.get("resources") or {}).get("limits") or {}
        if "cpu" in lim:
            cpu += q_milli(lim["cpu"])
        if "memory" in lim:
            mem += q_value(lim["memory"])
    for c in init_containers(pod):
        lim = (c.get("resources") or {}).get("limits") or {}
        if "cpu" in lim:
            cpu = max(cpu, q_milli(lim["cpu"]))
        if "memory" in lim:
            mem = max(mem, q_value(lim["memory"]))
    return cpu, mem
