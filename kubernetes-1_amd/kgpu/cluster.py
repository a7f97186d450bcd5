"""Synthetic clusters for the BASELINE.json configs.

Deterministic: a splitmix64 stream seeded with 0x5CED0001 drives every choice, so the same
(config, size) always yields the same objects on every host.  Objects are k8s-v1-shaped dicts, as
the reference's scheduler_perf fabricates them (nodes are API objects only; no kubelets).
"""
from . import compile as _c

CLUSTER_SEED = 0x5CED0001
M64 = (1 << 64) - 1
GI, MI = 1 << 30, 1 << 20
ZONE = "topology.kubernetes.io/zone"
HOSTNAME = "kubernetes.io/hostname"


class Rng:
    def __init__(self, seed=CLUSTER_SEED):
        self.s = seed & M64

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)

    def below(self, n):
        return self.next() % n

    def pick(self, seq):
        return seq[self.below(len(seq))]

    def chance(self, num, den):
        return self.below(den) < num


def node(name, cpu, mem, pods=110, eph=None, labels=None, taints=None):
    al = {"cpu": str(cpu), "memory": str(mem), "pods": str(pods)}
    if eph is not None:
        al["ephemeral-storage"] = str(eph)
    n = {"metadata": {"name": name}, "spec": {}, "status": {"allocatable": al, "capacity": dict(al)}}
    if labels:
        n["metadata"]["labels"] = dict(labels)
    if taints:
        n["spec"]["taints"] = list(taints)
    return n


def pod(name, cpu=None, mem=None, ns="default", labels=None, node_name=None, port=None, **spec):
    req = {}
    if cpu is not None:
        req["cpu"] = cpu
    if mem is not None:
        req["memory"] = mem
    c = {"name": "c", "image": "k8s.gcr.io/pause:3.2", "resources": {"requests": req} if req else {}}
    if port is not None:
        c["ports"] = [{"containerPort": port}]
    s = dict(spec)
    s["containers"] = [c]
    if node_name is not None:
        s["nodeName"] = node_name
    p = {"metadata": {"name": name, "namespace": ns, "uid": "uid-" + name}, "spec": s}
    if labels:
        p["metadata"]["labels"] = dict(labels)
    return p


# ----------------------------------------------------------------------------- (a)
def scheduling_basic(n_nodes=500, n_init=500, n_pods=1000):
    """scheduler_perf SchedulingBasic (performance-config.yaml:1-13): node-default.yaml nodes,
    pod-default.yaml pods (100m / 500Mi, containerPort 80 without hostPort), default profile.
    Init pods are returned unplaced: the caller schedules them first."""
    nodes = [node("scheduler-perf-%d" % i, "4", "32Gi", 110) for i in range(n_nodes)]
    init = [pod("init-%d" % i, "100m", "500Mi", port=80) for i in range(n_init)]
    pods = [pod("pod-%d" % i, "100m", "500Mi", port=80) for i in range(n_pods)]
    return nodes, init, pods, _c.Profile()


# ----------------------------------------------------------------------------- (b)
def fit_least_balanced(n_nodes=5000, n_pods=10000, seed=CLUSTER_SEED, zones=0):
    """Config (b): NodeResourcesFit + LeastAllocated + BalancedAllocation."""
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        labels = {ZONE: "zone%d" % (i % zones), HOSTNAME: "node%d" % i} if zones else None
        nodes.append(node("node%d" % i, str(r.pick([4, 8, 16, 32, 64])), "%dGi" % r.pick([16, 32, 64, 128, 256]),
                          110, "100Gi", labels=labels))
    pods = []
    for i in range(n_pods):
        if r.chance(1, 10):
            pods.append(pod("p%d" % i))
        else:
            pods.append(pod("p%d" % i, "%dm" % (100 * (1 + r.below(40))), "%dMi" % (128 * (1 + r.below(64)))))
    prof = _c.Profile(filters=["NodeResourcesFit"],
                      scores=[("NodeResourcesBalancedAllocation", 1), ("NodeResourcesLeastAllocated", 1)])
    return nodes, [], pods, prof


# ----------------------------------------------------------------------------- (c)
def taints_affinity_spread(n_nodes=5000, n_pods=10000, seed=CLUSTER_SEED, n_zones=10, spread=True):
    """Config (c): taints (10% dedicated=infra:NoSchedule, 20% spot=true:PreferNoSchedule),
    required NodeAffinity zone In {zone1,zone2,zone3}, PodTopologySpread on zone (DoNotSchedule)
    and hostname (ScheduleAnyway), default profile."""
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        taints = []
        if r.chance(1, 10):
            taints.append({"key": "dedicated", "value": "infra", "effect": "NoSchedule"})
        if r.chance(2, 10):
            taints.append({"key": "spot", "value": "true", "effect": "PreferNoSchedule"})
        nodes.append(node("node%d" % i, str(r.pick([4, 8, 16, 32, 64])), "%dGi" % r.pick([16, 32, 64, 128, 256]),
                          110, "100Gi", labels={ZONE: "zone%d" % (i % n_zones), HOSTNAME: "node%d" % i},
                          taints=taints))
    pods = []
    na = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
        {"matchExpressions": [{"key": ZONE, "operator": "In", "values": ["zone1", "zone2", "zone3"]}]}]}}}
    for i in range(n_pods):
        spec = {"affinity": na}
        if r.chance(1, 2):
            spec["tolerations"] = [{"key": "dedicated", "operator": "Equal", "value": "infra", "effect": "NoSchedule"}]
        if spread:
            sel = {"matchLabels": {"app": "web"}}
            spec["topologySpreadConstraints"] = [
                {"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "DoNotSchedule", "labelSelector": sel},
                {"maxSkew": 1, "topologyKey": HOSTNAME, "whenUnsatisfiable": "ScheduleAnyway", "labelSelector": sel}]
        pods.append(pod("p%d" % i, "%dm" % (100 * (1 + r.below(40))), "%dMi" % (128 * (1 + r.below(64))),
                        labels={"app": "web"}, **spec))
    return nodes, [], pods, _c.Profile()


# ----------------------------------------------------------------------------- (d)
_AFF_KINDS = ["nil", "req", "pref", "req_pref"]


def _pod_terms(label, topo_key, kind):
    """PodAffinityExists / PodAntiAffinityExists terms (testing/wrappers.go:260-336)."""
    term = {"labelSelector": {"matchExpressions": [{"key": label, "operator": "Exists"}]}, "topologyKey": topo_key}
    out = {}
    if kind in ("req", "req_pref"):
        out["requiredDuringSchedulingIgnoredDuringExecution"] = [dict(term)]
    if kind in ("pref", "req_pref"):
        out["preferredDuringSchedulingIgnoredDuringExecution"] = [{"weight": 1, "podAffinityTerm": dict(term)}]
    return out


def _affinity_combo(i, labels, tp_keys):
    label, tp = labels[i % len(labels)], tp_keys[i % len(tp_keys)]
    idx = i % 16
    aff, anti = _AFF_KINDS[idx // 4], _AFF_KINDS[idx % 4]
    a = {}
    if aff != "nil":
        a["podAffinity"] = _pod_terms(label, tp, aff)
    if anti != "nil":
        a["podAntiAffinity"] = _pod_terms(label, tp, anti)
    return a


def pod_affinity(n_nodes=5000, n_existing=5000, n_pods=10000):
    """Config (d): testing.MakeNodesAndPodsForPodAffinity (workload_prep.go:63-121): nodes labelled
    region i%3 / zone i%10 / node i, existing pods on node i%N carrying the 16 combinations of
    PodAffinityExists x PodAntiAffinityExists over labels foo/bar/baz and topology keys
    region/zone/node.  Nodes get node-default.yaml capacity (4 cpu, 32Gi, 110 pods); incoming pods
    (pod-default.yaml requests) carry label foo/bar/baz and cycle through the same 16 combinations."""
    labels, tp_keys = ["foo", "bar", "baz"], ["region", "zone", "node"]
    nodes = [node("node%d" % i, "4", "32Gi", 110,
                  labels={"region": "region%d" % (i % 3), "zone": "zone%d" % (i % 10), "node": "node%d" % i})
             for i in range(n_nodes)]
    existing = []
    for i in range(n_existing):
        a = _affinity_combo(i, labels, tp_keys)
        spec = {"affinity": a} if a else {}
        existing.append(pod("pod%d" % i, node_name="node%d" % (i % n_nodes), **spec))
    pods = []
    for i in range(n_pods):
        a = _affinity_combo(i, labels, tp_keys)
        spec = {"affinity": a} if a else {}
        pods.append(pod("p%d" % i, "100m", "500Mi", labels={labels[(i // 16) % 3]: ""}, **spec))
    return nodes, existing, pods, _c.Profile()


# ----------------------------------------------------------------------------- (e)
def sharded_spread(n_nodes=1_000_000, n_pods=10000, seed=CLUSTER_SEED, n_zones=64):
    """Config (e): the generator of (b)+(c) with zone = i % 64 -- config (b)'s
    node resources (cpu {4..64}, memory {16..256}Gi, 110 pods, 100Gi ephemeral) carrying config (c)'s
    taints (10% dedicated=infra:NoSchedule, 20% spot=true:PreferNoSchedule) and labels (zone, hostname),
    and config (c)'s pods (requests as (b), 50% tolerate `dedicated`, PodTopologySpread on zone
    (DoNotSchedule, maxSkew 1) and hostname (ScheduleAnyway), app=web) under the default profile.
    The required NodeAffinity admits the first 30% of the zones (zone1..zone19 of 64), the share
    (c)'s zone1..zone3 of 10 admits.  Meant for 1M nodes as contiguous shards over 8 GPUs."""
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        taints = []
        if r.chance(1, 10):
            taints.append({"key": "dedicated", "value": "infra", "effect": "NoSchedule"})
        if r.chance(2, 10):
            taints.append({"key": "spot", "value": "true", "effect": "PreferNoSchedule"})
        nodes.append(node("node%d" % i, str(r.pick(_CPUS)), "%dGi" % r.pick(_MEMS_GI),
                          110, "100Gi", labels={ZONE: "zone%d" % (i % n_zones), HOSTNAME: "node%d" % i},
                          taints=taints))
    return nodes, [], _spread_pods(r, n_pods, n_zones), _c.Profile()


_CPUS = [4, 8, 16, 32, 64]
_MEMS_GI = [16, 32, 64, 128, 256]


def _spread_pods(r, n_pods, n_zones):
    """Config (e)'s pods, drawn from r after the node draws."""
    admit = ["zone%d" % z for z in range(1, max(2, (3 * n_zones) // 10 + 1))]
    na = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
        {"matchExpressions": [{"key": ZONE, "operator": "In", "values": admit}]}]}}}
    sel = {"matchLabels": {"app": "web"}}
    tsc = [{"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "DoNotSchedule", "labelSelector": sel},
           {"maxSkew": 1, "topologyKey": HOSTNAME, "whenUnsatisfiable": "ScheduleAnyway", "labelSelector": sel}]
    pods = []
    for i in range(n_pods):
        spec = {"affinity": na, "topologySpreadConstraints": tsc}
        if r.chance(1, 2):
            spec["tolerations"] = [{"key": "dedicated", "operator": "Equal", "value": "infra", "effect": "NoSchedule"}]
        if r.chance(1, 10):
            pods.append(pod("p%d" % i, labels={"app": "web"}, **spec))
        else:
            pods.append(pod("p%d" % i, "%dm" % (100 * (1 + r.below(40))), "%dMi" % (128 * (1 + r.below(64))),
                            labels={"app": "web"}, **spec))
    return pods


def _splitmix_draws(seed, start, count):
    """Outputs start .. start+count-1 (0-based) of Rng(seed), vectorized: the k-th output is a pure
    function of the state seed + (k+1)*0x9E3779B97F4A7C15 (mod 2^64)."""
    import numpy as np
    with np.errstate(over="ignore"):
        k = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed & M64) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def sharded_spread_compiled(n_nodes=1_000_000, n_pods=10000, shard=None, n_hint=16, seed=CLUSTER_SEED, n_zones=64):
    """Config (e) straight to the engine's SoA columns: the cluster of sharded_spread(n_nodes,
    n_pods) compiled exactly as Compiler.register + compile_snapshot would compile its node objects
    (same dictionaries in the same order, same columns; tests/test_cluster_fast.py pins the equality),
    without building a million v1.Node dicts.  Each node draws 4 values (dedicated taint, spot taint,
    cpu, memory), so node i's draws are 4i..4i+3 and the columns are one vectorized splitmix64 pass.

    shard=(base, count) keeps only that slice of the rows (native.shard_range).  n_hint: the pods
    registered before the snapshot compile (GpuFramework's pods_hint).  Returns (compiler, (snap,
    arrays, order), pods, profile)."""
    import numpy as np
    N = n_nodes
    d = _splitmix_draws(seed, 0, 4 * N).reshape(N, 4) if N else np.zeros((0, 4), np.uint64)
    ded = (d[:, 0] % np.uint64(10)) < 1
    spot = (d[:, 1] % np.uint64(10)) < 2
    cpu = np.array(_CPUS, np.int64)[(d[:, 2] % np.uint64(5)).astype(np.int64)]
    mem = np.array(_MEMS_GI, np.int64)[(d[:, 3] % np.uint64(5)).astype(np.int64)]
    del d
    r = Rng(seed)
    r.s = (seed + 4 * N * 0x9E3779B97F4A7C15) & M64
    pods = _spread_pods(r, n_pods, n_zones)
    prof = _c.Profile()
    comp = _c.Compiler(prof)
    # Compiler.register(nodes, (), pods[:n_hint]) in node insertion order: labels (zone, then
    # hostname), taints by first appearance (dedicated before spot within a node), zone keys
    nz = min(N, n_zones)
    for i in range(nz):
        comp.nkeys.add(ZONE, "zone%d" % i)
    names = ["node%d" % i for i in range(N)]
    if N:
        hk = comp.nkeys.add_key(HOSTNAME)
        comp.nkeys.vals[hk].add_many(names)
    t_ded = ("dedicated", "infra", "NoSchedule")
    t_spot = ("spot", "true", "PreferNoSchedule")
    f_ded = int(np.argmax(ded)) if ded.any() else None
    f_spot = int(np.argmax(spot)) if spot.any() else None
    firsts = sorted([(f, 0, t) for f, t in ((f_ded, t_ded),) if f is not None] +
                    [(f, 1, t) for f, t in ((f_spot, t_spot),) if f is not None])
    for _, _, t in firsts:
        comp.taints.add(t)
    for i in range(nz):
        comp.zones.add(":\x00:zone%d" % i)
    for p in pods[:n_hint]:
        comp.register_pod(p)
    comp.ns.add("")
    # Snapshot.List(): node i sits in zone i % n_zones at position i // n_zones of that zone, so the
    # zone round robin (node_tree.go:147-170) lists the nodes in insertion order
    comp.set_order(names, first_wins=False)
    A = comp.empty_columns(N)
    A["alloc_cpu"][:] = cpu * 1000
    A["alloc_mem"][:] = mem * GI
    A["alloc_eph"][:] = 100 * GI
    A["alloc_pods"][:] = 110
    idx = np.arange(N, dtype=np.int64)
    A["label_val"][0] = idx % n_zones
    if N:
        A["label_val"][1] = idx
    A["zone_id"][:] = idx % n_zones
    for t, mask, col in ((t_ded, ded, "taint_nosched"), (t_spot, spot, "taint_prefer")):
        tid = comp.taints.get(t)
        if tid >= 0:
            A[col][tid // 64][mask] |= np.uint64(1 << (tid % 64))
    compiled = comp.snapshot_from_columns(A, shard)
    return comp, compiled, pods, prof


CONFIGS = {"a": scheduling_basic, "b": fit_least_balanced, "c": taints_affinity_spread, "d": pod_affinity,
           "e": sharded_spread}


def uneven_zones(sizes=(("a", 30), ("b", 2), ("c", 30)), n_pods=24):
    """Zones of uneven size for node-sharding tests: nodeTree's zone round robin
    (node_tree.go:147-170) exhausts the 2-node zone b early, so both of its nodes sit in the first
    contiguous shard of Snapshot.List().  b holds the smallest match count, so every other shard
    needs the first shard's pair registrations to see criticalPaths[0] (filtering.go:246-270):
    without the cross-shard union its zones a / c would pass the skew check that the cluster-wide
    minimum fails.  Pods: PodTopologySpread zone (DoNotSchedule) + hostname (ScheduleAnyway)."""
    nodes = []
    for z, n in sizes:
        nodes += [node("%s%d" % (z, i), "4", "32Gi", 110, labels={ZONE: z, HOSTNAME: "%s%d" % (z, i)})
                  for i in range(n)]
    existing = [pod("e%d" % i, "100m", "128Mi", labels={"app": "web"}, node_name=nn)
                for i, nn in enumerate(["a3", "a7", "a20", "c1", "c28"])]
    sel = {"matchLabels": {"app": "web"}}
    tsc = [{"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "DoNotSchedule", "labelSelector": sel},
           {"maxSkew": 1, "topologyKey": HOSTNAME, "whenUnsatisfiable": "ScheduleAnyway", "labelSelector": sel}]
    pods = [pod("p%d" % i, "100m", "128Mi", labels={"app": "web"}, topologySpreadConstraints=tsc)
            for i in range(n_pods)]
    return nodes, existing, pods, _c.Profile()
