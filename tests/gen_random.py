"""Seeded random clusters exercising every tier-1 plugin input (test infrastructure)."""
import random

ZONE = "topology.kubernetes.io/zone"
REGION = "topology.kubernetes.io/region"
HOST = "kubernetes.io/hostname"


def rnode(r, i, n_zones=3):
    al = {"cpu": "%dm" % r.choice([1000, 2000, 4000, 8000, 16000]), "memory": "%dMi" % r.choice([1024, 2048, 4096, 8192]),
          "pods": str(r.choice([3, 5, 10, 110]))}
    if r.random() < 0.5:
        al["ephemeral-storage"] = "%dGi" % r.choice([1, 10, 100])
    if r.random() < 0.3:
        al["example.com/gpu"] = str(r.choice([0, 1, 2, 4]))
    labels = {HOST: "n%d" % i}
    if r.random() < 0.9:
        labels[ZONE] = "z%d" % r.randrange(n_zones)
    if r.random() < 0.5:
        labels[REGION] = "r%d" % r.randrange(2)
    if r.random() < 0.5:
        labels["disk"] = r.choice(["ssd", "hdd", "nvme"])
    if r.random() < 0.5:
        labels["kernel"] = r.choice(["100", "200", "0300", "abc", "-5"])
    taints = []
    if r.random() < 0.3:
        taints.append({"key": "dedicated", "value": r.choice(["infra", "db"]), "effect": r.choice(["NoSchedule", "NoExecute"])})
    if r.random() < 0.4:
        taints.append({"key": "spot", "value": "true", "effect": "PreferNoSchedule"})
    if r.random() < 0.2:
        taints.append({"key": "noisy", "value": "", "effect": "PreferNoSchedule"})
    n = {"metadata": {"name": "n%d" % i, "labels": labels}, "spec": {}, "status": {"allocatable": al}}
    if taints:
        n["spec"]["taints"] = taints
    if r.random() < 0.05:
        n["spec"]["unschedulable"] = True
    if r.random() < 0.3:
        n["status"]["images"] = [{"names": ["img%d:latest" % r.randrange(4)], "sizeBytes": r.choice([10, 300, 900]) * 1024 * 1024}]
    if r.random() < 0.1:
        n["metadata"]["annotations"] = {"preferAvoidPods": [{"kind": "ReplicaSet", "uid": "rs%d" % r.randrange(3)}]}
    return n


def rpod(r, i, node_names=(), allow_node_name=True):
    c = {"name": "c", "image": "img%d" % r.randrange(6)}
    req = {}
    if r.random() < 0.8:
        req["cpu"] = "%dm" % r.choice([0, 50, 100, 250, 500, 1000, 3000])
    if r.random() < 0.8:
        req["memory"] = "%dMi" % r.choice([0, 64, 128, 512, 1024, 3000])
    if r.random() < 0.2:
        req["ephemeral-storage"] = "%dGi" % r.choice([1, 5, 50])
    if r.random() < 0.15:
        req["example.com/gpu"] = str(r.choice([1, 2]))
    c["resources"] = {"requests": req}
    if r.random() < 0.15:
        c["ports"] = [{"containerPort": 80, "hostPort": r.choice([8080, 9090]), "protocol": r.choice(["TCP", "UDP"]),
                       "hostIP": r.choice(["", "10.0.0.1"])}]
    spec = {"containers": [c]}
    if r.random() < 0.2:
        spec["initContainers"] = [{"name": "i", "resources": {"requests": {"cpu": "%dm" % r.choice([100, 2000])}}}]
    if r.random() < 0.1:
        spec["overhead"] = {"cpu": "%dm" % r.choice([10, 1500]), "memory": "10Mi"}
    tols = []
    if r.random() < 0.4:
        tols.append({"key": "dedicated", "operator": r.choice(["Equal", "Exists"]), "value": r.choice(["infra", "db"]),
                     "effect": r.choice(["", "NoSchedule", "NoExecute"])})
    if r.random() < 0.3:
        tols.append({"key": "spot", "operator": "Exists", "effect": r.choice(["", "PreferNoSchedule", "NoSchedule"])})
    if r.random() < 0.05:
        tols.append({"operator": "Exists"})
    if r.random() < 0.05:
        tols.append({"key": "node.kubernetes.io/unschedulable", "operator": "Exists", "effect": "NoSchedule"})
    if tols:
        spec["tolerations"] = tols
    if r.random() < 0.2:
        spec["nodeSelector"] = {"disk": r.choice(["ssd", "hdd", "tape"])}
    aff = {}
    if r.random() < 0.3:
        terms = []
        for _ in range(r.choice([1, 2])):
            op = r.choice(["In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"])
            if op in ("In", "NotIn"):
                e = {"key": r.choice([ZONE, "disk", "nokey"]), "operator": op, "values": r.sample(["z0", "z1", "ssd", "hdd", "zz"], 2)}
            elif op in ("Gt", "Lt"):
                e = {"key": "kernel", "operator": op, "values": [r.choice(["150", "50", "250"])]}
            else:
                e = {"key": r.choice(["disk", "kernel", "nokey"]), "operator": op}
            t = {"matchExpressions": [e]}
            if r.random() < 0.2 and node_names:
                t["matchFields"] = [{"key": "metadata.name", "operator": r.choice(["In", "NotIn"]),
                                     "values": [r.choice(list(node_names))]}]
            terms.append(t)
        aff["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": terms}
    if r.random() < 0.4:
        prefs = []
        for _ in range(r.choice([1, 2, 3])):
            op = r.choice(["In", "Exists", "Gt"])
            if op == "In":
                e = {"key": r.choice([ZONE, "disk"]), "operator": "In", "values": [r.choice(["z0", "z2", "ssd", "nvme"])]}
            elif op == "Gt":
                e = {"key": "kernel", "operator": "Gt", "values": ["99"]}
            else:
                e = {"key": r.choice(["disk", REGION]), "operator": "Exists"}
            prefs.append({"weight": r.choice([1, 5, 50, 100]), "preference": {"matchExpressions": [e]}})
        aff["preferredDuringSchedulingIgnoredDuringExecution"] = prefs
    if aff:
        spec["affinity"] = {"nodeAffinity": aff}
    if allow_node_name and r.random() < 0.03 and node_names:
        spec["nodeName"] = r.choice(list(node_names) + ["ghost"])
    md = {"name": "p%d" % i, "namespace": "default", "uid": "u%d" % i, "labels": {"app": r.choice(["a", "b"])}}
    if r.random() < 0.2:
        md["ownerReferences"] = [{"kind": "ReplicaSet", "uid": "rs%d" % r.randrange(3), "controller": True}]
    return {"metadata": md, "spec": spec}


def cluster(seed, n_nodes=20, n_existing=15, n_pods=30):
    r = random.Random(seed)
    nodes = [rnode(r, i) for i in range(n_nodes)]
    names = [n["metadata"]["name"] for n in nodes]
    existing = []
    for i in range(n_existing):
        p = rpod(r, 1000 + i, names, allow_node_name=False)
        p["spec"]["nodeName"] = r.choice(names)
        existing.append(p)
    pods = [rpod(r, i, names) for i in range(n_pods)]
    return nodes, existing, pods


# ---------------------------------------------------------------- topology workloads (PTS / IPA / DPTS)
APPS = ["web", "db", "cache"]


def _lsel(r):
    kind = r.random()
    if kind < 0.5:
        return {"matchLabels": {"app": r.choice(APPS)}}
    if kind < 0.7:
        return {"matchExpressions": [{"key": "app", "operator": "In", "values": r.sample(APPS, 2)}]}
    if kind < 0.85:
        return {"matchExpressions": [{"key": r.choice(["tier", "app"]), "operator": "Exists"}]}
    if kind < 0.95:
        return {"matchExpressions": [{"key": "app", "operator": "NotIn", "values": [r.choice(APPS)]}]}
    return {"matchExpressions": [{"key": "tier", "operator": "DoesNotExist"}]}


def _pod_term(r):
    t = {"labelSelector": _lsel(r), "topologyKey": r.choice([ZONE, HOST, REGION, "nokey"])}
    if r.random() < 0.15:
        t["namespaces"] = r.sample(["default", "other"], r.choice([1, 2]))
    return t


def _topo_spec(r, spec, md, p_tsc=0.5, p_aff=0.5):
    if r.random() < p_tsc:
        tsc = []
        for _ in range(r.choice([1, 1, 2])):
            tsc.append({"maxSkew": r.choice([1, 1, 2, 3]), "topologyKey": r.choice([ZONE, HOST, REGION, ZONE]),
                        "whenUnsatisfiable": r.choice(["DoNotSchedule", "ScheduleAnyway"]),
                        "labelSelector": _lsel(r)})
        spec["topologySpreadConstraints"] = tsc
    if r.random() < p_aff:
        a = spec.setdefault("affinity", {})
        for field in ("podAffinity", "podAntiAffinity"):
            if r.random() < 0.5:
                continue
            sub = {}
            if r.random() < 0.5:
                sub["requiredDuringSchedulingIgnoredDuringExecution"] = [_pod_term(r) for _ in range(r.choice([1, 2]))]
            if r.random() < 0.6:
                sub["preferredDuringSchedulingIgnoredDuringExecution"] = [
                    {"weight": r.choice([1, 10, 50, 100]), "podAffinityTerm": _pod_term(r)}
                    for _ in range(r.choice([1, 2]))]
            a[field] = sub
        if not a:
            del spec["affinity"]
    labels = {"app": r.choice(APPS)}
    if r.random() < 0.3:
        labels["tier"] = r.choice(["fe", "be"])
    md["labels"] = labels
    if r.random() < 0.2:
        md["namespace"] = "other"
    if r.random() < 0.05:
        md["deletionTimestamp"] = "2020-01-01T00:00:00Z"


def topo_cluster(seed, n_nodes=16, n_existing=24, n_pods=30):
    """Nodes over 3 zones / 2 regions (some unlabeled), existing pods with terms, incoming pods with
    spread constraints and (anti-)affinity, plus services / replica sets for DefaultPodTopologySpread."""
    r = random.Random(1000 + seed)
    nodes = [rnode(r, i) for i in range(n_nodes)]
    for n in nodes:  # generous capacity: topology plugins decide, not Fit
        n["status"]["allocatable"].update({"cpu": "64", "memory": "256Gi", "pods": "110"})
    names = [n["metadata"]["name"] for n in nodes]
    existing = []
    for i in range(n_existing):
        p = rpod(r, 1000 + i, names, allow_node_name=False)
        p["spec"]["nodeName"] = r.choice(names)
        _topo_spec(r, p["spec"], p["metadata"], p_tsc=0.0, p_aff=0.4)
        existing.append(p)
    pods = []
    for i in range(n_pods):
        p = rpod(r, i, names, allow_node_name=False)
        _topo_spec(r, p["spec"], p["metadata"])
        pods.append(p)
    services = [{"metadata": {"name": "svc-web", "namespace": "default"}, "spec": {"selector": {"app": "web"}}}]
    rss = [{"metadata": {"name": "rs-db", "namespace": "default"},
            "spec": {"selector": {"matchLabels": {"app": "db"}}}}]
    return nodes, existing, pods, services, rss
