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
