"""Evaluate golden fixture cases through the product's compile step (kgpu.compile) and either
the C restatement (oracle/c, CPU) or libkgpu.so (GPU).  Same result format as golden_runner."""
import copy

import numpy as np

from kgpu import abi, api
from kgpu.compile import Cluster, Profile
from kgpu.framework import GpuFramework

TIER1_SCORES = {"NodeResourcesLeastAllocated", "NodeResourcesMostAllocated", "NodeResourcesBalancedAllocation",
                "TaintToleration", "NodeAffinity", "ImageLocality", "NodePreferAvoidPods", "PodTopologySpread",
                "DefaultPodTopologySpread", "InterPodAffinity", "RequestedToCapacityRatio", "NodeResourceLimits"}
TIER1_FILTERS = {"NodeResourcesFit", "TaintToleration", "NodeAffinity", "NodeUnschedulable", "NodeName",
                 "NodePorts", "PodTopologySpread", "InterPodAffinity"}


def supported(c):
    k = c["kind"]
    if k == "score":
        # a cycle with one feasible node returns it unscored (generic_scheduler.go:184-191): plugin-level
        # tables over a single candidate are checked on the oracle only
        if c.get("filtered") is not None and len(c["filtered"]) < 2:
            return False
        return c["plugin"] in TIER1_SCORES
    if k == "filter":
        return c["plugin"] in TIER1_FILTERS
    if k in ("image_name", "node_tree", "node_tree_ops", "normalize", "broken_linear"):
        return True
    if k == "schedule":
        prof = c.get("profile") or {}
        # the fake plugins of generic_scheduler_test.go and the PVC basic checks are oracle-only
        if any(f not in TIER1_FILTERS for f in prof.get("filters", [])) or c.get("pvcs") or \
                any((p.get("spec") or {}).get("volumes") for p in c["schedule_pods"]):
            return False
        return all(n in TIER1_SCORES | {"DefaultPodTopologySpread"} for n, _ in prof.get("scores", []))
    return False


def _profile(c):
    a = c.get("args") or {}
    if c["kind"] == "score":
        # nodes outside the case's "filtered" list are made infeasible through NodeUnschedulable
        kw = dict(filters=["NodeUnschedulable"] if c.get("filtered") is not None else [], scores=[(c["plugin"], 1)])
        if c["plugin"] == "InterPodAffinity":
            kw["hard_pod_affinity_weight"] = a.get("hard_pod_affinity_weight", 1)
        if c["plugin"] == "NodeResourcesLeastAllocated":
            kw["least_resources"] = [tuple(r) for r in a.get("resources", [["cpu", 1], ["memory", 1]])]
        if c["plugin"] == "NodeResourcesMostAllocated":
            kw["most_resources"] = [tuple(r) for r in a.get("resources", [["cpu", 1], ["memory", 1]])]
        if c["plugin"] == "RequestedToCapacityRatio":
            kw["rtcr_resources"] = [tuple(r) for r in a["resources"]]
            kw["rtcr_shape"] = [tuple(x) for x in a["shape"]]
        return Profile(**kw)
    if c["kind"] == "filter":
        return Profile(filters=[c["plugin"]], scores=[], ignored_resources=a.get("ignored", []),
                       pts_default_constraints=a.get("default_constraints", []))
    p = c.get("profile") or {}
    return Profile(filters=[f for f in p.get("filters", Profile.DEFAULT_FILTERS) if f in abi.FILTER_IDS],
                   scores=[tuple(s) for s in p.get("scores", Profile.DEFAULT_SCORES)])


def normalize_case(c):
    """A helper/normalize_score_test.go row (DefaultNormalizeScore over given raw scores) as a score
    case of the plugin that normalizes with it: reverse -> TaintToleration (raw = the node's
    intolerable PreferNoSchedule taints, taint_toleration.go:123-157), not reverse -> NodeAffinity
    (raw = the summed weights of the matched preferred terms, node_affinity.go:66-111).  Node i
    carries raw score scores[i]; the product's normalize path must give the table's values."""
    assert c["max_priority"] == 100
    raws = [int(v) for _, v in c["scores"]]
    nodes, terms = [], []
    for i, v in enumerate(raws):
        meta = {"name": str(i)}
        spec = {}
        if c["reverse"]:
            spec["taints"] = [{"key": "t%d_%d" % (i, j), "value": "x", "effect": "PreferNoSchedule"} for j in range(v)]
        else:
            # v as terms of weight <= 100, each matched by this node's own label
            labels, left, j = {}, v, 0
            while left > 0:
                w = min(left, 100)
                labels["k%d_%d" % (i, j)] = "y"
                terms.append({"weight": w, "preference": {"matchExpressions": [
                    {"key": "k%d_%d" % (i, j), "operator": "In", "values": ["y"]}]}})
                left -= w
                j += 1
            meta["labels"] = labels
        nodes.append({"metadata": meta, "spec": spec, "status": {"allocatable": {}}})
    pod = {"metadata": {"name": "p", "namespace": ""}, "spec": {}}
    if terms:
        pod["spec"]["affinity"] = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": terms}}
    return {"kind": "score", "plugin": "TaintToleration" if c["reverse"] else "NodeAffinity", "normalize": True,
            "nodes": nodes, "pod": pod, "pods": [], "args": {}, "name": c["name"], "src": c["src"]}


def soa_eval(c, backend):
    if c["kind"] == "normalize":
        return soa_eval(normalize_case(c), backend)
    if c["kind"] == "broken_linear":
        ps = [p for p, _ in c["expect_values"]]
        if backend == "gpu":
            node = {"metadata": {"name": "n0"}, "spec": {}, "status": {"allocatable": {"cpu": "1"}}}
            fw = GpuFramework(Profile(filters=[], scores=[]), [node], [], device=0)
            try:
                vals = fw.engine.broken_linear(c["points"], ps)
            finally:
                fw.engine.close()
        else:
            from oracle import cref
            vals = cref.broken_linear(c["points"], ps)
        return {"values": [[p, v] for p, v in zip(ps, vals)]}
    if c["kind"] == "node_tree":
        return {"order": [api.name_of(n) for n in api.snapshot_order(c["nodes"])]}
    if c["kind"] == "node_tree_ops":
        from golden_runner import replay_node_tree
        return replay_node_tree(api.NodeTree(c["initial"]), c["ops"], lambda t, r: not t.remove_node(r))
    if c["kind"] == "image_name":
        # host-side: kgpu/compile.py interns normalized names before any image id reaches the device
        return {"name": api.normalized_image_name(c["input"])}
    try:
        prof = _profile(c)
    except ValueError as e:
        return {"error": str(e)}
    pods = [c["pod"]] if c["kind"] in ("score", "filter") else c["schedule_pods"]
    nodes = c["nodes"]
    if c["kind"] == "score" and c.get("filtered") is not None:
        keep = set(c["filtered"])
        nodes = copy.deepcopy(nodes)
        for n in nodes:
            if n["metadata"]["name"] not in keep:
                n.setdefault("spec", {})["unschedulable"] = True
    cluster = Cluster(c.get("services", []), c.get("rcs", []), c.get("rss", []), c.get("sss", []))
    fw = GpuFramework(prof, nodes, c.get("pods", []), cluster=cluster, pods_hint=pods,
                      create_engine=(backend == "gpu"))
    pod = pods[0]
    if backend == "gpu":
        cr = fw.cycle(pod, assume=False)
        res0 = cr.result
        words = {nm: 0 for nm in fw.order}
        for nm, st in cr.statuses.items():
            words[nm] = st
        statuses, scores = cr.statuses, cr.scores
    else:
        from oracle.cref import RefEngine
        q, pc, pnp, errs = fw.compile_pods([pod])
        ref = RefEngine(fw.config, fw.snap)
        res, st, raw, norm = ref.schedule(q, pc, diag=True)
        res0 = res[0]
        statuses = {}
        for i in np.nonzero(st)[0]:
            nm = fw.order[int(i)]
            statuses[nm] = fw.reasons(pod, nm, int(st[i]))
        scores = {}
        feas = np.nonzero(st == 0)[0]
        for name, w in prof.scores:
            sid = abi.SCORE_IDS[name]
            scores[name] = {fw.order[int(i)]: (int(raw[sid, i]), int(norm[sid, i])) for i in feas}
    if c["kind"] == "filter":
        out = {}
        for nm in fw.order:
            s = statuses.get(nm)
            out[nm] = {"code": 0, "reasons": []} if s is None else {"code": s[0], "reasons": s[2]}
        return {"filter": out}
    if c["kind"] == "score":
        sc = scores[c["plugin"]]
        return {"scores": {nm: (v[1] if c.get("normalize") else v[0]) if c["plugin"] in ("TaintToleration", "NodeAffinity") else v[1] for nm, v in sc.items()}}
    totals = {}
    for name, w in prof.scores:
        for nm, (r, nv) in scores[name].items():
            totals[nm] = totals.get(nm, 0) + nv * w
    node = int(res0["node"])
    return {"placements": [{"host": fw.order[node] if node >= 0 else None, "totals": totals,
                            "evaluated": int(res0["evaluated"]), "feasible": int(res0["feasible"])}]}
