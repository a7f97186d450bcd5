"""Evaluate one golden fixture case with the Python oracle (oracle/refsched).

Result format shared with the GPU-path evaluator (tests/gpu_runner.py):
    {"scores": {node: int}}  |  {"filter": {node: {"code": c, "reasons": [...]}}}  |
    {"error": message}       |  {"placements": [...]}
"""
from oracle.refsched import framework as F
from oracle.refsched import nodeinfo as NI
from oracle.refsched import plugins as P


def make_plugin(name, args, handle):
    a = args or {}
    if name == "NodeResourcesLeastAllocated":
        return P.LeastAllocated(handle, [tuple(r) for r in a.get("resources", [["cpu", 1], ["memory", 1]])])
    if name == "NodeResourcesMostAllocated":
        return P.MostAllocated(handle, [tuple(r) for r in a.get("resources", [["cpu", 1], ["memory", 1]])])
    if name == "NodeResourcesBalancedAllocation":
        return P.BalancedAllocation(handle)
    if name == "NodeResourcesFit":
        return P.Fit(a.get("ignored", []))
    if name == "TaintToleration":
        return P.TaintToleration(handle)
    if name == "NodeAffinity":
        return P.NodeAffinity(handle)
    if name == "NodeUnschedulable":
        return P.NodeUnschedulable()
    if name == "NodeName":
        return P.NodeName()
    if name == "NodePorts":
        return P.NodePorts()
    if name == "ImageLocality":
        return P.ImageLocality(handle)
    if name == "NodePreferAvoidPods":
        return P.NodePreferAvoidPods(handle)
    if name == "PodTopologySpread":
        return P.PodTopologySpread(handle, a.get("default_constraints", []))
    if name == "DefaultPodTopologySpread":
        return P.DefaultPodTopologySpread(handle)
    if name == "InterPodAffinity":
        return P.InterPodAffinity(handle, a.get("hard_pod_affinity_weight", 1))
    if name == "RequestedToCapacityRatio":
        return P.RequestedToCapacityRatio(handle, a["shape"], [tuple(r) for r in a["resources"]])
    if name == "NodeResourceLimits":
        return P.ResourceLimits(handle)
    raise KeyError(name)


def _handle(c):
    snap = NI.Snapshot(c["nodes"], c.get("pods", []), order=c.get("order", "given"))
    return F.Handle(snap, c.get("services", []), c.get("rcs", []), c.get("rss", []), c.get("sss", []))


def oracle_eval(c):
    kind = c["kind"]
    if kind in ("score", "filter"):
        h = _handle(c)
        try:
            pl = make_plugin(c["plugin"], c.get("args"), h)
        except ValueError as e:
            return {"error": str(e)}
        state = {}
        pod = c["pod"]
        if kind == "filter":
            if hasattr(pl, "prefilter"):
                st = pl.prefilter(state, pod)
                if not P.is_success(st):
                    return {"error": repr(st)}
            out = {}
            for ni in h.snapshot.list:
                st = pl.filter(state, pod, ni)
                out[NI.name(ni.node)] = {"code": P.code_of(st), "reasons": [] if st is None else st.reasons}
            return {"filter": out}
        nodes = [ni.node for ni in h.snapshot.list]
        names = c.get("filtered") or [NI.name(n) for n in nodes]
        fnodes = [h.snapshot.get(n).node for n in names]
        if hasattr(pl, "prescore"):
            st = pl.prescore(state, pod, fnodes)
            if not P.is_success(st):
                return {"error": repr(st)}
        scores = []
        for n in names:
            s, st = pl.score(state, pod, n)
            if not P.is_success(st):
                return {"error": repr(st)}
            scores.append([n, s])
        if c.get("normalize") and hasattr(pl, "normalize"):
            st = pl.normalize(state, pod, scores)
            if not P.is_success(st):
                return {"error": repr(st)}
        return {"scores": {n: s for n, s in scores}}
    if kind == "schedule":
        prof = profile_from_case(c)
        res = F.schedule_sequence(c["nodes"], c.get("pods", []), c["schedule_pods"], prof,
                                  c.get("services", []), c.get("rcs", []), c.get("rss", []), c.get("sss", []),
                                  pvcs=c.get("pvcs", []), order=c.get("order", "tree"))
        out = []
        for r in res:
            if isinstance(r, F.ScheduleError):
                e = {"host": None, "error": type(r).__name__, "message": str(r)}
                if isinstance(r, F.FitError):
                    e["fit"] = {n: [st.code, list(st.reasons)] for n, (_, st) in r.statuses.items()}
                out.append(e)
            else:
                out.append({"host": r.host, "totals": {n: s for n, s in r.totals}, "feasible": r.feasible,
                            "evaluated": r.evaluated})
        return {"placements": out}
    if kind == "select":
        idx = {n: i for i, (n, _) in enumerate(c["list"])}
        prof = F.Profile()
        hosts = set()
        try:
            for seq in range(16):
                hosts.add(F.select_host(c["list"], idx, prof, seq)[0])
        except F.ScheduleError as e:
            return {"error": str(e)}
        return {"hosts": sorted(hosts)}
    if kind == "num_feasible":
        gs = F.GenericScheduler(F.Framework(F.Profile(percentage_of_nodes_to_score=c["pct"], filters=[],
                                                      prefilters=[], prescores=[], scores=[]),
                                            F.Handle(NI.Snapshot([]))))
        return {"num": gs.num_feasible_nodes_to_find(c["num_all_nodes"])}
    if kind == "normalize":
        scores = [list(x) for x in c["scores"]]
        P.default_normalize_score(c["max_priority"], c["reverse"], scores)
        return {"scores": {str(i): s for i, (_, s) in enumerate(scores)}}
    if kind == "node_tree":
        return {"order": NI.node_tree_order(c["nodes"])}
    if kind == "node_tree_ops":
        return replay_node_tree(NI.NodeTreeRef(c["initial"]), c["ops"],
                                lambda t, r: t.remove_node(r) is not None)
    if kind == "pts_state":
        return pts_state(c)
    if kind == "ipa_state":
        return ipa_state(c)
    if kind == "run_score":
        return run_score(c)
    if kind == "run_filter":
        return run_filter(c)
    if kind == "preempt":
        return preempt_full(c)
    if kind == "broken_linear":
        pl = P.RequestedToCapacityRatio(None, [], [])
        pl.shape = [tuple(x) for x in c["points"]]
        return {"values": [[p, pl.broken_linear(p)] for p, _ in c["expect_values"]]}
    if kind in ("preempt_select", "preempt_pick"):
        return preempt_eval(c)
    if kind == "preempt_might_help":
        from oracle.refsched import preemption as PR
        nodes = [NI.NodeInfo({"metadata": {"name": n}}) for n in c["node_names"]]
        sts = {n: P.Status(code, "") for n, code in c["statuses"].items()}
        return {"hosts": sorted(NI.name(ni.node) for ni in PR.nodes_where_preemption_might_help(nodes, sts))}
    if kind == "image_name":
        return {"name": P.normalized_image_name(c["input"])}
    raise KeyError(kind)


def preempt_eval(c):
    """selectNodesForPreemption (+ pickOneNodeForPreemption) over every node of the snapshot, after
    the preemptor's PreFilter (generic_scheduler_test.go:1625-1646, 1909-1916)."""
    from oracle.refsched import preemption as PR
    prof = profile_from_case(c)
    snap = NI.Snapshot(c["nodes"], c.get("pods", []), order=c.get("order", "given"))
    fw = F.Framework(prof, F.Handle(snap))
    state = {}
    st = fw.run_prefilter(state, c["pod"])
    if st is not None:
        return {"error": repr(st)}
    now = PR.pod_start_time({"status": {"startTime": c["now"]}}, 0)
    n2v = PR.select_nodes_for_preemption(fw, None, state, c["pod"], snap.list, c.get("pdbs", []), now)
    out = {"victims": {n: {"pods": sorted(NI.name(p) for p in v), "pdb": nv} for n, (v, nv) in n2v.items()}}
    pick = PR.pick_one_node_for_preemption(n2v, now)
    out["hosts"] = [pick] if pick else []
    return out


def replay_node_tree(t, ops, remove_failed):
    """Apply a node_tree_ops sequence to a nodeTree implementation; shared by the oracle and the
    product's kgpu.api.NodeTree (tests/soa_runner.py)."""
    output, errors = [], []
    for op in ops:
        if op[0] == "add":
            t.add_node(op[1])
        elif op[0] == "remove":
            errors.append(bool(remove_failed(t, op[1])))
        elif op[0] == "update":
            t.update_node(op[1], op[2])
        else:
            output.append(t.next())
    tree = {z: list(t.tree[z]["nodes"]) for z in t.zones} if isinstance(t, NI.NodeTreeRef) else t.tree()
    return {"output": output, "tree": tree, "remove_errors": errors}


def _canon_selector(sel):
    """A selector as sorted (key, op, values) triples; "=" and "==" read as one operator."""
    if sel.nothing:
        return "nothing"
    return sorted([r.key, {"==": "="}.get(r.op, r.op), sorted(r.vals)] for r in sel.reqs)


def pts_state(c):
    """PodTopologySpread cycle state after PreFilter (+ AddPod/RemovePod) or PreScore."""
    h = _handle(c)
    pl = make_plugin("PodTopologySpread", c.get("args"), h)
    state, pod = {}, c["pod"]
    if c["op"] == "prescore":
        st = pl.prescore(state, pod, [ni.node for ni in h.snapshot.list])
        if not P.is_success(st):
            return {"error": repr(st)}
        s = state["PreScorePodTopologySpread"]
        return {"state": {"constraints": [[m, k, _canon_selector(sel)] for m, k, sel in s["constraints"]],
                          "ignored": sorted(s["ignored"]),
                          "pairs": sorted([k, v, n] for (k, v), n in s["counts"].items()),
                          "weights": list(s["weights"])}}
    st = pl.prefilter(state, pod)
    if not P.is_success(st):
        return {"error": repr(st)}
    if c["op"] in ("add", "remove"):
        ni = h.snapshot.get(c["op_node"])
        (pl.add_pod if c["op"] == "add" else pl.remove_pod)(state, pod, c["op_pod"], ni)
    s = state["PreFilterPodTopologySpread"]
    paths = {}
    for k, cp in s["paths"].items():
        p = [list(cp.p[0]), list(cp.p[1])]
        # filtering_test.go:50-55 criticalPaths.sort: equal counts compare alphabetically
        if p[0][1] == p[1][1] and p[0][0] > p[1][0]:
            p[0][0], p[1][0] = p[1][0], p[0][0]
        paths[k] = p
    return {"state": {"constraints": [[m, k, _canon_selector(sel)] for m, k, sel in s["constraints"]],
                      "paths": paths, "pairs": sorted([k, v, n] for (k, v), n in s["pairs"].items())}}


RUNNER_NODES = [{"metadata": {"name": "node1"}}, {"metadata": {"name": "node2"}}]  # framework_test.go:338-341


def run_score(c):
    """RunScorePlugins (framework.go:579-656) with the table's injected score plugins."""
    fw = F.Framework(profile_from_case(c), F.Handle(NI.Snapshot(RUNNER_NODES)))
    out, st = fw.run_score_plugins({}, {"metadata": {"name": ""}}, RUNNER_NODES)
    if st is not None:
        return {"error": ", ".join(st.reasons)}
    return {"run_scores": out}


def run_filter(c):
    """RunFilterPlugins + PluginToStatus.Merge (framework.go:477-502, interface.go:161-191)."""
    fw = F.Framework(profile_from_case(c), F.Handle(NI.Snapshot(RUNNER_NODES)))
    ni = NI.NodeInfo(RUNNER_NODES[0])
    sm = fw.run_filter_plugins({}, {"metadata": {"name": ""}}, ni, run_all_filters=c.get("run_all_filters", False))
    merged = F.merge_statuses(sm)
    return {"status_map": {k: {"code": v.code, "reasons": list(v.reasons)} for k, v in sm.items()},
            "merged": None if merged is None else {"code": merged.code, "reasons": list(merged.reasons)}}


def preempt_full(c):
    """genericScheduler.Preempt (generic_scheduler.go:252-351, extenders included) after a FitError with
    the case's statuses, then the second call of TestPreempt (:2440-2460) with the victims marked
    deleted and the preemptor nominated to the chosen node."""
    import copy
    import fake_plugins
    from oracle.refsched import preemption as PR
    c = copy.deepcopy(c)
    prof = profile_from_case(c)
    snap = NI.Snapshot(c["nodes"], c.get("pods", []), order=c.get("order", "given"))
    gs = F.GenericScheduler(F.Framework(prof, F.Handle(snap)))
    fe = F.FitError({n: (None, P.Status(code, "")) for n, code in c["statuses"].items()})
    now = PR.pod_start_time({"status": {"startTime": c["now"]}}, 0)
    pod = c["pod"]
    ext = fake_plugins.extenders(c.get("extenders"))
    node, victims, _ = PR.preempt(gs, pod, fe, c.get("pdbs", []), None, now, extenders=ext)
    names = {NI.name(v) for v in victims}
    for ni in snap.list:
        for pi in ni.pods:
            if NI.name(pi.pod) in names:
                pi.pod.setdefault("metadata", {})["deletionTimestamp"] = c["now"]
    pod.setdefault("status", {})["nominatedNodeName"] = node
    node2, victims2, _ = PR.preempt(gs, pod, fe, c.get("pdbs", []), None, now, extenders=ext)
    return {"preempt": {"node": node, "victims": sorted(names), "again": [node2, len(victims2)]}}


def ipa_state(c):
    """InterPodAffinity preFilterState maps after PreFilter, and for op add_remove after AddPod (with
    the two DeepEqual checks of filtering_test.go:1990-2030: AddPod's state equals PreFilter over a
    snapshot that holds the pod, RemovePod restores the original)."""
    def prefilter(pods):
        h = _handle(dict(c, pods=pods))
        pl = make_plugin("InterPodAffinity", c.get("args"), h)
        state = {}
        st = pl.prefilter(state, c["pod"])
        return pl, h, state, st

    def maps(state):
        s = state["PreFilterInterPodAffinity"]
        return {k: sorted([a, b, n] for (a, b), n in s[k].items()) for k in ("existing_anti", "aff", "anti")}

    pl, h, state, st = prefilter(c.get("pods", []))
    if not P.is_success(st):
        return {"error": repr(st)}
    m = maps(state)
    out = {"aff": m["aff"], "anti": m["anti"], "existing_anti": m["existing_anti"]}
    if c["op"] == "add_remove":
        ni = h.snapshot.get(c["op_node"])
        pl.add_pod(state, c["pod"], c["op_pod"], ni)
        added = maps(state)
        _, _, all_state, _ = prefilter(list(c.get("pods", [])) + [c["op_pod"]])
        pl.remove_pod(state, c["pod"], c["op_pod"], ni)
        out = {"aff": added["aff"], "anti": added["anti"], "existing_anti": added["existing_anti"],
               "add_equals_all": added == maps(all_state), "remove_restores": maps(state) == m}
    return {"ipa": out}


def profile_from_case(c):
    p = c.get("profile") or {}
    kw = {}
    for k in ("filters", "prefilters", "prescores"):
        if k in p:
            kw[k] = p[k]
    if "scores" in p:
        kw["scores"] = [tuple(s) for s in p["scores"]]
    for k in ("least_resources", "most_resources"):
        if k in p:
            kw[k] = [tuple(r) for r in p[k]]
    for k in ("hard_pod_affinity_weight", "ignored_resources", "pts_default_constraints",
              "percentage_of_nodes_to_score", "tie_break_mode", "seed"):
        if k in p:
            kw[k] = p[k]
    if "fake" in p:
        import fake_plugins
        kw["plugin_factories"] = fake_plugins.factories(p["fake"])
    if p.get("base") == "cluster_autoscaler":
        return F.cluster_autoscaler_profile(**kw)
    return F.Profile(**kw)


def check(c, got):
    """Compare a result against the case's expectations; returns a list of mismatches."""
    bad = []
    if "expect_error" in c:
        if "error" not in got or (c["expect_error"] and c["expect_error"] not in got["error"]):
            bad.append(("error", c["expect_error"], got))
        return bad
    if "error" in got:
        return [("unexpected error", got["error"])]
    if "expect_scores" in c:
        for n, s in c["expect_scores"].items():
            if got["scores"].get(n) != s:
                bad.append((n, s, got["scores"].get(n)))
    if "expect_filter" in c:
        for n, e in c["expect_filter"].items():
            g = got["filter"].get(n)
            if g is None or g["code"] != e["code"]:
                bad.append((n, e, g))
            elif "reasons" in e and e["reasons"] is not None and sorted(g["reasons"]) != sorted(e["reasons"]):
                bad.append((n, e, g))
    if "expect_possible" in c:
        if not set(got["hosts"]) <= set(c["expect_possible"]):
            bad.append(("hosts", c["expect_possible"], got["hosts"]))
    if "expect_set" in c and sorted(got.get("hosts") or []) != c["expect_set"]:
        bad.append(("set", c["expect_set"], got.get("hosts")))
    if "expect_victims" in c and got.get("victims") != c["expect_victims"]:
        bad.append(("victims", c["expect_victims"], got.get("victims")))
    if "expect_num" in c and got.get("num") != c["expect_num"]:
        bad.append(("num", c["expect_num"], got.get("num")))
    if "expect_state" in c:
        bad += _check_state(c["expect_state"], got.get("state") or {})
    if "expect_run_scores" in c and got.get("run_scores") != c["expect_run_scores"]:
        bad.append(("run_scores", c["expect_run_scores"], got.get("run_scores")))
    if "expect_status_map" in c:
        if got.get("status_map") != c["expect_status_map"]:
            bad.append(("status_map", c["expect_status_map"], got.get("status_map")))
        if got.get("merged") != c["expect_merged"]:
            bad.append(("merged", c["expect_merged"], got.get("merged")))
    if "expect_preempt" in c:
        g = got.get("preempt") or {}
        if g.get("node") != c["expect_preempt"]["node"] or g.get("victims") != c["expect_preempt"]["victims"]:
            bad.append(("preempt", c["expect_preempt"], g))
        again = g.get("again") or ["", 0]
        if again[0] and again[1] > 0:  # generic_scheduler_test.go:2455-2457
            bad.append(("preempted again", again))
    if "expect_ipa" in c:
        g = got.get("ipa") or {}
        for f in ("aff", "anti"):
            if g.get(f) != c["expect_ipa"][f]:
                bad.append((f, c["expect_ipa"][f], g.get(f)))
        if c.get("op") == "add_remove":
            for f in ("add_equals_all", "remove_restores"):
                if g.get(f) is not True:
                    bad.append((f, True, g.get(f)))
    for f in ("output", "tree", "remove_errors"):
        if "expect_" + f in c and got.get(f) != c["expect_" + f]:
            bad.append((f, c["expect_" + f], got.get(f)))
    if "expect_values" in c and got.get("values") != c["expect_values"]:
        bad.append(("values", c["expect_values"], got.get("values")))
    if "expect_name" in c and got.get("name") != c["expect_name"]:
        bad.append(("name", c["expect_name"], got.get("name")))
    if "expect_order" in c and got.get("order") != c["expect_order"]:
        bad.append(("order", c["expect_order"], got.get("order")))
    if "expect_hosts" in c:
        for i, allowed in enumerate(c["expect_hosts"]):
            h = got["placements"][i]["host"]
            if allowed is None:
                if h is not None:
                    bad.append((i, None, h))
            elif h not in allowed:
                bad.append((i, allowed, h))
    for i, want in enumerate(c.get("expect_messages") or []):
        if want is not None and want != got["placements"][i].get("message"):
            bad.append((i, "message", want, got["placements"][i].get("message")))
    for i, want in enumerate(c.get("expect_fit") or []):
        if want is not None and want != got["placements"][i].get("fit"):
            bad.append((i, "fit", want, got["placements"][i].get("fit")))
    for i, want in enumerate(c.get("expect_evaluated") or []):
        if want is not None and want != got["placements"][i].get("evaluated"):
            bad.append((i, "evaluated", want, got["placements"][i].get("evaluated")))
    if "expect_totals" in c:
        for i, tot in enumerate(c["expect_totals"]):
            if tot is None:
                continue
            g = got["placements"][i].get("totals", {})
            for n, s in tot.items():
                if g.get(n) != s:
                    bad.append((i, n, s, g.get(n)))
    return bad


def _check_state(want, got):
    import math
    from oracle.refsched import labels as L
    bad = []
    wc = [[m, k, _canon_selector(L.label_selector_as_selector(sel))] for m, k, sel in want.get("constraints", [])]
    if wc != got.get("constraints"):
        bad.append(("constraints", wc, got.get("constraints")))
    for f in ("paths", "ignored"):
        if f in want and want[f] != got.get(f):
            bad.append((f, want[f], got.get(f)))
    if sorted(map(list, want.get("pairs", []))) != got.get("pairs"):
        bad.append(("pairs", want.get("pairs"), got.get("pairs")))
    if "weight_sizes" in want:
        # scoring.go:260 topologyNormalizingWeight(size) = math.Log(float64(size + 2))
        w = [math.log(n + 2) for n in want["weight_sizes"]]
        g = got.get("weights") or []
        if len(w) != len(g) or any(abs(a - b) > 1e-15 * abs(a) for a, b in zip(w, g)):
            bad.append(("weights", w, g))
    return bad
