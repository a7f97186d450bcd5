"""Nominated-pod two-pass filter and preemption on the HIP path vs the oracle.

Reference: core/generic_scheduler.go:526-615 (addNominatedPods, podPassesFiltersOnNode),
:718-1056 (pickOneNodeForPreemption, selectNodesForPreemption, filterPodsWithPDBViolation,
selectVictimsOnNode, nodesWherePreemptionMightHelp, podEligibleToPreemptOthers).  The golden cases
are generic_scheduler_test.go's TestSelectNodesForPreemption / TestPickOneNodeForPreemption
(tests/golden/preemption.json); the random cases compare whole victim lists (in Victims.Pods
order), PDB violation counts and the picked node with oracle/refsched/preemption.py."""
import copy
import random

import numpy as np
import pytest

import gen_random
from conftest import load_golden
from kgpu import abi
from kgpu.compile import Cluster, Profile
from kgpu.framework import GpuFramework
from oracle.refsched import framework as F
from oracle.refsched import nodeinfo as NI
from oracle.refsched import plugins as P
from oracle.refsched import preemption as PR

NOW = 2_000_000_000 * 1_000_000_000
PRIOS = [-100, 0, 0, 100, 1000]


def _gpu_profile(c):
    p = c["profile"]
    return Profile(filters=[f for f in p["filters"] if f in abi.FILTER_IDS], scores=[])


GOLDEN = [c for c in load_golden("preemption") if c.get("gpu")]


@pytest.mark.gpu
@pytest.mark.parametrize("case", GOLDEN, ids=[c["name"][:60] for c in GOLDEN])
def test_golden_preemption_gpu(case):
    fw = GpuFramework(_gpu_profile(case), case["nodes"], case["pods"], pods_hint=[case["pod"]])
    now = PR.pod_start_time({"status": {"startTime": case["now"]}}, 0)
    n2v, pick = fw.select_nodes_for_preemption(case["pod"], case.get("pdbs", []), now)
    got = {n: {"pods": sorted(NI.name(p) for p in v), "pdb": nv} for n, (v, nv) in n2v.items()}
    if "expect_victims" in case:
        assert got == case["expect_victims"], (case["name"], got)
    if "expect_possible" in case:
        assert pick in case["expect_possible"], (case["name"], pick)
    fw.engine.close()


# ---------------------------------------------------------------- random parity
def _scenario(seed, topo):
    r = random.Random(7000 + seed)
    if topo:
        nodes, existing, pods, services, rss = gen_random.topo_cluster(seed, n_nodes=14, n_existing=40, n_pods=6)
        for n in nodes:  # tighter: resources and pod counts matter too
            n["status"]["allocatable"].update({"cpu": "4", "memory": "8Gi", "pods": str(r.choice([4, 6, 110]))})
    else:
        nodes, existing, pods = gen_random.cluster(seed, n_nodes=14, n_existing=40, n_pods=6)
        services, rss = [], []
    for p in existing + pods:
        p["spec"]["priority"] = r.choice(PRIOS)
        if r.random() < 0.7:
            p["status"] = {"startTime": "2019-01-0%dT01:01:01Z" % r.randrange(1, 8)}
    for p in pods:
        p["spec"]["priority"] = r.choice([500, 1000, 2000])
        p["spec"].pop("nodeName", None)
    pdbs = []
    for j in range(r.choice([0, 1, 2, 3])):
        sel = r.choice([{"matchLabels": {"app": r.choice(["a", "b", "web", "db"])}},
                        {"matchExpressions": [{"key": "app", "operator": "Exists"}]}, {}])
        pdbs.append({"namespace": r.choice(["default", "default", "other"]), "selector": sel,
                     "disruptionsAllowed": r.choice([0, 1, 2])})
    # nominated pods (pods that preempted earlier and wait), some above the preemptors' priority
    noms = []
    names = [n["metadata"]["name"] for n in nodes]
    for j in range(r.choice([0, 2, 4])):
        p = gen_random.rpod(r, 5000 + j, names, allow_node_name=False)
        if topo:
            gen_random._topo_spec(r, p["spec"], p["metadata"], p_tsc=0.0, p_aff=0.4)
        p["spec"]["priority"] = r.choice([0, 1000, 3000])
        noms.append((p, r.choice(names)))
    return nodes, existing, pods, services, rss, pdbs, noms


def _oracle_preempt(nodes, existing, pod, services, rss, pdbs, noms):
    snap = NI.Snapshot(nodes, existing)
    fw = F.Framework(F.Profile(), F.Handle(snap, services, (), rss))
    nominator = PR.Nominator()
    for p, nn in noms:
        nominator.add(p, nn)
    state = {}
    st = fw.run_prefilter(state, pod)
    if st is not None:
        return None
    potential = []
    for ni in snap.list:
        _, _, status = PR.pod_passes_filters_on_node(fw, nominator, state, pod, ni)
        if P.code_of(status) != P.UNRESOLVABLE:
            potential.append(ni)
    n2v = PR.select_nodes_for_preemption(fw, nominator, state, pod, potential, pdbs, NOW)
    return {n: ([NI.name(p) for p in v], nv) for n, (v, nv) in n2v.items()}, PR.pick_one_node_for_preemption(n2v, NOW)


@pytest.mark.gpu
@pytest.mark.parametrize("topo", [False, True], ids=["resources", "topology"])
@pytest.mark.parametrize("seed", range(6))
def test_select_victims_matches_oracle(seed, topo):
    nodes, existing, pods, services, rss, pdbs, noms = _scenario(seed, topo)
    fw = GpuFramework(Profile(), nodes, existing, cluster=Cluster(services=services, rss=rss),
                      pods_hint=pods + [p for p, _ in noms])
    if noms:
        fw.set_nominated(noms)
    checked = 0
    for pod in pods:
        want = _oracle_preempt(nodes, existing, pod, services, rss, pdbs, noms)
        if want is None:
            continue
        n2v, pick = fw.select_nodes_for_preemption(pod, pdbs, NOW)
        got = {n: ([NI.name(p) for p in v], nv) for n, (v, nv) in n2v.items()}
        assert got == want[0], (seed, NI.name(pod))
        assert pick == want[1], (seed, NI.name(pod), pick, want[1])
        checked += 1
    assert checked
    fw.engine.close()


@pytest.mark.gpu
@pytest.mark.parametrize("topo", [False, True], ids=["resources", "topology"])
@pytest.mark.parametrize("seed", range(6))
def test_nominated_two_pass_matches_oracle(seed, topo):
    """Scheduling cycles with a non-empty nominator: per-node statuses and the placement."""
    nodes, existing, pods, services, rss, pdbs, noms = _scenario(seed, topo)
    if not noms:
        r = random.Random(seed)
        p = gen_random.rpod(r, 6000, [n["metadata"]["name"] for n in nodes], allow_node_name=False)
        p["spec"]["priority"] = 3000
        noms = [(p, nodes[seed % len(nodes)]["metadata"]["name"])]
    fw = GpuFramework(Profile(), nodes, existing, cluster=Cluster(services=services, rss=rss),
                      pods_hint=pods + [p for p, _ in noms])
    fw.set_nominated(noms)
    snap = NI.Snapshot(nodes, existing)
    ofw = F.Framework(F.Profile(), F.Handle(snap, services, (), rss))
    nominator = PR.Nominator()
    for p, nn in noms:
        nominator.add(p, nn)
    gs = F.GenericScheduler(ofw, nominator)
    for i, pod in enumerate(pods):
        try:
            want = gs.schedule(pod, i)
            want_host, want_st = want.host, want.statuses
        except F.FitError as e:
            want_host, want_st = None, e.statuses
        cr = fw.cycle(pod, assume=False, seq=i)
        assert cr.host == want_host, (seed, i)
        got_codes = {n: s[0] for n, s in cr.statuses.items()}
        want_codes = {n: st.code for n, (_, st) in want_st.items()}
        assert got_codes == want_codes, (seed, i)
    fw.engine.close()


@pytest.mark.gpu
def test_nominated_batch_drops_placed_pods():
    """kgpu_schedule_batch with a nominator runs pod by pod and drops each assumed pod from it
    (scheduler.go:448): the oracle's scheduleOne loop with the same nominator agrees."""
    nodes, existing, pods, services, rss, pdbs, noms = _scenario(3, False)
    # nominate two of the batch's own pods: once placed they must stop counting on their nodes
    names = [n["metadata"]["name"] for n in nodes]
    noms = [(pods[0], names[0]), (pods[2], names[1])] + noms
    fw = GpuFramework(Profile(), nodes, existing, pods_hint=pods + [p for p, _ in noms])
    fw.set_nominated(noms)
    res = fw.schedule(pods, first_seq=0)
    snap = NI.Snapshot(nodes, existing)
    ofw = F.Framework(F.Profile(), F.Handle(snap))
    nominator = PR.Nominator()
    for p, nn in noms:
        nominator.add(p, nn)
    gs = F.GenericScheduler(ofw, nominator)
    for i, pod in enumerate(pods):
        try:
            r = gs.schedule(pod, i)
        except F.ScheduleError:
            assert res[i]["node"] < 0
            continue
        assert fw.host_of(int(res[i]["node"])) == r.host, i
        placed = copy.deepcopy(pod)
        placed["spec"]["nodeName"] = r.host
        snap.get(r.host).add_pod(placed)
        nominator.delete(pod)
    fw.engine.close()


@pytest.mark.gpu
def test_preempt_flow_and_eligibility():
    """Preempt: a FitError pod preempts on the device-picked node; PreemptNever and a terminating
    lower-priority pod on its nominated node make it ineligible."""
    nodes, existing, pods, services, rss, pdbs, noms = _scenario(1, False)
    fw = GpuFramework(Profile(), nodes, existing, pods_hint=pods)
    big = copy.deepcopy(pods[0])
    big["spec"]["containers"][0]["resources"] = {"requests": {"cpu": "900m", "memory": "900Mi"}}
    big["spec"]["priority"] = 100000
    cr = fw.cycle(big, assume=False)
    node, victims, clear = fw.preempt(big, cr.statuses, pdbs, NOW)
    want = _oracle_preempt(nodes, existing, big, services, rss, pdbs, [])
    assert node == want[1]
    if node:
        assert [NI.name(p) for p in victims] == want[0][node][0]
    never = copy.deepcopy(big)
    never["spec"]["preemptionPolicy"] = "Never"
    assert fw.preempt(never, cr.statuses, pdbs, NOW) == ("", [], [])
    fw.engine.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_many_pdbs_only_matching_ones_reach_the_engine(seed):
    """Preempt lists every PodDisruptionBudget of the cluster: 80 PDBs, most selecting no
    potential victim, the matching ones scattered past index 64.  The engine gets the matching subset
    renumbered in order (filterPodsWithPDBViolation walks only those), and the victims, violation
    counts and picked node equal the oracle's over the full list."""
    nodes, existing, pods, services, rss, pdbs, noms = _scenario(seed, False)
    r = random.Random(900 + seed)
    many = [{"namespace": "nowhere", "selector": {"matchLabels": {"app": "x%d" % j}}, "disruptionsAllowed": 0}
            for j in range(80)]
    for k, p in enumerate(pdbs):
        many[r.randrange(60, 80) if k % 2 else r.randrange(0, 80)] = p
    fw = GpuFramework(Profile(), nodes, existing, cluster=Cluster(services=services, rss=rss), pods_hint=pods)
    checked = 0
    for pod in pods:
        want = _oracle_preempt(nodes, existing, pod, services, rss, many, [])
        if want is None:
            continue
        n2v, pick = fw.select_nodes_for_preemption(pod, many, NOW)
        got = {n: ([NI.name(p) for p in v], nv) for n, (v, nv) in n2v.items()}
        assert got == want[0], (seed, NI.name(pod))
        assert pick == want[1], (seed, NI.name(pod))
        checked += 1
    assert checked
    fw.engine.close()


MIGHT_HELP = [c for c in load_golden("preemption") if c["kind"] == "preempt_might_help"]


@pytest.mark.parametrize("case", MIGHT_HELP, ids=[c["name"][:60] for c in MIGHT_HELP])
def test_golden_nodes_where_preemption_might_help(case):
    """TestNodesWherePreemptionMightHelp (generic_scheduler_test.go) through the product's host step
    (kgpu.framework.nodes_where_preemption_might_help), which Preempt uses to pick the nodes that get
    potential victims."""
    from kgpu.framework import nodes_where_preemption_might_help
    got = nodes_where_preemption_might_help(case["node_names"], case["statuses"])
    assert sorted(got) == case["expect_set"], (case["name"], got)


# ---------------------------------------------------------------- TestPreempt (generic_scheduler_test.go:2047)
PREEMPT = [c for c in load_golden("preemption") if c["kind"] == "preempt"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", PREEMPT, ids=[c["src"].rsplit(":", 1)[1] for c in PREEMPT])
def test_golden_preempt_gpu(case):
    """genericScheduler.Preempt through the product (GpuFramework.preempt: nodesWherePreemptionMightHelp,
    kgpu_select_victims on the device, the table's extenders), then the table's second call with the
    victims marked deleted and the preemptor nominated to the node: nothing more may be preempted."""
    import copy
    import fake_plugins
    case = copy.deepcopy(case)
    fw = GpuFramework(_gpu_profile(case), case["nodes"], case["pods"], pods_hint=[case["pod"]])
    now = PR.pod_start_time({"status": {"startTime": case["now"]}}, 0)
    statuses = {nn: (code, None, []) for nn, code in case["statuses"].items()}
    ext = fake_plugins.extenders(case.get("extenders"))
    pod = case["pod"]
    node, victims, _ = fw.preempt(pod, statuses, case.get("pdbs", []), now, extenders=ext)
    want = case["expect_preempt"]
    assert node == want["node"], (case["name"], node)
    names = sorted(NI.name(v) for v in victims)
    assert names == want["victims"], (case["name"], names)
    for pods in fw.node_pods.values():
        for p, _ in pods:
            if NI.name(p) in names:
                p["metadata"]["deletionTimestamp"] = case["now"]
    pod.setdefault("status", {})["nominatedNodeName"] = node
    node2, victims2, _ = fw.preempt(pod, statuses, case.get("pdbs", []), now, extenders=ext)
    assert not (node2 and victims2), (case["name"], node2, victims2)
    fw.engine.close()
