"""runAllFilters (framework/v1alpha1/framework.go:90,155-160,484-499; set from the legacy Policy's
AlwaysCheckAllPredicates, factory.go:107,278-281) -- KGPU_OPT_RUN_ALL_FILTERS.

With it, RunFilterPlugins runs every filter plugin on a node instead of stopping at the first failure,
and PluginToStatus.Merge (interface.go:162-191) folds their statuses: every failing plugin's reasons,
UnschedulableAndUnresolvable over Unschedulable.  Placements never change (a node is feasible iff every
plugin passes either way); the per-node statuses do -- the FitError message, the pod events, and which
nodes nodesWherePreemptionMightHelp (generic_scheduler.go:1014-1028) keeps.

CPU: the Python oracle's runner under the flag (placements unchanged, merged statuses).  GPU: every
cycle's merged status word and per-plugin words (kgpu_get_filter / kgpu_get_filter_all, formatted by
kgpu_filter_reasons) against the oracle, on random clusters with and without topology plugins and with
nominated pods (k_victims' pass 1 becomes a node's verdict), and preemption's candidate nodes."""
import random

import pytest

import gen_random
from kgpu import abi
from kgpu.compile import Cluster, Profile
from kgpu.framework import GpuFramework
from oracle.refsched import framework as F
from oracle.refsched import nodeinfo as NI
from oracle.refsched import plugins as P
from oracle.refsched import preemption as PR

NOW = 1_600_000_000


def _scenario(seed, topo, nominated):
    """A small tight cluster whose pods fail several plugins per node."""
    r = random.Random(9100 + seed)
    if topo:
        nodes, existing, pods, services, rss = gen_random.topo_cluster(seed, n_nodes=16, n_existing=40, n_pods=14)
    else:
        nodes, existing, pods = gen_random.cluster(seed, n_nodes=16, n_existing=30, n_pods=14)
        services, rss = [], []
    for n in nodes:
        n["status"]["allocatable"].update({"cpu": r.choice(["2", "4"]), "memory": r.choice(["4Gi", "8Gi"]),
                                           "pods": str(r.choice([3, 5, 110]))})
        if r.random() < 0.25:
            n.setdefault("spec", {})["unschedulable"] = True
    for p in existing + pods:
        p["spec"]["priority"] = r.choice([0, 100, 1000])
        p["status"] = {"startTime": "2019-01-0%dT01:01:01Z" % r.randrange(1, 8)}
    for p in pods:
        p["spec"].pop("nodeName", None)
        p["spec"]["priority"] = r.choice([500, 2000])
    noms = []
    if nominated:
        names = [n["metadata"]["name"] for n in nodes]
        for j in range(3):
            p = gen_random.rpod(r, 7000 + j, names, allow_node_name=False)
            if topo:
                gen_random._topo_spec(r, p["spec"], p["metadata"], p_tsc=0.0, p_aff=0.4)
            p["spec"]["priority"] = r.choice([1000, 3000])
            noms.append((p, r.choice(names)))
    return nodes, existing, pods, services, rss, noms


def _oracle(nodes, existing, services, rss, noms, run_all):
    snap = NI.Snapshot(nodes, existing)
    fw = F.Framework(F.Profile(run_all_filters=run_all), F.Handle(snap, services, (), rss))
    nominator = None
    if noms:
        nominator = PR.Nominator()
        for p, nn in noms:
            nominator.add(p, nn)
    return snap, fw, F.GenericScheduler(fw, nominator), nominator


def _oracle_cycle(gs, pod, seq):
    try:
        r = gs.schedule(pod, seq)
        return r.host, r.statuses
    except F.FitError as e:
        return None, e.statuses


# ---------------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("seed", range(4))
def test_oracle_run_all_keeps_placements_and_merges(seed):
    """The restated runner under runAllFilters: the same hosts as without it; every node's merged status
    names the first failing plugin, has at least its reasons, and is UnschedulableAndUnresolvable
    whenever some failing plugin is."""
    nodes, existing, pods, services, rss, noms = _scenario(seed, topo=seed % 2 == 1, nominated=False)
    _, fw1, gs1, _ = _oracle(nodes, existing, services, rss, noms, False)
    snap, fwa, gsa, _ = _oracle(nodes, existing, services, rss, noms, True)
    multi = 0
    for i, pod in enumerate(pods):
        state = {}
        fwa.run_prefilter(state, pod)
        per_node = {NI.name(ni.node): fwa.run_filter_plugins(state, pod, ni, run_all_filters=True) for ni in snap.list}
        h1, s1 = _oracle_cycle(gs1, pod, i)
        ha, sa = _oracle_cycle(gsa, pod, i)
        assert h1 == ha, (seed, i)
        assert set(s1) == set(sa)
        for nn, (plugin, st) in sa.items():
            first_plugin, first = s1[nn]
            assert plugin == first_plugin
            assert st.reasons[:len(first.reasons)] == first.reasons
            m = per_node.get(nn)
            if m:
                multi += len(m) > 1
                want = P.UNRESOLVABLE if any(s.code == P.UNRESOLVABLE for s in m.values()) else P.UNSCHEDULABLE
                assert st.code == want
                assert st.reasons == [r for s in m.values() for r in s.reasons]
    assert multi > 0, "no node failed more than one plugin: the scenario does not exercise the merge"


def test_profile_flag_reaches_engine_option():
    assert Profile(run_all_filters=True).run_all_filters and not Profile().run_all_filters
    assert abi.OPT_RUN_ALL_FILTERS == 20


# ---------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("nominated", [False, True], ids=["plain", "nominated"])
@pytest.mark.parametrize("topo", [False, True], ids=["resources", "topology"])
@pytest.mark.parametrize("seed", range(3))
def test_gpu_run_all_statuses_match_oracle(seed, topo, nominated):
    nodes, existing, pods, services, rss, noms = _scenario(seed, topo, nominated)
    fw = GpuFramework(Profile(run_all_filters=True), nodes, existing, cluster=Cluster(services=services, rss=rss),
                      pods_hint=pods + [p for p, _ in noms])
    if noms:
        fw.set_nominated(noms)
    snap, ofw, gs, _ = _oracle(nodes, existing, services, rss, noms, True)
    multi = 0
    for i, pod in enumerate(pods):
        per_node = None
        if not noms:  # RunFilterPlugins' PluginToStatus of every node (one pass)
            state = {}
            ofw.run_prefilter(state, pod)
            per_node = {NI.name(ni.node): ofw.run_filter_plugins(state, pod, ni, run_all_filters=True)
                        for ni in snap.list}
        want_host, want_st = _oracle_cycle(gs, pod, i)
        cr = fw.cycle(pod, assume=False, seq=i)
        assert cr.host == want_host, (seed, i)
        got = {nn: (code, plugin, list(rs)) for nn, (code, plugin, rs) in cr.statuses.items()}
        want = {nn: (st.code, plugin, list(st.reasons)) for nn, (plugin, st) in want_st.items()}
        assert got == want, (seed, i)
        if per_node is not None:
            for nn, per in cr.plugin_statuses.items():
                multi += len(per) > 1
                exp = {pl: (s.code, list(s.reasons)) for pl, s in per_node[nn].items()}
                assert {pl: (c, list(rs)) for pl, (c, rs) in per.items()} == exp, (seed, i, nn)
    if not noms:
        assert multi > 0, "no node failed more than one plugin"
    fw.engine.close()


@pytest.mark.gpu
@pytest.mark.parametrize("topo", [False, True], ids=["resources", "topology"])
@pytest.mark.parametrize("seed", range(3))
def test_gpu_run_all_preemption_candidates(seed, topo):
    """selectNodesForPreemption under the flag: nodesWherePreemptionMightHelp reads the merged code (a
    node whose first failure is Unschedulable but where another plugin is UnschedulableAndUnresolvable
    is skipped); the device's candidates, victims and PDB counts equal the oracle's."""
    nodes, existing, pods, services, rss, noms = _scenario(seed, topo, nominated=False)
    fw = GpuFramework(Profile(run_all_filters=True), nodes, existing, cluster=Cluster(services=services, rss=rss),
                      pods_hint=pods)
    checked = 0
    for pod in pods:
        snap = NI.Snapshot(nodes, existing)
        ofw = F.Framework(F.Profile(run_all_filters=True), F.Handle(snap, services, (), rss))
        state = {}
        if ofw.run_prefilter(state, pod) is not None:
            continue
        potential = []
        for ni in snap.list:
            _, _, status = PR.pod_passes_filters_on_node(ofw, PR.Nominator(), state, pod, ni)
            if P.code_of(status) != P.UNRESOLVABLE:
                potential.append(ni)
        n2v = PR.select_nodes_for_preemption(ofw, PR.Nominator(), state, pod, potential, [], NOW)
        want = {n: ([NI.name(p) for p in v], nv) for n, (v, nv) in n2v.items()}
        got_n2v, _ = fw.select_nodes_for_preemption(pod, [], NOW)
        got = {n: ([NI.name(p) for p in v], nv) for n, (v, nv) in got_n2v.items()}
        assert got == want, (seed, NI.name(pod))
        checked += 1
    assert checked
    fw.engine.close()
