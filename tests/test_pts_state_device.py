"""Topology-plugin PreFilter / PreScore STATE on the device against the reference's own state tables.

PodTopologySpread (tests/golden/podtopologyspread.json, kind pts_state): filtering_test.go:543
TestPreFilterState, :857/:1146 TestPreFilterStateAddPod / RemovePod and scoring_test.go:38
TestPreScoreStateEmptyNodes.  kgpu_debug_pts_state exports what the device builds for one pod: per value
of a constraint's key, whether the pair is registered and its count (TpPairToMatchNum /
TopologyPairToPodCounts), and criticalPaths[0].MatchNum (PreFilter) or the topology size behind
topologyNormalizingWeight (PreScore).

InterPodAffinity (tests/golden/interpodaffinity.json, kind ipa_state): filtering_test.go:1697
TestPreFilterStateAddRemovePod and :2045 TestGetTPMapMatchingIncomingAffinityAntiAffinity through
kgpu_debug_ipa_state (the three preFilterState maps).

The AddPod / RemovePod rows run as what the device actually does when a pod lands on or leaves a
node: a kgpu_apply_delta ADD_POD / REMOVE_POD through the host cache mirror (kgpu/cache.py, no
re-upload), then the state export of the next cycle.  For the inter-pod affinity rows the state after
the add must also equal the state of an engine uploaded with the pod already in place, and the
remove must restore the original state, as the reference test's two DeepEqual checks require
(filtering_test.go:1990-2030).  TestPreFilterStateRemovePod's "delete a non-existing pod" row has
no pod to remove from a cache: its state is the unchanged one, which is what the table expects."""
import copy

import numpy as np
import pytest

from conftest import load_golden
from kgpu.cache import SchedulerCache
from kgpu.compile import Cluster, Pools, Profile
from kgpu.framework import GpuFramework
from oracle.refsched.golog import go_log

PTS = [c for c in load_golden("podtopologyspread") if c["kind"] == "pts_state" and "expect_state" in c]
IPA = [c for c in load_golden("interpodaffinity") if c["kind"] == "ipa_state"]


def _uid(pod):
    """The cache keys pods by UID (framework.GetPodKey); the tables' pods have none: ns/name."""
    p = copy.deepcopy(pod)
    m = p.setdefault("metadata", {})
    m.setdefault("uid", "%s/%s" % (m.get("namespace", "") or "", m.get("name", "")))
    return p


def _cluster(case):
    return Cluster(case.get("services", []), case.get("rcs", []), case.get("rss", []), case.get("sss", []))


def _query(comp, pod):
    pools = Pools()
    q = comp.compile_pod(pod, pools)
    pc, _ = pools.finalize()
    return np.array([q]), pc


def _pts_check(case, engine, comp, q, pc, kind):
    want = case["expect_state"]
    nk = comp.nkeys
    pairs = {}
    for k, v, n in want["pairs"]:
        pairs.setdefault(k, {})[v] = n
    checked = 0
    for i, (max_skew, key, _sel) in enumerate(want["constraints"]):
        ki = nk.key(key)
        if ki < 0:  # no node carries the key: no pair can be registered
            assert not pairs.get(key), (case["name"], key)
            checked += 1
            continue
        D = len(nk.vals[ki].items)
        reg, cnt, scalar = engine.pts_state(q[0], pc, kind, i, D)
        got = {nk.vals[ki].items[v]: int(cnt[v]) for v in range(D) if reg[v]}
        if kind == 1 and key == "kubernetes.io/hostname":
            # scoring.go:83-86,196-198: hostname pairs are never registered; counts are per node at Score
            assert got == {}, (case["name"], got)
        else:
            assert got == pairs.get(key, {}), (case["name"], key, got)
        if kind == 0:
            assert scalar == want["paths"][key][0][1], (case["name"], key, scalar)
        elif scalar >= 0 and want.get("weights"):
            assert go_log(float(scalar + 2)) == want["weights"][i], (case["name"], key, scalar)
        checked += 1
    assert checked or not want["constraints"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", PTS, ids=["%s:%s" % (c["op"], c["name"][:50]) for c in PTS])
def test_pts_state_on_device(case):
    a = case.get("args") or {}
    # PreFilter: the filter alone; PreScore over every node (the tables pass the whole list as filtered)
    prescore = case["op"] == "prescore"
    prof = Profile(filters=[] if prescore else ["PodTopologySpread"],
                   scores=[("PodTopologySpread", 1)] if prescore else [],
                   pts_default_constraints=a.get("default_constraints", []))
    if case["op"] in ("add", "remove"):
        hint = [case["pod"], case["op_pod"]]
        cache = SchedulerCache(prof, case["nodes"], [_uid(p) for p in case.get("pods", [])], cluster=_cluster(case),
                               pods_hint=hint)
        try:
            if case["op"] == "add":
                cache.add_pod(_uid(case["op_pod"]))
            elif any(p["metadata"]["name"] == case["op_pod"]["metadata"]["name"] and
                     p["metadata"].get("namespace", "") == case["op_pod"]["metadata"].get("namespace", "")
                     for p in case.get("pods", [])):
                cache.remove_pod(_uid(case["op_pod"]))
            cache.sync()
            assert cache.uploads == 1  # the change went through kgpu_apply_delta
            q, pc = _query(cache.compiler, case["pod"])
            _pts_check(case, cache.engine, cache.compiler, q, pc, 0)
        finally:
            cache.close()
        return
    fw = GpuFramework(prof, case["nodes"], case.get("pods", []), cluster=_cluster(case), pods_hint=[case["pod"]])
    q, pc, _, errs = fw.compile_pods([case["pod"]])
    assert not errs
    _pts_check(case, fw.engine, fw.compiler, q, pc, 1 if prescore else 0)
    fw.engine.close()


IPA_KINDS = ("existing_anti", "aff", "anti")


def _ipa_maps(engine, comp, pod):
    q, pc = _query(comp, pod)
    nk = comp.nkeys
    D = max([len(d.items) for d in nk.vals] + [1])
    out = {k: {} for k in IPA_KINDS}
    for kind, key, counts in engine.ipa_state(q[0], pc, D):
        for v in np.nonzero(counts)[0]:
            pair = (nk.keys.items[key], nk.vals[key].items[int(v)])
            out[IPA_KINDS[kind]][pair] = out[IPA_KINDS[kind]].get(pair, 0) + int(counts[v])
    return {k: sorted([a, b, n] for (a, b), n in m.items()) for k, m in out.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("case", IPA, ids=["%s:%s" % (c["src"].rsplit(":", 1)[1], c["name"][:60]) for c in IPA])
def test_ipa_state_on_device(case):
    prof = Profile(filters=["InterPodAffinity"], scores=[])
    hint = [case["pod"]] + ([case["op_pod"]] if case["op"] == "add_remove" else [])
    cache = SchedulerCache(prof, case["nodes"], [_uid(p) for p in case.get("pods", [])], cluster=_cluster(case),
                           pods_hint=hint)
    try:
        before = _ipa_maps(cache.engine, cache.compiler, case["pod"])
        want = case["expect_ipa"]
        if case["op"] != "add_remove":
            assert before["aff"] == want["aff"] and before["anti"] == want["anti"], (case["name"], before)
            return
        cache.add_pod(_uid(case["op_pod"]))
        cache.sync()
        assert cache.uploads == 1  # the change went through kgpu_apply_delta
        after = _ipa_maps(cache.engine, cache.compiler, case["pod"])
        assert after["aff"] == want["aff"] and after["anti"] == want["anti"], (case["name"], after)
        # DeepEqual(allPodsState, state): an engine uploaded with the pod already in place
        fw = GpuFramework(prof, case["nodes"], list(case.get("pods", [])) + [case["op_pod"]], cluster=_cluster(case),
                          pods_hint=hint)
        assert _ipa_maps(fw.engine, fw.compiler, case["pod"]) == after, case["name"]
        fw.engine.close()
        cache.remove_pod(_uid(case["op_pod"]))
        cache.sync()
        assert _ipa_maps(cache.engine, cache.compiler, case["pod"]) == before, case["name"]
    finally:
        cache.close()
