"""PodTopologySpread PreFilter / PreScore STATE on the device against the reference's own state tables
(tests/golden/podtopologyspread.json, kind pts_state, transcribed from
podtopologyspread/filtering_test.go:543 TestPreFilterState and scoring_test.go:38 TestPreScoreStateEmptyNodes).

kgpu_debug_pts_state exports what the device builds for one pod: per value of a constraint's key,
whether the pair is registered and its count (TpPairToMatchNum / TopologyPairToPodCounts), and
criticalPaths[0].MatchNum (PreFilter) or the topology size behind topologyNormalizingWeight (PreScore).
The tables' AddPod / RemovePod cases (filtering_test.go:857,1146) update a PreFilter state in place;
the device applies those updates only inside the nominated / preemption passes (k_victims), whose
verdicts tests/test_preemption.py compares with the oracle's update_with_pod.  They run on the oracle
(tests/test_oracle_golden.py)."""
import pytest

from conftest import load_golden
from kgpu.compile import Cluster, Profile
from kgpu.framework import GpuFramework
from oracle.refsched.golog import go_log

CASES = [c for c in load_golden("podtopologyspread")
         if c["kind"] == "pts_state" and c["op"] in ("prefilter", "prescore") and "expect_state" in c]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=["%s:%s" % (c["op"], c["name"][:50]) for c in CASES])
def test_pts_state_on_device(case):
    a = case.get("args") or {}
    # PreFilter: the filter alone; PreScore over every node (the tables pass the whole list as filtered)
    prefilter = case["op"] == "prefilter"
    prof = Profile(filters=["PodTopologySpread"] if prefilter else [],
                   scores=[] if prefilter else [("PodTopologySpread", 1)],
                   pts_default_constraints=a.get("default_constraints", []))
    cluster = Cluster(case.get("services", []), case.get("rcs", []), case.get("rss", []), case.get("sss", []))
    fw = GpuFramework(prof, case["nodes"], case.get("pods", []), cluster=cluster, pods_hint=[case["pod"]])
    q, pc, _, errs = fw.compile_pods([case["pod"]])
    assert not errs
    want = case["expect_state"]
    kind = 0 if case["op"] == "prefilter" else 1
    nk = fw.compiler.nkeys
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
        reg, cnt, scalar = fw.engine.pts_state(q[0], pc, kind, i, D)
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
    fw.engine.close()
