"""R2: percentageOfNodesToScore -> numFeasibleNodesToFind + nextStartNodeIndex
(pkg/scheduler/core/generic_scheduler.go:379-399,424-495).

Determinism contract: findNodesThatPassFilters as run by ONE worker of parallelize.Until -- nodes
are checked from nextStartNodeIndex in rotated Snapshot.List() order, the first numNodesToFind
feasible nodes are kept, the next one that fits cancels the search, EvaluatedNodes =
len(filtered) + len(statuses) and nextStartNodeIndex advances by it.  The Python oracle (objects),
the C restatement (compiled SoA) and libkgpu.so (GPU) are compared placement by placement, so every
pod also checks the rotation the previous pods left behind."""
import numpy as np
import pytest

import gen_random
from kgpu import abi
from kgpu.compile import Cluster, Profile
from kgpu.framework import GpuFramework
from oracle.refsched import framework as F

import conftest

GOLDEN = [c for c in conftest.load_golden("generic") if c["kind"] == "num_feasible"]


def oracle_run(nodes, existing, pods, services, rss, pct, profile=None):
    prof = profile or F.Profile(percentage_of_nodes_to_score=pct)
    res = F.schedule_sequence(nodes, existing, pods, prof, services=services, rss=rss)
    out = []
    for r in res:
        if isinstance(r, F.FitError):
            out.append((None, 0, None, None))
        elif isinstance(r, F.ScheduleError):
            out.append(("error", None, None, None))
        else:
            tot = dict((n, s) for n, s in r.totals)
            out.append((r.host, r.feasible, tot.get(r.host) if len(r.totals) > 0 else None, r.evaluated))
    return out


def product_run(nodes, existing, pods, services, rss, pct, backend, threads=2, profile=None):
    prof = profile or Profile(percentage_of_nodes_to_score=pct)
    fw = GpuFramework(prof, nodes, existing, cluster=Cluster(services=services, rss=rss), pods_hint=pods,
                      create_engine=(backend == "gpu"))
    q, pc, pnp, errs = fw.compile_pods(pods)
    assert not errs
    if backend == "gpu":
        res, _ = fw.engine.schedule_batch(q, pc)
    else:
        from oracle.cref import RefEngine
        res = RefEngine(fw.config, fw.snap, threads=threads).schedule(q, pc)
    out = []
    for r in res:
        if r["node"] == -1:
            out.append((None, 0, None, None))
        elif r["node"] < -1:
            out.append(("error", None, None, None))
        else:
            out.append((fw.order[r["node"]], int(r["feasible"]), int(r["score"]) if r["scored"] else None,
                        int(r["evaluated"])))
    return out, res


def _cmp(want, got):
    for i, (w, g) in enumerate(zip(want, got)):
        assert w[0] == g[0], "pod %d: oracle %r, product %r" % (i, w, g)
        if w[0] not in (None, "error"):
            assert w[1] == g[1], "pod %d feasible %r vs %r" % (i, w, g)
            assert w[3] == g[3], "pod %d evaluated %r vs %r" % (i, w, g)
            if w[1] > 1:
                assert w[2] == g[2], "pod %d score %r vs %r" % (i, w, g)


def _cluster(seed, n_nodes):
    """A resource-constrained cluster where many nodes fail Fit, so that the cut position, the
    statuses counted before it and the rotation all matter."""
    from kgpu import cluster
    nodes, ex, pods, _ = cluster.fit_least_balanced(n_nodes=n_nodes, n_pods=40, seed=seed, zones=4)
    for i, n in enumerate(nodes):
        if i % 3 == 0:
            n["status"]["allocatable"]["cpu"] = "1"
    return nodes, ex, pods, [], []


@pytest.mark.parametrize("case", GOLDEN, ids=[c["name"][:40] for c in GOLDEN])
def test_num_feasible_golden_through_c_restatement(case):
    """TestNumFeasibleNodesToFind (generic_scheduler_test.go:2470-2519): all nodes feasible, so the
    feasible count of one cycle is numFeasibleNodesToFind(N)."""
    from kgpu import cluster
    n = case["num_all_nodes"]
    nodes = [cluster.node("n%d" % i, "4", "8Gi") for i in range(n)]
    pods = [cluster.pod("p", "100m", "100Mi")]
    got, res = product_run(nodes, [], pods, [], [], case["pct"], backend="ref",
                           profile=Profile(filters=["NodeResourcesFit"], scores=[("NodeResourcesLeastAllocated", 1)],
                                           percentage_of_nodes_to_score=case["pct"]))
    assert int(res[0]["feasible"]) == case["expect_num"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", GOLDEN, ids=[c["name"][:40] for c in GOLDEN])
def test_num_feasible_golden_gpu(case):
    from kgpu import cluster
    n = case["num_all_nodes"]
    nodes = [cluster.node("n%d" % i, "4", "8Gi") for i in range(n)]
    pods = [cluster.pod("p", "100m", "100Mi")]
    _, res = product_run(nodes, [], pods, [], [], case["pct"], backend="gpu",
                         profile=Profile(filters=["NodeResourcesFit"], scores=[("NodeResourcesLeastAllocated", 1)],
                                         percentage_of_nodes_to_score=case["pct"]))
    assert int(res[0]["feasible"]) == case["expect_num"]
    assert int(res[0]["evaluated"]) == case["expect_num"] if case["expect_num"] < n else n


@pytest.mark.parametrize("pct", [0, 30, 60])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_c_restatement_matches_python_oracle_pct(seed, pct):
    args = _cluster(seed, 700)
    _cmp(oracle_run(*args, pct=pct), product_run(*args, pct=pct, backend="ref")[0])


def _topo_cluster(cfg):
    from kgpu import cluster
    if cfg == "c":
        nodes, ex, pods, _ = cluster.taints_affinity_spread(n_nodes=400, n_pods=30)
    else:
        nodes, ex, pods, _ = cluster.pod_affinity(n_nodes=400, n_existing=400, n_pods=32)
    return nodes, ex, pods, [], []


@pytest.mark.parametrize("pct", [0, 40])
@pytest.mark.parametrize("cfg", ["c", "d"])
def test_c_restatement_matches_python_oracle_pct_topology(cfg, pct):
    """PTS / IPA / DPTS PreScore over the trimmed feasible set (topoSize, ignored nodes, normalize)."""
    args = _topo_cluster(cfg)
    _cmp(oracle_run(*args, pct=pct), product_run(*args, pct=pct, backend="ref")[0])


@pytest.mark.gpu
@pytest.mark.parametrize("pct", [0, 40])
@pytest.mark.parametrize("cfg", ["c", "d"])
def test_gpu_matches_oracle_pct_topology(cfg, pct):
    args = _topo_cluster(cfg)
    _cmp(oracle_run(*args, pct=pct), product_run(*args, pct=pct, backend="gpu")[0])


@pytest.mark.gpu
@pytest.mark.parametrize("pct", [0, 30, 60])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_gpu_matches_oracle_pct(seed, pct):
    args = _cluster(seed, 700)
    _cmp(oracle_run(*args, pct=pct), product_run(*args, pct=pct, backend="gpu")[0])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["b", "c", "d"])
def test_gpu_pct0_5k_nodes_matches_c_restatement(cfg):
    """The reference default (percentageOfNodesToScore 0: adaptive, 10% at 5000 nodes) on the
    BASELINE configs' clusters at full node count: every pod's node / feasible / evaluated / score."""
    from kgpu import cluster
    from oracle.cref import RefEngine
    if cfg == "b":
        nodes, ex, pods, prof = cluster.fit_least_balanced(n_nodes=5000, n_pods=300)
    elif cfg == "c":
        nodes, ex, pods, prof = cluster.taints_affinity_spread(n_nodes=5000, n_pods=200)
    else:
        nodes, ex, pods, prof = cluster.pod_affinity(n_nodes=5000, n_existing=5000, n_pods=160)
    prof.percentage_of_nodes_to_score = 0
    fw = GpuFramework(prof, nodes, ex, pods_hint=pods)
    q, pc, pnp, errs = fw.compile_pods(pods)
    assert not errs
    want = RefEngine(fw.config, fw.snap, threads=8).schedule(q, pc)
    got, _ = fw.engine.schedule_batch(q, pc)
    for f in ("node", "feasible", "evaluated", "scored", "score"):
        np.testing.assert_array_equal(want[f], got[f], err_msg=f)
    assert (got["feasible"][got["node"] >= 0] <= 500).all()


@pytest.mark.gpu
def test_gpu_fair_evaluation_rotation():
    """TestFairEvaluationForNodes (generic_scheduler_test.go:2533-2566): 500 nodes, percentage 30,
    every node fits; over 2 * (500 / 150 + 1) cycles each cycle keeps 150 nodes and
    nextStartNodeIndex advances by 150 (mod 500).  The kept window is read back from the per-node
    status words of kgpu_schedule_one."""
    from kgpu import cluster
    nodes = [cluster.node("%d" % i, "4", "8Gi") for i in range(500)]
    prof = Profile(filters=["NodeUnschedulable"], scores=[], percentage_of_nodes_to_score=30)
    pods = [cluster.pod("p")]
    fw = GpuFramework(prof, nodes, [], pods_hint=pods)
    q, pc, pnp, _ = fw.compile_pods(pods)
    k = 150
    for i in range(2 * (500 // k + 1)):
        res, _ = fw.engine.schedule_one(q[0], pc, seq=i, assume=False)
        assert int(res["feasible"]) == k and int(res["evaluated"]) == k
        words = fw.engine.filter_words(500)
        kept = set(np.nonzero(words == 0)[0].tolist())
        start = i * k % 500
        assert kept == {(start + j) % 500 for j in range(k)}, i
        assert set(np.nonzero(words == abi.STATUS_NOT_EVALUATED)[0].tolist()) == set(range(500)) - kept
