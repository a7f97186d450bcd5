"""Seeded random clusters with PodTopologySpread / InterPodAffinity / DefaultPodTopologySpread
constraints on the default profile: the Python oracle (objects) == the product's compile step + the
C restatement (oracle/c) == libkgpu.so on the GPU.  Every placement of the scheduleOne loop is
compared (node, feasible count, winner's total), so each pod also sees the previous pods' assumes
in its PTS counts and IPA terms."""
import numpy as np
import pytest

import gen_random
from kgpu.compile import Cluster, Profile
from kgpu.framework import GpuFramework
from oracle.refsched import framework as F

SEEDS = list(range(16))


def oracle_run(nodes, existing, pods, services, rss):
    res = F.schedule_sequence(nodes, existing, pods, F.Profile(), services=services, rss=rss)
    out = []
    for r in res:
        if isinstance(r, F.FitError):
            out.append((None, 0, None))
        elif isinstance(r, F.ScheduleError):
            out.append(("error", None, None))
        else:
            tot = dict((n, s) for n, s in r.totals)
            out.append((r.host, r.feasible, tot.get(r.host) if len(r.totals) > 0 else None))
    return out


def product_run(nodes, existing, pods, services, rss, backend, threads=2):
    fw = GpuFramework(Profile(), nodes, existing, cluster=Cluster(services=services, rss=rss), pods_hint=pods,
                      create_engine=(backend == "gpu"))
    if backend == "gpu":
        res = fw.schedule(pods, first_seq=0)
        rows = fw.engine.read_nodes(fw.snap.n_nodes)
    else:
        from oracle.cref import RefEngine
        q, pc, pnp, errs = fw.compile_pods(pods)
        assert not errs
        ref = RefEngine(fw.config, fw.snap, threads=threads)
        res = ref.schedule(q, pc)
        rows = ref.read_nodes()
    out = []
    for r in res:
        if r["node"] == -1:
            out.append((None, 0, None))
        elif r["node"] < -1:
            out.append(("error", None, None))
        else:
            out.append((fw.order[r["node"]], int(r["feasible"]), int(r["score"]) if r["scored"] else None))
    return out, rows


def _cmp(want, got):
    for i, (w, g) in enumerate(zip(want, got)):
        assert w[0] == g[0], "pod %d: oracle %r, product %r" % (i, w, g)
        if w[0] not in (None, "error"):
            assert w[1] == g[1], "pod %d feasible %r vs %r" % (i, w, g)
            if w[1] > 1:
                assert w[2] == g[2], "pod %d score %r vs %r" % (i, w, g)


@pytest.mark.parametrize("seed", SEEDS)
def test_c_restatement_matches_python_oracle_topology(seed):
    args = gen_random.topo_cluster(seed)
    want = oracle_run(*args)
    got, _ = product_run(*args, backend="ref")
    _cmp(want, got)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_gpu_matches_oracle_topology(seed):
    args = gen_random.topo_cluster(seed)
    want = oracle_run(*args)
    got, rows = product_run(*args, backend="gpu")
    _cmp(want, got)
    _, rows_c = product_run(*args, backend="ref")
    for k in rows:
        np.testing.assert_array_equal(rows[k], rows_c[k], err_msg=k)


def _config_case(name):
    from kgpu import cluster
    if name == "c":
        nodes, ex, pods, _ = cluster.taints_affinity_spread(n_nodes=60, n_pods=80)
    else:
        nodes, ex, pods, _ = cluster.pod_affinity(n_nodes=60, n_existing=60, n_pods=48)
    return nodes, ex, pods, [], []


@pytest.mark.parametrize("cfg", ["c", "d"])
def test_c_restatement_matches_python_oracle_bench_configs(cfg):
    args = _config_case(cfg)
    _cmp(oracle_run(*args), product_run(*args, backend="ref")[0])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c", "d"])
def test_gpu_matches_oracle_bench_configs(cfg):
    args = _config_case(cfg)
    _cmp(oracle_run(*args), product_run(*args, backend="gpu")[0])


@pytest.mark.parametrize("hint", [0, 4])
def test_compile_order_independent(hint):
    """Selectors compiled before any pod carries their label keys / values still match pods
    compiled later (the snapshot is compiled with only `hint` incoming pods registered)."""
    from kgpu import cluster
    from oracle.cref import RefEngine
    nodes, ex, pods, _ = cluster.pod_affinity(n_nodes=40, n_existing=40, n_pods=48)
    want = oracle_run(nodes, ex, pods, [], [])
    fw = GpuFramework(Profile(), nodes, ex, pods_hint=pods[:hint], create_engine=False)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    res = RefEngine(fw.config, fw.snap).schedule(q, pc)
    got = [(None, 0, None) if r["node"] == -1 else (fw.order[r["node"]], int(r["feasible"]),
                                                    int(r["score"]) if r["scored"] else None) for r in res]
    _cmp(want, got)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c", "d"])
@pytest.mark.parametrize("fused", [1, 0])
def test_gpu_topology_multiblock_fused_and_unfused(cfg, fused):
    # 3000 nodes = 47 one-wave workgroups: the fused kernel's grid barriers order phases across
    # workgroups (and XCDs); the six-launch variant is the reference schedule of the same phases
    from kgpu import abi, cluster
    from oracle.cref import RefEngine
    if cfg == "c":
        nodes, ex, pods, prof = cluster.taints_affinity_spread(n_nodes=3000, n_pods=120)
    else:
        nodes, ex, pods, prof = cluster.pod_affinity(n_nodes=3000, n_existing=3000, n_pods=96)
    fw = GpuFramework(prof, nodes, ex, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    ref = RefEngine(fw.config, fw.snap, threads=4)
    want = ref.schedule(q, pc)
    fw.engine.set_option(abi.OPT_TOPO_FUSED, fused)
    got, _ = fw.engine.schedule_batch(q, pc)
    for f in ("node", "feasible", "scored", "score"):
        np.testing.assert_array_equal(want[f], got[f], err_msg=f)
    rows, rows_c = fw.engine.read_nodes(fw.snap.n_nodes), ref.read_nodes()
    for k in rows:
        np.testing.assert_array_equal(rows[k], rows_c[k], err_msg=k)
