"""Parity at the BASELINE.json sizes: every pod of configs (a)-(d) through libkgpu.so against the C
restatement of the reference (oracle/c), with the workloads bench.py measures.  Compared per pod:
chosen node, FeasibleNodes, the scored flag and the winner's total score; after the batch every
node's Requested / NonZeroRequested / pod count."""
import numpy as np
import pytest

from kgpu.framework import GpuFramework


def _workload(cfg):
    from kgpu import cluster
    if cfg == "a":
        nodes, init, pods, prof = cluster.scheduling_basic(n_nodes=500, n_init=500, n_pods=1000)
        return nodes, [], init + pods, prof
    if cfg == "b":
        return cluster.fit_least_balanced(n_nodes=5000, n_pods=10000)
    if cfg == "c":
        return cluster.taints_affinity_spread(n_nodes=5000, n_pods=10000)
    return cluster.pod_affinity(n_nodes=5000, n_existing=5000, n_pods=10000)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["a", "b", "c", "d"])
def test_gpu_full_size_config_matches_c_restatement(cfg):
    from oracle.cref import RefEngine
    nodes, ex, pods, prof = _workload(cfg)
    fw = GpuFramework(prof, nodes, ex, pods_hint=pods[:16])
    q, pc, pnp, errs = fw.compile_pods(pods)
    assert not errs
    ref = RefEngine(fw.config, fw.snap, threads=16)
    want = ref.schedule(q, pc)
    got = np.concatenate([fw.engine.schedule_batch(q[k:k + 1000], pc, first_seq=k)[0] for k in range(0, len(q), 1000)])
    for f in ("node", "feasible", "scored", "score"):
        bad = np.nonzero(want[f] != got[f])[0]
        assert len(bad) == 0, "config %s: %s differs at pods %s" % (cfg, f, bad[:5])
    rows_w, rows_g = ref.read_nodes(), fw.engine.read_nodes(fw.snap.n_nodes)
    for k in rows_w:
        np.testing.assert_array_equal(rows_w[k], rows_g[k], err_msg=k)
    assert (got["node"] >= 0).sum() > 0


@pytest.mark.gpu
def test_gpu_config_d_48k_nodes_matches_c_restatement():
    """Config (d) at 48,000 nodes and 48,000 existing pods: the InterPodAffinity k_tbatch with more
    than 64 workgroups (the four-granules-per-lane statistics sweep), 300 pods against oracle/c."""
    from kgpu import cluster
    from oracle.cref import RefEngine
    nodes, ex, pods, prof = cluster.pod_affinity(n_nodes=48000, n_existing=48000, n_pods=300)
    fw = GpuFramework(prof, nodes, ex, pods_hint=pods[:16])
    q, pc, pnp, errs = fw.compile_pods(pods)
    assert not errs
    ref = RefEngine(fw.config, fw.snap, threads=16)
    want = ref.schedule(q, pc)
    got = np.concatenate([fw.engine.schedule_batch(q[k:k + 150], pc, first_seq=k)[0] for k in (0, 150)])
    for f in ("node", "feasible", "scored", "score"):
        bad = np.nonzero(want[f] != got[f])[0]
        assert len(bad) == 0, "config d 48k: %s differs at pods %s" % (f, bad[:5])
    rows_w, rows_g = ref.read_nodes(), fw.engine.read_nodes(fw.snap.n_nodes)
    for k in rows_w:
        np.testing.assert_array_equal(rows_w[k], rows_g[k], err_msg=k)
    assert (got["node"] >= 0).sum() > 0
    fw.engine.close()
