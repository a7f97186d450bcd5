"""Node sharding on the device: the sharded launch sequence -- per-pod shard pack,
RCCL all-gather of the shard winners (and of the DefaultNormalizeScore maxima), cluster-wide
resolve + assume by the owning rank -- against the C restatement on the unsharded snapshot.

The GPU box has one MI355X and RCCL refuses two ranks on one device, so the device tests run a
one-rank communicator: every pod still goes through k_shard_pack -> ncclAllGather -> prev_winner
over the gathered records, and every topology pod through the per-phase ncclAllReduce of its
histograms, registration slots, sizes and score extremes (multi-rank: unmeasured on hardware).  The multi-rank combine rule itself is covered on the CPU with gloo
(test_shard_cpu.py)."""
import numpy as np
import pytest

import gen_random
from kgpu import cluster, native
from kgpu.compile import Profile
from kgpu.framework import GpuFramework

NO_TOPO = Profile(filters=["NodeUnschedulable", "NodeResourcesFit", "NodeName", "NodePorts", "NodeAffinity",
                           "TaintToleration"],
                  scores=[("NodeResourcesBalancedAllocation", 1), ("ImageLocality", 1),
                          ("NodeResourcesLeastAllocated", 1), ("NodeAffinity", 1), ("NodePreferAvoidPods", 10000),
                          ("TaintToleration", 1)])


def _sharded(prof, nodes, existing, pods):
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods, shard=(0, 1))
    fw.init_comm(0, 1, native.comm_unique_id())
    return fw


def _check(prof, nodes, existing, pods, chunks=1):
    from oracle.cref import RefEngine
    fw = _sharded(prof, nodes, existing, pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    want = RefEngine(fw.config, fw.snap, threads=4).schedule(q, pc)
    step = (len(q) + chunks - 1) // chunks
    got = np.concatenate([fw.engine.schedule_batch(q[s:s + step], pc, first_seq=s)[0]
                          for s in range(0, len(q), step)])
    for f in ("node", "feasible", "scored", "score"):
        np.testing.assert_array_equal(want[f], got[f], err_msg=f)
    return fw, got


@pytest.mark.gpu
def test_sharded_fit_least_balanced():
    nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=700, n_pods=500)
    _, got = _check(prof, nodes, existing, pods, chunks=3)
    assert (got["node"] >= 0).all()


@pytest.mark.gpu
def test_sharded_normalize_pass():
    # PreferNoSchedule taints: TaintToleration's DefaultNormalizeScore maximum is exchanged per pod
    nodes, existing, pods, _ = cluster.taints_affinity_spread(n_nodes=400, n_pods=300, spread=False)
    _check(NO_TOPO, nodes, existing, pods)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 5, 9])
def test_sharded_random(seed):
    nodes, existing, pods = gen_random.cluster(seed)
    _check(NO_TOPO, nodes, existing, pods)


@pytest.mark.gpu
def test_sharded_cycle_diagnostics():
    nodes, existing, pods = gen_random.cluster(4)
    fw = _sharded(NO_TOPO, nodes, existing, pods)
    ref = GpuFramework(NO_TOPO, nodes, existing, pods_hint=pods)
    for p in pods[:6]:
        a, b = fw.cycle(p, assume=True), ref.cycle(p, assume=True)
        assert a.host == b.host
        assert a.statuses == b.statuses
        assert a.scores == b.scores


@pytest.mark.gpu
def test_sharded_topology_config_c():
    # PodTopologySpread (zone DoNotSchedule, hostname ScheduleAnyway) + taints + NodeAffinity: the
    # histograms, sizes and score extremes go through the per-phase RCCL all-reduces
    nodes, existing, pods, prof = cluster.taints_affinity_spread(n_nodes=500, n_pods=200)
    _check(prof, nodes, existing, pods, chunks=2)


@pytest.mark.gpu
def test_sharded_topology_config_d():
    nodes, existing, pods, prof = cluster.pod_affinity(n_nodes=300, n_existing=300, n_pods=150)
    _check(prof, nodes, existing, pods)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 3])
def test_sharded_topology_random(seed):
    nodes, existing, pods, services, rss = gen_random.topo_cluster(seed, n_nodes=60, n_existing=80, n_pods=40)
    from kgpu.compile import Cluster
    from oracle.cref import RefEngine
    prof = Profile()
    fw = GpuFramework(prof, nodes, existing, cluster=Cluster(services, rss=rss), pods_hint=pods, shard=(0, 1))
    fw.init_comm(0, 1, native.comm_unique_id())
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    want = RefEngine(fw.config, fw.snap, threads=4).schedule(q, pc)
    got, _ = fw.engine.schedule_batch(q, pc)
    for f in ("node", "feasible", "scored", "score"):
        np.testing.assert_array_equal(want[f], got[f], err_msg=f)


@pytest.mark.gpu
def test_sharded_reupload_keeps_communicator():
    # cache.UpdateSnapshot re-uploads the mirror; the communicator and exchange buffers survive it
    nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=300, n_pods=120)
    fw = _sharded(prof, nodes, existing, pods)
    q, pc, _, _ = fw.compile_pods(pods)
    a, _ = fw.engine.schedule_batch(q, pc)
    fw.engine.upload(fw.snap, fw.arrays)
    b, _ = fw.engine.schedule_batch(q, pc)
    np.testing.assert_array_equal(a["node"], b["node"])
