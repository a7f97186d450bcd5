"""The persistent topology kernel (k_tbatch: device-resident domain histograms, two granule rounds
per pod) against the C restatement of the reference (oracle/c) on seeded random clusters large
enough for several workgroups, at every geometry (rows per lane 1 and 2), and against the per-pod
topology launches it replaces.  Pods the kernel does not carry (two ScheduleAnyway constraints, a
DoNotSchedule constraint on kubernetes.io/hostname) fall back inside the same batch, so the runs
also check the hand-over of histogram state between the two paths."""
import numpy as np
import pytest

import gen_random
from kgpu import abi
from kgpu.compile import Cluster, Profile
from kgpu.framework import GpuFramework


def _big(seed, n_nodes=1500, n_existing=600, n_pods=80):
    nodes, ex, pods, services, rss = gen_random.topo_cluster(seed, n_nodes=n_nodes, n_existing=n_existing,
                                                             n_pods=n_pods)
    return nodes, ex, pods, services, rss


def _run(args, tfast=1, groups=0, threads=4, geo=None, ahead=None, wlab=None, poll_sleep=None):
    from oracle.cref import RefEngine
    nodes, ex, pods, services, rss = args
    fw = GpuFramework(Profile(), nodes, ex, cluster=Cluster(services=services, rss=rss), pods_hint=pods)
    q, pc, pnp, errs = fw.compile_pods(pods)
    assert not errs
    want = RefEngine(fw.config, fw.snap, threads=threads)
    w = want.schedule(q, pc)
    fw.engine.set_option(abi.OPT_TOPO_PERSISTENT, tfast)
    if groups:
        fw.engine.set_option(abi.OPT_PERSIST_GROUPS, groups)
    if geo is not None:
        fw.engine.set_option(abi.OPT_TBATCH_GEO, geo)
    if ahead is not None:
        fw.engine.set_option(abi.OPT_TOPO_AHEAD, ahead)
    if wlab is not None:
        fw.engine.set_option(abi.OPT_TBATCH_WLAB, wlab)
    if poll_sleep is not None:
        fw.engine.set_option(abi.OPT_TBATCH_POLL_SLEEP, poll_sleep)
    got, _ = fw.engine.schedule_batch(q, pc)
    return fw, w, got, want.read_nodes(), fw.engine.read_nodes(fw.snap.n_nodes)


def _check(w, got, rows_w, rows_g):
    for f in ("node", "feasible", "scored", "score"):
        bad = np.nonzero(w[f] != got[f])[0]
        assert len(bad) == 0, "%s differs at pods %s: want %s got %s" % (f, bad[:5], w[f][bad[:5]], got[f][bad[:5]])
    for k in rows_w:
        np.testing.assert_array_equal(rows_w[k], rows_g[k], err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("groups", [0, 2])
@pytest.mark.parametrize("seed", range(8))
def test_gpu_tbatch_random_matches_c_restatement(seed, groups):
    fw, w, got, rw, rg = _run(_big(seed), tfast=1, groups=groups)
    _check(w, got, rw, rg)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(16))
def test_gpu_tbatch_small_clusters(seed):
    """One workgroup, most lanes idle, every plugin input of gen_random.topo_cluster."""
    fw, w, got, rw, rg = _run(gen_random.topo_cluster(seed, n_nodes=40, n_existing=60, n_pods=60), tfast=1)
    _check(w, got, rw, rg)


@pytest.mark.gpu
@pytest.mark.parametrize("wlab", [0, 1])
@pytest.mark.parametrize("seed", [3])
def test_gpu_tbatch_winner_labels_switch(seed, wlab):
    """KGPU_OPT_TBATCH_WLAB 0 / 1: the winner's label values from global memory or from the run's LDS
    copy of every node's: both against the C restatement."""
    fw, w, got, rw, rg = _run(_big(seed, n_nodes=1200, n_existing=500, n_pods=70), tfast=1, wlab=wlab)
    _check(w, got, rw, rg)


@pytest.mark.gpu
@pytest.mark.parametrize("poll_sleep", [0, 1])
@pytest.mark.parametrize("groups", [0, 2])
@pytest.mark.parametrize("seed", [1, 6])
def test_gpu_tbatch_poll_sleep_switch(seed, groups, poll_sleep):
    """KGPU_OPT_TBATCH_POLL_SLEEP 0 / 1: statistics sweeps back to back or with a sleep between, against
    the C restatement."""
    fw, w, got, rw, rg = _run(_big(seed), tfast=1, groups=groups, poll_sleep=poll_sleep)
    _check(w, got, rw, rg)


@pytest.mark.gpu
@pytest.mark.parametrize("ahead", [0, 1])
@pytest.mark.parametrize("seed", [2, 5])
def test_gpu_tbatch_ahead_switch(seed, ahead):
    """KGPU_OPT_TOPO_AHEAD 0 (every pod evaluated after the previous assume) and 1 (the next pod's
    non-topology half evaluated while the statistics travel): both against the C restatement."""
    fw, w, got, rw, rg = _run(_big(seed, n_nodes=900, n_existing=400, n_pods=60), tfast=1, ahead=ahead)
    _check(w, got, rw, rg)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c", "d"])
@pytest.mark.parametrize("groups", [0, 3])
def test_gpu_tbatch_bench_configs_3000(cfg, groups):
    from kgpu import cluster
    if cfg == "c":
        nodes, ex, pods, _ = cluster.taints_affinity_spread(n_nodes=3000, n_pods=400)
    else:
        nodes, ex, pods, _ = cluster.pod_affinity(n_nodes=3000, n_existing=3000, n_pods=320)
    fw, w, got, rw, rg = _run((nodes, ex, pods, [], []), tfast=1, groups=groups, threads=8)
    _check(w, got, rw, rg)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 4])
def test_gpu_tbatch_geometry_256(seed):
    """KGPU_OPT_TBATCH_GEO 0: 256 threads x 1 row per lane (four waves, one per SIMD; six
    workgroups at 1,500 nodes)."""
    fw, w, got, rw, rg = _run(_big(seed), tfast=1, geo=0)
    _check(w, got, rw, rg)


def test_rank40_inverse_constants():
    """k_tbatch recovers the winning node from its packed key: rank40 (tiebreak.py) is a bijection
    on 40 bits and rank40_inv undoes it (the same constants as kgpu_kernels.hip)."""
    import random
    M = (1 << 40) - 1
    C1, C2 = 0xD6E8FEB865, 0x94D049BB13
    I1, I2 = 0xB38E39396D, 0x38E12D471B
    assert (C1 * I1) & M == 1 and (C2 * I2) & M == 1
    from oracle.refsched import tiebreak
    r = random.Random(7)
    for _ in range(2000):
        k, idx = r.getrandbits(64), r.getrandbits(20)
        x = tiebreak.rank40(k, idx) if hasattr(tiebreak, "rank40") else None
        if x is None:
            pytest.skip("tiebreak.rank40 not exposed")
        x ^= (k >> 24) & M
        x ^= x >> 23
        x = (x * I2) & M
        x ^= (x >> 19) ^ (x >> 38)
        x = (x * I1) & M
        x ^= k & M
        assert x == idx


@pytest.mark.gpu
@pytest.mark.parametrize("ahead", [0, 1])
def test_gpu_tbatch_repeated_affinity_terms(ahead):
    """A pod with two identical required podAffinity terms (seed 20359's pod 18) is assumed inside the run; a
    later pod (24) that the terms match scores them once per term (processExistingPod).  The run's histogram
    delta used to be applied once per column, so pod 24's InterPodAffinity score came out 1 high
    (tools/stress_parity.py found it; 1000701 against oracle/c's 1000700)."""
    fw, w, got, rw, rg = _run(gen_random.topo_cluster(20359, n_nodes=16, n_existing=24, n_pods=30), tfast=1,
                              ahead=ahead)
    _check(w, got, rw, rg)
