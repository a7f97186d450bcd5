"""The persistent batch kernel (k_batch) against the one-launch-per-pod path and the C restatement.

Both device paths and the oracle must agree on every placement, feasible count and winning score,
and on the assumed node rows afterwards.  KGPU_OPT_PERSIST_GROUPS caps the grid so that small
clusters also run the 2-, 4- and 8-rows-per-lane variants and multi-workgroup exchanges."""
import numpy as np
import pytest

import gen_random
from kgpu import abi, cluster
from kgpu.compile import Profile
from kgpu.framework import GpuFramework

ROW_KEYS = ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods")


def _ref(fw, q, pc, threads=4):
    from oracle.cref import RefEngine
    ref = RefEngine(fw.config, fw.snap, threads=threads)
    return ref.schedule(q, pc), ref.read_nodes()


def _gpu(fw, q, pc, persistent=1, groups=0, chunks=1, geo=0):
    fw.engine.upload(fw.snap, fw.arrays)
    fw.engine.set_option(abi.OPT_PERSISTENT, persistent)
    fw.engine.set_option(abi.OPT_PERSIST_GROUPS, groups)
    fw.engine.set_option(abi.OPT_BATCH_GEO, geo)
    out = []
    step = (len(q) + chunks - 1) // chunks
    for s in range(0, len(q), step):
        res, _ = fw.engine.schedule_batch(q[s:s + step], pc, first_seq=s)
        out.append(res)
    return np.concatenate(out), fw.engine.read_nodes(fw.snap.n_nodes)


def _same(a, b, what):
    for f in ("node", "feasible", "scored", "score"):
        np.testing.assert_array_equal(a[f], b[f], err_msg="%s: %s" % (what, f))


def _rows(a, b, what):
    for k in ROW_KEYS:
        np.testing.assert_array_equal(a[k], b[k], err_msg="%s: %s" % (what, k))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 3, 7, 11])
def test_persistent_random_clusters(seed):
    nodes, existing, pods = gen_random.cluster(seed)
    fw = GpuFramework(Profile(), nodes, existing, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    want, want_rows = _ref(fw, q, pc)
    for persistent, groups in ((0, 0), (1, 0), (1, 1), (1, 2)):
        got, rows = _gpu(fw, q, pc, persistent, groups)
        _same(want, got, "persistent=%d groups=%d" % (persistent, groups))
        _rows(want_rows, rows, "persistent=%d groups=%d" % (persistent, groups))


@pytest.mark.gpu
@pytest.mark.parametrize("groups", [0, 5, 2])
def test_persistent_fit_least_balanced(groups):
    # config (b) shape at 3,000 nodes: no cap = 12 workgroups of 256 threads x 1 row; a cap of 5
    # forces 3 workgroups of 1024 x 1, a cap of 2 forces 2 workgroups of 512 threads x 4 rows
    nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=3000, n_pods=600)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16])
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    want, want_rows = _ref(fw, q, pc, threads=8)
    got, rows = _gpu(fw, q, pc, 1, groups, chunks=3)
    _same(want, got, "groups=%d" % groups)
    _rows(want_rows, rows, "groups=%d" % groups)


@pytest.mark.gpu
def test_persistent_mixed_with_normalize_pods():
    # taints + preferred node affinity: pods whose normalize maxima vary take the two-launch path,
    # the rest run persistently, interleaved in one batch
    nodes, existing, pods, prof = cluster.taints_affinity_spread(n_nodes=1500, n_pods=400, spread=False)
    for i, p in enumerate(pods):
        if i % 3:  # tolerating every PreferNoSchedule taint makes the TaintToleration maximum constant
            p["spec"].setdefault("tolerations", []).append({"key": "spot", "operator": "Exists"})
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16])
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    want, want_rows = _ref(fw, q, pc, threads=8)
    for persistent in (1, 0):
        got, rows = _gpu(fw, q, pc, persistent, 0)
        _same(want, got, "persistent=%d" % persistent)
        _rows(want_rows, rows, "persistent=%d" % persistent)


@pytest.mark.gpu
@pytest.mark.parametrize("geo", [0, 1, 2])
def test_persistent_geometries(geo):
    # KGPU_OPT_BATCH_GEO: 64, 128 and 192 row threads per workgroup (one, two and three row waves
    # beside the communication wave) on the config (b) shape and on random clusters
    nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=2500, n_pods=500)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16])
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    want, want_rows = _ref(fw, q, pc, threads=8)
    got, rows = _gpu(fw, q, pc, 1, 0, chunks=2, geo=geo)
    _same(want, got, "geo=%d" % geo)
    _rows(want_rows, rows, "geo=%d" % geo)
    nodes, existing, pods = gen_random.cluster(5)
    fw = GpuFramework(Profile(), nodes, existing, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    want, want_rows = _ref(fw, q, pc)
    got, rows = _gpu(fw, q, pc, 1, 0, geo=geo)
    _same(want, got, "random geo=%d" % geo)
    _rows(want_rows, rows, "random geo=%d" % geo)
