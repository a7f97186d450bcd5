"""Pipelined batches (kgpu_schedule_batch_submit / kgpu_schedule_batch_wait): consecutive batches of the
scheduleOne loop with batch k+1 staged and launched while batch k runs.  Placements, FeasibleNodes,
scores and the final node rows must equal the synchronous kgpu_schedule_batch path and the C restatement
(oracle/c); a batch the pipeline does not carry (a normalize pod, a short batch) runs synchronously inside
submit in queue order; other calls are refused while batches are in flight."""
import numpy as np
import pytest

from kgpu import abi, cluster
from kgpu.compile import Profile
from kgpu.framework import GpuFramework
from kgpu.native import KgpuError


def _same(a, b, what):
    for f in ("node", "feasible", "scored", "score"):
        np.testing.assert_array_equal(a[f], b[f], err_msg="%s: %s" % (what, f))


def _pipelined(e, q, pc, cuts):
    out = []
    stats = abi.Stats()
    for a, b in zip(cuts[:-1], cuts[1:]):
        e.schedule_batch_submit(q[a:b], pc, first_seq=a, stats=stats)
        if e.pipelined() > 1:
            out.append(e.schedule_batch_wait()[0])
    while e.pipelined():
        out.append(e.schedule_batch_wait()[0])
    return np.concatenate(out), stats


@pytest.mark.gpu
@pytest.mark.parametrize("nodes", [5000, 40000])
def test_pipelined_batches_match_sync_and_oracle(nodes):
    from oracle.cref import RefEngine
    n_pods = 2400
    ns, ex, pods, prof = cluster.fit_least_balanced(n_nodes=nodes, n_pods=n_pods)
    fw = GpuFramework(prof, ns, ex, pods_hint=pods[:16])
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    cuts = [0, 700, 1400, 1401, 1500, 2400]  # a one-pod batch (short: synchronous) inside the stream
    got, stats = _pipelined(fw.engine, q, pc, cuts)
    assert stats.pods == n_pods and stats.scheduled == int((got["node"] >= 0).sum())
    rows_p = fw.engine.read_nodes(fw.snap.n_nodes)
    ref = RefEngine(fw.config, fw.snap, threads=16)
    _same(ref.schedule(q, pc), got, "pipelined vs oracle/c")
    rows_w = ref.read_nodes()
    for k in rows_w:
        np.testing.assert_array_equal(rows_w[k], rows_p[k], err_msg=k)
    # the synchronous path on a fresh upload: the same records
    fw.engine.upload(fw.snap, fw.arrays)
    sync = np.concatenate([fw.engine.schedule_batch(q[a:b], pc, first_seq=a)[0] for a, b in zip(cuts[:-1], cuts[1:])])
    _same(sync, got, "pipelined vs synchronous")
    fw.engine.close()


@pytest.mark.gpu
def test_pipeline_with_normalize_pods_and_guards():
    """Default profile: pods with preferred NodeAffinity terms need the normalize pass, so their batches
    run synchronously inside submit; placements stay those of the C restatement in queue order.  While
    a batch is in flight any other call is refused."""
    from oracle.cref import RefEngine
    nodes, _, pods, _ = cluster.fit_least_balanced(n_nodes=3000, n_pods=1200, zones=4)
    pref = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 5, "preference": {"matchExpressions": [
            {"key": cluster.ZONE, "operator": "In", "values": ["zone1"]}]}}]}}
    for i in (450, 900):
        pods[i] = cluster.pod("pref%d" % i, "200m", "256Mi", affinity=pref)
    prof = Profile(filters=["NodeResourcesFit", "NodeAffinity"],
                   scores=[("NodeResourcesBalancedAllocation", 1), ("NodeResourcesLeastAllocated", 1), ("NodeAffinity", 1)])
    fw = GpuFramework(prof, nodes, [], pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    e = fw.engine
    e.schedule_batch_submit(q[:300], pc, first_seq=0)
    with pytest.raises(KgpuError) as ex:
        e.schedule_one(q[300], pc, seq=300)
    assert ex.value.code == abi.E_STATE
    first = e.schedule_batch_wait()[0]
    got, _ = _pipelined(e, q, pc, [300, 400, 800, 1000, 1200])
    got = np.concatenate([first, got])
    _same(RefEngine(fw.config, fw.snap, threads=16).schedule(q, pc), got, "pipelined vs oracle/c")
    fw.engine.close()
