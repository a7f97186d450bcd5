"""kgpu_prepare_pods: pod classes registered ahead of need (the drop-in
cycle's tail was the first cycle of each pod class, a host pass plus a k_class_init launch on the cycle).

* Placements: a kgpu_schedule_one loop (assume on) over config-(d)- and config-(c)-shaped clusters gives the
  same nodes as oracle/c whether the pods' classes were prepared first or met on their own cycles.
* After preparing every pod, the cycles launch no k_class_init (kgpu_debug_counters out[3]).
* The device pod table (k_class_init's input) is sent incrementally: classes met after many assumes and
  forgets count exactly (placements vs oracle/c) with at most the first upload of the whole table.
* prepare is a no-op outside a topology profile and rejects a call before any upload."""
import numpy as np
import pytest

from kgpu import cluster, native
from kgpu.framework import GpuFramework
from oracle.cref import RefEngine


def _workload(kind, n_nodes=600, n_pods=96):
    if kind == "d":
        return cluster.pod_affinity(n_nodes=n_nodes, n_existing=n_nodes, n_pods=n_pods)
    return cluster.taints_affinity_spread(n_nodes=n_nodes, n_pods=n_pods)


def _oracle(fw, q, pc):
    ref = RefEngine(fw.config, fw.snap)
    out = ref.schedule(q, pc)
    ref.close()
    return out["node"]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["d", "c"])
@pytest.mark.parametrize("prepare", [False, True])
def test_prepare_keeps_placements(kind, prepare):
    nodes, existing, pods, prof = _workload(kind)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16], device=0)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    want = _oracle(fw, q, pc)
    eng = fw.engine
    if prepare:
        eng.prepare_pods(q, pc)
    before = eng.counters()
    got = [int(eng.schedule_one(q[i], pc, seq=i, assume=True)[0]["node"]) for i in range(len(q))]
    after = eng.counters()
    assert np.array_equal(np.array(got), want), "placements differ from oracle/c"
    if prepare:
        assert after["class_inits"] == before["class_inits"], "a cycle met a class prepare_pods did not register"
    eng.close()


@pytest.mark.gpu
def test_pod_table_incremental_after_assumes_and_forgets():
    """Classes first met after assumes (rows appended) and forgets (rows changed in place) count the
    device pod table as it is: placements equal oracle/c on the cluster the same assumes leave."""
    nodes, existing, pods, prof = _workload("d", n_nodes=400, n_pods=128)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16], device=0)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    eng = fw.engine
    # the first 48 pods: assume, then forget every third (RemovePod on the device rows)
    slots = []
    for i in range(48):
        res, slot = eng.schedule_one(q[i], pc, seq=i, assume=True)
        slots.append((i, slot, int(res["node"])))
    for i, slot, node in slots[::3]:
        if node >= 0:
            eng.forget(slot)
    import copy
    placed = []
    for i, slot, node in slots:
        if i % 3 != 0 and node >= 0:
            p = copy.deepcopy(pods[i])
            p["spec"]["nodeName"] = fw.order[node]
            placed.append(p)
    # the oracle: a fresh snapshot of the cluster those assumes and forgets leave, the remaining pods in order
    fw2 = GpuFramework(prof, nodes, list(existing) + placed, pods_hint=pods[:16], create_engine=False)
    q2, pc2, _, errs2 = fw2.compile_pods(pods[48:])
    assert not errs2
    ref = RefEngine(fw2.config, fw2.snap)
    want = [fw2.order[int(x)] if int(x) >= 0 else None for x in ref.schedule(q2, pc2, first_seq=48)["node"]]
    ref.close()
    got = []
    for i in range(48, len(q)):
        n = int(eng.schedule_one(q[i], pc, seq=i, assume=True)[0]["node"])
        got.append(fw.order[n] if n >= 0 else None)
    assert got == want
    assert eng.counters()["pod_table_full_uploads"] <= 1
    eng.close()


@pytest.mark.gpu
def test_prepare_noop_outside_topology_profile():
    nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=64, n_pods=16)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods, device=0)
    q, pc, _, _ = fw.compile_pods(pods)
    fw.engine.prepare_pods(q, pc)
    assert fw.engine.counters()["class_inits"] == 0
    fw.engine.close()


def test_prepare_exported():
    """CPU: the entry point is exported and bound (kgpu.h declares it)."""
    assert "kgpu_prepare_pods" in native.EXPORTS
    assert hasattr(native.lib(), "kgpu_prepare_pods")
