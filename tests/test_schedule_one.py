"""kgpu_schedule_one -- the drop-in plugin's per-cycle call -- over a sequence of pods with assume.

A one-pod diagnostic cycle takes the short path: the query rides in the launch arguments, the
DevState is re-sent only when it changed, k_final's last workgroup resolves the pod and applies
the assume, and the record lands in pinned host memory.  The sequence must place, count and score
every pod as the C restatement does (genericScheduler.Schedule + assume per pod,
core/generic_scheduler.go:146-209, scheduler.go:555-567), and leave the same node rows.  A batch
call in the middle puts a different DevState image on the device, which the next cycle must
notice."""
import numpy as np
import pytest

import gen_random
from kgpu import abi, cluster
from kgpu.compile import Profile
from kgpu.framework import GpuFramework

ROW_KEYS = ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods")


def _ref(fw, q, pc):
    from oracle.cref import RefEngine
    ref = RefEngine(fw.config, fw.snap, threads=4)
    return ref.schedule(q, pc), ref.read_nodes()


def _case(name):
    if name == "fit":
        nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=700, n_pods=160)
        return nodes, existing, pods, prof
    nodes, existing, pods = gen_random.cluster(int(name[len("random"):]))
    return nodes, existing, pods, Profile()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["fit", "random0", "random7"])
def test_schedule_one_sequence_matches_oracle(name):
    nodes, existing, pods, prof = _case(name)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    want, want_rows = _ref(fw, q, pc)
    fw.engine.upload(fw.snap, fw.arrays)
    got = np.zeros(len(q), abi.RESULT)
    mid = len(q) // 2
    for i in range(len(q)):
        if i == mid:
            res, _ = fw.engine.schedule_batch(q[i:i + 1], pc, first_seq=i)
            got[i] = res[0]
            continue
        got[i], _ = fw.engine.schedule_one(q[i], pc, seq=i, assume=True)
    for f in ("node", "feasible", "scored", "score"):
        np.testing.assert_array_equal(want[f], got[f], err_msg="%s: %s" % (name, f))
    rows = fw.engine.read_nodes(fw.snap.n_nodes)
    for k in ROW_KEYS:
        np.testing.assert_array_equal(want_rows[k], rows[k], err_msg="%s: %s" % (name, k))


@pytest.mark.gpu
@pytest.mark.parametrize("zc", [0, 1])
@pytest.mark.parametrize("name", ["fit", "random0", "random7"])
def test_schedule_one_per_pod_pools(name, zc):
    """The Go shim's shape: every cycle's pod compiled on its own (its own pools block, different from the
    last cycle's).  KGPU_OPT_ZEROCOPY_POOLS 1: a one-launch cycle's k_eval reads them from pinned host
    memory, rewritten every cycle; 0: they ride in the cycle's copy.  Both against the C restatement of
    the same sequence (compiled as one batch), placements and node rows."""
    nodes, existing, pods, prof = _case(name)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    want, want_rows = _ref(fw, q, pc)
    fw.engine.upload(fw.snap, fw.arrays)
    fw.engine.set_option(abi.OPT_ZEROCOPY_POOLS, zc)
    got = np.zeros(len(q), abi.RESULT)
    for i, pod in enumerate(pods):
        qi, pci, _, errs = fw.compile_pods([pod])
        assert not errs
        got[i], _ = fw.engine.schedule_one(qi[0], pci, seq=i, assume=True)
    for f in ("node", "feasible", "scored", "score"):
        np.testing.assert_array_equal(want[f], got[f], err_msg="%s: %s" % (name, f))
    rows = fw.engine.read_nodes(fw.snap.n_nodes)
    for k in ROW_KEYS:
        np.testing.assert_array_equal(want_rows[k], rows[k], err_msg="%s: %s" % (name, k))


@pytest.mark.gpu
def test_schedule_one_without_assume_leaves_rows():
    nodes, existing, pods, prof = _case("fit")
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods[:20])
    assert not errs
    fw.engine.upload(fw.snap, fw.arrays)
    before = fw.engine.read_nodes(fw.snap.n_nodes)
    first, _ = fw.engine.schedule_one(q[0], pc, seq=0, assume=False)
    for i in range(1, 20):
        fw.engine.schedule_one(q[i], pc, seq=0, assume=False)
    again, _ = fw.engine.schedule_one(q[0], pc, seq=0, assume=False)
    after = fw.engine.read_nodes(fw.snap.n_nodes)
    for k in ROW_KEYS:
        np.testing.assert_array_equal(before[k], after[k], err_msg=k)
    assert first["node"] == again["node"] and first["score"] == again["score"]
