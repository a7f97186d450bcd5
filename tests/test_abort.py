"""Persistent-run abort (KGPU_OPT_ABORT_AT): a run that gives up mid-batch must fail the batch,
invalidate the device mirror (later cycles refused until the next upload), and leave an engine
that, after re-upload, schedules exactly as the C restatement does.

The hook raises the abort word from workgroup 0 at a chosen pod, which is what a workgroup that
lost co-residency does after kSpinTimeout (kgpu_kernels.hip, poll_row / tpoll_slot)."""
import time

import numpy as np
import pytest

from kgpu import abi, cluster
from kgpu.compile import Profile
from kgpu.framework import GpuFramework
from kgpu.native import KgpuError


def _ref(fw, q, pc):
    from oracle.cref import RefEngine
    ref = RefEngine(fw.config, fw.snap, threads=4)
    return ref.schedule(q, pc)


def _abort_then_recover(fw, q, pc, at, groups=0, must_abort=True):
    """(aborted, placements after recovery).  A hook index that falls on a pod scheduled by the
    per-pod launches (no persistent run holds it) does not abort: must_abort=False accepts that."""
    e = fw.engine
    e.upload(fw.snap, fw.arrays)
    e.set_option(abi.OPT_PERSIST_GROUPS, groups)
    e.set_option(abi.OPT_ABORT_AT, at)
    try:
        res, _ = e.schedule_batch(q, pc)
    except KgpuError as ex:
        assert ex.code == abi.E_DEVICE, ex
        assert "re-upload" in str(ex)
    else:
        e.set_option(abi.OPT_ABORT_AT, -1)
        assert not must_abort, "the abort hook at pod %d did not abort the batch" % at
        return False, res
    e.set_option(abi.OPT_ABORT_AT, -1)
    with pytest.raises(KgpuError):      # the mirror is invalid until the next upload
        e.schedule_batch(q[:1], pc)
    e.upload(fw.snap, fw.arrays)
    got, _ = e.schedule_batch(q, pc)
    return True, got


def _same(a, b):
    for f in ("node", "feasible", "scored", "score"):
        np.testing.assert_array_equal(a[f], b[f], err_msg=f)


@pytest.mark.gpu
@pytest.mark.parametrize("at,groups", [(0, 0), (37, 0), (37, 3), (199, 0)])
def test_abort_k_batch(at, groups):
    nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=700, n_pods=200)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    _same(_ref(fw, q, pc), _abort_then_recover(fw, q, pc, at, groups)[1])


@pytest.mark.gpu
@pytest.mark.parametrize("at", [0, 45])
def test_abort_k_tbatch(at):
    nodes, existing, pods, prof = cluster.taints_affinity_spread(n_nodes=600, n_pods=120)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    _same(_ref(fw, q, pc), _abort_then_recover(fw, q, pc, at)[1])


def _mixed_batch():
    """Config (b)-style pods under the default profile with two pods carrying preferred
    NodeAffinity terms: their normalize maxima are not constant, so they run as per-pod launches
    and split the batch into three persistent k_batch runs."""
    nodes, _, pods, _ = cluster.fit_least_balanced(n_nodes=700, n_pods=200, zones=4)
    pref = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 5, "preference": {"matchExpressions": [
            {"key": cluster.ZONE, "operator": "In", "values": ["zone1"]}]}}]}}
    for i in (60, 130):
        pods[i] = cluster.pod("pref%d" % i, "200m", "256Mi", affinity=pref)
    return nodes, pods


@pytest.mark.gpu
def test_abort_in_one_of_several_runs():
    """An abort in any of a batch's persistent runs must surface (one abort word per
    batch, OR-ed on the device), and an abort hook on a per-pod launch must leave the batch exact."""
    nodes, pods = _mixed_batch()
    fw = GpuFramework(Profile(), nodes, [], pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    want = _ref(fw, q, pc)
    for at, must in ((10, True), (60, False), (100, True), (130, False), (190, True)):
        ab, got = _abort_then_recover(fw, q, pc, at, must_abort=must)
        assert ab == must, at
        _same(want, got)


@pytest.mark.gpu
@pytest.mark.parametrize("point", [1, 2])
def test_allocation_failure_invalidates_and_recovers(point):
    """Fault injection (kgpu_debug_fail_alloc): a std::bad_alloc thrown inside kgpu_schedule_batch
    -- at the batch staging (1) or inside the topology plans (2) -- comes back through the C ABI as
    KGPU_E_NOMEM, the mirror is invalidated (KGPU_E_STATE until the next upload), and after the
    re-upload the engine schedules exactly as the C restatement."""
    from kgpu import native
    nodes, existing, pods, prof = cluster.taints_affinity_spread(n_nodes=300, n_pods=60)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    e = fw.engine
    native.debug_fail_alloc(point)
    try:
        with pytest.raises(KgpuError) as ex:
            e.schedule_batch(q, pc)
    finally:
        native.debug_fail_alloc(0)
    assert ex.value.code == abi.E_NOMEM, ex.value
    assert "invalidated" in str(ex.value)
    with pytest.raises(KgpuError) as ex2:
        e.schedule_batch(q[:1], pc)
    assert ex2.value.code == abi.E_STATE
    # an allocation failure inside the upload itself: reported, and the next upload recovers
    native.debug_fail_alloc(1)
    try:
        with pytest.raises(KgpuError) as ex3:
            e.upload(fw.snap, fw.arrays)
    finally:
        native.debug_fail_alloc(0)
    assert ex3.value.code == abi.E_NOMEM
    e.upload(fw.snap, fw.arrays)
    got, _ = e.schedule_batch(q, pc)
    _same(_ref(fw, q, pc), got)


@pytest.mark.gpu
@pytest.mark.parametrize("at", [5, 120])
def test_lds_handoff_timeout_recovers(at):
    """An LDS hand-off that never completes (KGPU_OPT_SKIP_RELEASE_AT: the candidate row is staged
    but its release skipped): the waiting wave times out after kSpinTimeout and raises the
    abort word, the batch fails with KGPU_E_DEVICE, the mirror is invalidated, and after the
    re-upload the engine schedules exactly as the C restatement."""
    nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=700, n_pods=200)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    e = fw.engine
    # 128 row threads: two row waves, so the candidate row crosses waves through LDS (one row wave
    # reads it from the candidate lane directly and has no such hand-off)
    e.set_option(abi.OPT_BATCH_GEO, 1)
    e.set_option(abi.OPT_SKIP_RELEASE_AT, at)
    with pytest.raises(KgpuError) as ex:
        e.schedule_batch(q, pc)
    assert ex.value.code == abi.E_DEVICE and "re-upload" in str(ex.value)
    e.set_option(abi.OPT_SKIP_RELEASE_AT, -1)
    with pytest.raises(KgpuError):
        e.schedule_batch(q[:1], pc)
    e.upload(fw.snap, fw.arrays)
    got, _ = e.schedule_batch(q, pc)
    _same(_ref(fw, q, pc), got)


def _hold_case(kind):
    if kind == "batch":
        nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=700, n_pods=160)
    else:
        nodes, existing, pods, prof = cluster.taints_affinity_spread(n_nodes=600, n_pods=60)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    return fw, q, pc


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["batch", "tbatch"])
def test_missing_workgroup_retried_cooperatively(kind):
    """Persistent kernels go out as ordinary launches (KGPU_OPT_COOPERATIVE 0).  A workgroup that never
    starts (KGPU_OPT_HOLD_GROUP: it leaves at once) makes the others' pod-0 spins time out before any
    pod resolved -- a clean abort: the call is issued again with a cooperative launch, returns the C
    restatement's placements, and the mirror stays valid (the next call needs no re-upload)."""
    fw, q, pc = _hold_case(kind)
    e = fw.engine
    want = _ref(fw, q, pc)
    e.set_option(abi.OPT_HOLD_GROUP, 1)
    got1, _ = e.schedule_batch(q[:80], pc, first_seq=0)
    e.set_option(abi.OPT_HOLD_GROUP, -1)
    c = e.counters()
    assert c["coop_retries"] == 1 and c["coop_launches"] >= 1, c
    got2, _ = e.schedule_batch(q[80:], pc, first_seq=80)
    assert e.counters()["coop_retries"] == 1
    _same(want, np.concatenate([got1, got2]))


@pytest.mark.gpu
def test_missing_workgroup_one_pod_cycle():
    """The same for a kgpu_schedule_one cycle of a topology pod (a one-pod k_tbatch run whose abort word
    travels through the pinned result block), in the middle of a sequence of cycles with assume and the
    resident topology state on: every placement and the final node rows equal the C restatement's."""
    from oracle.cref import RefEngine
    fw, q, pc = _hold_case("tbatch_one")
    e = fw.engine
    got = []
    for i in range(len(q)):
        if i == 7:
            e.set_option(abi.OPT_HOLD_GROUP, 0)
        t0 = time.perf_counter()
        res, _ = e.schedule_one(q[i], pc, seq=i, assume=True)
        if i == 7:
            e.set_option(abi.OPT_HOLD_GROUP, -1)
            # the spin timeout (0.5 s) and the cooperative re-issue; the host stops waiting on the completion
            # word as soon as it holds the abort code (it used to spin out its 2 s bound first: ADVICE r5)
            assert time.perf_counter() - t0 < 1.5
        got.append(res)
    assert e.counters()["coop_retries"] == 1
    ref = RefEngine(fw.config, fw.snap, threads=4)
    want = ref.schedule(q, pc)
    _same(want, np.array(got, dtype=abi.RESULT))
    rows_w, rows_g = ref.read_nodes(), e.read_nodes(fw.snap.n_nodes)
    for k in rows_w:
        np.testing.assert_array_equal(rows_w[k], rows_g[k], err_msg=k)


@pytest.mark.gpu
def test_abort_one_pod_cycle_recovers():
    """A one-pod topology cycle (kgpu_schedule_one's k_tbatch run, abort word through the pinned result
    block) that aborts after its workgroups started (KGPU_OPT_ABORT_AT): KGPU_E_DEVICE, the mirror is
    invalid until the next upload, and after it the cycles match the C restatement."""
    from oracle.cref import RefEngine
    fw, q, pc = _hold_case("tbatch_one")
    e = fw.engine
    for i in range(5):
        e.schedule_one(q[i], pc, seq=i, assume=True)
    e.set_option(abi.OPT_ABORT_AT, 0)
    t0 = time.perf_counter()
    with pytest.raises(KgpuError) as ex:
        e.schedule_one(q[5], pc, seq=5, assume=True)
    assert time.perf_counter() - t0 < 1.5  # no 2 s spin on a completion word that holds an abort code
    assert ex.value.code == abi.E_DEVICE and "re-upload" in str(ex.value)
    e.set_option(abi.OPT_ABORT_AT, -1)
    assert e.counters()["coop_retries"] == 0  # a run that started everywhere is not issued again
    with pytest.raises(KgpuError):
        e.schedule_one(q[5], pc, seq=5, assume=True)
    e.upload(fw.snap, fw.arrays)
    got = [e.schedule_one(q[i], pc, seq=i, assume=True)[0] for i in range(len(q))]
    _same(RefEngine(fw.config, fw.snap, threads=4).schedule(q, pc), np.array(got, dtype=abi.RESULT))
