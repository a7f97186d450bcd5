"""Pod overhead (RuntimeClass) in the two resource sums that treat it differently, through the one
compile libkgpu ships (kgpu_compile.cpp), the compile the Go shim calls too:

  * NodeInfo.AddPod's NonZeroRequested delta (kgpu_pod_query.nz, the on-device assume): calculateResource
    adds the overhead CPU as Quantity.MilliValue() (pkg/scheduler/framework/v1alpha1/types.go:571-580);
  * the scorers' pod request (kgpu_pod_query.score_req): calculatePodResourceRequest adds every overhead
    quantity as Quantity.Value(), whole cores rounded up for CPU (noderesources/resource_allocation.go:135-139).

A 250m CPU overhead therefore adds 250 to the node's NonZeroRequested but 1 to the scorer's request.  The
round-5 Go shim added the scorer's 1 on assume (Weak 1); the GPU case below places a second
pod differently under that error.  Expected values come from the Python restatement (oracle/refsched), which
reads the pod objects, not the compiled queries."""
import numpy as np
import pytest

from kgpu import abi, cluster
from kgpu.compile import Compiler, Pools, Profile
from oracle.refsched import framework as F
from oracle.refsched import nodeinfo as NI
from oracle.refsched import plugins as P


def _pod(name, cpu, overhead=None, init_cpu=None):
    p = cluster.pod(name, cpu)
    if overhead:
        p["spec"]["overhead"] = dict(overhead)
    if init_cpu:
        p["spec"]["initContainers"] = [{"name": "i", "image": "busybox", "resources": {"requests": {"cpu": init_cpu}}}]
    return p


CASES = [_pod("a", "100m", {"cpu": "250m", "memory": "1Mi"}), _pod("b", None, {"cpu": "250m"}),
         _pod("c", "1", {"cpu": "1500m"}), _pod("d", "300m", {"cpu": "250m"}, init_cpu="700m"),
         _pod("e", "2", {"memory": "10Mi"}), _pod("f", "2")]


@pytest.mark.parametrize("i", range(len(CASES)))
def test_compiled_requests_follow_both_reference_sums(i):
    pod = CASES[i]
    comp = Compiler(Profile())
    comp.register([cluster.node("n0", "4", "8Gi")], (), [pod])
    comp.compile_snapshot([cluster.node("n0", "4", "8Gi")])
    q = comp.compile_pod(pod, Pools())
    res, n0c, n0m = NI.calculate_resource(pod)
    assert (int(q["nz"][0]), int(q["nz"][1])) == (n0c, n0m)
    fit = NI.compute_pod_resource_request(pod)
    assert (int(q["req"][0]), int(q["req"][1])) == (fit.milli_cpu, fit.memory)
    want = [P._pod_score_request(pod, r) for r in ("cpu", "memory")]
    assert [int(q["score_req"][0]), int(q["score_req"][1])] == want


def test_overhead_cpu_rounding_differs_between_the_sums():
    q = Compiler(Profile()).compile_pod(CASES[0], Pools())
    assert int(q["nz"][0]) == 100 + 250      # MilliValue
    assert int(q["score_req"][0]) == 100 + 1  # Value(): 250m rounds up to one core


def _overhead_cluster():
    """Node b carries 1100m of NonZeroRequested CPU; node a is empty.  Pod p1 (1000m + 250m overhead)
    lands on a.  For p2 (the same), LeastAllocated compares a at 1250 + 1001 against b at 1100 + 1001: b
    wins.  With the overhead assumed as Value() (a at 1001 + 1001) a would win instead."""
    nodes = [cluster.node("a", "4", "8Gi"), cluster.node("b", "4", "8Gi")]
    existing = [cluster.pod("e0", "1100m", node_name="b")]
    pods = [_pod("p1", "1", {"cpu": "250m"}), _pod("p2", "1", {"cpu": "250m"})]
    prof = Profile(filters=["NodeResourcesFit"], scores=[("NodeResourcesLeastAllocated", 1)])
    return nodes, existing, pods, prof


def test_overhead_placements_oracle():
    nodes, existing, pods, prof = _overhead_cluster()
    oprof = F.Profile(filters=prof.filters, prefilters=["NodeResourcesFit"], prescores=[], scores=prof.scores)
    want = [r.host for r in F.schedule_sequence(nodes, existing, pods, oprof)]
    assert want == ["a", "b"]


@pytest.mark.gpu
def test_gpu_overhead_assume_two_pods_one_batch():
    """Both pods in one kgpu_schedule_batch (on-device assume between them): placements as the Python
    restatement's, and the device's NonZeroRequested rows as NodeInfo.AddPod leaves them."""
    from kgpu.framework import GpuFramework
    from oracle.cref import RefEngine
    nodes, existing, pods, prof = _overhead_cluster()
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods)
    res = fw.schedule(pods, first_seq=0)
    assert [fw.host_of(int(n)) for n in res["node"]] == ["a", "b"]
    rows = fw.engine.read_nodes(fw.snap.n_nodes)
    idx = {nm: i for i, nm in enumerate(fw.order)}
    nz = {"a": 0, "b": NI.calculate_resource(existing[0])[1]}
    for p, host in zip(pods, ("a", "b")):
        nz[host] += NI.calculate_resource(p)[1]
    assert int(rows["nz_cpu"][idx["a"]]) == nz["a"] == 1250
    assert int(rows["nz_cpu"][idx["b"]]) == nz["b"] == 2350
    q, pc, _, _ = fw.compile_pods(pods)
    fw2 = GpuFramework(prof, nodes, existing, pods_hint=pods, create_engine=False)
    ref = RefEngine(fw2.config, fw2.snap)
    want = ref.schedule(q, pc)
    assert np.array_equal(want["node"], res["node"])
    rw = ref.read_nodes()
    for k in rw:
        np.testing.assert_array_equal(rw[k], rows[k], err_msg=k)
