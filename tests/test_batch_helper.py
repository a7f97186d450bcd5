"""KGPU_OPT_BATCH_HELPER: on config (b)'s profile (NodeResourcesFit + BalancedAllocation +
LeastAllocated) and its one-row-wave geometry, a helper wave evaluates LeastAllocated and the
tie-break rank of every row beside the row wave's Fit + Balanced, and follows the candidate and the
winner to keep its copies of the rows assumed.

With the helper on and off, the persistent kernel must give the C restatement's placements, feasible
counts, scores and final node rows on: the (b) shape; a tie-heavy cluster (identical nodes and pods:
the rank decides every pod); and pods with host ports or extended resources, whose assume changes
memory-resident columns, so the next pod's variant B does not apply and the winning row is evaluated
again by the row wave alone (the slow path)."""
import numpy as np
import pytest

from kgpu import abi, cluster
from kgpu.framework import GpuFramework

ROW_KEYS = ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods")


def _case(name):
    nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=2000, n_pods=500)
    if name == "ties":
        nodes = [cluster.node("n%d" % i, "16", "64Gi", 110, "100Gi") for i in range(1500)]
        pods = [cluster.pod("p%d" % i, "500m", "1Gi") for i in range(500)]
    elif name == "slow":
        for i, n in enumerate(nodes):
            if i % 3 == 0:
                n["status"]["allocatable"]["example.com/dev"] = "4"
                n["status"]["capacity"]["example.com/dev"] = "4"
        for i, p in enumerate(pods):
            c = p["spec"]["containers"][0]
            if i % 7 == 3:
                c["ports"] = [{"containerPort": 8080, "hostPort": 8000 + i % 5, "protocol": "TCP"}]
            if i % 11 == 5:
                c.setdefault("resources", {}).setdefault("requests", {})["example.com/dev"] = "1"
    return nodes, existing, pods, prof


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["b", "ties", "slow"])
def test_batch_helper_matches_oracle(name):
    nodes, existing, pods, prof = _case(name)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16])
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    from oracle.cref import RefEngine
    ref = RefEngine(fw.config, fw.snap, threads=8)
    want, want_rows = ref.schedule(q, pc), ref.read_nodes()
    for helper in (1, 0):
        e = fw.engine
        e.upload(fw.snap, fw.arrays)
        e.set_option(abi.OPT_BATCH_HELPER, helper)
        out = []
        for s in range(0, len(q), 200):
            res, _ = e.schedule_batch(q[s:s + 200], pc, first_seq=s)
            out.append(res)
        got = np.concatenate(out)
        for f in ("node", "feasible", "scored", "score"):
            np.testing.assert_array_equal(want[f], got[f], err_msg="%s helper=%d: %s" % (name, helper, f))
        rows = e.read_nodes(fw.snap.n_nodes)
        for k in ROW_KEYS:
            np.testing.assert_array_equal(want_rows[k], rows[k], err_msg="%s helper=%d: %s" % (name, helper, k))
