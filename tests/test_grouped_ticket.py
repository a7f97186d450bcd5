"""One-pod cycles on grids around resolve_tail's grouped-ticket threshold (kTicketSplit = 128 workgroups of 64
nodes): below it one counter, from it 8 group counters (blockIdx mod 8, uneven group sizes when the grid is
not a multiple of 8) and a top counter.  Every kgpu_schedule_one cycle -- k_eval alone, or k_eval + k_final
for pods that need the normalize pass -- against the C restatement (oracle/c) of the same sequence:
placements, feasible counts, scores and the assumed node rows."""
import numpy as np
import pytest

import gen_random
from kgpu.compile import Profile
from kgpu.framework import GpuFramework


@pytest.mark.gpu
@pytest.mark.parametrize("n_nodes", [127 * 64, 128 * 64, 128 * 64 + 8, 131 * 64 + 5, 1023 * 64 + 1])
def test_schedule_one_around_the_ticket_split(n_nodes):
    from oracle.cref import RefEngine
    nodes, ex, pods = gen_random.cluster(7 + n_nodes % 97, n_nodes=n_nodes, n_existing=n_nodes // 4, n_pods=24)
    fw = GpuFramework(Profile(), nodes, ex, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    ref = RefEngine(fw.config, fw.snap, threads=8)
    want = ref.schedule(q, pc)
    got = {f: [] for f in ("node", "feasible", "scored", "score")}
    for i, pod in enumerate(pods):
        qi, pci, _, errs = fw.compile_pods([pod])  # the Go shim's shape: the pod's own pools
        assert not errs
        r, _ = fw.engine.schedule_one(qi[0], pci, seq=i, assume=True)
        for f in got:
            got[f].append(int(r[f]))
    for f in got:
        np.testing.assert_array_equal(np.asarray(want[f]), np.asarray(got[f]), err_msg=f)
    rows_w, rows_g = ref.read_nodes(), fw.engine.read_nodes(fw.snap.n_nodes)
    for k in rows_w:
        np.testing.assert_array_equal(rows_w[k], rows_g[k], err_msg=k)
    fw.engine.close()
