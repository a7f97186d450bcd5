"""Config (e) at its real per-GPU size: one 125,000-node GPU's worth of the 1M-node cluster (the
columnar generator bench.py uses, cluster.sharded_spread_compiled) through the persistent topology
kernel k_tbatch, against the C restatement of the reference (oracle/c) pod for pod.

125k nodes at 512 rows per workgroup is 245 workgroups: the statistics poll's 4-granules-per-lane
branch (65-256 workgroups) is exercised, which nothing at 5k nodes reaches.  The per-workgroup
phase trace proves the run went through k_tbatch with that many workgroups.

Semantics: PodTopologySpread PreFilter / Filter / Score (podtopologyspread/filtering.go:198-328,
scoring.go:59-257), TaintToleration, NodeAffinity and the resource scorers, then selectHost with
the build's tie-break (generic_scheduler.go:217-238)."""
import numpy as np
import pytest

from kgpu import abi, cluster
from kgpu.framework import GpuFramework


@pytest.mark.gpu
def test_e_125k_shard_k_tbatch_matches_c_restatement():
    from oracle.cref import RefEngine
    comp, compiled, pods, prof = cluster.sharded_spread_compiled(n_nodes=125_000, n_pods=320)
    fw = GpuFramework(prof, None, pods_hint=pods[:16], compiled=(comp, compiled))
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    ref = RefEngine(fw.config, fw.snap, threads=16)
    want = ref.schedule(q, pc)
    fw.engine.set_option(abi.OPT_PHASE_TRACE, 1)
    got = np.concatenate([fw.engine.schedule_batch(q[k:k + 160], pc, first_seq=k)[0] for k in (0, 160)])
    trace = fw.engine.wg_trace(160)
    fw.engine.set_option(abi.OPT_PHASE_TRACE, 0)
    assert trace.shape[0] == 160 and trace.shape[1] > 64, trace.shape  # k_tbatch, > 64 workgroups
    for f in ("node", "feasible", "scored", "score"):
        bad = np.nonzero(want[f] != got[f])[0]
        assert len(bad) == 0, "%s differs at pods %s: want %s got %s" % (f, bad[:5], want[f][bad[:5]], got[f][bad[:5]])
    rows_w, rows_g = ref.read_nodes(), fw.engine.read_nodes(fw.snap.n_nodes)
    for k in rows_w:
        np.testing.assert_array_equal(rows_w[k], rows_g[k], err_msg=k)
    placed = int((got["node"] >= 0).sum())
    assert placed > 300, placed
    fw.engine.close()
