"""The short cycle's staging arena (KGPU_OPT_ARENA_BYTES): a one-pod or small-batch call stages its
changed pools, topology plans, DevState + queries and a one-pod persistent topology run's tables and
zeroed words in one pinned block and moves them with ONE copy; items that do not fit take copies of
their own, and k_tbatch's abort word then goes back through a read-back copy.

Every arena size -- the default 1 MiB, a few KiB (some items staged, the rest copied on their own,
and the one-pod k_tbatch's zeroed words beyond it) and 0 (nothing staged but DevState and queries) --
must give the C restatement's placements, feasible counts, scores and node rows over a sequence of
kgpu_schedule_one cycles with assume and a few short batches, and the same diagnostic status words
and per-plugin scores for the last cycle."""
import numpy as np
import pytest

import gen_random
from kgpu import abi, cluster
from kgpu.compile import Profile
from kgpu.framework import GpuFramework

ROW_KEYS = ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods")


def _case(name):
    if name == "spread":
        return cluster.taints_affinity_spread(n_nodes=300, n_pods=70)
    if name == "affinity":
        return cluster.pod_affinity(n_nodes=200, n_existing=200, n_pods=70)
    nodes, existing, pods = gen_random.cluster(7)
    return nodes, existing, pods, Profile()


def _run(fw, q, pc, cap):
    e = fw.engine
    e.upload(fw.snap, fw.arrays)
    e.set_option(abi.OPT_ARENA_BYTES, cap)
    got = np.zeros(len(q), abi.RESULT)
    i = 0
    while i < len(q):
        if i % 20 == 10:  # a short batch of five pods (one copy for all of them)
            res, _ = e.schedule_batch(q[i:i + 5], pc, first_seq=i)
            got[i:i + 5] = res
            i += 5
            continue
        got[i], _ = e.schedule_one(q[i], pc, seq=i, assume=True)
        i += 1
    rows = e.read_nodes(fw.snap.n_nodes)
    e.schedule_one(q[0], pc, seq=len(q), assume=False)  # a diagnostic cycle on the final rows
    words = e.filter_words(fw.snap.n_nodes)
    scores = {s: e.scores(s, fw.snap.n_nodes) for s in range(abi.NUM_SCORES)}
    return got, rows, words, scores


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["spread", "affinity", "random7"])
def test_arena_sizes_match_oracle(name):
    nodes, existing, pods, prof = _case(name)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    from oracle.cref import RefEngine
    ref = RefEngine(fw.config, fw.snap, threads=4)
    want, want_rows = ref.schedule(q, pc), ref.read_nodes()
    base = None
    for cap in (1 << 20, 4096, 512, 0):
        got, rows, words, scores = _run(fw, q, pc, cap)
        for f in ("node", "feasible", "scored", "score"):
            np.testing.assert_array_equal(want[f], got[f], err_msg="%s cap=%d: %s" % (name, cap, f))
        for k in ROW_KEYS:
            np.testing.assert_array_equal(want_rows[k], rows[k], err_msg="%s cap=%d: %s" % (name, cap, k))
        if base is None:
            base = (words, scores)
        else:
            np.testing.assert_array_equal(base[0], words, err_msg="%s cap=%d: status words" % (name, cap))
            for s in base[1]:
                for a, b in zip(base[1][s], scores[s]):
                    np.testing.assert_array_equal(a, b, err_msg="%s cap=%d: plugin %d" % (name, cap, s))
