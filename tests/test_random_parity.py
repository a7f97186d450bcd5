"""Seeded random clusters: Python oracle (objects) == product compile + C restatement == libkgpu.

Every placement of the scheduleOne loop is compared (node, feasible count, winner's total
score), and after the loop the assumed node rows are compared too."""
import numpy as np
import pytest

import gen_random
from oracle.refsched import framework as F
from kgpu.compile import Profile
from kgpu.framework import GpuFramework

SEEDS = list(range(12))


def oracle_run(nodes, existing, pods):
    res = F.schedule_sequence(nodes, existing, pods, F.Profile())
    out = []
    for r in res:
        if isinstance(r, F.FitError):
            out.append((None, 0, None))
        elif isinstance(r, F.ScheduleError):
            out.append(("error", None, None))
        else:
            tot = dict((n, s) for n, s in r.totals)
            out.append((r.host, r.feasible, tot.get(r.host) if len(r.totals) > 0 else None))
    return out


def product_run(nodes, existing, pods, backend):
    fw = GpuFramework(Profile(), nodes, existing, pods_hint=pods, create_engine=(backend == "gpu"))
    if backend == "gpu":
        res = fw.schedule(pods, first_seq=0)
        rows = fw.engine.read_nodes(fw.snap.n_nodes)
    else:
        from oracle.cref import RefEngine
        q, pc, pnp, errs = fw.compile_pods(pods)
        assert not errs
        ref = RefEngine(fw.config, fw.snap, threads=2)
        res = ref.schedule(q, pc)
        rows = ref.read_nodes()
    out = []
    for r in res:
        if r["node"] == -1:
            out.append((None, 0, None))
        elif r["node"] < -1:
            out.append(("error", None, None))
        else:
            out.append((fw.order[r["node"]], int(r["feasible"]), int(r["score"]) if r["scored"] else None))
    return out, rows, fw


def _cmp(want, got):
    for i, (w, g) in enumerate(zip(want, got)):
        assert w[0] == g[0], "pod %d: oracle host %r, product %r" % (i, w, g)
        if w[0] not in (None, "error"):
            assert w[1] == g[1], "pod %d feasible %r vs %r" % (i, w, g)
            if w[1] > 1:
                assert w[2] == g[2], "pod %d score %r vs %r" % (i, w, g)


@pytest.mark.parametrize("seed", SEEDS)
def test_c_restatement_matches_python_oracle(seed):
    nodes, existing, pods = gen_random.cluster(seed)
    want = oracle_run(nodes, existing, pods)
    got, rows, fw = product_run(nodes, existing, pods, "ref")
    _cmp(want, got)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_gpu_matches_python_oracle_and_c(seed):
    nodes, existing, pods = gen_random.cluster(seed)
    want = oracle_run(nodes, existing, pods)
    got, rows, fw = product_run(nodes, existing, pods, "gpu")
    _cmp(want, got)
    got_c, rows_c, _ = product_run(nodes, existing, pods, "ref")
    for k in rows:
        np.testing.assert_array_equal(rows[k], rows_c[k], err_msg=k)
