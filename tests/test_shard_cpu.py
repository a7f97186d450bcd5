"""Node sharding on the CPU: world_size-2 gloo ranks.

* Shard compile: every rank's contiguous slice of Snapshot.List() (native.shard_range) holds
  exactly the rows of the unsharded snapshot, with node_base / n_total_nodes set for global
  indices (ImageLocality, NodeName and the tie-break hash all use the global index).
* Combine rule: per pod each rank packs its shard's best key (score << 40 | rank40 over the
  GLOBAL node index) and its feasible count, the records are all-gathered (gloo here, RCCL on the
  device), and the max key over ranks must be the unsharded selectHost winner with the summed
  feasible count.  Per-node scores come from the C restatement on the full cluster state, so the
  test checks the exchange protocol, not the scorers."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from kgpu import cluster, native
from kgpu.framework import GpuFramework

COLS = ("alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "req_cpu", "req_mem", "nz_cpu", "nz_mem", "num_pods")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _workload(name):
    if name == "basic":  # identical nodes: every placement is decided by the tie-break hash
        nodes, init, pods, prof = cluster.scheduling_basic(n_nodes=61, n_init=0, n_pods=40)
        return nodes, [], pods, prof
    nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=101, n_pods=60)
    return nodes, existing, pods, prof


def _rank_main(rank, world, port, name, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.cref import RefEngine
        from oracle.refsched import tiebreak
        nodes, existing, pods, prof = _workload(name)
        full = GpuFramework(prof, nodes, existing, pods_hint=pods, create_engine=False)
        shard = GpuFramework(prof, nodes, existing, pods_hint=pods, create_engine=False, shard=(rank, world))
        base, cnt = shard.shard
        N = full.snap.n_nodes
        assert (shard.snap.node_base, shard.snap.n_nodes, shard.snap.n_total_nodes) == (base, cnt, N)
        for c in COLS:
            np.testing.assert_array_equal(shard.arrays[c], full.arrays[c][base:base + cnt], err_msg=c)
        spans = [None] * world
        dist.all_gather_object(spans, (base, cnt))
        assert sorted(spans) == [(rank * N // world, (rank + 1) * N // world - rank * N // world)
                                 for rank in range(world)]
        assert sum(c for _, c in spans) == N

        cfg = full.config
        weights = {cfg.scores[i]: max(int(cfg.score_weights[i]), 1) for i in range(cfg.n_scores)}
        q, pc, _, errs = full.compile_pods(pods)
        assert not errs
        want = RefEngine(cfg, full.snap).schedule(q, pc)
        ref = RefEngine(cfg, full.snap)
        for k in range(len(q)):
            res, status, _, norm = ref.schedule(q[k:k + 1], pc, first_seq=k, diag=True)
            tk = tiebreak.pod_key(cfg.seed, k)
            best, best_g, feas = 0, -1, 0
            for n in range(base, base + cnt):
                if status[n]:
                    continue
                feas += 1
                total = sum(w * int(norm[s][n]) for s, w in weights.items()) if weights else 1
                key = (total << 40) | tiebreak.rank40(tk, n)
                if key > best:
                    best, best_g = key, n
            recs = [None] * world
            dist.all_gather_object(recs, (best, best_g, feas))
            top = max(recs)
            assert sum(r[2] for r in recs) == int(res[0]["feasible"]) == int(want["feasible"][k])
            assert top[1] == int(res[0]["node"]) == int(want["node"][k]), "pod %d" % k
        out.put((rank, "ok"))
    except Exception as e:  # surfaced by the parent
        out.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["fit", "basic"])
def test_shard_combine_gloo_world2(name):
    world = 2
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, name, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    got = dict(out.get(timeout=5) for _ in range(world))
    assert got == {0: "ok", 1: "ok"}, got
    assert all(p.exitcode == 0 for p in procs)


def test_shard_range_partition():
    for n in (1, 7, 100, 1_000_000):
        for w in (1, 2, 3, 8):
            spans = [native.shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and sum(c for _, c in spans) == n
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
