"""Node sharding on the CPU: world_size-2 gloo ranks.

* Shard compile: every rank's contiguous slice of Snapshot.List() (native.shard_range) holds
  exactly the rows of the unsharded snapshot, with node_base / n_total_nodes set for global
  indices (ImageLocality, NodeName and the tie-break hash all use the global index).
* Combine rule: per pod each rank scores only ITS shard (a fresh shard compile of the current
  cluster state through the C restatement), exchanges the DefaultNormalizeScore maxima and packs
  its best key (score << 40 | rank40 over the GLOBAL node index) with its feasible count; the
  records are all-gathered (gloo here, RCCL on the device), and the max key over ranks must be the
  unsharded selectHost winner with the summed feasible count, pod after pod.
* PreferNoSchedule taints on one shard only: the OR-exchanged union equals the cluster's, so the
  normalize decision is the same on every rank."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from kgpu import cluster, native
from kgpu.framework import GpuFramework

COLS = ("alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "req_cpu", "req_mem", "nz_cpu", "nz_mem", "num_pods")


def _rendezvous_file():
    """A fresh path for torch.distributed's FileStore (the file must not exist yet)."""
    import tempfile
    return os.path.join(tempfile.mkdtemp(prefix="kgpu_rdv_"), "store")


def _workload(name):
    if name == "basic":  # identical nodes: every placement is decided by the tie-break hash
        nodes, init, pods, prof = cluster.scheduling_basic(n_nodes=61, n_init=0, n_pods=40)
        return nodes, [], pods, prof
    if name == "prefer_one_shard":
        # PreferNoSchedule taints only on the second half of Snapshot.List() (rank 1's shard): the
        # TaintToleration normalize decision must still be the same on both ranks
        nodes, existing, pods, _ = cluster.taints_affinity_spread(n_nodes=80, n_pods=30, spread=False)
        for i, n in enumerate(nodes):
            n["spec"]["taints"] = ([{"key": "spot", "value": "true", "effect": "PreferNoSchedule"}]
                                   if i >= 40 and i % 3 == 0 else [])
        from kgpu.compile import Profile
        prof = Profile(filters=["NodeUnschedulable", "NodeResourcesFit", "NodeName", "NodePorts", "NodeAffinity",
                                "TaintToleration"],
                       scores=[("NodeResourcesBalancedAllocation", 1), ("ImageLocality", 1),
                               ("NodeResourcesLeastAllocated", 1), ("NodeAffinity", 1),
                               ("NodePreferAvoidPods", 10000), ("TaintToleration", 1)])
        return nodes, existing, pods, prof
    nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=101, n_pods=60)
    return nodes, existing, pods, prof


def _rank_main(rank, world, port, name, out):
    """Each rank holds only its shard: a fresh shard compile of the cluster state (node_base /
    n_total_nodes), scored by the C restatement; the ranks exchange their PreferNoSchedule unions,
    normalize maxima and best keys over gloo exactly as kgpu_comm_init / k_shard_pack /
    ncclAllGather do, and the combined winner must be the unsharded scheduleOne's, pod by pod."""
    # a rendezvous file, not a port: a free-port probe can race another process for the port
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        import copy
        from kgpu import abi
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
        assert sorted(spans) == [(r * N // world, (r + 1) * N // world - r * N // world) for r in range(world)]
        # the cluster-wide PreferNoSchedule union (kgpu_comm_init's OR exchange)
        local_union = int(np.bitwise_or.reduce(shard.arrays["taint_prefer"], axis=1).sum()) if cnt else 0
        unions = [None] * world
        dist.all_gather_object(unions, local_union)
        global_union = 0
        for u in unions:
            global_union |= u
        assert global_union == int(np.bitwise_or.reduce(full.arrays["taint_prefer"], axis=1).sum())

        cfg = full.config
        order = full.order
        weights = {cfg.scores[i]: max(int(cfg.score_weights[i]), 1) for i in range(cfg.n_scores)}
        q, pc, _, errs = full.compile_pods(pods)
        assert not errs
        want = RefEngine(cfg, full.snap).schedule(q, pc)
        placed = []
        for k in range(len(pods)):
            # this rank's shard of the current cluster state (existing + pods placed so far)
            sfw = GpuFramework(prof, nodes, list(existing) + placed, pods_hint=pods, create_engine=False,
                               shard=(rank, world))
            sq, spc, _, _ = sfw.compile_pods([pods[k]])
            _, status, raw, _ = RefEngine(sfw.config, sfw.snap).schedule(sq, spc, first_seq=k, diag=True)
            feas = [n for n in range(cnt) if not status[n]]
            # DefaultNormalizeScore maxima over the whole cluster (k_shard_pack stat + all-gather)
            mt = max([int(raw[abi.S_TAINT][n]) for n in feas], default=0)
            mn = max([int(raw[abi.S_NODE_AFFINITY][n]) for n in feas], default=0)
            stats = [None] * world
            dist.all_gather_object(stats, (mt, mn))
            mt, mn = max(s[0] for s in stats), max(s[1] for s in stats)
            tk = tiebreak.pod_key(cfg.seed, k)
            best, best_g = 0, -1
            for n in feas:
                total = 0
                for s, w in weights.items():
                    v = int(raw[s][n])
                    if s == abi.S_TAINT:
                        v = 100 if mt == 0 else 100 - (100 * v) // mt
                    elif s == abi.S_NODE_AFFINITY:
                        v = v if mn == 0 else (100 * v) // mn
                    total += w * v
                key = ((total if weights else 1) << 40) | tiebreak.rank40(tk, base + n)
                if key > best:
                    best, best_g = key, base + n
            recs = [None] * world
            dist.all_gather_object(recs, (best, best_g, len(feas)))
            top = max(recs)
            assert sum(r[2] for r in recs) == int(want["feasible"][k]), "pod %d" % k
            assert top[1] == int(want["node"][k]), "pod %d: shards chose %d, unsharded %d" % (k, top[1], want["node"][k])
            if top[1] >= 0:
                p = copy.deepcopy(pods[k])
                p["spec"]["nodeName"] = order[top[1]]
                placed.append(p)
        out.put((rank, "ok"))
    except Exception as e:  # surfaced by the parent
        out.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["fit", "basic", "prefer_one_shard"])
def test_shard_combine_gloo_world2(name):
    world = 2
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _rendezvous_file()
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
