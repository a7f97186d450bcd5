"""Node sharding of TOPOLOGY pods (PodTopologySpread / InterPodAffinity) with the
persistent topology kernel's cross-rank exchange over xGMI mailboxes (k_tbatch XG + the init
reduction), two ranks in two processes on ONE GPU: each rank holds one contiguous shard of
Snapshot.List(); the IPC-mapped mailboxes are written by the other rank exactly as over xGMI.

No RCCL communicator is created: a topology pod the XG kernel did not take would need the per-pod
RCCL pipeline and fail the batch, so a green run means every pod went through k_tbatch XG.

Per pod the ranks must agree with the unsharded engine AND with the C restatement (oracle/c) on the
whole cluster: placements, feasible counts, scores; after the batches each rank's node rows must
equal the unsharded rows of its shard.  The cross-shard semantics under test are the reference's
cluster-wide maps: TpPairToMatchNum / criticalPaths (podtopologyspread/filtering.go:246-270) and the
inter-pod (anti-)affinity maps (interpodaffinity/filtering.go:166-271) built from every shard."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from kgpu import cluster, native
from kgpu.framework import GpuFramework

E_NODES = 20000  # config (e) over two ranks: 10k-node shards (each rank compiles its own, as bench.py does)
COLS = ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods")


def _rendezvous_file():
    """A fresh path for torch.distributed's FileStore (the file must not exist yet)."""
    import tempfile
    return os.path.join(tempfile.mkdtemp(prefix="kgpu_rdv_"), "store")


def _workload(name):
    if name == "spread":   # config (c): taints, required NodeAffinity, PTS zone (hard) + hostname (soft)
        nodes, existing, pods, prof = cluster.taints_affinity_spread(n_nodes=1200, n_pods=160)
    elif name == "affinity":  # config (d): existing pods' and incoming pods' (anti-)affinity terms
        nodes, existing, pods, prof = cluster.pod_affinity(n_nodes=900, n_existing=900, n_pods=128)
    elif name == "sharded_e":  # config (e): (b)+(c) generator, zone = i % 64
        nodes, existing, pods, prof = cluster.sharded_spread(n_nodes=E_NODES, n_pods=160)
    else:  # a zone whose nodes all sit in rank 0's shard holds the critical path
        nodes, existing, pods, prof = cluster.uneven_zones()
    return nodes, existing, pods, prof


def _run(fw, pods, batches):
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    out = []
    step = (len(pods) + batches - 1) // batches
    for b in range(0, len(pods), step):
        res, _ = fw.engine.schedule_batch(q[b:b + step], pc, first_seq=b)
        out.append(res)
    res = np.concatenate(out)
    rows = fw.engine.read_nodes(fw.snap.n_nodes)
    return res, rows


def _rank_main(rank, world, port, name, out):
    # a rendezvous file, not a port: a free-port probe can race another process for the port
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        if name == "sharded_e":
            # the columnar generator, sliced to this rank's shard, as bench.py runs config (e); the
            # unsharded reference run below compiles the same cluster from node objects
            comp, compiled, pods, prof = cluster.sharded_spread_compiled(
                n_nodes=E_NODES, n_pods=160, shard=native.shard_range(E_NODES, world, rank))
            fw = GpuFramework(prof, None, pods_hint=pods[:16], device=0, shard=(rank, world),
                              compiled=(comp, compiled))
        else:
            nodes, existing, pods, prof = _workload(name)
            fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16], device=0, shard=(rank, world))
        h = fw.engine.xgmi_handle(world)
        hs = [None] * world
        dist.all_gather_object(hs, h)
        fw.engine.xgmi_init(world, rank, b"".join(hs))
        assert fw.engine.xgmi_active()
        res, rows = _run(fw, pods, 2)
        np.savez(out, node=res["node"], feasible=res["feasible"], score=res["score"], scored=res["scored"],
                 base=fw.snap.node_base, **rows)
        fw.engine.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["spread", "affinity", "sharded_e", "uneven"])
def test_xgmi_topology_two_ranks_one_gpu(name, tmp_path):
    from oracle.cref import RefEngine
    nodes, existing, pods, prof = _workload(name)
    world = 2
    ctx = mp.get_context("spawn")
    port = _rendezvous_file()
    outs = [str(tmp_path / ("r%d.npz" % r)) for r in range(world)]
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, name, outs[r])) for r in range(world)]
    for p in procs:
        p.start()
    try:
        for p in procs:
            p.join(240)
            assert p.exitcode == 0, "rank exited with %r" % p.exitcode
    finally:
        for p in procs:  # a rank left waiting for a dead peer must not outlive the test
            if p.is_alive():
                p.kill()
                p.join(10)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16], device=0)
    q, pc, _, _ = fw.compile_pods(pods)
    ref = RefEngine(fw.config, fw.snap, threads=4).schedule(q, pc)
    want, rows = _run(fw, pods, 2)
    fw.engine.close()
    placed = int((want["node"] >= 0).sum())
    assert placed > len(pods) // 2, placed
    for f in ("node", "feasible", "score", "scored"):
        assert np.array_equal(want[f], ref[f]), (name, "unsharded vs oracle", f)
    for r in range(world):
        got = np.load(outs[r])
        for f in ("node", "feasible", "score", "scored"):
            assert np.array_equal(got[f], want[f]), (name, r, f, np.nonzero(got[f] != want[f])[0][:5])
        base = int(got["base"])
        n = len(got["num_pods"])
        for c in COLS:
            assert np.array_equal(got[c], rows[c][base:base + n]), (name, r, c)
