"""Node sharding with the persistent kernel's granules exchanged through peer stores (xGMI mailbox
rings, kgpu_xgmi_handle / kgpu_xgmi_init), two ranks in two processes on ONE GPU: the IPC-mapped
mailbox of each rank is written by the other exactly as over xGMI (the same code path; only the
fabric differs).  Each rank holds one contiguous shard of Snapshot.List(); the handles travel over
gloo.  Every rank must return the unsharded engine's placements, feasible counts and scores pod
after pod, and its shard's node rows must equal the unsharded rows after the batches."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from kgpu import abi, cluster, native
from kgpu.framework import GpuFramework

COLS = ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods")


def _rendezvous_file():
    """A fresh path for torch.distributed's FileStore (the file must not exist yet)."""
    import tempfile
    return os.path.join(tempfile.mkdtemp(prefix="kgpu_rdv_"), "store")


def _workload(name):
    if name == "basic":  # identical nodes: the tie-break hash decides every placement
        nodes, init, pods, prof = cluster.scheduling_basic(n_nodes=1500, n_init=0, n_pods=500)
        return nodes, [], pods, prof
    if name == "first_max":
        nodes, init, pods, prof = cluster.scheduling_basic(n_nodes=900, n_init=0, n_pods=300)
        prof.tie_break_mode = 1
        return nodes, [], pods, prof
    nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=2000, n_pods=600)
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
        nodes, existing, pods, prof = _workload(name)
        fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16], device=0, shard=(rank, world))
        h = fw.engine.xgmi_handle(world)
        hs = [None] * world
        dist.all_gather_object(hs, h)
        fw.engine.xgmi_init(world, rank, b"".join(hs))
        assert fw.engine.xgmi_active()
        res, rows = _run(fw, pods, 3)
        np.savez(out, node=res["node"], feasible=res["feasible"], score=res["score"], scored=res["scored"],
                 base=fw.snap.node_base, **rows)
        fw.engine.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["fit", "basic", "first_max"])
def test_xgmi_mailbox_two_ranks_one_gpu(name, tmp_path):
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
            p.join(180)
            assert p.exitcode == 0, "rank exited with %r" % p.exitcode
    finally:
        for p in procs:  # a rank left waiting for a dead peer must not outlive the test
            if p.is_alive():
                p.kill()
                p.join(10)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16], device=0)
    want, rows = _run(fw, pods, 3)
    fw.engine.close()
    assert (want["node"] >= 0).sum() > 0
    for r in range(world):
        got = np.load(outs[r])
        for f in ("node", "feasible", "score", "scored"):
            assert np.array_equal(got[f], want[f]), (name, r, f, np.nonzero(got[f] != want[f])[0][:5])
        base = int(got["base"])
        n = len(got["num_pods"])
        for c in COLS:
            assert np.array_equal(got[c], rows[c][base:base + n]), (name, r, c)
