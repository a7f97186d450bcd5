"""Node-sharded persistent runs over the xGMI mailbox rings with W ranks as W processes on ONE GPU
(the only multi-rank setup a one-GPU box allows: RCCL refuses two ranks on one device, so the IPC
handles travel over gloo).  Config (b): --nodes per rank, 10 x 1000 pods, timed like bench.py
(barrier + synchronize, max over ranks).  Peers share one GPU here, so the number prices the
mailbox protocol (system-scope peer stores, ring polling) without the xGMI fabric."""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-1_amd")]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_main(rank, world, port, args, q_out):
    import numpy as np
    import torch
    import torch.distributed as dist
    from kgpu import cluster
    from kgpu.framework import GpuFramework
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def say(*a):
        print("[rank %d %.2fs]" % (rank, time.time() - T0), *a, file=sys.stderr, flush=True)
    T0 = time.time()
    B, K = args.pods_per_step, args.steps
    nodes, ex, pods, prof = cluster.fit_least_balanced(n_nodes=args.nodes * world, n_pods=B * K)
    fw = GpuFramework(prof, nodes, ex, pods_hint=pods[:16], device=0, shard=(rank, world))
    hs = [None] * world
    dist.all_gather_object(hs, fw.engine.xgmi_handle(world))
    fw.engine.xgmi_init(world, rank, b"".join(hs))
    say("mailbox ready")
    q, pc, _, _ = fw.compile_pods(pods)
    eng = fw.engine
    say("compiled")

    def run():
        dist.barrier()
        eng.upload(fw.snap, fw.arrays)
        say("warmup")
        eng.schedule_batch(q[:B], pc, first_seq=0)  # warmup
        say("warmup done")
        dist.barrier()
        eng.upload(fw.snap, fw.arrays)
        dist.barrier()
        t0 = time.perf_counter()
        out = []
        for k in range(K):
            r, _ = eng.schedule_batch(q[k * B:(k + 1) * B], pc, first_seq=k * B)
            out.append(r)
            say("step", k)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        dist.barrier()
        return t, np.concatenate(out)

    t, res = run()
    ts = [None] * world
    dist.all_gather_object(ts, t)
    if rank == 0:
        q_out.put({"tool": "xgmi_bench", "ranks_on_one_gpu": world, "nodes_per_rank": args.nodes,
                   "pods": B * K, "pods_per_s": round(B * K / max(ts), 1), "us_per_pod": round(1e6 * max(ts) / (B * K), 3),
                   "placed": int((res["node"] >= 0).sum())})
    eng.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--pods-per-step", type=int, default=1000)
    args = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    qo = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=rank_main, args=(r, args.ranks, port, args, qo)) for r in range(args.ranks)]
    for p in procs:
        p.start()
    rec = qo.get(timeout=600)
    for p in procs:
        p.join(120)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
