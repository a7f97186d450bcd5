"""Probe: sharded path across a snapshot re-upload, with and without torch's GPU runtime active."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-1_amd")]
mode = sys.argv[1]
if mode.startswith("torch"):
    import torch
from kgpu import cluster, native
from kgpu.framework import GpuFramework

nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=500, n_pods=200)
fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16], shard=(0, 1))
fw.init_comm(0, 1, native.comm_unique_id())
q, pc, _, _ = fw.compile_pods(pods)
a, _ = fw.engine.schedule_batch(q[:100], pc)
print(mode, "batch 1 ok", flush=True)
if mode == "torch_sync":
    torch.cuda.synchronize()
    print(mode, "torch sync ok", flush=True)
if mode != "noreup":
    fw.engine.upload(fw.snap, fw.arrays)
    print(mode, "re-upload ok", flush=True)
b, _ = fw.engine.schedule_batch(q[:100], pc)
print(mode, "batch 2 ok", (a["node"] == b["node"]).all() if mode != "noreup" else "", flush=True)
