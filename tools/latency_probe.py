"""Per-call latency of kgpu_schedule_one (the drop-in plugin's per-cycle call) on configs (b), (c), (d), and
"t" = (c) without its spread constraints (tolerations and node-affinity terms in the pools, one k_eval launch).

Run under `rocprofv3 --hip-trace --kernel-trace --stats` to see where a call's time goes
(API calls, copies, launches, synchronisation)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-1_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=300)
    ap.add_argument("--config", default="b")
    ap.add_argument("--zc", type=int, default=None, help="KGPU_OPT_ZEROCOPY_POOLS (default: the library's, 1)")
    ap.add_argument("--prepare", type=int, default=1,
                    help="1: kgpu_prepare_pods over the measured pods first (the drop-in registers its queue's pod "
                         "classes at upload); 0: each class is met on its first cycle")
    ap.add_argument("--per-pod-pools", type=int, default=0,
                    help="1: every pod compiled on its own, with its own pools block (the Go shim's shape)")
    args = ap.parse_args()
    from kgpu import cluster
    from kgpu.framework import GpuFramework
    if args.config == "b":
        nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=args.nodes, n_pods=args.pods)
    elif args.config == "t":  # (c) without the spread constraints: taints, tolerations, node affinity (k_eval)
        nodes, existing, pods, prof = cluster.taints_affinity_spread(n_nodes=args.nodes, n_pods=args.pods, spread=False)
    elif args.config == "c":
        nodes, existing, pods, prof = cluster.taints_affinity_spread(n_nodes=args.nodes, n_pods=args.pods)
    else:
        nodes, existing, pods, prof = cluster.pod_affinity(n_nodes=args.nodes, n_existing=args.nodes, n_pods=args.pods)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16])
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    eng = fw.engine
    if args.zc is not None:
        from kgpu import abi
        eng.set_option(abi.OPT_ZEROCOPY_POOLS, args.zc)
    for i in range(20):  # warm
        eng.schedule_one(q[i], pc, seq=i, assume=False)
    if args.prepare:
        eng.prepare_pods(q, pc)
    lat = []
    own = [fw.compile_pods([p])[:2] for p in pods] if args.per_pod_pools else None
    for i in range(len(q)):
        qi, pci = (own[i][0][0], own[i][1]) if own else (q[i], pc)
        t = time.perf_counter()
        eng.schedule_one(qi, pci, seq=i, assume=True)
        lat.append((time.perf_counter() - t) * 1e6)
    la = np.array(lat)
    print("kgpu_schedule_one config %s %d nodes%s%s: p50 %.1f us, p99 %.1f us, mean %.1f us"
          % (args.config, args.nodes, " (classes prepared)" if args.prepare else "",
             " (per-pod pools)" if args.per_pod_pools else "", np.percentile(la, 50),
             np.percentile(la, 99), la.mean()))
    eng.close()


if __name__ == "__main__":
    main()
