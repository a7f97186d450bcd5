#!/usr/bin/env python3
"""Device-side timeline of the topology kgpu_schedule_one cycle's one-pod k_tbatch run
(KGPU_OPT_PHASE_TRACE, s_memrealtime 10 ns ticks), workgroup 0 and the last workgroup:
entry -> pod loop start (LDS replicas, label values and node rows loaded) -> the pod's phases
(prefilter, rows, stats publish, stats wait, normalize + key publish, key wait, assume) -> exit,
medians over the cycles; plus the host wall time per cycle with and without the resident topology
state (KGPU_OPT_TOPO_RESIDENT)."""
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
    ap.add_argument("--pods", type=int, default=200)
    ap.add_argument("--config", default="c")
    args = ap.parse_args()
    from kgpu import abi, cluster
    from kgpu.framework import GpuFramework
    if args.config == "c":
        nodes, ex, pods, prof = cluster.taints_affinity_spread(n_nodes=args.nodes, n_pods=args.pods)
    else:
        nodes, ex, pods, prof = cluster.pod_affinity(n_nodes=args.nodes, n_existing=args.nodes, n_pods=args.pods)
    fw = GpuFramework(prof, nodes, ex, pods_hint=pods[:16])
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    eng = fw.engine
    for resident in (0, 1):
        eng.upload(fw.snap, fw.arrays)
        eng.set_option(abi.OPT_TOPO_RESIDENT, resident)
        eng.set_option(abi.OPT_PHASE_TRACE, 0)
        for i in range(10):
            eng.schedule_one(q[i], pc, seq=i, assume=False)
        lat = []
        for i in range(len(q)):
            t = time.perf_counter()
            eng.schedule_one(q[i], pc, seq=i, assume=True)
            lat.append((time.perf_counter() - t) * 1e6)
        la = np.array(lat)
        hits, misses = eng.topo_resident()
        print("config %s %d nodes, resident %d: kgpu_schedule_one p50 %.1f us, p99 %.1f us, mean %.1f us "
              "(resident hits %d, misses %d)" % (args.config, args.nodes, resident, np.percentile(la, 50),
                                                  np.percentile(la, 99), la.mean(), hits, misses))
        # device timeline of traced cycles
        eng.set_option(abi.OPT_PHASE_TRACE, 1)
        rows = []
        for i in range(40):
            eng.schedule_one(q[i], pc, seq=len(q) + i, assume=False)
            t = eng.phase_trace(2).astype(np.float64) * 10.0  # [2][2][8] ns
            rows.append(t)
        eng.set_option(abi.OPT_PHASE_TRACE, 0)
        t = np.array(rows)  # [cycles][2 rows][2 wg][8]
        names = ["entry->loop", "prefilter", "rows", "stats_pub", "stats_wait", "score_pub", "key_wait", "assume",
                 "end->exit"]
        for w, wn in ((0, "wg0"), (1, "wglast")):
            run = t[:, 1, w, :]
            pod = t[:, 0, w, :]
            ph = [run[:, 1] - run[:, 0]] + [pod[:, k + 1] - pod[:, k] for k in range(7)] + [run[:, 2] - pod[:, 7]]
            total = run[:, 2] - run[:, 0]
            print("  %s: run %.0f ns | " % (wn, np.median(total)) +
                  "  ".join("%s %.0f" % (nm, np.median(v)) for nm, v in zip(names, ph)))
        # entry skew between the workgroups (dispatch)
        print("  entry skew last-wg minus wg0: %.0f ns" % np.median(t[:, 1, 1, 0] - t[:, 1, 0, 0]))
    eng.close()


if __name__ == "__main__":
    main()
