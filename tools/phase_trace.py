#!/usr/bin/env python3
"""Per-pod phase breakdown of the persistent batch kernel (s_memrealtime, 10 ns ticks).

phases per pipeline iteration i.  Row wave 0: eval = pod i evaluated (variant A on every row,
variant B on the spare lane); partials = wave reductions; wait = barrier (c), i.e. the slowest
row wave and the communication wave; post = pod i-1 assumed, pod i's candidate row staged; next =
loop overhead.  Communication wave: poll_vs_rows = pod i-1 resolved minus wave 0's partials of
pod i (positive: the granule hop, not the evaluation, sets the pace); publish = pod i published
after the later of its partials and pod i-1's resolution; hop = latest publish of pod i (of the
two traced workgroups) to pod i seen resolved."""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-1_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=1000)
    ap.add_argument("--config", default="b")
    ap.add_argument("--groups", type=int, default=0, help="KGPU_OPT_PERSIST_GROUPS cap (0: one per CU)")
    ap.add_argument("--batch-geo", type=int, default=None, help="KGPU_OPT_BATCH_GEO")
    args = ap.parse_args()
    import numpy as np
    from kgpu import abi, cluster
    from kgpu.framework import GpuFramework
    if args.config == "b":
        nodes, ex, pods, prof = cluster.fit_least_balanced(n_nodes=args.nodes, n_pods=args.pods)
    else:
        nodes, init, pods, prof = cluster.scheduling_basic(n_nodes=args.nodes, n_init=args.nodes, n_pods=args.pods)
        ex, pods = [], init + pods
    fw = GpuFramework(prof, nodes, ex, pods_hint=pods[:16])
    q, pc, _, errs = fw.compile_pods(pods)
    eng = fw.engine
    eng.schedule_batch(q[:64], pc)
    eng.upload(fw.snap, fw.arrays)
    eng.set_option(abi.OPT_PHASE_TRACE, 1)
    if args.batch_geo is not None:
        eng.set_option(abi.OPT_BATCH_GEO, args.batch_geo)
    if args.groups:
        eng.set_option(abi.OPT_PERSIST_GROUPS, args.groups)
    eng.schedule_batch(q, pc)
    t = eng.phase_trace(len(q) + 1).astype(np.float64) * 10.0  # ns
    t = t[1:-1]  # steady state: skip the prologue and epilogue iterations
    for w, name in ((0, "wg0"), (1, "wglast")):
        a = t[:, w, :]
        per = np.diff(a[:, 0])
        ph = {"eval": a[:, 5] - a[:, 0], "partials": a[:, 1] - a[:, 5],
              "wait": a[:, 2] - a[:, 1], "post": a[:, 4] - a[:, 2], "next": a[1:, 0] - a[:-1, 4],
              "poll_vs_rows": a[1:, 7] - a[1:, 1],
              "publish": a[1:, 3] - np.maximum(a[1:, 6], a[1:, 7])}
        print("groups<=%d %s: per-pod %.0f ns | " % (args.groups, name, np.median(per)) +
              "  ".join("%s %.0f" % (k, np.median(v)) for k, v in ph.items()) + " (medians, ns)")
    # hop: latest publish of pod i (of the two traced workgroups) -> pod i seen resolved by the
    # communication wave (stamp 7 of iteration i+1)
    pub = np.maximum(t[:-1, 0, 3], t[:-1, 1, 3])
    res0, res1 = t[1:, 0, 7], t[1:, 1, 7]
    print("publish skew (wg0 - wglast) %.0f ns; hop to wg0 %.0f ns, to wglast %.0f ns (medians)"
          % (np.median(t[:, 0, 3] - t[:, 1, 3]), np.median(res0 - pub), np.median(res1 - pub)))

if __name__ == "__main__":
    main()
