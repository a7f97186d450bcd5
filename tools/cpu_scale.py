#!/usr/bin/env python3
"""CPU baseline scaling: the C restatement (oracle/c) at several worker counts on one workload, with
KGPU_REF_PHASES=1 printing where each worker count's time goes (prefilter, the two parallel sections,
the serial feasible list, normalize + totals + selectHost + assume).
  python3 tools/cpu_scale.py <b|c|d> <nodes> <pods> <threads,threads,...>"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "kubernetes-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from kgpu import cluster  # noqa: E402
from kgpu.framework import GpuFramework  # noqa: E402
from oracle.cref import RefEngine  # noqa: E402


def main():
    cfg, n, S = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    if cfg == "b":
        nodes, ex, pods, prof = cluster.fit_least_balanced(n_nodes=n, n_pods=S)
    elif cfg == "c":
        nodes, ex, pods, prof = cluster.taints_affinity_spread(n_nodes=n, n_pods=S)
    else:
        nodes, ex, pods, prof = cluster.pod_affinity(n_nodes=n, n_existing=n, n_pods=S)
    fw = GpuFramework(prof, nodes, ex, pods_hint=pods[:16], create_engine=False)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    base = None
    for th in [int(x) for x in sys.argv[4].split(",")]:
        ref = RefEngine(fw.config, fw.snap, threads=th)
        t = time.perf_counter()
        res = ref.schedule(q, pc)
        dt = time.perf_counter() - t
        ref.close()
        if base is None:
            base = res["node"].copy()
        same = bool((res["node"] == base).all())
        print("config %s, %d nodes: %2d thread(s) %9.1f pods/s  (placements %s)"
              % (cfg, n, th, S / dt, "equal" if same else "DIFFER"), flush=True)


if __name__ == "__main__":
    main()
