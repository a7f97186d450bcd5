#!/usr/bin/env python3
"""Where a batch-path mismatch comes from: the same pod sequence cut into two batches at several points (the
second batch starts from the state the first left), each against oracle/c.
  python tools/repro/batch_splits.py --seed 20359 --pod 24"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "kubernetes-1_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=20359)
    ap.add_argument("--pod", type=int, default=24)
    a = ap.parse_args()
    import gen_random
    from kgpu.compile import Cluster, Profile
    from kgpu.framework import GpuFramework
    from oracle.cref import RefEngine
    nodes, ex, pods, services, rss = gen_random.topo_cluster(a.seed, n_nodes=16, n_existing=24, n_pods=30)
    k = a.pod
    want = None
    for cut in [0, 1, 5, 10, 15, 20, 21, 22, 23, 24]:
        fw = GpuFramework(Profile(), nodes, ex, cluster=Cluster(services=services, rss=rss), pods_hint=pods)
        q, pc, _, errs = fw.compile_pods(pods)
        if want is None:
            want = RefEngine(fw.config, fw.snap, threads=2).schedule(q, pc)
        if cut:
            fw.engine.schedule_batch(q[:cut], pc)
        got, _ = fw.engine.schedule_batch(q[cut:k + 1], pc, first_seq=cut)
        print("cut %2d: pod %d node %d score %d (oracle %d %d)" % (cut, k, got["node"][-1], got["score"][-1],
                                                                   want["node"][k], want["score"][k]), flush=True)
        fw.engine.close()


if __name__ == "__main__":
    main()
