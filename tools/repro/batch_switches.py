#!/usr/bin/env python3
"""One seeded topology cluster through the batch path under each k_tbatch switch, against oracle/c: which
switch a mismatch depends on.  python tools/repro/batch_switches.py --seed 20359"""
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
    ap.add_argument("--nodes", type=int, default=16)
    ap.add_argument("--existing", type=int, default=24)
    ap.add_argument("--pods", type=int, default=30)
    a = ap.parse_args()
    import gen_random
    from kgpu import abi
    from kgpu.compile import Cluster, Profile
    from kgpu.framework import GpuFramework
    from oracle.cref import RefEngine
    nodes, ex, pods, services, rss = gen_random.topo_cluster(a.seed, n_nodes=a.nodes, n_existing=a.existing,
                                                             n_pods=a.pods)
    runs = [("default", {}), ("ahead 0", {abi.OPT_TOPO_AHEAD: 0}), ("wlab 0", {abi.OPT_TBATCH_WLAB: 0}),
            ("poll_sleep 0", {abi.OPT_TBATCH_POLL_SLEEP: 0}), ("resident 0", {abi.OPT_TOPO_RESIDENT: 0}),
            ("geo 0 (256x1)", {abi.OPT_TBATCH_GEO: 0}), ("geo 2 (512x2)", {abi.OPT_TBATCH_GEO: 2}),
            ("topo persistent 0", {abi.OPT_TOPO_PERSISTENT: 0})]
    want = None
    for name, opts in runs:
        fw = GpuFramework(Profile(), nodes, ex, cluster=Cluster(services=services, rss=rss), pods_hint=pods)
        q, pc, _, errs = fw.compile_pods(pods)
        assert not errs
        if want is None:
            want = RefEngine(fw.config, fw.snap, threads=2).schedule(q, pc)
        for k, v in opts.items():
            fw.engine.set_option(k, v)
        got, _ = fw.engine.schedule_batch(q, pc)
        bad = [(i, int(want["node"][i]), int(got["node"][i]), int(want["score"][i]), int(got["score"][i]))
               for i in range(len(q)) if want["node"][i] != got["node"][i] or want["score"][i] != got["score"][i]]
        print("%-18s %s" % (name, bad if bad else "identical"), flush=True)
        fw.engine.close()


if __name__ == "__main__":
    main()
