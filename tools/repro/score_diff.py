#!/usr/bin/env python3
"""Per-plugin normalized scores of one pod of a seeded topology cluster on the GPU against the Python oracle:
the batch path places pods [0, k), then a kgpu_schedule_one diagnostic cycle (no assume) of pod k reads every
plugin's normalized row (kgpu_get_scores).  python tools/repro/score_diff.py --seed 20359 --pod 24"""
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
    ap.add_argument("--nodes", type=int, default=16)
    ap.add_argument("--existing", type=int, default=24)
    ap.add_argument("--pods", type=int, default=30)
    a = ap.parse_args()
    import gen_random
    from kgpu import abi
    from kgpu.compile import Cluster, Profile
    from kgpu.framework import GpuFramework
    from oracle.refsched import framework as F
    nodes, ex, pods, services, rss = gen_random.topo_cluster(a.seed, n_nodes=a.nodes, n_existing=a.existing,
                                                             n_pods=a.pods)
    res = F.schedule_sequence(nodes, ex, pods, F.Profile(), services=services, rss=rss)
    fw = GpuFramework(Profile(), nodes, ex, cluster=Cluster(services=services, rss=rss), pods_hint=pods)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    got, _ = fw.engine.schedule_batch(q[:a.pod + 1], pc)
    print("batch pod %d: node %s score %d (oracle %s %s)" % (a.pod, fw.order[got["node"][a.pod]] if got["node"][a.pod] >= 0
                                                             else None, got["score"][a.pod], res[a.pod].host,
                                                             dict(res[a.pod].totals).get(res[a.pod].host)))
    fw2 = GpuFramework(Profile(), nodes, ex, cluster=Cluster(services=services, rss=rss), pods_hint=pods)
    q2, pc2, _, _ = fw2.compile_pods(pods)
    fw2.engine.schedule_batch(q2[:a.pod], pc2)
    r, _ = fw2.engine.schedule_one(q2[a.pod], pc2, seq=a.pod, assume=False)
    print("schedule_one pod %d: node %s score %d" % (a.pod, fw2.order[r["node"]] if r["node"] >= 0 else None, r["score"]))
    n = fw2.snap.n_nodes
    for plugin, rows in res[a.pod].scores.items():
        sid = abi.SCORE_IDS.get(plugin)
        if sid is None:
            continue
        raw, norm = fw2.engine.scores(sid, n)
        want = [(nm, v) for nm, v in rows]
        gotn = [(nm, int(norm[fw2.order.index(nm)]), int(raw[fw2.order.index(nm)])) for nm, _ in rows]
        print("  %-34s oracle(weighted) %s" % (plugin, [v for _, v in want]))
        print("  %-34s gpu norm          %s  raw %s" % ("", [v for _, v, _ in gotn], [r for _, _, r in gotn]))

if __name__ == "__main__":
    main()
