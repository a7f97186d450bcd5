#!/usr/bin/env python3
"""Seeded parity sweep on the GPU, wider than the test suite: many random clusters (tests/gen_random.py) at
several sizes, every placement, feasible count and score of libkgpu's batch path (k_batch / k_tbatch with
on-device assume) and of its per-pod drop-in path (kgpu_schedule_one) against the C restatement of the
reference (oracle/c), and the assumed node rows after the run.  Prints one line per family and a JSON
summary; exits non-zero on the first mismatch.  Checker only: the product path is what is measured.

  python tools/stress_parity.py --seeds 60 --start 1000      (GPU box)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "kubernetes-1_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

FIELDS = ("node", "feasible", "scored", "score")


def _compare(tag, seed, want, got, rows_w=None, rows_g=None):
    for f in FIELDS:
        bad = np.nonzero(np.asarray(want[f]) != np.asarray(got[f]))[0]
        if len(bad):
            raise AssertionError("%s seed %d: %s differs at pods %s (want %s, got %s)" %
                                 (tag, seed, f, bad[:5].tolist(), np.asarray(want[f])[bad[:5]].tolist(),
                                  np.asarray(got[f])[bad[:5]].tolist()))
    if rows_w is not None:
        for k in rows_w:
            if not np.array_equal(rows_w[k], rows_g[k]):
                raise AssertionError("%s seed %d: node rows %s differ" % (tag, seed, k))


def make_profile(variant):
    """The scheduler profile a sweep runs under (--variant): the default, or one setting changed."""
    from kgpu.compile import Profile
    if variant == "pct":  # percentageOfNodesToScore: numFeasibleNodesToFind and nextStartNodeIndex (k_cut)
        return Profile(percentage_of_nodes_to_score=40)
    if variant == "hpaw":  # InterPodAffinity's hardPodAffinityWeight
        return Profile(hard_pod_affinity_weight=5)
    if variant == "tie1":  # the first-max tie-break mode
        return Profile(tie_break_mode=1)
    if variant == "most":  # MostAllocated, RequestedToCapacityRatio and ResourceLimits in the score set
        scores = [s for s in Profile.DEFAULT_SCORES if s[0] != "NodeResourcesLeastAllocated"]
        return Profile(scores=scores + [("NodeResourcesMostAllocated", 1), ("RequestedToCapacityRatio", 2),
                                        ("NodeResourceLimits", 1)])
    if variant == "fit":  # config (b)'s profile: k_batch's helper-wave instantiation on random pods
        return Profile(filters=["NodeResourcesFit"], scores=[("NodeResourcesLeastAllocated", 1),
                                                             ("NodeResourcesBalancedAllocation", 1)])
    return Profile()


def run_family(tag, make, seeds, one_pod_every, variant="default"):
    from kgpu.compile import Cluster
    from kgpu.framework import GpuFramework
    from oracle.cref import RefEngine
    pods_total = 0
    t0 = time.time()
    for s in seeds:
        spec = make(s)
        nodes, ex, pods = spec[:3]
        cl = Cluster(services=spec[3], rss=spec[4]) if len(spec) > 3 else None
        kw = {"cluster": cl} if cl is not None else {}
        # batch path
        fw = GpuFramework(make_profile(variant), nodes, ex, pods_hint=pods, **kw)
        q, pc, _, errs = fw.compile_pods(pods)
        assert not errs, errs
        ref = RefEngine(fw.config, fw.snap, threads=8)
        want = ref.schedule(q, pc)
        got, _ = fw.engine.schedule_batch(q, pc)
        _compare(tag + " batch", s, want, got, ref.read_nodes(), fw.engine.read_nodes(fw.snap.n_nodes))
        fw.engine.close()
        pods_total += len(pods)
        # drop-in path: one kgpu_schedule_one per pod, each with its own pools (the Go shim's shape)
        if one_pod_every and s % one_pod_every == 0:
            fw = GpuFramework(make_profile(variant), nodes, ex, pods_hint=pods, **kw)
            got1 = {f: [] for f in FIELDS}
            for i, pod in enumerate(pods):
                qi, pci, _, errs = fw.compile_pods([pod])
                assert not errs, errs
                r, _ = fw.engine.schedule_one(qi[0], pci, seq=i, assume=True)
                for f in FIELDS:
                    got1[f].append(int(r[f]))
            _compare(tag + " schedule_one", s, want, got1, ref.read_nodes(), fw.engine.read_nodes(fw.snap.n_nodes))
            fw.engine.close()
        if hasattr(ref, "close"):
            ref.close()
        print("  %s seed %d: %d pods ok" % (tag, s, len(pods)), flush=True)  # progress (the box's silence limit)
    line = {"family": tag, "variant": variant, "clusters": len(seeds), "pods": pods_total,
            "seconds": round(time.time() - t0, 1)}
    print(json.dumps(line), flush=True)
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=40)
    ap.add_argument("--start", type=int, default=1000, help="first seed (the test suite uses small seeds)")
    ap.add_argument("--one-pod-every", type=int, default=4, help="also run every k-th cluster one pod at a time")
    ap.add_argument("--variant", default="default", choices=["default", "pct", "hpaw", "tie1", "most", "fit"],
                    help="the profile setting the sweep changes (make_profile)")
    ap.add_argument("--long-runs", action="store_true", help="two families of long topology runs instead")
    ap.add_argument("--long-generic", action="store_true", help="two families of long generic batches instead")
    a = ap.parse_args()
    import gen_random
    seeds = list(range(a.start, a.start + a.seeds))
    fams = [
        ("generic 20 nodes", lambda s: gen_random.cluster(s, n_nodes=20, n_existing=15, n_pods=30)),
        ("generic 700 nodes", lambda s: gen_random.cluster(s, n_nodes=700, n_existing=400, n_pods=60)),
        ("generic 5000 nodes", lambda s: gen_random.cluster(s, n_nodes=5000, n_existing=2000, n_pods=40)),
        # 141 one-pod workgroups: resolve_tail's grouped tickets (uneven groups)
        ("generic 9000 nodes", lambda s: gen_random.cluster(s, n_nodes=9000, n_existing=3000, n_pods=30)),
        ("topology 16 nodes", lambda s: gen_random.topo_cluster(s, n_nodes=16, n_existing=24, n_pods=30)),
        ("topology 1500 nodes", lambda s: gen_random.topo_cluster(s, n_nodes=1500, n_existing=600, n_pods=60)),
        ("topology 6000 nodes", lambda s: gen_random.topo_cluster(s, n_nodes=6000, n_existing=3000, n_pods=40)),
    ]
    if a.long_generic:  # batches longer than a short cycle: the persistent k_batch
        fams = [("generic 700 nodes, 400 pods", lambda s: gen_random.cluster(s, n_nodes=700, n_existing=400,
                                                                            n_pods=400)),
                ("generic 5000 nodes, 300 pods", lambda s: gen_random.cluster(s, n_nodes=5000, n_existing=2000,
                                                                             n_pods=300))]
    if a.long_runs:  # long k_tbatch runs: more in-run assumes between a pod and the pods it affects
        fams = [("topology 200 nodes, 200 pods", lambda s: gen_random.topo_cluster(s, n_nodes=200, n_existing=150,
                                                                                  n_pods=200)),
                ("topology 1500 nodes, 300 pods", lambda s: gen_random.topo_cluster(s, n_nodes=1500, n_existing=900,
                                                                                   n_pods=300))]
    out = []
    for tag, make in fams:
        n = len(seeds) if not any(k in tag for k in ("5000", "6000", "9000")) else max(4, len(seeds) // 5)
        out.append(run_family(tag, make, seeds[:n], a.one_pod_every, a.variant))
    print(json.dumps({"stress_parity": "ok", "families": out}))


if __name__ == "__main__":
    main()
