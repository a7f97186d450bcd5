#!/usr/bin/env python3
"""Per-cycle cost of the drop-in boundary with and without batch-ahead (kgpu/ahead.py).

The scheduler loop of tests/test_ahead.py without deviations: pods pop in queue order, each placed
pod is assumed in the host cache mirror (kgpu/cache.py).  Per cycle it times the whole
Go-equivalent cycle (sync + compile + device call + assume bookkeeping) and the engine calls alone,
for per-pod cycles (SchedulerCache.schedule: UpdateSnapshot + kgpu_schedule_one) and for
batch-ahead (one kgpu_schedule_batch per `depth` pods, then adoption).  Placements must agree."""
import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-1_amd")]


def run(cfg, n_nodes, n_pods, depth):
    import numpy as np
    from kgpu import cluster
    from kgpu.ahead import BatchAhead
    from kgpu.cache import SchedulerCache
    if cfg == "b":
        nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=n_nodes, n_pods=n_pods)
    elif cfg == "c":
        nodes, existing, pods, prof = cluster.taints_affinity_spread(n_nodes=n_nodes, n_pods=n_pods)
    else:
        nodes, existing, pods, prof = cluster.pod_affinity(n_nodes=n_nodes, n_existing=n_nodes, n_pods=n_pods)
    for i, p in enumerate(pods):
        p["metadata"]["uid"] = "q%d" % i
    out = {}
    hosts = {}
    for mode in ("per_pod", "ahead"):
        cache = SchedulerCache(prof, nodes, existing, pods_hint=pods[:32])
        queue = list(pods)
        ahead = BatchAhead(cache, lambda: queue, depth=depth) if mode == "ahead" else None
        eng = cache.engine
        calls = {"t": 0.0}
        for name in ("schedule_one", "schedule_batch", "apply_delta", "adopt_pod", "forget"):
            f = getattr(eng, name)

            def wrap(*a, _f=f, **k):
                t0 = time.perf_counter()
                try:
                    return _f(*a, **k)
                finally:
                    calls["t"] += time.perf_counter() - t0
            setattr(eng, name, wrap)
        cyc = []
        got = []
        seq = 0
        while queue:
            pod = queue.pop(0)
            t0 = time.perf_counter()
            host, _ = ahead.schedule(pod, seq) if ahead is not None else cache.schedule(pod, seq=seq)
            if host is not None:
                placed = copy.deepcopy(pod)
                placed["spec"]["nodeName"] = host
                cache.assume_pod(placed)
            cyc.append(time.perf_counter() - t0)
            got.append(host)
            seq += 1
        c = np.array(cyc[5:]) * 1e6
        out[mode] = {"cycles": len(cyc), "p50_us": round(float(np.median(c)), 2),
                     "p99_us": round(float(np.percentile(c, 99)), 2), "mean_us": round(float(c.mean()), 2),
                     "engine_us_per_cycle": round(calls["t"] * 1e6 / len(cyc), 2)}
        if ahead is not None:
            out[mode]["stats"] = dict(ahead.stats)
            ahead.close()
        hosts[mode] = got
        cache.close()
    out["placements_equal"] = hosts["per_pod"] == hosts["ahead"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="b")
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=2000)
    ap.add_argument("--depth", type=int, default=256)
    a = ap.parse_args()
    r = run(a.config, a.nodes, a.pods, a.depth)
    r.update(config=a.config, nodes=a.nodes, pods=a.pods, depth=a.depth)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
