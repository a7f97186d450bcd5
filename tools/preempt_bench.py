"""Latency of kgpu_select_victims (selectNodesForPreemption + pickOneNodeForPreemption) on config (b)
clusters with pod priorities: every node holds low-priority pods, the preemptor fits nowhere without
evicting.  Prints one JSON line per node count (wall clock per call, host compile excluded)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-1_amd")]

import numpy as np  # noqa: E402

from kgpu import abi, cluster  # noqa: E402
from kgpu.framework import GpuFramework  # noqa: E402


def main():
    for n_nodes in [int(x) for x in (sys.argv[1:] or ["5000", "100000"])]:
        nodes, ex, pods, prof = cluster.fit_least_balanced(n_nodes=n_nodes, n_pods=2 * n_nodes)
        r = np.random.default_rng(5)
        names = [n["metadata"]["name"] for n in nodes]
        existing = []
        for i, p in enumerate(pods):  # two pods per node, priorities 0..2, fixed start times
            p = dict(p)
            p["metadata"] = dict(p["metadata"], uid="v%d" % i)
            p["spec"] = dict(p["spec"], nodeName=names[i % n_nodes], priority=int(r.integers(0, 3)))
            p["status"] = {"startTime": "2019-01-0%dT01:01:01Z" % (1 + i % 7)}
            existing.append(p)
        pre = {"metadata": {"name": "preemptor", "namespace": "default", "uid": "pre"},
               "spec": {"priority": 1000, "containers": [{"name": "c", "resources": {"requests": {"cpu": "60", "memory": "200Gi"}}}]}}
        t0 = time.time()
        fw = GpuFramework(prof, nodes, existing, pods_hint=[pre])
        t_up = time.time() - t0
        # device part alone: compile the preemptor and victims once, time the C call
        prio = 1000
        cand = [(nn, p, slot) for nn in fw.order for p, slot in fw.node_pods.get(nn, []) if p["spec"]["priority"] < prio]
        q, pc, _, _ = fw.compile_pods([pre] + [p for _, p, _ in cand])
        index = {nn: i for i, nn in enumerate(fw.order)}
        vic = np.zeros(len(cand), abi.VICTIM)
        for i, (nn, p, slot) in enumerate(cand):
            vic[i] = (index[nn], slot, i, 0, 0, 0)
        lat = []
        for k in range(12):
            t1 = time.perf_counter()
            out, vout, chosen = fw.engine.select_victims(q[0], pc, vic, q[1:], np.zeros(0, np.int32), fw.snap.n_nodes)
            lat.append((time.perf_counter() - t1) * 1e3)
        lat = np.array(lat[2:])
        print(json.dumps({"call": "kgpu_select_victims", "nodes": n_nodes, "potential_victims": len(cand),
                          "fits": int(out["fits"].sum()), "chosen": fw.order[chosen] if chosen >= 0 else None,
                          "ms_median": round(float(np.median(lat)), 3), "ms_min": round(float(lat.min()), 3),
                          "setup_s": round(t_up, 1)}), flush=True)
        fw.engine.close()


if __name__ == "__main__":
    main()
