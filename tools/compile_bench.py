#!/usr/bin/env python3
"""Per-pod cost of the pod compile (the PreFilter-time host work of a scheduling cycle).

  c_us_per_pod      kgpu_compile_pods over descriptors built beforehand: libkgpu's C++ compile alone,
                    what the Go shim pays after its marshalling (desc.go)
  marshal_us_per_pod  building the kgpu_pod_desc descriptors from the v1-shaped dicts (Python; the Go
                    shim's desc.go does the same copies in Go)
  py_us_per_pod     Compiler.compile_pods (marshal + C compile, the Python mirror's and the extender's path)
  one_us_per_pod    Compiler.compile_pod one pod at a time (the extender's per-cycle path)

No GPU: runs here and on the box.  python tools/compile_bench.py --config c --nodes 5000 --pods 2000
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "kubernetes-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def compile_costs(fw, pods, reps=3):
    """{c_us_per_pod, marshal_us_per_pod, py_us_per_pod, one_us_per_pod} for `pods` on framework fw's compiler."""
    import ctypes as C

    import numpy as np
    from kgpu import abi, cdesc
    from kgpu.compile import Pools

    comp = fw.compiler
    L = cdesc.lib()
    n = len(pods)
    best = {}

    def keep(k, v):
        best[k] = min(best.get(k, float("inf")), v)

    for _ in range(reps):
        cdesc.clear_cache()
        cdesc._STR.clear()
        cdesc._Q.clear()
        t = time.perf_counter()
        descs = cdesc._arr(cdesc.PodDesc, [comp.pod_desc(p) for p in pods])
        keep("marshal_us_per_pod", (time.perf_counter() - t) / n * 1e6)
        pools = Pools()
        q = np.zeros(n, abi.QUERY)
        st = np.zeros(n, np.int32)
        t = time.perf_counter()
        rc = L.kgpu_compile_pods(comp._cc, pools.h, descs, n, q.ctypes.data, st.ctypes.data)
        keep("c_us_per_pod", (time.perf_counter() - t) / n * 1e6)
        assert rc == 0, comp._err()
        t = time.perf_counter()
        fw.compile_pods(pods)
        keep("py_us_per_pod", (time.perf_counter() - t) / n * 1e6)
        m = min(n, 200)
        pools = Pools()
        t = time.perf_counter()
        for p in pods[:m]:
            comp.compile_pod(p, pools)
        keep("one_us_per_pod", (time.perf_counter() - t) / m * 1e6)
    return {k: round(v, 3) for k, v in best.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="b")
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=2000)
    a = ap.parse_args()
    import bench
    from kgpu.framework import GpuFramework
    nodes, existing, init, pods, prof = bench._object_workload(a.config, a.nodes, a.pods)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16], device=0, create_engine=False)
    out = compile_costs(fw, pods)
    out.update({"config": a.config, "nodes": a.nodes, "pods": len(pods)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
