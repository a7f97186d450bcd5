#!/usr/bin/env python3
"""cProfile of the HTTP extender's verbs (kgpu/extender.py) per pod, in process: where a
filter -> prioritize -> bind cycle spends its host time.  GPU box:
  python tools/extender_profile.py --config b --nodes 5000 --pods 40
"""
import argparse
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "kubernetes-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="b")
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=40)
    a = ap.parse_args()
    import bench
    nodes, existing, init, pods, prof = bench._object_workload(a.config, a.nodes, a.pods)
    bench.extender_cycles(prof, nodes, existing, pods[:2], 0)  # code objects, first sync
    pr = cProfile.Profile()
    pr.enable()
    rec = bench.extender_cycles(prof, nodes, existing, pods, 0)
    pr.disable()
    print(rec)
    pstats.Stats(pr).sort_stats("cumulative").print_stats(35)


if __name__ == "__main__":
    main()
