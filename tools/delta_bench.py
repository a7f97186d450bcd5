"""Cost of keeping the device mirror coherent: kgpu_apply_delta vs a full re-upload.

Builds config (c)'s cluster (taints, zones, hostname labels, default profile) at --nodes nodes with
--existing running pods in a kgpu.cache.SchedulerCache, then times each kind of cache event:
host side (Python mirror + compile + the C call) and the C call alone, median of --reps syncs.
Writes one JSON line per event kind to stdout.

    python tools/delta_bench.py --nodes 100000 --existing 100000 --reps 20
"""
import argparse
import copy
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-1_amd"))

from kgpu import cluster  # noqa: E402
from kgpu.cache import SchedulerCache  # noqa: E402
from kgpu.compile import Profile  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=100000)
    ap.add_argument("--existing", type=int, default=100000)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    nodes, _, pods, _ = cluster.taints_affinity_spread(n_nodes=args.nodes, n_pods=args.existing + 2000)
    existing = []
    for i, p in enumerate(pods[:args.existing]):
        p = copy.deepcopy(p)
        p["spec"]["nodeName"] = nodes[(i * 7919) % len(nodes)]["metadata"]["name"]
        existing.append(p)
    fresh = pods[args.existing:]
    t0 = time.perf_counter()
    c = SchedulerCache(Profile(), nodes, existing, pods_hint=fresh[:10])
    t_build = time.perf_counter() - t0
    eng = c.engine
    call_t = []
    orig = eng.apply_delta

    def timed(batch, gen, n, keep=()):
        a = time.perf_counter()
        r = orig(batch, gen, n, keep)
        call_t.append(time.perf_counter() - a)
        return r

    eng.apply_delta = timed
    out = []

    def measure(kind, fn, reps=args.reps):
        host = []
        call_t.clear()
        for k in range(reps):
            fn(k)
            a = time.perf_counter()
            c.sync()
            host.append(time.perf_counter() - a)
        rec = {"event": kind, "nodes": len(c.list), "reps": reps,
               "sync_ms_median": round(1e3 * statistics.median(host), 4),
               "apply_delta_call_ms_median": round(1e3 * statistics.median(call_t), 4) if call_t else None,
               "uploads": c.uploads}
        out.append(rec)
        print(json.dumps(rec), flush=True)

    names = list(c.list)
    fi = iter(range(len(fresh)))

    def add_one(k):
        p = copy.deepcopy(fresh[next(fi)])
        p["spec"]["nodeName"] = names[(k * 104729) % len(names)]
        c.add_pod(p)
        added.append(p)

    added = []
    measure("pod_add", add_one)
    measure("pod_remove", lambda k: c.remove_pod(added.pop()))

    def add_100(k):
        for j in range(100):
            add_one(k * 100 + j)
    measure("pod_add_x100", add_100, reps=5)

    def node_update(k):
        nm = names[(k * 7) % len(names)]
        old = c.nodes[nm]
        new = copy.deepcopy(old)
        new["status"]["allocatable"]["cpu"] = str(8 + k % 4)
        new["spec"]["taints"] = [{"key": "spot", "value": "true", "effect": "PreferNoSchedule"}] if k % 2 else []
        c.update_node(old, new)
    measure("node_update", node_update)

    def node_add(k):
        n = cluster.node("extra%d" % k, "16", "64Gi", 110, "100Gi",
                         labels={cluster.ZONE: "zone%d" % (k % 10), cluster.HOSTNAME: "extra%d" % k})
        c.add_node(n)
    measure("node_add", node_add, reps=5)

    # full re-upload of the same state (compile + kgpu_upload_snapshot), for comparison
    host = []
    for k in range(3):
        a = time.perf_counter()
        c._upload(list(c.list))
        host.append(time.perf_counter() - a)
    up_call = []
    for k in range(3):
        snap, arrays = c._snap
        a = time.perf_counter()
        eng.upload(snap, arrays, c.generation)
        up_call.append(time.perf_counter() - a)
    rec = {"event": "full_reupload", "nodes": len(c.list), "compile_and_upload_ms_median": round(1e3 * statistics.median(host), 2),
           "upload_call_ms_median": round(1e3 * statistics.median(up_call), 2), "mirror_build_s": round(t_build, 2)}
    print(json.dumps(rec), flush=True)
    c.close()


if __name__ == "__main__":
    main()
