#!/usr/bin/env python3
"""HBM traffic per launch of the dominant kernel from per-pass rocprofv3 --pmc runs
(tools/gpu_r5_prof.sh -> gpurun_out/<run>/pmc_<config>_<nodes>_<COUNTER>/run_counter_collection.csv):
k_batch for configs a and b, k_tbatch for configs c, d and e.

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch; FETCH_SIZE is doubled per the gfx950 correction in
MI355X_MICROARCH.md (HBM section).  Writes profiles/<tag>_pmc_traffic.json (keys
'<config>:<nodes>:<pods_per_launch>', as bench.py reads them) and copies the counter CSVs to
profiles/<tag>_pmc_<config><nodes>_<COUNTER>.csv.

Usage: tools/pmc_summary.py <gpurun_out run dir> <tag> [pods_per_launch]"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"a": "k_batch", "b": "k_batch", "c": "k_tbatch", "d": "k_tbatch", "e": "k_tbatch"}


def mean_kib(path, kernel):
    # the persistent kernel itself (k_batch<...> / k_tbatch<...>), not k_batch_fixup / k_tbatch_init
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Kernel_Name"].split("(")[0].split("<")[0].endswith("::" + kernel)]
    return sum(vals) / len(vals), len(vals)


def main():
    run, tag = sys.argv[1], sys.argv[2]
    pods = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    out = {"_doc": __doc__.strip().replace("\n", " ")}
    # every pmc_<config>_<nodes>_<COUNTER> pass directory of the run
    pairs = sorted({(e.split("_")[1], int(e.split("_")[2])) for e in os.listdir(run)
                    if e.startswith("pmc_") and len(e.split("_")) >= 4})
    for cfg, nodes in pairs:
        d = {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            src = os.path.join(run, "pmc_%s_%d_%s" % (cfg, nodes, ctr), "run_counter_collection.csv")
            if not os.path.exists(src):
                break
            d[ctr] = mean_kib(src, KERNELS[cfg])
            shutil.copy(src, os.path.join(ROOT, "profiles", "%s_pmc_%s%d_%s.csv" % (tag, cfg, nodes, ctr)))
        if len(d) < 2:
            continue
        fetch, nf = d["FETCH_SIZE"]
        write, nw = d["WRITE_SIZE"]
        out["%s:%d:%d" % (cfg, nodes, pods)] = {
            "kernel": KERNELS[cfg], "launches": [nf, nw], "fetch_kib_raw": fetch, "write_kib": write,
            "traffic_bytes_per_launch": int(round((2.0 * fetch + write) * 1024))}
    with open(os.path.join(ROOT, "profiles", "%s_pmc_traffic.json" % tag), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
