#!/usr/bin/env python3
"""HBM traffic per launch of the dominant kernel from per-pass rocprofv3 --pmc runs
(tools/gpu_pmc1.sh -> gpurun_out/pmc2_<config>_<nodes>_<COUNTER>/run_counter_collection.csv).

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch; FETCH_SIZE is doubled per the gfx950
correction in MI355X_MICROARCH.md (HBM section).  Writes profiles/r02_pmc_traffic.json (keys
'<config>:<nodes>:<pods_per_launch>', as bench.py reads them) and copies the counter CSVs to
profiles/r02_pmc_<config><nodes>_<COUNTER>.csv."""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_batch"


def mean_kib(path):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"]]
    return sum(vals) / len(vals), len(vals)


def main():
    out = {"_doc": __doc__.strip().replace("\n", " ")}
    pods = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    for cfg, nodes in (("b", 5000), ("b", 100000)):
        d = {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            src = os.path.join(ROOT, "gpurun_out", "pmc2_%s_%d_%s" % (cfg, nodes, ctr), "run_counter_collection.csv")
            if not os.path.exists(src):
                break
            d[ctr] = mean_kib(src)
            shutil.copy(src, os.path.join(ROOT, "profiles", "r02_pmc_%s%d_%s.csv" % (cfg, nodes, ctr)))
        if len(d) < 2:
            continue
        fetch, nf = d["FETCH_SIZE"]
        write, nw = d["WRITE_SIZE"]
        out["%s:%d:%d" % (cfg, nodes, pods)] = {
            "kernel": KERNEL, "launches": [nf, nw], "fetch_kib_raw": fetch, "write_kib": write,
            "traffic_bytes_per_launch": int(round((2.0 * fetch + write) * 1024))}
    with open(os.path.join(ROOT, "profiles", "r02_pmc_traffic.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
