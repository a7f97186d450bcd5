#!/usr/bin/env python3
"""One kgpu_schedule_one cycle, call by call, from a rocprofv3 `--hip-trace --kernel-trace` run of
tools/latency_probe.py: every cycle starts with the entry's hipSetDevice.  Prints the median over the
last `--cycles` cycles of each step's start offset and duration (API calls on the calling thread,
kernels on the device), then the median cycle length.

    python tools/cycle_timeline.py gpurun_out/<run>/lat_trace_c [--cycles 100]"""
import argparse
import csv
import glob
import os
import statistics


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--cycles", type=int, default=100)
    a = ap.parse_args()
    api = rows(glob.glob(os.path.join(a.dir, "*hip_api_trace.csv"))[0])
    ker = rows(glob.glob(os.path.join(a.dir, "*kernel_trace.csv"))[0])
    ev = [("api", r["Function"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in api
          if not r["Function"].startswith("__hip")]
    ev += [("gpu", r["Kernel_Name"].split("(")[0][:60], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
           for r in ker]
    ev.sort(key=lambda e: e[2])
    starts = [e[2] for e in ev if e[0] == "api" and e[1] == "hipSetDevice"]
    starts = starts[-(a.cycles + 1):]
    cyc = []
    for s, t in zip(starts, starts[1:]):
        cyc.append([(k, n, b - s, e - b) for (k, n, b, e) in ev if s <= b < t])
    sig = [tuple((k, n) for k, n, _, _ in c) for c in cyc]
    common = statistics.mode(sig)
    same = [c for c, sg in zip(cyc, sig) if sg == common]
    print("cycles %d, %d with the common shape; median cycle %.1f us" %
          (len(cyc), len(same), statistics.median(t - s for s, t in zip(starts, starts[1:])) / 1e3))
    for j, (k, n) in enumerate(common):
        off = statistics.median(c[j][2] for c in same) / 1e3
        dur = statistics.median(c[j][3] for c in same) / 1e3
        print("%8.1f us  %7.1f us  %-3s %s" % (off, dur, k, n))


if __name__ == "__main__":
    main()
