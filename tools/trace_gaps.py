#!/usr/bin/env python3
"""Idle time between consecutive kernels of a rocprofv3 kernel trace.

Reads the `*kernel_trace.csv` a `rocprofv3 --kernel-trace --output-format csv`
run wrote and reports, per kernel name, how often the GPU sat idle right
before that kernel started and for how long in total (gaps under --max-us
only: longer ones are the host between steps / timed regions).  A gap in
front of `duplicate_lds_kernel` is the host's K read-back in the forward.

usage: python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv [--max-us 200]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--max-us", type=float, default=200.0)
    args = ap.parse_args()
    path = args.trace
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    gaps = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    idle = 0.0
    for (s0, e0, _n0), (s1, e1, n1) in zip(rows, rows[1:]):
        g = (s1 - max(e0, s0)) / 1000.0
        if 0 < g < args.max_us:
            key = n1.split("(")[0][:80]
            gaps[key][0] += 1
            gaps[key][1] += g
            idle += g
        busy += (e1 - s1) / 1000.0
    out = {"trace": path, "kernels": len(rows), "busy_us": round(busy, 1), "idle_us_short_gaps": round(idle, 1),
           "by_next_kernel": {k: {"gaps": v[0], "total_us": round(v[1], 1), "avg_us": round(v[1] / v[0], 2)}
                              for k, v in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:15]}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
