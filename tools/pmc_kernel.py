#!/usr/bin/env python3
"""Mean of every counter per kernel from rocprofv3 --pmc counter_collection
CSVs (one or more passes), for kernels whose name contains a substring.

usage: python tools/pmc_kernel.py <dir-or-csv> [...] [--match render_bwd] [--json]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--json", action="store_true")
    args = ap.parse_args()
    files = []
    for p in args.paths:
        files += sorted(glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True)) \
            if os.path.isdir(p) else [p]
    vals = defaultdict(lambda: defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if args.match and args.match not in k:
                continue
            k = k.split("(")[0][:90]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
    if args.json:
        print(json.dumps(out, indent=1))
        return
    for k, cs in out.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"  {c:28s} {v:16.1f}")


if __name__ == "__main__":
    main()
