#!/usr/bin/env python3
"""Turn tools/pmc_calib's two rocprofv3 passes into per-pattern factors:
counted bytes (FETCH_SIZE or WRITE_SIZE, KiB -> B) per byte the lanes asked
for and per 128-B line / 64-B row touched.  Writes profiles/<tag>_pmc_calib.json.

usage: python tools/pmc_calib.py --tag r02n [--src gpurun_out]
  expects <src>/calib.json (the probe's stdout),
          <src>/pmc_calib_fetch/run_counter_collection.csv,
          <src>/pmc_calib_write/run_counter_collection.csv
"""
import argparse
import csv
import json
import os


def counter_by_kernel(path: str, counter: str) -> dict:
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            out[name] = out.get(name, 0.0) + float(r["Counter_Value"]) * 1024.0
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--src", default="gpurun_out")
    a = ap.parse_args()
    probe = json.load(open(os.path.join(a.src, "calib.json")))["patterns"]
    fetch = counter_by_kernel(os.path.join(a.src, "pmc_calib_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counter_by_kernel(os.path.join(a.src, "pmc_calib_write", "run_counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for name, p in probe.items():
        k = p["kernel"]
        f, w = fetch.get(k), write.get(k)
        units = p.get("lines", p.get("rows"))
        unit = "line128" if "lines" in p else "row64"
        res[name] = {"asked_bytes": p["bytes"], unit: units,
                     "FETCH_bytes": f, "WRITE_bytes": w,
                     "FETCH_per_asked_byte": None if f is None else round(f / p["bytes"], 4),
                     "WRITE_per_asked_byte": None if w is None else round(w / p["bytes"], 4),
                     f"FETCH_per_{unit}": None if f is None else round(f / units, 2),
                     f"WRITE_per_{unit}": None if w is None else round(w / units, 2)}
    out = {"tag": a.tag, "source": "tools/pmc_calib.hip (1 GiB buffer, each line touched once)",
           "note": "counted bytes per asked byte; a factor of 0.5 on stream16 reproduces MI355X_MICROARCH.md "
                   "section HBM's x2 FETCH correction", "patterns": res}
    os.makedirs("profiles", exist_ok=True)
    dst = os.path.join("profiles", f"{a.tag}_pmc_calib.json")
    with open(dst, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
