#!/usr/bin/env python3
"""Summarise rocprofv3 runs into profiles/ (committed evidence).

Inputs (written by tools/gpu_session.sh under gpurun_out/):
  prof_<config>/run_kernel_stats.csv             --kernel-trace --stats
  pmc_<config>_fetch/run_counter_collection.csv  --pmc FETCH_SIZE (own pass)
  pmc_<config>_write/run_counter_collection.csv  --pmc WRITE_SIZE (own pass)
  pmc_<config>_valu/run_counter_collection.csv   --pmc SQ_INSTS_VALU (own pass)
  build_digest.txt                                the source digest of the build that ran

Everything is keyed by the FULL kernel name first ("kernels"); a stage
("sort_tiles", "amr_render", ...) is then the launch-weighted sum over its
kernels per invocation of the stage:

    stage value = sum_k (mean value per launch of kernel k x launches of k)
                  / launches of the stage's most-launched kernel

so a stage made of several kernels (sort_tiles = sort_tiles_small<E> for
each E + sort_tiles_wide, launched once each per forward) reports their sum,
never one of them and never a mean mixing different kernels.  Durations
(kernel_avg_us) follow the same rule from the --stats table.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads half the bytes of a wide
coalesced stream, so per_launch_hbm_bytes = 2 x FETCH + WRITE.  For gather
patterns that factor overstates (profiles/r02n_pmc_calib.json); bench.py
uses the raw values with its gather calibration for the blend kernels.  Any
stage whose traffic / duration implies more than 6.3 TB/s is listed under
"implausible" (a mapping error, not evidence).

The summary records the configuration key (P, W, H, tile) and the build
digest; bench.py attaches a summary only to a line of the same
configuration AND the same build.

usage: python tools/pmc_summary.py --tag r03a [--src gpurun_out] [--config cfg3_amr_1080p_1M]
"""
import argparse
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict

# substring of the kernel name -> stage (first match wins; more specific first)
STAGES = [
    ("render_bwd_kernel", "render_bwd"),
    ("render_fwd_kernel", "render"),
    ("duplicate_lds_kernel", "duplicate"),
    ("band_stage_kernel", "duplicate"),
    ("band_split_kernel", "duplicate"),
    ("duplicate_kernel", "duplicate"),
    ("count_tiles_kernel", "count_tiles"),
    ("backward_gaussians_kernel", "bwd_gauss"),
    ("backward_gaussians_drgb_kernel", "bwd_gauss"),
    ("sh_backward_kernel", "bwd_gauss"),
    ("preprocess_kernel", "preprocess"),
    ("sort_tiles_small_kernel", "sort_tiles"),
    ("sort_tiles_wide_kernel", "sort_tiles"),
    ("sort_tiles_large_kernel", "sort_tiles"),
    ("sort_tiles_radix_kernel", "sort_tiles"),
    ("sort_tiles_bucket_kernel", "sort_tiles"),
    ("sort_tiles_mixed_kernel", "sort_tiles"),
    ("tile_scan", "tile_scan"),
    ("amr_region_render_kernel<1", "amr_render"),
    ("amr_region_render_kernel<4", "amr_render_once"),
    ("amr_region_lists_kernel", "amr_lists"),
    ("amr_levels_kernel", "amr_levels"),
    ("amr_interpolate_kernel", "amr_interp"),
    ("multiview_backward", "multiview_bwd"),
    ("pack_view_grads_kernel", "pack_view"),
]

PLAUSIBLE_MAX_BPS = 6.3e12  # above this a stage's bytes / time is not a measurement


def stage_of(name: str):
    for k, v in STAGES:
        if k in name:
            return v
    return None


def short_name(name: str) -> str:
    """Kernel name without the argument list ("void ns::k<1, 4>(int, ...)" -> "ns::k<1, 4>")."""
    n = re.sub(r"^void\s+", "", name.strip())
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return n[:i]
    return n


def counter_by_kernel(path: str, counter: str) -> dict:
    """{short kernel name: [value per dispatch]} of one --pmc pass."""
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        vals[short_name(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return dict(vals)


def stats_by_kernel(path: str) -> dict:
    """{short kernel name: (calls, average ns)} of a --stats table."""
    out = {}
    for r in csv.DictReader(open(path)):
        out[short_name(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]))
    return out


def stage_sum(per_kernel: dict) -> dict:
    """per_kernel: {kernel: (launches, mean value per launch)} -> {stage:
    value per stage invocation}, the launch-weighted sum over the stage's
    kernels divided by the launches of its most-launched kernel."""
    groups = defaultdict(list)
    for k, (n, mean) in per_kernel.items():
        st = stage_of(k)
        if st and n > 0:
            groups[st].append((n, mean))
    out = {}
    for st, xs in groups.items():
        primary = max(n for n, _ in xs)
        out[st] = sum(n * m for n, m in xs) / primary
    return out


def summarise(fetch=None, write=None, valu=None, stats=None) -> dict:
    """The per-kernel and per-stage tables from the parsed passes (each a
    {kernel: [values]} dict, stats a {kernel: (calls, avg ns)} dict)."""
    res = {"kernels": {}, "per_launch_hbm_bytes": {}, "raw_kib": {}, "implausible": {}}
    kern = res["kernels"]

    def mean(xs):
        return sum(xs) / len(xs)

    for field, src in (("FETCH_SIZE_kib", fetch), ("WRITE_SIZE_kib", write), ("SQ_INSTS_VALU", valu)):
        for k, xs in (src or {}).items():
            if stage_of(k):
                kern.setdefault(k, {"stage": stage_of(k)})[field] = {"launches": len(xs), "mean": mean(xs)}
    for k, (calls, avg) in (stats or {}).items():
        if stage_of(k):
            kern.setdefault(k, {"stage": stage_of(k)})["stats"] = {"calls": calls, "avg_us": avg / 1e3}

    def stage_of_field(field):
        return stage_sum({k: (v[field]["launches"], v[field]["mean"]) for k, v in kern.items() if field in v})

    fk, wk = stage_of_field("FETCH_SIZE_kib"), stage_of_field("WRITE_SIZE_kib")
    for st in sorted(set(fk) & set(wk)):
        res["raw_kib"][st] = {"FETCH_SIZE": fk[st], "WRITE_SIZE": wk[st],
                              "kernels": sorted(k for k, v in kern.items() if v["stage"] == st)}
        res["per_launch_hbm_bytes"][st] = (2.0 * fk[st] + wk[st]) * 1024.0
    if valu:
        res["per_launch_valu_instructions"] = stage_of_field("SQ_INSTS_VALU")
    if stats:
        res["kernel_avg_us"] = stage_sum({k: (v["stats"]["calls"], v["stats"]["avg_us"])
                                          for k, v in kern.items() if "stats" in v})
        for st, b in res["per_launch_hbm_bytes"].items():
            us = res["kernel_avg_us"].get(st)
            if us and b / (us * 1e-6) > PLAUSIBLE_MAX_BPS:
                res["implausible"][st] = {"bytes": b, "avg_us": us, "implied_TBps": b / (us * 1e-6) / 1e12}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--src", default="gpurun_out")
    ap.add_argument("--out", default="profiles")
    ap.add_argument("--config", default="cfg2_1080p_1M", help="bench.py configuration of the pmc_<config>_* passes")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    pre = os.path.join(args.src, f"pmc_{args.config}_")

    def load(kind, counter):
        p = pre + kind + os.sep + "run_counter_collection.csv"
        return counter_by_kernel(p, counter) if os.path.exists(p) else None

    stats_p = os.path.join(args.src, f"prof_{args.config}", "run_kernel_stats.csv")
    stats = stats_by_kernel(stats_p) if os.path.exists(stats_p) else None
    res = summarise(load("fetch", "FETCH_SIZE"), load("write", "WRITE_SIZE"), load("valu", "SQ_INSTS_VALU"), stats)
    c = bench.CONFIGS[args.config]
    dig_p = os.path.join(args.src, "build_digest.txt")
    res.update({"tag": args.tag, "units": "per stage invocation (launch-weighted sum over the stage's kernels)",
                "fetch_correction": 2.0, "config_name": args.config,
                "config": bench.config_key(c["P"], c["W"], c["H"], c["tile"], c.get("views", 1)),
                "build": open(dig_p).read().strip() if os.path.exists(dig_p) else bench.build_digest(),
                "note": "per_launch_hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB (MI355X_MICROARCH.md §HBM)"})
    name = args.config.split("_")[0]
    if stats is not None:
        shutil.copy(stats_p, os.path.join(args.out, f"{args.tag}_{name}_kernel_stats.csv"))
    out = os.path.join(args.out, f"{args.tag}_{name}_pmc_summary.json")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: res[k] for k in ("build", "config", "kernel_avg_us", "per_launch_hbm_bytes", "implausible")
                      if k in res}, indent=1, sort_keys=True))
    if res["implausible"]:
        print("WARNING: implausible stages (check STAGES):", sorted(res["implausible"]), file=sys.stderr)


if __name__ == "__main__":
    main()
