#!/usr/bin/env python3
"""Summarise rocprofv3 runs into profiles/ (committed evidence).

Inputs (written by tools/gpu_session.sh under gpurun_out/):
  prof_<config>/run_kernel_stats.csv             --kernel-trace --stats
  pmc_<config>_fetch/run_counter_collection.csv  --pmc FETCH_SIZE (own pass)
  pmc_<config>_write/run_counter_collection.csv  --pmc WRITE_SIZE (own pass)
  pmc_<config>_valu/run_counter_collection.csv   --pmc SQ_INSTS_VALU (own pass)

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads exactly half the bytes of
a wide (16 B/lane) coalesced stream, so the corrected read side is
2 x FETCH_SIZE.  That factor is calibrated only for 16-B/lane streams; the
raw values are kept next to the corrected ones.  Infinity-Cache hits are
counted as well (they are L2 misses), so traffic is "beyond-L2" bytes.

Per-configuration passes (tools/gpu_session.sh pmc2 / pmc3 / pmc4, prof2 /
prof3 / prof4) live in pmc_<config>_{fetch,write,valu}/ and
prof_<config>/; the summary then records the
configuration key (P, W, H, tile) that bench.py matches before it attaches
any traffic to a roofline.

usage: python tools/pmc_summary.py --tag r02 [--src gpurun_out] [--config cfg3_amr_1080p_1M]
"""
import argparse
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

STAGES = {
    "render_bwd_kernel": "render_bwd",
    "render_fwd_kernel": "render",
    "duplicate_kernel": "duplicate",
    "duplicate_lds_kernel": "duplicate",
    "count_tiles_kernel": "count_tiles",
    "backward_gaussians_kernel": "bwd_gauss",
    "preprocess_kernel": "preprocess",
    "sort_tiles_small_kernel": "sort_tiles",
    "sort_tiles_large_kernel": "sort_tiles_large",
    "tile_scan_kernel": "tile_scan",
    "amr_region_render_kernel<1,": "amr_render",
    "amr_region_render_kernel<4,": "amr_render_once",
    "amr_region_lists_kernel": "amr_lists",
    "sort_tiles_wide_kernel": "sort_tiles",
    "amr_quad_render_kernel<1>": "amr_render",
    "amr_quad_render_kernel<4>": "amr_render_once",
    "amr_quad_lists_kernel": "amr_lists",
    "amr_render_kernel": "amr_render",
    "amr_levels_kernel": "amr_levels",
    "amr_interpolate_kernel": "amr_interp",
    "multiview_backward_kernel": "multiview_bwd",
    "pack_view_grads_kernel": "pack_view",
}


def stage_of(name: str):
    for k, v in STAGES.items():
        if k in name:
            return v
    return None


def per_kernel(path, counter):
    vals = defaultdict(list)
    durs = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        st = stage_of(r["Kernel_Name"])
        if st:
            vals[st].append(float(r["Counter_Value"]))
            durs[st].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return vals, durs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--src", default="gpurun_out")
    ap.add_argument("--out", default="profiles")
    ap.add_argument("--config", default="cfg2_1080p_1M", help="bench.py configuration of the pmc_<config>_* passes")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    res = {"tag": args.tag, "units": "bytes per launch", "fetch_correction": 2.0,
           "note": "traffic = (2*FETCH_SIZE + WRITE_SIZE) KiB per launch (MI355X_MICROARCH.md §HBM)",
           "per_launch_hbm_bytes": {}, "raw_kib": {}}
    pre = f"pmc_{args.config}_"
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    c = bench.CONFIGS[args.config]
    res["config_name"] = args.config
    res["config"] = bench.config_key(c["P"], c["W"], c["H"], c["tile"])
    f = os.path.join(args.src, pre + "fetch", "run_counter_collection.csv")
    w = os.path.join(args.src, pre + "write", "run_counter_collection.csv")
    if os.path.exists(f) and os.path.exists(w):
        fv, _ = per_kernel(f, "FETCH_SIZE")
        wv, _ = per_kernel(w, "WRITE_SIZE")
        for st in sorted(set(fv) & set(wv)):
            fk = sum(fv[st]) / len(fv[st])
            wk = sum(wv[st]) / len(wv[st])
            res["raw_kib"][st] = {"FETCH_SIZE": fk, "WRITE_SIZE": wk, "launches": len(fv[st])}
            res["per_launch_hbm_bytes"][st] = (2.0 * fk + wk) * 1024.0
    # VALU issue: SQ_INSTS_VALU per launch (wave-instructions; own pass, see
    # tools/gpu_session.sh pmc_valu) -- the roofline of the blend kernels.
    v = os.path.join(args.src, pre + "valu", "run_counter_collection.csv")
    if os.path.exists(v):
        res["per_launch_valu_instructions"] = {}
        vv, _ = per_kernel(v, "SQ_INSTS_VALU")
        for st, xs in vv.items():
            res["per_launch_valu_instructions"][st] = sum(xs) / len(xs)
    stats = os.path.join(args.src, f"prof_{args.config}", "run_kernel_stats.csv")
    name = args.config.split("_")[0]
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(args.out, f"{args.tag}_{name}_kernel_stats.csv"))
        res["kernel_avg_us"] = {}
        for r in csv.DictReader(open(stats)):
            st = stage_of(r["Name"])
            if st:
                res["kernel_avg_us"][st] = float(r["AverageNs"]) / 1e3
    out = os.path.join(args.out, f"{args.tag}_{name}_pmc_summary.json")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
