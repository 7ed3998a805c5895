#!/usr/bin/env python3
"""Wave-cycle attribution of the blend kernels from rocprofv3 --pmc passes
(tools/gpu_session.sh sqc<N> / sqd<N>) into profiles/.

Per kernel (mean per launch over the passes' dispatches):
  * the disjoint split of SQ_WAVE_CYCLES (MI355X_MICROARCH.md SQ table):
      active  = SQ_ACTIVE_INST_ANY   (issuing)
      parked  = SQ_WAIT_ANY          (s_waitcnt / barrier)
      stalled = SQ_WAIT_INST_ANY     (issue-stalled; SQ_WAIT_INST_LDS is its LDS part)
    and the fraction of SQ_WAVE_CYCLES the three account for;
  * the issue mix inside `active`: SQ_ACTIVE_INST_{VALU,SCA,LDS} / WAVE_CYCLES;
  * LDS: instructions and bank-conflict cycles per instruction;
  * L2: TCC hit rate (TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)).
All SQ cycle counters are quad-cycles summed over the chip (the same unit in
every ratio here).

usage: python tools/sq_summary.py --tag r06a --config cfg2_1080p_1M [--src gpurun_out] [--kernels render_bwd_kernel render_fwd_kernel]
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short_name  # noqa: E402


def load(path):
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        vals[short_name(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def summarise(passes, want):
    out = {}
    for vals in passes:
        for k, cs in vals.items():
            if not any(w in k for w in want):
                continue
            d = out.setdefault(k, {})
            for c, xs in cs.items():
                d[c] = {"launches": len(xs), "mean": sum(xs) / len(xs)}
    res = {}
    for k, d in out.items():
        m = {c: v["mean"] for c, v in d.items()}
        r = {"counters": d}
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            act, park, stall = m.get("SQ_ACTIVE_INST_ANY"), m.get("SQ_WAIT_ANY"), m.get("SQ_WAIT_INST_ANY")
            if None not in (act, park, stall):
                r["wave_cycles"] = {"active": act / wc, "parked_waitcnt_barrier": park / wc,
                                    "issue_stalled": stall / wc, "accounted": (act + park + stall) / wc}
                if "SQ_WAIT_INST_LDS" in m:
                    r["wave_cycles"]["issue_stalled_lds"] = m["SQ_WAIT_INST_LDS"] / wc
                r["active_mix"] = {n: m[c] / wc for n, c in (("valu", "SQ_ACTIVE_INST_VALU"),
                                                               ("scalar", "SQ_ACTIVE_INST_SCA"),
                                                               ("lds", "SQ_ACTIVE_INST_LDS")) if c in m}
        if "SQ_INSTS_LDS" in m and m["SQ_INSTS_LDS"]:
            r["lds"] = {"insts": m["SQ_INSTS_LDS"],
                        "bank_conflict_cycles_per_inst": m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_INSTS_LDS"]}
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            tot = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
            r["l2"] = {"hit": m["TCC_HIT_sum"], "miss": m["TCC_MISS_sum"], "hit_rate": m["TCC_HIT_sum"] / tot if tot else None}
        res[k] = r
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--config", default="cfg2_1080p_1M")
    ap.add_argument("--src", default="gpurun_out")
    ap.add_argument("--out", default="profiles")
    ap.add_argument("--kernels", nargs="*", default=["render_bwd_kernel", "render_fwd_kernel"])
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    passes = []
    for p in ("sqc", "sqd"):
        f = os.path.join(a.src, f"{p}{a.config[3]}_{a.config}", "run_counter_collection.csv")
        if os.path.exists(f):
            passes.append(load(f))
    res = summarise(passes, a.kernels)
    dig = os.path.join(a.src, "build_digest.txt")
    res["_meta"] = {"tag": a.tag, "config": a.config, "note": a.note,
                    "build": open(dig).read().strip() if os.path.exists(dig) else None,
                    "units": "SQ cycle counters in quad-cycles summed over the chip; means per launch"}
    name = a.config.split("_")[0]
    out = os.path.join(a.out, f"{a.tag}_{name}_sq_counters.json")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, r in res.items():
        if k != "_meta":
            print(k, json.dumps({x: r.get(x) for x in ("wave_cycles", "active_mix", "lds", "l2")}, indent=None))


if __name__ == "__main__":
    main()
