#!/usr/bin/env python3
"""Per-frame timeline of the config-3 5-step frame from a rocprofv3 kernel
trace: for every frame (preprocess ... the 4th amr_region_render_kernel<1>)
the span, the summed kernel time, and the median idle gap in front of each
kernel of the frame.

usage: python tools/frame_gaps.py gpurun_out/trace_cfg3/run_kernel_trace.csv
"""
import csv
import statistics
import sys
from collections import defaultdict


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "").replace("gsamd::", "")[:48]


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    frames = []
    i = 0
    while i < len(ks):
        if ks[i][0].startswith("preprocess_kernel"):
            j, nstep = i + 1, 0
            while j < len(ks) and not ks[j][0].startswith("preprocess_kernel"):
                if ks[j][0].startswith("amr_region_render_kernel<1>"):
                    nstep += 1
                    if nstep == 4:
                        break
                j += 1
            if nstep == 4 and j < len(ks):
                frames.append(ks[i:j + 1])
                i = j + 1
                continue
        i += 1
    if not frames:
        print("no 5-step frames found")
        return
    # frames of the timed fused loop: the most common kernel sequence
    sig = defaultdict(list)
    for f in frames:
        sig[tuple(k[0] for k in f)].append(f)
    seq, fs = max(sig.items(), key=lambda kv: len(kv[1]))
    fs = fs[len(fs) // 4:]  # past the ramp
    span = [(f[-1][2] - f[0][1]) / 1e3 for f in fs]
    busy = [sum(k[2] - k[1] for k in f) / 1e3 for f in fs]
    print(f"{len(fs)} frames of {len(seq)} kernels: span median {statistics.median(span):.1f} us, "
          f"kernels {statistics.median(busy):.1f} us")
    for p, name in enumerate(seq):
        gap = statistics.median([(f[p][1] - f[p - 1][2]) / 1e3 if p else 0.0 for f in fs])
        dur = statistics.median([(f[p][2] - f[p][1]) / 1e3 for f in fs])
        print(f"  {name:48s} gap {gap:6.1f} us  kernel {dur:6.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
