#!/usr/bin/env python3
"""Where render_bwd's waves wait: runs the blend
backward at a config's size under the instrumented variants ("bwd_variant"
12 = the default, 13 = its late-tail form) and prints, per variant, the
fractions of all wave-cycles spent in the record waits at the batch heads,
in the id waits ahead of the next batch's gathers and in the staging reduces
(s_memtime brackets, gs_debug_bwd_probe), beside the event times of the
plain and the instrumented kernels.

usage: python tools/bwd_probe.py [--P 1000000 --W 1920 --H 1080] [--iters 20]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import gaussian_splatting_with_eye_tracking_amd as pkg
    from gaussian_splatting_with_eye_tracking_amd import _C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    lib = ctypes.CDLL(os.path.join(os.path.dirname(pkg.__file__), "libgsplat_amd.so"))
    lib.gs_debug_bwd_probe.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    lib.gs_debug_bwd_probe.restype = ctypes.c_int

    dev = torch.device("cuda:0")
    cam = S.make_camera(args.W, args.H)
    sc = S.make_scene(args.P, cam, seed=0)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(sc, k))).to(dev)
         for k in ("means3D", "opacities", "shs", "scales", "rotations")}
    bg = torch.zeros(3, device=dev)
    vm = torch.from_numpy(cam.world_view_transform).to(dev)
    pm = torch.from_numpy(cam.full_proj_transform).to(dev)
    cp = torch.from_numpy(cam.camera_center).to(dev)
    e = torch.Tensor([])
    dpix = torch.from_numpy(S.make_cotangent(args.H, args.W, 1)).to(dev)
    K, color, radii, geom, binning, img = C.rasterize_gaussians(
        bg, t["means3D"], e, t["opacities"], t["scales"], t["rotations"], 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy,
        args.H, args.W, t["shs"], 3, cp, False, False)

    def backward():
        return C.rasterize_gaussians_backward(bg, t["means3D"], radii, e, t["scales"], t["rotations"], 1.0, e, vm, pm,
                                              cam.tanfovx, cam.tanfovy, dpix, t["shs"], 3, cp, geom, K, binning, img,
                                              False)

    buf = (ctypes.c_ulonglong * 8)()
    out = {"P": args.P, "W": args.W, "H": args.H, "iters": args.iters, "variants": {}}
    variants = [2, 3, 12, 13]
    times = {v: [] for v in variants}
    probes = {v: np.zeros(8, dtype=np.float64) for v in (12, 13)}
    try:
        for _ in range(args.rounds):
            for v in variants:
                C.set_tuning("bwd_variant", v)
                backward()
                torch.cuda.synchronize()
                if v in probes:
                    assert lib.gs_debug_bwd_probe(buf, 1) == 0
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.iters):
                    backward()
                b.record()
                torch.cuda.synchronize()
                times[v].append(a.elapsed_time(b) / args.iters)
                if v in probes:
                    assert lib.gs_debug_bwd_probe(buf, 1) == 0
                    probes[v] += np.array(list(buf), dtype=np.float64)
    finally:
        C.set_tuning("bwd_variant", -1)
    for v in variants:
        rec = {"backward_ms_median": float(np.median(times[v])), "backward_ms_min": float(np.min(times[v]))}
        if v in probes:
            p = probes[v]
            rec.update(wave_cycles_per_wave=p[0] / max(p[5], 1), batches_per_wave=p[4] / max(p[5], 1),
                       frac_record_wait=p[1] / p[0], frac_id_wait=p[2] / p[0], frac_stage_reduce=p[3] / p[0],
                       record_wait_cycles_per_batch=p[1] / max(p[4], 1), id_wait_cycles_per_batch=p[2] / max(p[4], 1))
        out["variants"][str(v)] = rec
        print(v, json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
