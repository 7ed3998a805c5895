#!/usr/bin/env python3
"""Host-side cost of the config-3 frame (gaussian_renderer_amr render()'s five
_RasterizeGaussians calls + the four image sums): per call, the time the
Python call takes to return (it returns after enqueueing, except foveaStep 0,
which reads K back), next to the frame's wall time.  When the host time per
frame approaches the wall time, the frame is host-bound.

usage: python tools/host_overhead.py [--frames 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=50)
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    args = ap.parse_args()
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    from diff_gaussian_rasterization_amr import GaussianRasterizationSettings as AS, _RasterizeGaussians as AR
    dev = torch.device("cuda:0")
    cam = S.make_camera(args.W, args.H)
    sc = S.make_scene(args.P, cam, seed=0)
    st = AS(image_height=args.H, image_width=args.W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
            bg=torch.zeros(3, device=dev), scale_modifier=1.0,
            viewmatrix=torch.from_numpy(cam.world_view_transform).to(dev),
            projmatrix=torch.from_numpy(cam.full_proj_transform).to(dev), sh_degree=3,
            campos=torch.from_numpy(cam.camera_center).to(dev), prefiltered=False, debug=False)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(sc, k))).to(dev)
         for k in ("means3D", "opacities", "shs", "scales", "rotations")}
    e = torch.empty(0, device=dev)
    u8 = torch.empty(0, dtype=torch.uint8, device=dev)
    m2 = torch.zeros_like(t["means3D"])
    a = (t["means3D"], m2, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    host = np.zeros(9)  # step 0..4 calls, 4 adds

    def frame(rec):
        t0 = time.perf_counter()
        c, _, gb, bb, ib = AR.apply(*a, 0, e, u8, u8, u8, False, st)
        t1 = time.perf_counter()
        rec[0] += t1 - t0
        acc = c
        for k in range(1, 5):
            t0 = time.perf_counter()
            c, _, gb, bb, ib = AR.apply(*a, k, acc, gb, bb, ib, False, st)
            t1 = time.perf_counter()
            acc = acc + c
            t2 = time.perf_counter()
            rec[k] += t1 - t0
            rec[4 + k] += t2 - t1
        return acc

    with torch.no_grad():
        scratch = np.zeros(9)
        for _ in range(5):
            frame(scratch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.frames):
            frame(host)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    host_us = host / args.frames * 1e6
    print(json.dumps({"frames": args.frames, "wall_ms_per_frame": round(wall / args.frames * 1e3, 4),
                      "host_us_per_call": {"step0 (incl. K readback wait)": round(host_us[0], 1),
                                           **{f"step{k}": round(host_us[k], 1) for k in range(1, 5)},
                                           **{f"add{k}": round(host_us[4 + k], 1) for k in range(1, 5)}},
                      "host_us_steps1to4_and_adds": round(float(host_us[1:].sum()), 1)}))


if __name__ == "__main__":
    main()
