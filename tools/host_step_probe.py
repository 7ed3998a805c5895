#!/usr/bin/env python3
"""Host time of each call of the config-3 5-step frame (no syncs inside the
frame): where the host spends its time between GPU launches.

usage: python3 tools/host_step_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import bench
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    dev = torch.device("cuda:0")
    W, H, P = 1920, 1080, 1_000_000
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=0)
    st = bench.raster_settings(cam, dev, "diff_gaussian_rasterization_amr")
    t = bench.device_params(sc, dev, False)
    e = torch.empty(0, device=dev)
    u8 = torch.empty(0, dtype=torch.uint8, device=dev)
    a = (t["means3D"], torch.zeros_like(t["means3D"]), t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    rec = []
    with torch.no_grad():
        for it in range(30):
            ts = [time.perf_counter()]
            c_, _r, gb, bb, ib = _RasterizeGaussians.apply(*a, 0, e, u8, u8, u8, False, st)
            ts.append(time.perf_counter())
            acc = c_
            for k in range(1, 5):
                c_, _, gb, bb, ib = _RasterizeGaussians.apply(*a, k, acc, gb, bb, ib, False, st)
                ts.append(time.perf_counter())
                acc = acc + c_
                ts.append(time.perf_counter())
            torch.cuda.synchronize()
            ts.append(time.perf_counter())
            if it >= 10:
                rec.append(np.diff(ts) * 1e6)
    r = np.median(np.array(rec), axis=0)
    names = ["step0"] + [x for k in range(1, 5) for x in (f"step{k}", f"add{k}")] + ["sync_wait"]
    for n, v in zip(names, r):
        print(f"{n:10s} {v:8.1f} us")
    print("frame host total (to sync end)", round(float(np.sum(r)), 1))


if __name__ == "__main__":
    main()
