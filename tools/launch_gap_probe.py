#!/usr/bin/env python3
"""Launch-gap probe: does a kernel of this library start later after a
torch (foreign) kernel than after one of its own?  Runs config 3's
progressive step 1 repeatedly, (a) back to back, (b) each followed by a
torch add, (c) each followed by a torch add and then the library's tiny
set_tuning-free zero launch (gs_zero_words), under rocprofv3
--kernel-trace; prints the mean gap before each kernel kind.

usage: rocprofv3 --kernel-trace -d gpurun_out/gap -o run --output-format csv -- python3 tools/launch_gap_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    import bench
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    dev = torch.device("cuda:0")
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    W, H, P = 1920, 1080, 1_000_000
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=0)
    st = bench.raster_settings(cam, dev, "diff_gaussian_rasterization_amr")
    t = bench.device_params(sc, dev, False)
    e = torch.empty(0, device=dev)
    u8 = torch.empty(0, dtype=torch.uint8, device=dev)
    a = (t["means3D"], torch.zeros_like(t["means3D"]), t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    with torch.no_grad():
        c0, _, gb, bb, ib = _RasterizeGaussians.apply(*a, 0, e, u8, u8, u8, False, st)
        acc = c0
        torch.cuda.synchronize()
        for mode in range(3):
            for _ in range(20):
                c1, _, gb, bb, ib = _RasterizeGaussians.apply(*a, 1, acc, gb, bb, ib, False, st)
                if mode >= 1:
                    acc = acc + c1
                if mode == 2:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
