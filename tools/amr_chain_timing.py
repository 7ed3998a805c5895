"""Diagnostic: 5-step frame wall time, fused vs literal sequence (config 3).

usage: python tools/amr_chain_timing.py [mode ...]   modes: fused chain inline once (default: all)
(under rocprofv3 --kernel-trace with one mode, tools/frame_gaps.py splits the frame)"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from diff_gaussian_rasterization_amr import _RasterizeGaussians  # noqa: E402
from gaussian_splatting_with_eye_tracking_amd import rasterization_amr as RA  # noqa: E402

P, W, H = 1_000_000, 1920, 1080
args = bench.parse_args(["--no-cpu-baseline"])
ctx = bench.Ctx(1, 0, 0, False, torch.device("cuda:0"), args)
sc, cam = ctx.scene(P, W, H)
st = bench.raster_settings(cam, ctx.dev, "diff_gaussian_rasterization_amr")
t = bench.device_params(sc, ctx.dev, False)
e = torch.empty(0, device=ctx.dev)
u8 = torch.empty(0, dtype=torch.uint8, device=ctx.dev)
a = (t["means3D"], torch.zeros_like(t["means3D"]), t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)


def inline():
    c_, _r, gb, bb, ib = _RasterizeGaussians.apply(*a, 0, e, u8, u8, u8, False, st)
    acc = c_
    for k in range(1, 5):
        c_, _, gb, bb, ib = _RasterizeGaussians.apply(*a, k, acc, gb, bb, ib, False, st)
        acc = acc + c_
    return acc


fns = {"fused": lambda: RA.render_steps(*a, st, fused=True), "chain": lambda: RA.render_steps(*a, st, fused=False),
       "inline": inline,
       "once": lambda: RA.GaussianRasterizer(st)(means3D=a[0], means2D=a[1], opacities=a[4], shs=a[2], scales=a[5],
                                                 rotations=a[6], foveaStep=-2, interpolate_image=True)}
if sys.argv[1:2] == ["frames"]:
    # the bench's order (fused frames, then 10 chain frames, then timed chains
    # of growing length): the fixed per-measurement overhead is the intercept
    with torch.no_grad():
        for _ in range(100):
            fns["fused"]()
        for _ in range(10):
            fns["chain"]()
        for n in (20, 50, 100, 20, 50, 100):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                fns["chain"]()
            torch.cuda.synchronize()
            print("chain", n, "%.4f ms/frame" % ((time.perf_counter() - t0) / n * 1e3), flush=True)
    sys.exit(0)
want = sys.argv[1:] or list(fns)
fns = {k: v for k, v in fns.items() if k in want}
with torch.no_grad():
    for _ in range(300):
        for f in fns.values():
            f()
    for rep in range(3):
        for name, f in fns.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(50):
                f()
            torch.cuda.synchronize()
            print(rep, name, "%.4f ms/frame" % ((time.perf_counter() - t0) / 50 * 1e3), flush=True)
