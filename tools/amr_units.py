#!/usr/bin/env python3
"""Config 3 AMR work units: per-step distribution of the 8x8-region sub-list
lengths of the units each progressive step renders (the step time follows
its longest unit, render.hip amr_region_render_kernel).  GPU box tool."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from gaussian_splatting_with_eye_tracking_amd import _C  # noqa: E402
from gaussian_splatting_with_eye_tracking_amd import synthetic as S  # noqa: E402


def main():
    P, W, H = 1_000_000, 1920, 1080
    dev = torch.device("cuda", 0)
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=0)
    st = bench.raster_settings(cam, dev, "diff_gaussian_rasterization_amr")
    t = bench.device_params(sc, dev, False)
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    e = torch.empty(0, device=dev)
    u8 = torch.empty(0, dtype=torch.uint8, device=dev)
    m2 = torch.zeros_like(t["means3D"])
    a = (t["means3D"], m2, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    with torch.no_grad():
        c0, _, gb, bb, ib = _RasterizeGaussians.apply(*a, 0, e, u8, u8, u8, False, st)
        torch.cuda.synchronize()
    K = int(_C.parse_buffers(gb, bb, ib, P, 0, W, H, 32)["hdr"][0].item())
    d = _C.parse_buffers(gb, bb, ib, P, K, W, H, 32)
    rng = d["ranges"].cpu().numpy().astype(np.int64)
    n = rng[:, 1] - rng[:, 0]
    lv = np.minimum(d["levels"].cpu().numpy(), 4)
    rc = d["region_count"].cpu().numpy().astype(np.int64)
    out = {"K": K, "tiles": int(n.size), "tile_n": {"mean": float(n.mean()), "max": int(n.max())},
           "region_cnt": {"mean": float(rc.mean()), "max": int(rc.max()), "p99": float(np.percentile(rc, 99)),
                          "sum_over_K": float(rc.sum() / max(K, 1))}}
    for k in range(1, 5):
        act = lv >= k
        wave_max = rc[act].reshape(-1, 4, 4)  # rows of regions; a wave = a quadrant: regions (2r..2r+1, 2c..2c+1)
        q = np.stack([rc[act][:, [0, 1, 4, 5]], rc[act][:, [2, 3, 6, 7]], rc[act][:, [8, 9, 12, 13]],
                      rc[act][:, [10, 11, 14, 15]]], 1).max(-1)
        out[f"step{k}"] = {"tiles": int(act.sum()), "unit_max_list": {"max": int(q.max()), "p99": float(np.percentile(q, 99)),
                                                                     "mean": float(q.mean())},
                           "sum_unit_max": int(q.sum())}
        del wave_max
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
