#!/usr/bin/env python3
"""One-GPU cost of the data-parallel view exchange (data_parallel.py) at
config 2: stage 1 (blend backward + view record) and the multi-view
parameter backward for V = 1, 2, 4, 8 gathered records (records of
different yawed views, config 5), next to the single-view per-Gaussian
backward (bwd_gauss) it replaces.  The all-gather itself needs N GPUs."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from gaussian_splatting_with_eye_tracking_amd import _C
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    dev = torch.device("cuda:0")
    P, W, H = 1_000_000, 1920, 1080
    cam0 = S.make_camera(W, H)
    sc = S.make_scene(P, cam0, seed=0)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(sc, k))).to(dev)
         for k in ("means3D", "opacities", "shs", "scales", "rotations")}
    e = torch.empty(0, device=dev)
    recs = []
    for v in range(8):
        cam = S.make_orbit_camera(W, H, (v - 3.5) * 5.0)
        st = GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
            bg=torch.zeros(3, device=dev), scale_modifier=1.0,
            viewmatrix=torch.from_numpy(cam.world_view_transform).to(dev),
            projmatrix=torch.from_numpy(cam.full_proj_transform).to(dev), sh_degree=3,
            campos=torch.from_numpy(cam.camera_center).to(dev), prefiltered=False, debug=False)
        dpix = torch.from_numpy(S.make_cotangent(H, W, 100 + v)).to(dev)
        fwd = _C.rasterize_gaussians(st.bg, t["means3D"], e, t["opacities"], t["scales"], t["rotations"], 1.0, e,
                                     st.viewmatrix, st.projmatrix, st.tanfovx, st.tanfovy, H, W, t["shs"], 3,
                                     st.campos, False, False)
        recs.append(DP.view_record(st, fwd[2], fwd[3], fwd[0], fwd[4], fwd[5], dpix))
        if v == 0:
            st0, fwd0, dpix0 = st, fwd, dpix
    views = torch.stack(recs)
    torch.cuda.synchronize()

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    out = {"P": P, "W": W, "H": H}
    out["full_backward_ms"] = timeit(lambda: _C.rasterize_gaussians_backward(
        st0.bg, t["means3D"], fwd0[2], e, t["scales"], t["rotations"], 1.0, e, st0.viewmatrix, st0.projmatrix,
        st0.tanfovx, st0.tanfovy, dpix0, t["shs"], 3, st0.campos, fwd0[3], fwd0[0], fwd0[4], fwd0[5], False))
    out["stage1_view_record_ms"] = timeit(lambda: DP.view_record(st0, fwd0[2], fwd0[3], fwd0[0], fwd0[4], fwd0[5],
                                                                 dpix0))
    for V in (1, 2, 4, 8):
        vv = views[:V].contiguous()
        out[f"multiview_V{V}_ms"] = timeit(lambda: DP.multiview_param_grads(vv, t["means3D"], t["shs"], 3,
                                                                            t["scales"], t["rotations"]))
    out["view_record_MB"] = DP.view_record_numel(P) * 4 / 1e6
    out["param_grads_MB"] = 59 * 4 * P / 1e6
    print(json.dumps(out))


if __name__ == "__main__":
    main()
