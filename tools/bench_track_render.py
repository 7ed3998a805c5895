#!/usr/bin/env python3
"""The whole eye-tracking -> foveated-render loop on 1 x MI355X (what the
reference's track_render.py sketches with TODOs):

  8-bit eye frame (host) -> upload -> gamma + CLAHE + normalise (GPU) ->
  RITnet segmentation (GPU) -> pupil centroid (24-B read-back) -> fovea
  centre on the 1080p screen -> AMR step 0 (preprocess, binning, levels) ->
  fovea discs clamp the tile levels -> AMR steps 1..4 summed -> frame.

RITnet runs with random weights of the reference's shapes (the checkpoint is
not part of this repository: timing only); the scene is config 3's synthetic
1M Gaussians.  Prints one JSON line.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import ritnet_oracle as R
    from diff_gaussian_rasterization_amr import GaussianRasterizationSettings, _RasterizeGaussians
    from gaussian_splatting_with_eye_tracking_amd import eye_tracking as E
    from gaussian_splatting_with_eye_tracking_amd import rasterization_amr as RA
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S

    dev = torch.device("cuda:0")
    eye = np.load(os.path.join(ROOT, "tests", "golden", "eye_pins.npz"))["eye"]
    net = E.RITnet(R.random_state_dict(0))
    P, W, H = 1_000_000, 1920, 1080
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=0)
    st = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, bg=torch.zeros(3, device=dev),
        scale_modifier=1.0, viewmatrix=torch.from_numpy(cam.world_view_transform).to(dev),
        projmatrix=torch.from_numpy(cam.full_proj_transform).to(dev), sh_degree=3,
        campos=torch.from_numpy(cam.camera_center).to(dev), prefiltered=False, debug=False)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(sc, k))).to(dev)
         for k in ("means3D", "opacities", "shs", "scales", "rotations")}
    e = torch.empty(0, device=dev)
    u8 = torch.empty(0, dtype=torch.uint8, device=dev)
    a = (t["means3D"], torch.zeros_like(t["means3D"]), t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)

    def frame(gray):
        _, _, fovea = E.track(net, gray, (W, H))
        c, _, gb, bb, ib = _RasterizeGaussians.apply(*a, 0, e, u8, u8, u8, False, st)
        # no pupil found (possible with random weights): the reference's
        # image-centre discs
        centres, radii = RA.reference_foveae(W, H, fovea)
        RA.apply_fovea_levels(ib, W, H, centres, radii)
        acc = c
        for k in range(1, 5):
            ck, _, gb, bb, ib = _RasterizeGaussians.apply(*a, k, acc, gb, bb, ib, False, st)
            acc = acc + ck
        return acc, fovea

    with torch.no_grad():
        for _ in range(3):
            frame(eye)
        torch.cuda.synchronize()
        n = 30
        t0 = time.perf_counter()
        for _ in range(n):
            img, fovea = frame(eye)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        t0 = time.perf_counter()
        for _ in range(n):
            E.track(net, eye, (W, H))
        torch.cuda.synchronize()
        dt_track = (time.perf_counter() - t0) / n
    print(json.dumps({"metric": "eye frame -> foveated 1080p frame (track + 5-step AMR with fovea levels)",
                      "frames_per_s": round(1.0 / dt, 1), "ms_per_frame": round(dt * 1e3, 3),
                      "track_ms": round(dt_track * 1e3, 3), "render_ms": round((dt - dt_track) * 1e3, 3),
                      "fovea": None if fovea is None else [round(v, 2) for v in fovea],
                      "config": {"eye": "640x400 (reference eye.png)", "ritnet_weights": "random (timing only)",
                                 "P": P, "width": W, "height": H}}))


if __name__ == "__main__":
    main()
