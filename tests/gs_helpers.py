"""Shared test helpers: build identical inputs for the HIP path and the oracle,
and tolerance checks with the tolerances of BASELINE.json's north_star."""
from __future__ import annotations

import numpy as np

from gaussian_splatting_with_eye_tracking_amd import synthetic as S

# north_star: image L1 < 1e-5, gradients within 1e-4 relative.
IMAGE_L1_TOL = 1e-5
GRAD_REL_TOL = 1e-4


def scene_and_camera(P: int, W: int, H: int, seed: int = 0, **kw):
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=seed, **kw)
    return sc, cam


def torch_settings(cam, device="cuda", bg=(0.0, 0.0, 0.0), sh_degree=3, scale_modifier=1.0, debug=False,
                   amr=False):
    import torch
    if amr:
        from diff_gaussian_rasterization_amr import GaussianRasterizationSettings
    else:
        from diff_gaussian_rasterization import GaussianRasterizationSettings
    return GaussianRasterizationSettings(
        image_height=int(cam.image_height), image_width=int(cam.image_width), tanfovx=cam.tanfovx,
        tanfovy=cam.tanfovy, bg=torch.tensor(bg, dtype=torch.float32, device=device), scale_modifier=scale_modifier,
        viewmatrix=torch.from_numpy(cam.world_view_transform).to(device),
        projmatrix=torch.from_numpy(cam.full_proj_transform).to(device), sh_degree=sh_degree,
        campos=torch.from_numpy(cam.camera_center).to(device), prefiltered=False, debug=debug)


def scene_tensors(sc, device="cuda", requires_grad=False):
    import torch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device).requires_grad_(requires_grad)  # noqa: E731
    return dict(means3D=t(sc.means3D), opacities=t(sc.opacities), shs=t(sc.shs), scales=t(sc.scales),
                rotations=t(sc.rotations))


def image_l1(a, b) -> float:
    return float(np.mean(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))))


def rel_err(a, b) -> float:
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    den = np.linalg.norm(b)
    if den == 0:
        return float(np.linalg.norm(a))
    return float(np.linalg.norm(a - b) / den)
