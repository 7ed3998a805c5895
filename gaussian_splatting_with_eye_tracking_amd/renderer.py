"""The renderer glue -- the drop-in for ``gaussian_renderer``
(``gaussian_renderer/__init__.py``, SURVEY §2 L3: the caller of the
rasterizer in train.py / render.py / fps_test.py).

``render(viewpoint_camera, pc, pipe, bg_color, scaling_modifier=1.0,
override_color=None, starter=None, ender=None)`` -> the reference's dict
(``render``, ``viewspace_points``, ``visibility_filter``, ``radii``), through
``rasterization.GaussianRasterizer``.  Duck-typed arguments as in
``renderer_amr`` (which shares ``_operands``).
"""
from __future__ import annotations

import math

import torch

from .rasterization import GaussianRasterizationSettings, GaussianRasterizer
from .sh_utils import eval_sh


def _operands(viewpoint_camera, pc, pipe, bg_color, scaling_modifier, override_color):
    """Settings and rasterizer operands, as the reference renderers build them
    (gaussian_renderer/__init__.py:25-84, gaussian_renderer_amr/__init__.py:33-96,
    :620-700)."""
    xyz = pc.get_xyz
    screenspace_points = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True, device=xyz.device) + 0
    try:
        screenspace_points.retain_grad()
    except RuntimeError:  # (no graph under torch.no_grad())
        pass
    settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=math.tan(viewpoint_camera.FoVx * 0.5), tanfovy=math.tan(viewpoint_camera.FoVy * 0.5), bg=bg_color,
        scale_modifier=scaling_modifier, viewmatrix=viewpoint_camera.world_view_transform,
        projmatrix=viewpoint_camera.full_proj_transform, sh_degree=pc.active_sh_degree,
        campos=viewpoint_camera.camera_center, prefiltered=False, debug=pipe.debug)
    scales = rotations = cov3D_precomp = None
    if pipe.compute_cov3D_python:
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales, rotations = pc.get_scaling, pc.get_rotation
    shs = colors_precomp = None
    if override_color is not None:
        colors_precomp = override_color
    elif pipe.convert_SHs_python:
        feats = pc.get_features
        shs_view = feats.transpose(1, 2).view(-1, 3, (pc.max_sh_degree + 1) ** 2)
        dir_pp = xyz - viewpoint_camera.camera_center.repeat(feats.shape[0], 1)
        dirs = dir_pp / dir_pp.norm(dim=1, keepdim=True)
        colors_precomp = torch.clamp_min(eval_sh(pc.active_sh_degree, shs_view, dirs) + 0.5, 0.0)
    else:
        shs = pc.get_features
    return screenspace_points, settings, dict(means3D=xyz, opacities=pc.get_opacity, shs=shs,
                                              colors_precomp=colors_precomp, scales=scales, rotations=rotations,
                                              cov3D_precomp=cov3D_precomp)


def render(viewpoint_camera, pc, pipe, bg_color: torch.Tensor, scaling_modifier=1.0, override_color=None,
           starter=None, ender=None):
    """gaussian_renderer/__init__.py:18-113."""
    pts, st, op = _operands(viewpoint_camera, pc, pipe, bg_color, scaling_modifier, override_color)
    rasterizer = GaussianRasterizer(raster_settings=st)
    if starter is not None:
        starter.record()
    image, radii = rasterizer(means2D=pts, **op)
    if ender is not None:
        ender.record()
    return {"render": image, "viewspace_points": pts, "visibility_filter": radii > 0, "radii": radii}
