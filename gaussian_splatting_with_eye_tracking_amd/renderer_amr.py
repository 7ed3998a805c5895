"""The foveated renderer glue -- the drop-in for ``gaussian_renderer_amr``
(``gaussian_renderer_amr/__init__.py``, SURVEY §8 row B8: the caller of the
AMR rasterizer).

* ``render(viewpoint_camera, pc, pipe, bg_color, scaling_modifier=1.0,
  override_color=None, starter=None, ender=None, starters=None, enders=None,
  interpolate_image=False)`` -- the 5-step foveated frame
  (``__init__.py:24-608``): foveaStep 0..4 on one set of buffers, the step
  images summed.  Here through ``rasterization_amr.render_steps``: without an
  autograd graph (the fps harnesses run under ``torch.no_grad()``) the steps
  add their pixels into the running image in the kernel (same bits, no
  per-step image + full-image torch add); with one, the literal apply-and-add
  sequence, so ``loss.backward()`` works as with the reference's graph.
* ``render_once(...)`` -- one foveaStep -2 call with interpolation
  (``__init__.py:612-749``).

``pc`` is any object with the reference GaussianModel's accessors
(``get_xyz``, ``get_opacity``, ``get_scaling``, ``get_rotation``,
``get_features``, ``get_covariance(scaling_modifier)``, ``active_sh_degree``,
``max_sh_degree``), ``viewpoint_camera`` one with ``FoVx``, ``FoVy``,
``image_height``, ``image_width``, ``world_view_transform``,
``full_proj_transform``, ``camera_center``, and ``pipe`` one with ``debug``,
``compute_cov3D_python``, ``convert_SHs_python``.  Returns the reference's
dict: ``render``, ``viewspace_points``, ``visibility_filter``, ``radii``.
"""
from __future__ import annotations

import torch

from .rasterization_amr import GaussianRasterizer, render_steps
from .renderer import _operands


def _empty_like_device(t, ref):
    return torch.empty(0, device=ref.device) if t is None else t


def render(viewpoint_camera, pc, pipe, bg_color: torch.Tensor, scaling_modifier=1.0, override_color=None,
           starter=None, ender=None, starters=None, enders=None, interpolate_image=False, fovea_levels=None):
    """gaussian_renderer_amr/__init__.py:24-608.  ``fovea_levels`` (extension,
    SURVEY §8(f) rank 4): a callable on the step-0 image buffer run before
    step 1 (e.g. ``lambda ib: apply_fovea_levels(ib, W, H, centres, radii)``,
    the reference's line-244 TODO)."""
    pts, st, op = _operands(viewpoint_camera, pc, pipe, bg_color, scaling_modifier, override_color)
    x = op["means3D"]
    if starter is not None:
        starter.record()
    image, radii, _, _, _ = render_steps(
        x, pts, _empty_like_device(op["shs"], x), _empty_like_device(op["colors_precomp"], x), op["opacities"],
        _empty_like_device(op["scales"], x), _empty_like_device(op["rotations"], x),
        _empty_like_device(op["cov3D_precomp"], x), st, interpolate_image=interpolate_image, starters=starters,
        enders=enders, after_step0=fovea_levels)
    if ender is not None:
        ender.record()
    return {"render": image, "viewspace_points": pts, "visibility_filter": radii > 0, "radii": radii}


def render_once(viewpoint_camera, pc, pipe, bg_color: torch.Tensor, scaling_modifier=1.0, override_color=None,
                starter=None, ender=None):
    """gaussian_renderer_amr/__init__.py:612-749: one foveaStep -2 call
    (every tile to its level, interpolated)."""
    pts, st, op = _operands(viewpoint_camera, pc, pipe, bg_color, scaling_modifier, override_color)
    rasterizer = GaussianRasterizer(raster_settings=st)
    if starter is not None:
        starter.record()
    image, radii, _, _, _ = rasterizer(means2D=pts, foveaStep=int(-2), **op)
    if ender is not None:
        ender.record()
    return {"render": image, "viewspace_points": pts, "visibility_filter": radii > 0, "radii": radii}
