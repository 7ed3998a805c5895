"""Autograd wrapper of the base rasterizer -- the drop-in for
``submodules/diff-gaussian-rasterization/diff_gaussian_rasterization/__init__.py``.

Same public names, argument order, return values and error behaviour as the
reference (``base/.../__init__.py:21-221``):

* ``rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities,
  scales, rotations, cov3Ds_precomp, raster_settings)``;
* ``_RasterizeGaussians.forward -> (color [3,H,W], radii [P] int32)`` and a
  backward returning gradients in input order, ``means2D``'s gradient being
  dL/d(NDC xy) with a zero third column;
* ``GaussianRasterizationSettings`` (NamedTuple) and ``GaussianRasterizer``
  (nn.Module) with ``markVisible`` and the "exactly one of" checks raising
  ``Exception``.

The native calls go to the MI355X extension ``_C`` (C ABI underneath).
"""
from __future__ import annotations

from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C


def cpu_deep_copy_tuple(input_tuple):
    return tuple(item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


def _call(fn, args, debug: bool, dump: str, what: str):
    """debug mode: snapshot the arguments and re-raise (base/.../__init__.py:83-90)."""
    if not debug:
        return fn(*args)
    cpu_args = cpu_deep_copy_tuple(args)
    try:
        return fn(*args)
    except Exception as ex:
        torch.save(cpu_args, dump)
        print(f"\nAn error occured in {what}. Please forward {dump} for debugging.")
        raise ex


def _hint_forward_only(tensors) -> bool:
    """No backward can follow this call (grad mode off, or no input requires a
    gradient): tell the next native forward, which then skips what only the
    backward reads (the SH-derivative rows).  Returns whether
    the one-shot hint was set; the caller clears it once the call is over
    (_clear_hint), so a forward that raised before consuming it cannot hand
    it to a later training forward."""
    if not (torch.is_grad_enabled() and any(isinstance(t, torch.Tensor) and t.requires_grad for t in tensors)):
        _C.set_thread_option("fwd_no_grad", 1)
        return True
    return False


def _clear_hint(hinted: bool) -> None:
    if hinted:
        _C.set_thread_option("fwd_no_grad", 0)


class _RasterizeGaussians(torch.autograd.Function):
    @classmethod
    def apply(cls, *args):
        hinted = _hint_forward_only(args[:8])
        try:
            return super().apply(*args)
        finally:
            _clear_hint(hinted)

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        s = raster_settings
        args = (s.bg, means3D, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
                s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree,
                s.campos, s.prefiltered, s.debug)
        num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer = _call(
            _C.rasterize_gaussians, args, s.debug, "snapshot_fw.dump", "forward")
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer,
                              binningBuffer, imgBuffer)
        # radii (int32) never carries a gradient: without this autograd fills a
        # zero int tensor of P elements for it on every backward (~6 us at 1M)
        ctx.set_materialize_grads(False)
        return color, radii

    @staticmethod
    def backward(ctx, grad_out_color, _):
        if grad_out_color is None:  # the image took no part in the loss
            return (None,) * 9
        s = ctx.raster_settings
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer, binningBuffer,
         imgBuffer) = ctx.saved_tensors
        args = (s.bg, means3D, radii, colors_precomp, scales, rotations, s.scale_modifier, cov3Ds_precomp,
                s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, grad_out_color, sh, s.sh_degree, s.campos,
                geomBuffer, ctx.num_rendered, binningBuffer, imgBuffer, s.debug)
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh,
         grad_scales, grad_rotations) = _call(_C.rasterize_gaussians_backward_lean, args, s.debug,
                                              "snapshot_bw.dump", "backward")
        return (grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_opacities, grad_scales,
                grad_rotations, grad_cov3Ds_precomp, None)


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


def _check_exactly_one(shs, colors_precomp, scales, rotations, cov3D_precomp):
    """base/.../__init__.py:191-195"""
    if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
        raise Exception('Please provide excatly one of either SHs or precomputed colors!')
    if ((scales is None or rotations is None) and cov3D_precomp is None) or \
            ((scales is not None or rotations is not None) and cov3D_precomp is not None):
        raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')


def _or_empty(t):
    return torch.Tensor([]) if t is None else t


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            s = self.raster_settings
            visible = _C.mark_visible(positions, s.viewmatrix, s.projmatrix)
        return visible

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        _check_exactly_one(shs, colors_precomp, scales, rotations, cov3D_precomp)
        return rasterize_gaussians(means3D, means2D, _or_empty(shs), _or_empty(colors_precomp), opacities,
                                   _or_empty(scales), _or_empty(rotations), _or_empty(cov3D_precomp),
                                   self.raster_settings)
