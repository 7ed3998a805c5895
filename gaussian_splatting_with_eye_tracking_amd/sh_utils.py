"""Spherical-harmonics colour in torch -- the renderers' ``convert_SHs_python``
path (``utils/sh_utils.py:eval_sh``, used by ``gaussian_renderer*/__init__.py``
when ``pipe.convert_SHs_python``).

Real SH basis up to degree 4 with the usual normalisation constants; the
terms are accumulated in the same order as the reference so a float32 call
gives the same bits (tests/test_renderer_amr.py pins it against
tests/golden/ref_pins.npz and sh4_pins.npz, generated from the reference by
tools/make_golden.py).  (The rasterizer itself, like the reference's CUDA,
takes SH degree <= 3.)
"""
from __future__ import annotations

import torch

_C0 = 0.28209479177387814
_C1 = 0.4886025119029199
_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
       1.445305721320277, -0.5900435899266435)
_C4 = (2.5033429417967046, -1.7701307697799304, 0.9461746957575601, -0.6690465435572892, 0.10578554691520431,
       -0.6690465435572892, 0.47308734787878004, -1.7701307697799304, 0.6258357354491761)


def eval_sh(deg: int, sh: torch.Tensor, dirs: torch.Tensor) -> torch.Tensor:
    """Colour of SH coefficients ``sh`` [..., C, (deg + 1)^2 or more] along unit
    directions ``dirs`` [..., 3] -> [..., C] (no +0.5 offset, no clamp)."""
    if not 0 <= deg <= 4:
        raise ValueError("eval_sh: degree 0..4")
    if sh.shape[-1] < (deg + 1) ** 2:
        raise ValueError(f"eval_sh: degree {deg} needs {(deg + 1) ** 2} coefficients, got {sh.shape[-1]}")
    out = _C0 * sh[..., 0]
    if deg == 0:
        return out
    x, y, z = dirs[..., 0:1], dirs[..., 1:2], dirs[..., 2:3]
    out = out - _C1 * y * sh[..., 1] + _C1 * z * sh[..., 2] - _C1 * x * sh[..., 3]
    if deg == 1:
        return out
    xx, yy, zz = x * x, y * y, z * z
    xy, yz, xz = x * y, y * z, x * z
    out = (out + _C2[0] * xy * sh[..., 4] + _C2[1] * yz * sh[..., 5] + _C2[2] * (2.0 * zz - xx - yy) * sh[..., 6]
           + _C2[3] * xz * sh[..., 7] + _C2[4] * (xx - yy) * sh[..., 8])
    if deg == 2:
        return out
    out = (out + _C3[0] * y * (3 * xx - yy) * sh[..., 9] + _C3[1] * xy * z * sh[..., 10]
           + _C3[2] * y * (4 * zz - xx - yy) * sh[..., 11] + _C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[..., 12]
           + _C3[4] * x * (4 * zz - xx - yy) * sh[..., 13] + _C3[5] * z * (xx - yy) * sh[..., 14]
           + _C3[6] * x * (xx - 3 * yy) * sh[..., 15])
    if deg == 3:
        return out
    return (out + _C4[0] * xy * (xx - yy) * sh[..., 16] + _C4[1] * yz * (3 * xx - yy) * sh[..., 17]
            + _C4[2] * xy * (7 * zz - 1) * sh[..., 18] + _C4[3] * yz * (7 * zz - 3) * sh[..., 19]
            + _C4[4] * (zz * (35 * zz - 30) + 3) * sh[..., 20] + _C4[5] * xz * (7 * zz - 3) * sh[..., 21]
            + _C4[6] * (xx - yy) * (7 * zz - 1) * sh[..., 22] + _C4[7] * xz * (xx - 3 * yy) * sh[..., 23]
            + _C4[8] * (xx * (xx - 3 * yy) - yy * (3 * xx - yy)) * sh[..., 24])
