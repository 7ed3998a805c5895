"""``diff_gaussian_rasterization_amr._C`` (amr/ext.cpp): ``rasterize_gaussians``
takes the AMR signature (foveaStep, out_color_precomp, the three precomputed
buffers and interpolate_image inserted before ``debug``,
amr/rasterize_points.h:39-53)."""
from gaussian_splatting_with_eye_tracking_amd._C import amr_rasterize_gaussians as rasterize_gaussians  # noqa: F401
from gaussian_splatting_with_eye_tracking_amd._C import mark_visible, rasterize_gaussians_backward  # noqa: F401
