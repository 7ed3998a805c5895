"""Drop-in replacement for the reference package ``diff_gaussian_rasterization``
(submodules/diff-gaussian-rasterization), backed by the MI355X HIP kernels in
``gaussian_splatting_with_eye_tracking_amd``.  ``gaussian_renderer`` imports it
unchanged."""
from gaussian_splatting_with_eye_tracking_amd.rasterization import (  # noqa: F401
    GaussianRasterizationSettings, GaussianRasterizer, _RasterizeGaussians, cpu_deep_copy_tuple,
    rasterize_gaussians)

from . import _C  # noqa: F401,E402
