"""Drop-in replacement for ``diff_gaussian_rasterization_amr``
(submodules/diff-gaussian-rasterization-amr).  ``gaussian_renderer_amr``
imports ``GaussianRasterizationSettings``, ``GaussianRasterizer`` and
``_RasterizeGaussians`` from here unchanged."""
from gaussian_splatting_with_eye_tracking_amd.rasterization import cpu_deep_copy_tuple  # noqa: F401
from gaussian_splatting_with_eye_tracking_amd.rasterization_amr import (  # noqa: F401
    GaussianRasterizationSettings, GaussianRasterizer, _RasterizeGaussians, rasterize_gaussians)

from . import _C  # noqa: F401,E402
