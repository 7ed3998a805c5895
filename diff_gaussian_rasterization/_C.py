"""``diff_gaussian_rasterization._C`` (base/ext.cpp:15-19): the three bound
functions, served by the MI355X extension."""
from gaussian_splatting_with_eye_tracking_amd._C import (  # noqa: F401
    mark_visible, rasterize_gaussians, rasterize_gaussians_backward)
