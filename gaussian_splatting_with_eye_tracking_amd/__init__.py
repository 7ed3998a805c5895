"""MI355X-native (gfx950) differentiable Gaussian rasterizer with AMR foveated
tile culling -- the hot path of XinShuo-ph/gaussian_splatting_with_eye_tracking
(submodules/diff-gaussian-rasterization, -amr and simple-knn), rebuilt as
hand-written HIP kernels behind a C ABI (include/gsplat_amd.h) and a thin
PyTorch binding.

The drop-in packages ``diff_gaussian_rasterization``,
``diff_gaussian_rasterization_amr`` and ``simple_knn`` at the repository root
re-export the reference API from here.

There is no CPU fallback: importing ``_C`` fails loudly if the native
extension has not been built (run ``python
gaussian_splatting_with_eye_tracking_amd/build.py`` or
``__graft_entry__.build()``).
"""
from __future__ import annotations

import importlib
import os

__version__ = "0.1.0"

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))


def _load_native():
    try:
        import torch  # noqa: F401  (the extension links libtorch)
        return importlib.import_module(__name__ + "._C")
    except ImportError as e:  # pragma: no cover - exercised only when unbuilt
        raise ImportError(
            "gaussian_splatting_with_eye_tracking_amd: the native HIP extension is not built "
            f"({e}). Build it with `python gaussian_splatting_with_eye_tracking_amd/build.py` or `__graft_entry__.build()`.") from e


_C = _load_native()

from .rasterization import (GaussianRasterizationSettings, GaussianRasterizer,  # noqa: E402
                            rasterize_gaussians, _RasterizeGaussians)

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians",
           "_C", "native_library_paths"]


def native_library_paths() -> list[str]:
    """The in-tree shared objects the product path loads."""
    return [os.path.join(_PKG_DIR, "libgsplat_amd.so"), _C.__file__]
