"""CPU ORACLE-SIDE BASELINE (test/bench infrastructure only): the reference's
CPU AMR path, AMR_test.py, restated with numpy/scipy.

BASELINE.json's north_star asks for "the AMR_test.py CPU path timed on the
host cores in the same run" next to the GPU numbers.  The script itself
cannot run here or on the GPU box (module-level code that loads a trained
scene, needs torchvision and CUDA), so this module restates its
CPU section line for line on inputs the bench supplies:

  AMR_test.py:115-136  project the Gaussian centres (points @ viewM for the
                       depth, geom_transform_points with full_proj for x/y,
                       ndc2Pix) and keep those inside the image with z > 0.2;
  AMR_test.py:166-186  count centres per 16-px tile, tiles_num = W//16 + 1,
                       with the script's per-tile boolean-mask loop;
  AMR_test.py:191-195  level = floor(1.5 * log10(count + 1)) + 1, clipped to 4;
  AMR_test.py:245-258  accurate pixels every 2^(4 - level) px inside each tile
                       (tile end clamped to W-1 / H-1, exclusive);
  AMR_test.py:259-280  scipy.interpolate.griddata(linear) of each channel of
                       the rendered image from the accurate pixels to all
                       pixels (three separate calls, as the script does).

The rendered image the script interpolates comes from the GPU rasterizer in
the reference (AMR_test.py:60); here the caller passes one (the bench uses the
CPU oracle's forward render).  Nothing in the product path imports this.
"""
from __future__ import annotations

import time
from itertools import product

import numpy as np

TILE_LEVEL = 4      # AMR_test.py:27
AMR_FACTOR = 1.5    # AMR_test.py:30


def ndc2pix(v, S):
    """AMR_test.py:108-109."""
    return ((v + 1.0) * S - 1.0) * 0.5


def project_centres(means3D: np.ndarray, world_view: np.ndarray, full_proj: np.ndarray, W: int, H: int):
    """AMR_test.py:115-136 (torch in the script, numpy here, float32)."""
    P = means3D.shape[0]
    hom = np.concatenate([means3D.astype(np.float32), np.ones((P, 1), np.float32)], axis=1)
    points_view = hom @ world_view.astype(np.float32)
    out = hom @ full_proj.astype(np.float32)
    proj = out[:, :3] / (out[:, 3:] + np.float32(1e-7))   # utils/graphics_utils.py:22-29
    x = ndc2pix(proj[:, 0], W)
    y = ndc2pix(proj[:, 1], H)
    mask = (x >= 0) & (x < W) & (y >= 0) & (y < H) & (points_view[:, 2] > 0.2)
    return x[mask], y[mask]


def tile_counts(x: np.ndarray, y: np.ndarray, W: int, H: int) -> np.ndarray:
    """AMR_test.py:166-186, including its O(tiles x points) mask loop."""
    step = 2 ** TILE_LEVEL
    nx = W // step + 1
    ny = H // step + 1
    tx = (x // step).astype(int)
    ty = (y // step).astype(int)
    counts = np.zeros((nx, ny))
    for i in range(nx):
        for j in range(ny):
            counts[i, j] = np.sum((tx == i) & (ty == j))
    return counts


def tile_levels(counts: np.ndarray) -> np.ndarray:
    """AMR_test.py:191-195."""
    lv = np.floor(AMR_FACTOR * np.log10(counts + 1)).astype(int) + 1
    lv[lv > 4] = 4
    return lv


def accurate_points(levels: np.ndarray, W: int, H: int) -> np.ndarray:
    """AMR_test.py:245-258: (x, y) of the exactly rendered pixels."""
    step = 2 ** TILE_LEVEL
    pts = []
    nx, ny = levels.shape
    for i in range(nx):
        for j in range(ny):
            sx, ex = i * step, min((i + 1) * step, W - 1)
            sy, ey = j * step, min((j + 1) * step, H - 1)
            st = 2 ** (TILE_LEVEL - int(levels[i, j]))
            pts.extend(product(range(sx, ex, st), range(sy, ey, st)))
    return np.array(pts)


def interpolate(image: np.ndarray, pts: np.ndarray, W: int, H: int) -> np.ndarray:
    """AMR_test.py:259-280: griddata(linear) per channel; returns [3, H, W]
    (NaN outside the convex hull of the accurate points, as griddata gives)."""
    from scipy import interpolate as si
    all_points = np.array(list(product(range(W), range(H))))
    out = []
    for c in range(3):
        chan = image[c].T  # the script transposes to [W, H]
        vals = chan[pts[:, 0], pts[:, 1]]
        out.append(si.griddata(pts, vals, all_points, method="linear"))
    return np.stack(out).reshape(3, W, H).transpose(0, 2, 1)


def run(means3D, world_view, full_proj, image, W: int, H: int) -> dict:
    """The whole CPU section with wall times per part (seconds)."""
    t0 = time.perf_counter()
    x, y = project_centres(means3D, world_view, full_proj, W, H)
    t1 = time.perf_counter()
    counts = tile_counts(x, y, W, H)
    levels = tile_levels(counts)
    pts = accurate_points(levels, W, H)
    t2 = time.perf_counter()
    img = interpolate(image, pts, W, H)
    t3 = time.perf_counter()
    return {"levels": levels, "counts": counts, "accurate_points": pts, "image": img,
            "seconds": {"project": t1 - t0, "binning_levels": t2 - t1, "griddata": t3 - t2, "total": t3 - t0}}
