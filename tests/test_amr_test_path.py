"""The AMR_test.py CPU-path restatement (oracle/amr_test_path.py) used as the
north_star's CPU baseline.  CPU only.

Pins: the projection against the reference's own geom_transform_points
vectors (tests/golden/ref_pins.npz); the level formula on hand-computed
counts; griddata(linear) reproducing the image exactly at the accurate
pixels; the per-tile mask loop against a bincount.
"""
import os

import numpy as np
import pytest

import amr_test_path as A
from gaussian_splatting_with_eye_tracking_amd import synthetic as S

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_level_formula_known_answers():
    counts = np.array([[0, 1, 2, 3], [4, 9, 10, 20], [21, 99, 100, 1000]], float)
    # floor(1.5 * log10(c + 1)) + 1, clipped to 4
    exp = np.array([[1, 1, 1, 1], [2, 2, 2, 2], [3, 4, 4, 4]])  # 1.5*log10(22) = 2.01, 1.5*log10(100) = 3
    np.testing.assert_array_equal(A.tile_levels(counts), exp)


def test_tile_count_loop_equals_bincount():
    rng = np.random.default_rng(0)
    W, H = 200, 120
    x = rng.uniform(0, W, 3000).astype(np.float32)
    y = rng.uniform(0, H, 3000).astype(np.float32)
    c = A.tile_counts(x, y, W, H)
    nx, ny = W // 16 + 1, H // 16 + 1
    ref = np.bincount((x // 16).astype(int) * ny + (y // 16).astype(int), minlength=nx * ny).reshape(nx, ny)
    np.testing.assert_array_equal(c, ref)


def test_projection_matches_reference_geom_transform_points():
    """project_centres' x/y path is the reference's geom_transform_points
    (vectors made from /root/reference/utils/graphics_utils.py:22-29)."""
    pins = np.load(os.path.join(GOLD, "ref_pins.npz"))
    pts, M, ref = pins["gtp_points"], pins["gtp_full_proj"], pins["gtp_out"]
    W, H = 640, 480
    x, y = A.project_centres(pts, np.eye(4, dtype=np.float32), M, W, H)
    keep = ((A.ndc2pix(ref[:, 0], W) >= 0) & (A.ndc2pix(ref[:, 0], W) < W) & (A.ndc2pix(ref[:, 1], H) >= 0)
            & (A.ndc2pix(ref[:, 1], H) < H) & (pts[:, 2] > 0.2))
    np.testing.assert_allclose(x, A.ndc2pix(ref[keep, 0], W), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(y, A.ndc2pix(ref[keep, 1], H), rtol=1e-5, atol=1e-3)


def test_accurate_points_and_interpolation_exact_at_samples():
    W, H = 64, 48
    levels = np.array([[1, 2, 3, 4]] * (W // 16 + 1))[:, : H // 16 + 1]
    pts = A.accurate_points(levels, W, H)
    # inside tile (0, 0) with level 1 the stride is 8: (0,0), (0,8), (8,0), (8,8)
    t00 = [tuple(p) for p in pts if p[0] < 16 and p[1] < 16]
    assert sorted(t00) == [(0, 0), (0, 8), (8, 0), (8, 8)]
    rng = np.random.default_rng(1)
    img = rng.uniform(0, 1, (3, H, W)).astype(np.float32)
    out = A.interpolate(img, pts, W, H)
    assert out.shape == (3, H, W)
    for c in range(3):
        np.testing.assert_allclose(out[c][pts[:, 1], pts[:, 0]], img[c][pts[:, 1], pts[:, 0]], rtol=0, atol=1e-6)


def test_run_on_config1_sample():
    """Config 1 (10k Gaussians, 256x256) end to end on a synthetic image."""
    W, H = 256, 256
    cam = S.make_camera(W, H)
    sc = S.make_scene(10000, cam, seed=0)
    img = np.random.default_rng(2).uniform(0, 1, (3, H, W)).astype(np.float32)
    r = A.run(sc.means3D, cam.world_view_transform, cam.full_proj_transform, img, W, H)
    assert r["levels"].min() >= 1 and r["levels"].max() <= 4
    assert r["counts"].sum() > 0
    assert np.isfinite(r["image"]).mean() > 0.9
    assert r["seconds"]["total"] > 0
