"""How many (pixel, Gaussian) evaluations the blends spend per useful one, by
culling granularity -- a CPU study on the config-2 scene (oracle forward).

For every 16x16 tile and every entry of its list below the tile's largest
n_contrib, a pixel is "live" when the entry is one of its contributors
(index < n_contrib) and alpha >= 1/255 there (base/cr/backward.cu:
460-480).  Reported: live pairs, and the evaluations a wave-per-tile blend
performs when it skips whole pixel groups with no live pixel --
  none:   every pixel (256 per entry)
  strip:  4 rows x 16 columns (the current row groups, 64 px)
  quad:   8 x 8 quadrants (64 px)
  half:   2 rows x 16 columns / 4 x 8 (32 px, a half-wave group)
and for the forward (a wave per group, entries below the group's largest
n_contrib whose alpha >= 1/255 ellipse reaches the group): fstrip / fquad.
usage: python tools/cull_stats.py [--P 1000000 --W 1920 --H 1080]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--tiles", type=int, default=0, help="sample every k-th tile (0: all)")
    a = ap.parse_args()
    import oracle as O
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    O.set_threads(O.host_threads(8))
    cam = S.make_camera(a.W, a.H)
    sc = S.make_scene(a.P, cam, seed=0)
    t0 = time.time()
    r = O.forward(O.settings_from_camera(cam), sc.means3D, sc.opacities, shs=sc.shs, scales=sc.scales,
                  rotations=sc.rotations)
    print(f"oracle forward {time.time() - t0:.1f} s, K={r.num_rendered}", flush=True)
    W, H = a.W, a.H
    gx, gy = (W + 15) // 16, (H + 15) // 16
    nc = r.n_contrib.reshape(H, W)
    xy = r.means2D
    co = r.conic_opacity
    py, px = np.mgrid[0:16, 0:16]
    strip = (py // 4).reshape(-1)
    quad = ((py // 8) * 2 + px // 8).reshape(-1)
    half = (py // 2).reshape(-1)  # 8 groups of 2 rows x 16
    half8 = ((py // 4) * 2 + px // 8).reshape(-1)  # 8 groups of 4 rows x 8
    tot = dict(live=0, none=0, strip=0, quad=0, half=0, half8=0, entries=0, fstrip=0, fquad=0)
    step = max(1, a.tiles)
    for t in range(0, gx * gy, step):
        tx, ty = t % gx, t // gx
        x0, y0 = tx * 16, ty * 16
        pix_x = (x0 + px).reshape(-1).astype(np.float32)
        pix_y = (y0 + py).reshape(-1).astype(np.float32)
        inside = (pix_x < W) & (pix_y < H)
        ncp = np.zeros(256, np.int64)
        ncp[inside] = nc[np.minimum(pix_y[inside].astype(int), H - 1), np.minimum(pix_x[inside].astype(int), W - 1)]
        last = int(ncp.max()) if inside.any() else 0
        if last == 0:
            continue
        beg = int(r.ranges[t, 0])
        ids = r.point_list[beg:beg + last]
        g = xy[ids]
        c = co[ids]
        dx = g[:, 0:1] - pix_x[None, :]
        dy = g[:, 1:2] - pix_y[None, :]
        power = -0.5 * (c[:, 0:1] * dx * dx + c[:, 2:3] * dy * dy) - c[:, 1:2] * dx * dy
        alpha = np.minimum(0.99, c[:, 3:4] * np.exp(power))
        live = (power <= 0) & (alpha >= 1.0 / 255.0) & (np.arange(last)[:, None] < ncp[None, :]) & inside[None, :]
        # the forward: wave g evaluates the entries below the largest
        # n_contrib of its pixels whose alpha >= 1/255 ellipse reaches the group
        geo = (power <= 0) & (alpha >= 1.0 / 255.0) & inside[None, :]
        for name, grp in (("fstrip", strip), ("fquad", quad)):
            for k in range(4):
                sel = grp == k
                if not inside[sel].any():
                    continue
                mx = int(ncp[sel].max())
                tot[name] += int(geo[:mx, sel].any(axis=1).sum()) * 64
        tot["live"] += int(live.sum())
        tot["entries"] += last
        tot["none"] += last * 256
        for name, grp, n in (("strip", strip, 4), ("quad", quad, 4), ("half", half, 8), ("half8", half8, 8)):
            any_g = np.zeros((last, n), bool)
            for k in range(n):
                any_g[:, k] = live[:, grp == k].any(axis=1)
            tot[name] += int(any_g.sum()) * (256 // n)
    print(tot)
    for k in ("none", "strip", "quad", "half", "half8", "fstrip", "fquad"):
        print(f"{k:6s} evaluations {tot[k] / 1e6:9.1f} M  per live pair {tot[k] / max(1, tot['live']):.2f}")


if __name__ == "__main__":
    main()
