"""Deterministic synthetic scenes and cameras (SURVEY.md §8(d) generator).

No datasets or trained .ply models exist offline, so every benchmark and
parity case runs on this generator.  Camera matrices follow the reference's
conventions exactly:

* ``getWorld2View2`` / ``getProjectionMatrix``: ``utils/graphics_utils.py:38-77``
* ``world_view_transform = W2V.T``, ``full_proj = wv @ proj.T``,
  ``camera_center = inverse(wv)[3, :3]``: ``scene/cameras.py:54-57``
* activations (exp scale, normalised quaternion, sigmoid opacity, SH layout
  [P, 16, 3]): ``scene/gaussian_model.py:95-118``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


def get_world2view2(R: np.ndarray, t: np.ndarray, translate=np.zeros(3), scale: float = 1.0) -> np.ndarray:
    """utils/graphics_utils.py:38-49 (float64 math, float32 result)."""
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    cam_center = C2W[:3, 3]
    cam_center = (cam_center + translate) * scale
    C2W[:3, 3] = cam_center
    Rt = np.linalg.inv(C2W)
    return np.float32(Rt)


def get_projection_matrix(znear: float, zfar: float, fovX: float, fovY: float) -> np.ndarray:
    """utils/graphics_utils.py:51-71 (torch.zeros(4,4) is float32 there)."""
    tanHalfFovY = math.tan((fovY / 2))
    tanHalfFovX = math.tan((fovX / 2))
    top = tanHalfFovY * znear
    bottom = -top
    right = tanHalfFovX * znear
    left = -right
    P = np.zeros((4, 4), dtype=np.float32)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


@dataclass
class Camera:
    """The subset of ``scene/cameras.py:Camera`` the rasterizer consumes."""
    image_width: int
    image_height: int
    FoVx: float
    FoVy: float
    world_view_transform: np.ndarray  # [4,4] f32, row-vector convention (transposed)
    full_proj_transform: np.ndarray  # [4,4] f32
    camera_center: np.ndarray  # [3] f32

    @property
    def tanfovx(self) -> float:
        return math.tan(self.FoVx * 0.5)

    @property
    def tanfovy(self) -> float:
        return math.tan(self.FoVy * 0.5)


def make_camera(W: int, H: int, R: np.ndarray | None = None, T: np.ndarray | None = None,
                fovx_deg: float = 60.0, znear: float = 0.01, zfar: float = 100.0) -> Camera:
    if R is None:
        R = np.eye(3)
    if T is None:
        T = np.zeros(3)
    FoVx = math.radians(fovx_deg)
    FoVy = 2.0 * math.atan(math.tan(FoVx * 0.5) * H / W)
    wv = get_world2view2(R, T).T.copy()  # cameras.py:54 (.transpose(0,1))
    proj = get_projection_matrix(znear, zfar, FoVx, FoVy).T.copy()  # cameras.py:55
    full = (wv.astype(np.float32) @ proj.astype(np.float32)).astype(np.float32)  # cameras.py:56 (bmm in f32)
    center = np.linalg.inv(wv.astype(np.float64))[3, :3].astype(np.float32)  # cameras.py:57
    return Camera(W, H, FoVx, FoVy, wv.astype(np.float32), full, center)


def make_orbit_camera(W: int, H: int, yaw_deg: float, center=(0.0, 0.0, 11.0)) -> Camera:
    """Camera yawed by ``yaw_deg`` about the vertical axis through ``center``
    (config 5: views at ±(0..3.5)·5°).  R is camera-to-world rotation (COLMAP
    convention of ``getWorld2View2``: W2V rotation = R^T)."""
    a = math.radians(yaw_deg)
    Ry = np.array([[math.cos(a), 0.0, math.sin(a)], [0.0, 1.0, 0.0], [-math.sin(a), 0.0, math.cos(a)]])
    c = np.asarray(center, dtype=np.float64)
    cam_pos = c - Ry @ c  # rotate the identity camera (at origin) about c
    # world->view: x_v = R^T x_w + t, with t = -R^T cam_pos
    t = -Ry.T @ cam_pos
    return make_camera(W, H, R=Ry, T=t)


def config5_yaws(n_views: int = 8) -> list[float]:
    """±(0..3.5)·5°: -17.5 .. +17.5 step 5."""
    return [(-3.5 + v) * 5.0 for v in range(n_views)]


@dataclass
class Scene:
    means3D: np.ndarray  # [P,3] f32
    scales: np.ndarray  # [P,3] f32 (activated: exp)
    rotations: np.ndarray  # [P,4] f32 (normalised (r,x,y,z))
    opacities: np.ndarray  # [P,1] f32 (activated: sigmoid)
    shs: np.ndarray  # [P,16,3] f32
    sh_degree: int = 3

    @property
    def P(self) -> int:
        return int(self.means3D.shape[0])


def make_scene(P: int, cam: Camera, seed: int = 0, sh_degree: int = 3, depth_range=(2.0, 20.0),
               spread: float = 1.1, log_scale_mean: float = math.log(0.01), log_scale_std: float = 0.4,
               opacity_std: float = 1.5) -> Scene:
    """SURVEY §8(d) generator: depth z~U(2,20); x = z·tanfovx·U(-1.1,1.1);
    y = z·tanfovy·U(-1.1,1.1); log-scale ~ N(ln 0.01, 0.4); rotation =
    normalised N(0,1)^4; opacity = sigmoid(N(0,1.5)); SH DC ~ N(0,0.5), rest
    ~ N(0,0.1)."""
    rng = np.random.default_rng(seed)
    z = rng.uniform(depth_range[0], depth_range[1], P)
    x = z * cam.tanfovx * rng.uniform(-spread, spread, P)
    y = z * cam.tanfovy * rng.uniform(-spread, spread, P)
    means = np.stack([x, y, z], axis=1).astype(np.float32)
    scales = np.exp(rng.normal(log_scale_mean, log_scale_std, (P, 3))).astype(np.float32)
    q = rng.normal(0.0, 1.0, (P, 4))
    q = q / np.linalg.norm(q, axis=1, keepdims=True)
    rot = q.astype(np.float32)
    opac = (1.0 / (1.0 + np.exp(-rng.normal(0.0, opacity_std, (P, 1))))).astype(np.float32)
    M = (sh_degree + 1) ** 2
    shs = np.empty((P, 16 if sh_degree <= 3 else M, 3), dtype=np.float32)
    shs[:, 0, :] = rng.normal(0.0, 0.5, (P, 3))
    shs[:, 1:, :] = rng.normal(0.0, 0.1, (P, shs.shape[1] - 1, 3))
    return Scene(means, scales, rot, opac, shs, sh_degree)


def make_cotangent(H: int, W: int, seed: int = 1) -> np.ndarray:
    """dL/dpix ~ N(0,1), [3,H,W] f32."""
    return np.random.default_rng(seed).normal(0.0, 1.0, (3, H, W)).astype(np.float32)


# Fovea centre for config 3: RITnet ground-truth pupil centroid from the
# reference fixture eye_label_gt.npy, (x, y) = (361.74, 248.19) of a 640x400
# eye image.  Passed through like the reference, which
# computes fovea centres but never feeds them to the rasterizer
# (gaussian_renderer_amr/__init__.py:99-106).
PUPIL_CENTROID_XY = (361.74, 248.19)
EYE_IMAGE_WH = (640, 400)


def fovea_center(W: int, H: int) -> tuple[float, float]:
    return (PUPIL_CENTROID_XY[0] / EYE_IMAGE_WH[0] * W, PUPIL_CENTROID_XY[1] / EYE_IMAGE_WH[1] * H)
