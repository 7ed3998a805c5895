"""ctypes driver for the CPU oracle (gs_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() may
import this module, and only as the checker: the product path
(gaussian_splatting_with_eye_tracking_amd + the drop-in packages) never
imports, links or executes anything under oracle/.

The driver strings the restated stages together exactly like the reference
orchestrators:
  * base forward:  base/cr/rasterizer_impl.cu:198-336
  * base backward: base/cr/rasterizer_impl.cu:340-434, base/rasterize_points.cu:117-196
  * AMR forward:   amr/cr/rasterizer_impl.cu:296-694
  * simple-knn:    knn/simple_knn.cu:185-221
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libgs_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
                os.path.join(_HERE, "gs_oracle.c")):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
    return _lib


def set_threads(n: int) -> None:
    """Host threads of the C loops (OpenMP).  1 = serial, the order the golden
    fixtures were frozen with; n > 1 parallelises the independent loops and
    sums the blend backward per band of tile rows (gs_oracle.c)."""
    lib().orc_set_threads(ctypes.c_int(int(n)))


def get_threads() -> int:
    return int(lib().orc_get_threads())


def host_threads(cap: int = 16) -> int:
    """Threads this process may use: its CPU affinity (the GPU box's share,
    not the whole machine's os.cpu_count()), capped."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, min(cap, n))


def _p(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "oracle arrays must be C-contiguous"
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


@dataclass
class Settings:
    """Mirror of GaussianRasterizationSettings (base/.../__init__.py:157-169)."""
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: np.ndarray
    scale_modifier: float
    viewmatrix: np.ndarray
    projmatrix: np.ndarray
    sh_degree: int
    campos: np.ndarray
    prefiltered: bool = False
    debug: bool = False


def settings_from_camera(cam, bg=(0.0, 0.0, 0.0), sh_degree=3, scale_modifier=1.0) -> Settings:
    return Settings(cam.image_height, cam.image_width, cam.tanfovx, cam.tanfovy,
                    np.asarray(bg, np.float32), scale_modifier, cam.world_view_transform,
                    cam.full_proj_transform, sh_degree, cam.camera_center)


@dataclass
class ForwardResult:
    num_rendered: int
    color: np.ndarray
    radii: np.ndarray
    means2D: np.ndarray
    depths: np.ndarray
    cov3D: np.ndarray
    rgb: np.ndarray
    clamped: np.ndarray
    conic_opacity: np.ndarray
    tiles_touched: np.ndarray
    point_offsets: np.ndarray
    point_list_keys: np.ndarray
    point_list: np.ndarray
    ranges: np.ndarray
    final_T: np.ndarray
    n_contrib: np.ndarray
    block: int
    extra: dict = field(default_factory=dict)


def _c_float(x):
    return ctypes.c_float(float(x))


def preprocess_and_bin(s: Settings, means3D, opacities, shs=None, colors_precomp=None, scales=None,
                       rotations=None, cov3D_precomp=None, block: int = 16) -> ForwardResult:
    """base/cr/rasterizer_impl.cu:222-318 (everything before the blend)."""
    L = lib()
    means3D = _f32(means3D)
    P = means3D.shape[0]
    W, H = int(s.image_width), int(s.image_height)
    focal_y = np.float32(H / (2.0 * np.float32(s.tanfovy)))
    focal_x = np.float32(W / (2.0 * np.float32(s.tanfovx)))
    # rasterizer_impl.cu:222-223: focal computed in float: height / (2.0f * tan_fovy)
    tfx = np.float32(s.tanfovx)
    tfy = np.float32(s.tanfovy)
    focal_y = np.float32(np.float32(H) / (np.float32(2.0) * tfy))
    focal_x = np.float32(np.float32(W) / (np.float32(2.0) * tfx))
    shs = _f32(shs)
    M = 0 if shs is None or shs.size == 0 else shs.shape[1]
    if shs is not None and shs.size == 0:
        shs = None
    colors_precomp = _f32(colors_precomp)
    if colors_precomp is not None and colors_precomp.size == 0:
        colors_precomp = None
    scales = _f32(scales)
    if scales is not None and scales.size == 0:
        scales = None
    rotations = _f32(rotations)
    if rotations is not None and rotations.size == 0:
        rotations = None
    cov3D_precomp = _f32(cov3D_precomp)
    if cov3D_precomp is not None and cov3D_precomp.size == 0:
        cov3D_precomp = None
    opac = _f32(opacities).reshape(-1)
    radii = np.zeros(P, np.int32)
    means2D = np.zeros((P, 2), np.float32)
    depths = np.zeros(P, np.float32)
    cov3D = np.zeros((P, 6), np.float32)
    rgb = np.zeros((P, 3), np.float32)
    clamped = np.zeros((P, 3), np.uint8)
    conic = np.zeros((P, 4), np.float32)
    touched = np.zeros(P, np.uint32)
    L.orc_preprocess(
        ctypes.c_int(P), ctypes.c_int(int(s.sh_degree)), ctypes.c_int(M), _p(means3D), _p(scales),
        _c_float(s.scale_modifier), _p(rotations), _p(opac), _p(shs), _p(clamped), _p(cov3D_precomp),
        _p(colors_precomp), _p(_f32(s.viewmatrix)), _p(_f32(s.projmatrix)), _p(_f32(s.campos)),
        ctypes.c_int(W), ctypes.c_int(H), ctypes.c_float(tfx), ctypes.c_float(tfy),
        ctypes.c_float(focal_x), ctypes.c_float(focal_y), ctypes.c_int(block), ctypes.c_int(block),
        _p(radii), _p(means2D), _p(depths), _p(cov3D), _p(rgb), _p(conic), _p(touched),
        ctypes.c_int(int(s.prefiltered)))
    offsets = np.zeros(P, np.uint32)
    L.orc_inclusive_scan_u32(ctypes.c_int(P), _p(touched), _p(offsets))
    K = int(offsets[-1]) if P > 0 else 0
    keys = np.zeros(max(K, 1), np.uint64)
    vals = np.zeros(max(K, 1), np.uint32)
    L.orc_duplicate_with_keys(ctypes.c_int(P), _p(means2D), _p(depths), _p(offsets), _p(radii),
                              ctypes.c_int(W), ctypes.c_int(H), ctypes.c_int(block), ctypes.c_int(block),
                              _p(keys), _p(vals))
    gx, gy = (W + block - 1) // block, (H + block - 1) // block
    T = gx * gy
    L.orc_get_higher_msb.restype = ctypes.c_uint32
    bit = int(L.orc_get_higher_msb(ctypes.c_uint32(T)))
    L.orc_sort_pairs_u64(ctypes.c_int(K), _p(keys), _p(vals), ctypes.c_int(32 + bit))
    ranges = np.zeros((T, 2), np.uint32)
    L.orc_identify_tile_ranges(ctypes.c_int(K), _p(keys), ctypes.c_int(T), _p(ranges))
    return ForwardResult(K, np.zeros((3, H, W), np.float32), radii, means2D, depths, cov3D, rgb, clamped,
                         conic, touched, offsets, keys[:K].copy(), vals[:K].copy(), ranges,
                         np.zeros(H * W, np.float32), np.zeros(H * W, np.uint32), block,
                         extra={"colors_precomp": colors_precomp, "M": M, "focal_x": focal_x,
                                "focal_y": focal_y})


def forward(s: Settings, means3D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
            cov3D_precomp=None, block: int = 16) -> ForwardResult:
    """Base forward (rasterizer_impl.cu:198-336); block = 32 blends every
    pixel with the AMR path's 32-px tile lists (the state the AMR render
    leaves at every pixel it renders)."""
    r = preprocess_and_bin(s, means3D, opacities, shs, colors_precomp, scales, rotations, cov3D_precomp, block)
    W, H = int(s.image_width), int(s.image_height)
    feats = r.extra["colors_precomp"] if r.extra["colors_precomp"] is not None else r.rgb
    lib().orc_render_forward(ctypes.c_int(W), ctypes.c_int(H), ctypes.c_int(block), ctypes.c_int(block),
                             _p(r.ranges), _p(r.point_list), _p(r.means2D), _p(np.ascontiguousarray(feats)),
                             _p(r.conic_opacity), _p(r.final_T), _p(r.n_contrib), _p(_f32(s.bg)), _p(r.color))
    return r


def _bwd_inputs(means3D, shs, colors_precomp, scales, rotations, cov3D_precomp):
    none_if_empty = lambda a: None if a is None or np.asarray(a).size == 0 else _f32(a)  # noqa: E731
    return (_f32(means3D), none_if_empty(shs), none_if_empty(colors_precomp), none_if_empty(scales),
            none_if_empty(rotations), none_if_empty(cov3D_precomp))


def _per_gaussian_backward(s: Settings, fwd: ForwardResult, means3D, shs, scales, rotations, cov3D_precomp,
                           g_mean2D, g_conic, g_col) -> dict:
    """computeCov2DCUDA + preprocessCUDA backward (base/cr/backward.cu:144-396)
    of the blend-level gradients given: a linear map of them."""
    L = lib()
    P = means3D.shape[0]
    M = 0 if shs is None else shs.shape[1]
    g_mean3D = np.zeros((P, 3), np.float32)
    g_cov = np.zeros((P, 6), np.float32)
    g_sh = np.zeros((P, M, 3), np.float32)
    g_scale = np.zeros((P, 3), np.float32)
    g_rot = np.zeros((P, 4), np.float32)
    cov_ptr = cov3D_precomp if cov3D_precomp is not None else fwd.cov3D
    fx, fy = fwd.extra["focal_x"], fwd.extra["focal_y"]
    L.orc_cov2d_backward(ctypes.c_int(P), _p(means3D), _p(fwd.radii), _p(np.ascontiguousarray(cov_ptr)),
                         ctypes.c_float(fx), ctypes.c_float(fy), ctypes.c_float(np.float32(s.tanfovx)),
                         ctypes.c_float(np.float32(s.tanfovy)), _p(_f32(s.viewmatrix)), _p(g_conic),
                         _p(g_mean3D), _p(g_cov))
    L.orc_preprocess_backward(ctypes.c_int(P), ctypes.c_int(int(s.sh_degree)), ctypes.c_int(M), _p(means3D),
                              _p(fwd.radii), _p(shs), _p(fwd.clamped), _p(scales), _p(rotations),
                              _c_float(s.scale_modifier), _p(_f32(s.projmatrix)), _p(_f32(s.campos)),
                              _p(g_mean2D), _p(g_mean3D), _p(g_col), _p(g_cov), _p(g_sh), _p(g_scale),
                              _p(g_rot))
    return {"dL_dmeans3D": g_mean3D, "dL_dcov3D": g_cov, "dL_dsh": g_sh, "dL_dscales": g_scale,
            "dL_drotations": g_rot}


def backward(s: Settings, fwd: ForwardResult, means3D, dL_dpix, shs=None, colors_precomp=None, scales=None,
             rotations=None, cov3D_precomp=None, block: int = 16) -> dict:
    """Base backward (rasterize_points.cu:117-196 + rasterizer_impl.cu:340-434).
    Returns the 8 gradients of _C.rasterize_gaussians_backward plus dL_dconic."""
    means3D, shs, colors_precomp, scales, rotations, cov3D_precomp = _bwd_inputs(
        means3D, shs, colors_precomp, scales, rotations, cov3D_precomp)
    P = means3D.shape[0]
    W, H = int(s.image_width), int(s.image_height)
    g_mean2D = np.zeros((P, 3), np.float32)
    g_conic = np.zeros((P, 2, 2), np.float32)
    g_opac = np.zeros((P, 1), np.float32)
    g_col = np.zeros((P, 3), np.float32)
    colors = colors_precomp if colors_precomp is not None else fwd.rgb
    lib().orc_render_backward(ctypes.c_int(W), ctypes.c_int(H), ctypes.c_int(block), ctypes.c_int(block),
                              _p(fwd.ranges), _p(fwd.point_list), _p(_f32(s.bg)), _p(fwd.means2D),
                              _p(fwd.conic_opacity), _p(np.ascontiguousarray(colors)), _p(fwd.final_T),
                              _p(fwd.n_contrib), _p(_f32(dL_dpix)), ctypes.c_int(P), _p(g_mean2D), _p(g_conic),
                              _p(g_opac), _p(g_col))
    out = _per_gaussian_backward(s, fwd, means3D, shs, scales, rotations, cov3D_precomp, g_mean2D, g_conic, g_col)
    out.update({"dL_dmeans2D": g_mean2D, "dL_dcolors": g_col, "dL_dopacity": g_opac, "dL_dconic": g_conic})
    return out


def _tie_terms(s: Settings, fwd: ForwardResult, dL_dpix, colors):
    P = fwd.radii.shape[0]
    W, H = int(s.image_width), int(s.image_height)
    A = np.zeros((P, 9), np.float64)
    counts = np.zeros(4, np.int64)
    lib().orc_render_tie_allowance(ctypes.c_int(W), ctypes.c_int(H), ctypes.c_int(fwd.block),
                                   ctypes.c_int(fwd.block), _p(fwd.ranges), _p(fwd.point_list), _p(_f32(s.bg)),
                                   _p(fwd.means2D), _p(fwd.conic_opacity), _p(np.ascontiguousarray(colors)),
                                   _p(_f32(dL_dpix)), ctypes.c_int(P), _p(A), _p(counts))
    return A, counts


def _abs_terms(s: Settings, fwd: ForwardResult, dL_dpix, colors):
    P = fwd.radii.shape[0]
    W, H = int(s.image_width), int(s.image_height)
    S = np.zeros((P, 9), np.float64)
    lib().orc_render_backward_abs(ctypes.c_int(W), ctypes.c_int(H), ctypes.c_int(fwd.block), ctypes.c_int(fwd.block),
                                  _p(fwd.ranges), _p(fwd.point_list), _p(_f32(s.bg)), _p(fwd.means2D),
                                  _p(fwd.conic_opacity), _p(np.ascontiguousarray(colors)), _p(fwd.final_T),
                                  _p(fwd.n_contrib), _p(_f32(dL_dpix)), ctypes.c_int(P), _p(S))
    return S


def _propagate(s: Settings, fwd: ForwardResult, means3D, shs, scales, rotations, cov3D_precomp, A) -> dict:
    """Allowances [P, 9] on the nine blend-level terms -> allowances on every
    returned gradient: the terms' own tensors directly; the per-Gaussian
    gradients after the blend are a linear map J of the terms, so theirs is
    sum_k |J (A_k e_k)| over the nine terms k (the bound of |J v| over every
    v with |v_k| <= A_k)."""
    P = A.shape[0]
    Af = A.astype(np.float32)
    out = {"dL_dcolors": A[:, 0:3].copy(), "dL_dopacity": A[:, 8:9].copy(),
           "dL_dmeans2D": np.concatenate([A[:, 3:5], np.zeros((P, 1))], 1),
           "dL_dconic": np.stack([A[:, 5:7], np.stack([np.zeros(P), A[:, 7]], 1)], 1)}
    M = 0 if shs is None else shs.shape[1]
    down = {"dL_dmeans3D": np.zeros((P, 3)), "dL_dcov3D": np.zeros((P, 6)), "dL_dsh": np.zeros((P, M, 3)),
            "dL_dscales": np.zeros((P, 3)), "dL_drotations": np.zeros((P, 4))}
    for k in range(8):  # (the opacity term, k = 8, feeds no per-Gaussian gradient after the blend)
        if not Af[:, k].any():
            continue
        g_mean2D = np.zeros((P, 3), np.float32)
        g_conic = np.zeros((P, 2, 2), np.float32)
        g_col = np.zeros((P, 3), np.float32)
        if k < 3:
            g_col[:, k] = Af[:, k]
        elif k < 5:
            g_mean2D[:, k - 3] = Af[:, k]
        else:
            g_conic.reshape(P, 4)[:, (0, 1, 3)[k - 5]] = Af[:, k]
        r = _per_gaussian_backward(s, fwd, means3D, shs, scales, rotations, cov3D_precomp, g_mean2D, g_conic, g_col)
        for n in down:
            down[n] += np.abs(r[n].astype(np.float64))
    out.update(down)
    return out


def tie_allowance(s: Settings, fwd: ForwardResult, means3D, dL_dpix, shs=None, colors_precomp=None, scales=None,
                  rotations=None, cov3D_precomp=None) -> tuple:
    """Test support (gs_oracle.c orc_render_tie_allowance): per gradient
    element, the total jump the near-tie blend decisions can make -- each
    decision taken within float32 rounding of its threshold replayed the
    other way, one at a time, |gradient(flipped) - gradient(as taken)| summed,
    then carried through the per-Gaussian backward (_propagate).  Returns
    ({tensor name: allowance shaped like the gradient}, {counts})."""
    means3D, shs, colors_precomp, scales, rotations, cov3D_precomp = _bwd_inputs(
        means3D, shs, colors_precomp, scales, rotations, cov3D_precomp)
    colors = colors_precomp if colors_precomp is not None else fwd.rgb
    A, counts = _tie_terms(s, fwd, dL_dpix, colors)
    out = _propagate(s, fwd, means3D, shs, scales, rotations, cov3D_precomp, A)
    return out, {"tie_pixels": int(counts[0]), "power": int(counts[1]), "alpha": int(counts[2]), "T": int(counts[3]),
                 "gaussians": int(np.count_nonzero(A.any(1)))}


# Accumulation allowance per blend-level term: (ACC_SQRT sqrt(n) + ACC_ULPS)
# x 2^-24 x sum|terms|, n the tiles the Gaussian touches.  The GPU forms a
# Gaussian's per-pixel terms in float32 (hardware exp, T rebuilt by a
# reciprocal step by step down the pixel's chain) and adds them in its own
# order -- a tree of partial sums per tile (<= 256 pixels, ~8 levels), then
# the n tile partials by float atomics in arrival order -- where the oracle
# forms them with libm expf and a division and sums in double.  The error of
# such a sum is a multiple of 2^-24 sum|terms|: ~8 ulps per tile tree times
# ~sqrt(n) for the n partials' random-sign roundings (worst case ~n), plus the
# terms' own few-ulp differences.  It matters where the terms cancel -- a
# large Gaussian whose gradient is a small difference of many pixels' terms
# -- and the constants (16 sqrt(n) + 32 ulps) are twice the largest multiple
# measured on the GPU (tests record it as acc_multiple_needed).
ACC_SQRT = 16.0
ACC_ULPS = 32.0


def grad_allowance(s: Settings, fwd: ForwardResult, means3D, dL_dpix, shs=None, colors_precomp=None, scales=None,
                   rotations=None, cov3D_precomp=None, parts: bool = False) -> tuple:
    """Test support: the element-wise gradient tests' allowance -- the
    near-tie jumps (tie_allowance) plus the float32 accumulation allowance
    (ACC_SQRT sqrt(tiles touched) + ACC_ULPS) 2^-24 sum|terms| of every
    blend-level term (orc_render_backward_abs), carried together through the
    per-Gaussian backward (the propagation is linear in non-negative
    allowances, so the parts add).  Returns ({tensor: allowance}, {counts});
    with parts=True the first is {"tie": ..., "acc_sqrt": ..., "acc_ulp": ...}
    (the tie jumps; 2^-24 sqrt(n) sum|terms|; 2^-24 sum|terms|)."""
    means3D, shs, colors_precomp, scales, rotations, cov3D_precomp = _bwd_inputs(
        means3D, shs, colors_precomp, scales, rotations, cov3D_precomp)
    colors = colors_precomp if colors_precomp is not None else fwd.rgb
    A, counts = _tie_terms(s, fwd, dL_dpix, colors)
    S = _abs_terms(s, fwd, dL_dpix, colors) * 2.0 ** -24
    sq = np.sqrt(fwd.tiles_touched.astype(np.float64))[:, None]
    info = {"tie_pixels": int(counts[0]), "power": int(counts[1]), "alpha": int(counts[2]), "T": int(counts[3]),
            "gaussians": int(np.count_nonzero(A.any(1))), "acc_sqrt": ACC_SQRT, "acc_ulps": ACC_ULPS}
    prop = lambda X: _propagate(s, fwd, means3D, shs, scales, rotations, cov3D_precomp, X)  # noqa: E731
    if parts:
        return {"tie": prop(A), "acc_sqrt": prop(sq * S), "acc_ulp": prop(S)}, info
    return prop(A + (ACC_SQRT * sq + ACC_ULPS) * S), info


def combine_allowance(parts: dict, acc_sqrt: float = ACC_SQRT, acc_ulps: float = ACC_ULPS) -> dict:
    """grad_allowance(parts=True)'s parts -> one allowance per tensor."""
    return {n: parts["tie"][n] + acc_sqrt * parts["acc_sqrt"][n] + acc_ulps * parts["acc_ulp"][n]
            for n in parts["tie"]}


def mark_visible(means3D, viewmatrix, projmatrix) -> np.ndarray:
    means3D = _f32(means3D)
    out = np.zeros(means3D.shape[0], np.uint8)
    lib().orc_mark_visible(ctypes.c_int(means3D.shape[0]), _p(means3D), _p(_f32(viewmatrix)),
                           _p(_f32(projmatrix)), _p(out))
    return out.astype(bool)


# ------------------------------------------------------------------- AMR ---
@dataclass
class AMRState:
    """The opaque step-to-step state of the AMR path (geom/binning/image buffers)."""
    fwd: ForwardResult
    n_intersections: np.ndarray
    n_intersections_sorted: np.ndarray
    percentile_values: np.ndarray
    levels: np.ndarray
    levels_last: np.ndarray
    levels_current: np.ndarray
    final_T: np.ndarray
    n_contrib: np.ndarray


def amr_forward(s: Settings, means3D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None, foveaStep: int = 0, out_color_precomp=None, state: AMRState | None = None,
                interpolate_image: bool = True):
    """amr/cr/rasterizer_impl.cu:296-694. Returns (color, radii, state)."""
    L = lib()
    W, H = int(s.image_width), int(s.image_height)
    N = W * H
    if foveaStep >= 1:
        st = state
        fwd = st.fwd
        T = fwd.ranges.shape[0]
        orc_fovea(L, foveaStep, T, st)
        color = np.zeros((3, H, W), np.float32)
        feats = fwd.extra["colors_precomp"] if fwd.extra["colors_precomp"] is not None else fwd.rgb
        L.orc_amr_render(ctypes.c_int(W), ctypes.c_int(H), _p(fwd.ranges), _p(st.levels_current),
                         _p(st.levels_last), _p(fwd.point_list), _p(fwd.means2D), _p(np.ascontiguousarray(feats)),
                         _p(fwd.conic_opacity), _p(st.final_T), _p(st.n_contrib), _p(_f32(s.bg)), _p(color),
                         ctypes.c_int(foveaStep))
        if interpolate_image:
            pre = _f32(out_color_precomp)
            L.orc_amr_interpolate(ctypes.c_int(W), ctypes.c_int(H), _p(st.levels_current), _p(st.levels_last),
                                  _p(st.final_T), _p(st.n_contrib), _p(color), ctypes.c_int(foveaStep), _p(pre))
        return color, np.zeros(fwd.radii.shape, np.int32), st
    fwd = preprocess_and_bin(s, means3D, opacities, shs, colors_precomp, scales, rotations, cov3D_precomp, 32)
    T = fwd.ranges.shape[0]
    st = AMRState(fwd, np.zeros(T, np.uint32), np.zeros(T, np.uint32), np.zeros(3, np.uint32),
                  np.zeros(T, np.uint32), np.zeros(T, np.uint32), np.zeros(T, np.uint32),
                  np.zeros(N, np.float32), np.zeros(N, np.uint32))
    L.orc_amr_levels(ctypes.c_int(T), _p(fwd.ranges), _p(st.n_intersections), _p(st.n_intersections_sorted),
                     _p(st.percentile_values), _p(st.levels))
    color = np.zeros((3, H, W), np.float32)
    if foveaStep == 0:
        return color, fwd.radii, st
    orc_fovea(L, foveaStep, T, st)
    feats = fwd.extra["colors_precomp"] if fwd.extra["colors_precomp"] is not None else fwd.rgb
    L.orc_amr_render(ctypes.c_int(W), ctypes.c_int(H), _p(fwd.ranges), _p(st.levels), _p(st.levels_last),
                     _p(fwd.point_list), _p(fwd.means2D), _p(np.ascontiguousarray(feats)), _p(fwd.conic_opacity),
                     _p(st.final_T), _p(st.n_contrib), _p(_f32(s.bg)), _p(color), ctypes.c_int(foveaStep))
    if interpolate_image:
        L.orc_amr_interpolate(ctypes.c_int(W), ctypes.c_int(H), _p(st.levels), _p(st.levels_last),
                              _p(st.final_T), _p(st.n_contrib), _p(color), ctypes.c_int(foveaStep), _p(color))
    return color, fwd.radii, st


def orc_fovea(L, step, T, st: AMRState):
    L.orc_amr_fovea_levels(ctypes.c_int(step), ctypes.c_int(T), _p(st.levels_last), _p(st.levels_current),
                           _p(st.levels))


def fovea_levels(levels, W: int, H: int, centres, radii, min_level: int = 1, replace: bool = False):
    """Extension beyond parity (no reference implementation exists): the
    fovea-driven level rule of csrc/amr.hip fovea_override_kernel, restated.
    It implements the reference's TODO (gaussian_renderer_amr/__init__.py:244)
    with its unused fovea discs (:98-106).  Tile rectangle [x0, x1] x [y0, y1]
    in pixel coordinates; inside disc k when the float32 squared distance from
    the centre to the rectangle is <= radius^2 (float32)."""
    tile = 32
    gx = (W + tile - 1) // tile
    out = np.asarray(levels, np.uint32).copy()
    f32 = np.float32
    for t in range(out.shape[0]):
        tx, ty = t % gx, t // gx
        x0, y0 = f32(tx * tile), f32(ty * tile)
        x1, y1 = f32(min(tx * tile + tile, W)) - f32(1), f32(min(ty * tile + tile, H)) - f32(1)
        F = 0
        for k, (c, r) in enumerate(zip(centres, radii)):
            cx, cy, rr = f32(c[0]), f32(c[1]), f32(r)
            dx = max(x0 - cx, cx - x1, f32(0))
            dy = max(y0 - cy, cy - y1, f32(0))
            if f32(dx * dx) + f32(dy * dy) > f32(rr * rr):
                break
            F = k + 1
        f = max(F, min_level)
        out[t] = f if replace else min(int(out[t]), f)
    return out


def amr_render_foveated(s: Settings, scene_kwargs: dict, interpolate_image: bool = False, levels_hook=None):
    """gaussian_renderer_amr/__init__.py:24-608: steps 0..4, summing the partial
    images.  ``levels_hook(levels) -> levels`` (extension) rewrites the step-0
    tile levels before the progressive steps."""
    c0, radii, st = amr_forward(s, foveaStep=0, **scene_kwargs)
    if levels_hook is not None:
        st.levels[:] = levels_hook(st.levels)
    acc = c0.copy()
    steps = [c0]
    for k in range(1, 5):
        interp = interpolate_image if k == 4 else False
        ck, _, st = amr_forward(s, foveaStep=k, out_color_precomp=acc, state=st, interpolate_image=interp,
                                **scene_kwargs)
        steps.append(ck)
        acc = acc + ck
    return acc, radii, st, steps


def amr_render_once(s: Settings, scene_kwargs: dict):
    """gaussian_renderer_amr/__init__.py:612-749: one call with foveaStep=-2, interpolate=True."""
    return amr_forward(s, foveaStep=-2, interpolate_image=True, **scene_kwargs)


def amr_pixel_rounds(W: int, H: int) -> np.ndarray:
    """amr/cr/forward.cu:313-339: the AMR round of every pixel, [H, W]."""
    ys, xs = np.mgrid[0:H, 0:W]
    ox, oy = xs & 1, ys & 1
    return np.where(ox == 0, np.where(oy == 0, 1, 4), np.where(oy == 0, 3, 2)).astype(np.uint32)


def amr_tile_levels_per_pixel(levels, W: int, H: int) -> np.ndarray:
    tgx = (W + 31) // 32
    ys, xs = np.mgrid[0:H, 0:W]
    return np.minimum(np.asarray(levels, np.uint32)[(ys // 32) * tgx + xs // 32], 4)


def amr_interp_fold(dL_dpix, levels, W: int, H: int) -> np.ndarray:
    """Adjoint of render_once's interpolation (amr/cr/forward.cu:520-648): a
    pixel with round > level copies its 2x2 cell's (0,0) (levels 1, 2) or
    (1,1) (level 3) pixel, so its cotangent moves there (copies summed in
    round order, as csrc/amr.hip amr_interp_fold_kernel)."""
    g = np.asarray(dL_dpix, np.float32)
    out = np.zeros_like(g)
    rnd = amr_pixel_rounds(W, H)
    lvl = amr_tile_levels_per_pixel(levels, W, H)
    order = [(0, 0), (1, 1), (1, 0), (0, 1)]  # (dx, dy) of rounds 1..4
    for cy in range(0, H, 2):
        for cx in range(0, W, 2):
            L = int(lvl[cy, cx])
            o = 1 if L in (3, 4) else 0
            sx, sy = cx + o, cy + o
            src_in = sx < W and sy < H
            fold = np.zeros(3, np.float32)
            for r, (dx, dy) in enumerate(order):
                px, py = cx + dx, cy + dy
                if px >= W or py >= H:
                    continue
                if r + 1 <= L:
                    out[:, py, px] = g[:, py, px]
                elif src_in:
                    fold = (fold + g[:, py, px]).astype(np.float32)
            if src_in and L < 4:
                out[:, sy, sx] = (out[:, sy, sx] + fold).astype(np.float32)
    return out


def amr_backward(s: Settings, scene_kwargs: dict, dL_dpix, foveaStep: int, levels,
                 interpolate_image: bool = False) -> dict:
    """Extension beyond parity (the reference's AMR backward is unreachable):
    the gradients of one AMR call's image.  Every pixel the AMR render blends
    gets the state of a 32-px-tile base blend, so the backward is the base
    backward on the 32-px binning with the cotangent kept on the rendered
    pixels only -- foveaStep k > 0: round k where level >= k; < 0
    (render_once): round <= level, after folding the interpolation copies."""
    W, H = int(s.image_width), int(s.image_height)
    kw = dict(scene_kwargs)
    means3D = kw.pop("means3D")
    opacities = kw.pop("opacities")
    fwd = forward(s, means3D, opacities, block=32, **kw)
    g = np.asarray(dL_dpix, np.float32)
    if interpolate_image:
        if foveaStep > 0:
            raise ValueError("interpolate_image is differentiated for render_once only")
        g = amr_interp_fold(g, levels, W, H)
    rnd = amr_pixel_rounds(W, H)
    lvl = amr_tile_levels_per_pixel(levels, W, H)
    keep = (rnd == foveaStep) & (lvl >= foveaStep) if foveaStep > 0 else rnd <= lvl
    g = np.where(keep[None], g, np.float32(0)).astype(np.float32)
    return backward(s, fwd, means3D, g, block=32, **kw)


# ------------------------------------------------------------- simple-knn ---
def dist_cuda2(points) -> np.ndarray:
    pts = _f32(points)
    P = pts.shape[0]
    out = np.zeros(P, np.float32)
    lib().orc_knn(ctypes.c_int(P), _p(pts), _p(out), None, None, None)
    return out


def knn_intermediates(points):
    pts = _f32(points)
    P = pts.shape[0]
    nb = (P + 1023) // 1024
    out = np.zeros(P, np.float32)
    morton = np.zeros(P, np.uint32)
    idx = np.zeros(P, np.uint32)
    boxes = np.zeros((max(nb, 1), 6), np.float32)
    lib().orc_knn(ctypes.c_int(P), _p(pts), _p(out), _p(morton), _p(idx), _p(boxes))
    return out, morton, idx, boxes[:nb]
