"""GPU parity: the HIP path (through the drop-in API / C ABI) against the CPU
oracle on identical seeded inputs.

Bars (BASELINE.json north_star): tile keys / point_list / ranges and every
integer buffer bit-exact; preprocess floats bit-exact (same op order, no
contraction); image L1 < 1e-5; gradients within 1e-4 relative (L2 norm).
"""
import numpy as np
import pytest

import gs_helpers as G

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CASES = [
    ("g1_64_32x32", 64, 32, 32, 3),
    ("cfg1_10k_256", 10000, 256, 256, 0),
    ("ragged_3k_250x130", 3000, 250, 130, 7),
    ("dense_20k_128", 20000, 128, 128, 11),  # large tiles: exercises the merge-sort path
    ("grid_17k_tiles", 3000, 2112, 2080, 5),  # T = 17160 > kLdsTiles: device-atomic binning path
]


def _gpu_forward(sc, cam, colors_precomp=None, cov3D_precomp=None, bg=(0.0, 0.0, 0.0), keep_scales=False):
    import gaussian_splatting_with_eye_tracking_amd._C as C
    s = G.torch_settings(cam, bg=bg)
    t = G.scene_tensors(sc)
    e = torch.Tensor([])
    sh = t["shs"] if colors_precomp is None else e
    col = e if colors_precomp is None else torch.from_numpy(colors_precomp).cuda()
    scales = t["scales"] if cov3D_precomp is None or keep_scales else e
    rots = t["rotations"] if cov3D_precomp is None or keep_scales else e
    cov = e if cov3D_precomp is None else torch.from_numpy(cov3D_precomp).cuda()
    out = C.rasterize_gaussians(s.bg, t["means3D"], col, t["opacities"], scales, rots, s.scale_modifier, cov,
                                s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh,
                                s.sh_degree, s.campos, s.prefiltered, s.debug)
    torch.cuda.synchronize()
    return s, t, out


def _oracle_forward(sc, cam, colors_precomp=None, cov3D_precomp=None, bg=(0.0, 0.0, 0.0), keep_scales=False):
    import oracle as O
    s = O.settings_from_camera(cam, bg=bg)
    both = cov3D_precomp is None or keep_scales
    kw = dict(shs=sc.shs if colors_precomp is None else None, colors_precomp=colors_precomp,
              scales=sc.scales if both else None,
              rotations=sc.rotations if both else None, cov3D_precomp=cov3D_precomp)
    return s, O.forward(s, sc.means3D, sc.opacities, **kw), kw


@pytest.mark.parametrize("name,P,W,H,seed", CASES)
def test_forward_buffers_bit_exact(name, P, W, H, seed):
    _forward_buffers_bit_exact(name, P, W, H, seed)


def _forward_buffers_bit_exact(name, P, W, H, seed):
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(P, W, H, seed)
    C.set_thread_option("store_cov3d", 1)  # the geometry buffer's cov3D is written on request only
    try:
        _, _, (K, color, radii, geom, binning, img) = _gpu_forward(sc, cam)
    finally:
        C.set_thread_option("store_cov3d", 0)
    _, ref, _ = _oracle_forward(sc, cam)
    assert K == ref.num_rendered
    d = C.parse_buffers(geom, binning, img, P, K, W, H, 16)
    np.testing.assert_array_equal(radii.cpu().numpy(), ref.radii)
    vis = ref.radii > 0
    np.testing.assert_array_equal(d["depths"].cpu().numpy()[vis], ref.depths[vis])
    np.testing.assert_array_equal(d["means2D"].cpu().numpy()[vis], ref.means2D[vis])
    np.testing.assert_array_equal(d["conic_opacity"].cpu().numpy()[vis], ref.conic_opacity[vis])
    np.testing.assert_array_equal(d["rgb"].cpu().numpy()[vis], ref.rgb[vis])
    np.testing.assert_array_equal(d["cov3D"].cpu().numpy()[vis], ref.cov3D[vis])
    cb = d["clamped_bits"].cpu().numpy()[vis]
    ref_cb = (ref.clamped[vis] * np.array([1, 2, 4], np.uint8)).sum(1)
    np.testing.assert_array_equal(cb, ref_cb)
    np.testing.assert_array_equal(d["tiles_touched"].cpu().numpy().astype(np.uint32), ref.tiles_touched)
    np.testing.assert_array_equal(d["ranges"].cpu().numpy().astype(np.uint32), ref.ranges)
    if K:
        np.testing.assert_array_equal(d["point_list"].cpu().numpy().astype(np.uint32), ref.point_list)
        np.testing.assert_array_equal(d["point_list_keys"].cpu().numpy().view(np.uint64), ref.point_list_keys)


@pytest.mark.parametrize("name,P,W,H,seed", CASES)
def test_forward_image(name, P, W, H, seed):
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(P, W, H, seed)
    _, _, (K, color, radii, geom, binning, img) = _gpu_forward(sc, cam, bg=(0.1, 0.2, 0.3))
    _, ref, _ = _oracle_forward(sc, cam, bg=(0.1, 0.2, 0.3))
    assert G.image_l1(color.cpu().numpy(), ref.color) < G.IMAGE_L1_TOL
    d = C.parse_buffers(geom, binning, img, P, K, W, H, 16)
    ncont = d["n_contrib"].cpu().numpy().astype(np.uint32)
    assert np.mean(ncont != ref.n_contrib) < 1e-3  # exp is hardware v_exp_f32 vs libm expf
    assert G.image_l1(d["accum_alpha"].cpu().numpy(), ref.final_T) < G.IMAGE_L1_TOL


@pytest.mark.parametrize("name,P,W,H,seed", CASES[:3])
@pytest.mark.parametrize("variant", ["sh", "colors_precomp", "cov3D_precomp", "cov3D_precomp_and_scales"])
def test_backward_parity(name, P, W, H, seed, variant):
    # cov3D_precomp_and_scales: both covariance inputs, as the raw binding and
    # the C ABI accept them -- the forward renders the precomputed covariance,
    # the backward's cov2D step must read it (base/cr/backward.cu:160,
    # rasterizer_impl.cu:411) while the scales / rotations still receive the
    # cov3D backward (backward.cu:395-396).  The covariance is deliberately not
    # the one the scales would give.
    import oracle as O
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    sc, cam = G.scene_and_camera(P, W, H, seed)
    colors = None
    cov = None
    if variant == "colors_precomp":
        colors = np.random.default_rng(seed + 5).uniform(0, 1, (P, 3)).astype(np.float32)
    both = variant == "cov3D_precomp_and_scales"
    if variant.startswith("cov3D_precomp"):
        _, r0, _ = _oracle_forward(sc, cam)
        cov = r0.cov3D.copy()
        # invisible Gaussians have no computed cov3D: give them a valid one
        cov[r0.radii <= 0] = np.array([1e-4, 0, 0, 1e-4, 0, 1e-4], np.float32)
        if both:
            cov *= np.float32(1.3)
    bg = (0.2, 0.1, 0.05)
    s, t, (K, color, radii, geom, binning, img) = _gpu_forward(sc, cam, colors, cov, bg=bg, keep_scales=both)
    os_, ref, kw = _oracle_forward(sc, cam, colors, cov, bg=bg, keep_scales=both)
    dpix = S.make_cotangent(H, W, seed + 1)
    import gaussian_splatting_with_eye_tracking_amd._C as C
    e = torch.Tensor([])
    sh = t["shs"] if colors is None else e
    colt = e if colors is None else torch.from_numpy(colors).cuda()
    scales = t["scales"] if cov is None or both else e
    rots = t["rotations"] if cov is None or both else e
    covt = e if cov is None else torch.from_numpy(cov).cuda()
    grads = C.rasterize_gaussians_backward(s.bg, t["means3D"], radii, colt, scales, rots, s.scale_modifier, covt,
                                           s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy,
                                           torch.from_numpy(dpix).cuda(), sh, s.sh_degree, s.campos, geom, K, binning,
                                           img, False)
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    rg = O.backward(os_, ref, sc.means3D, dpix, **kw)
    for n, g in zip(names, grads):
        gg = g.cpu().numpy()
        assert gg.shape == rg[n].shape, n
        assert np.all(np.isfinite(gg)), n
        assert G.rel_err(gg, rg[n]) < G.GRAD_REL_TOL, (n, G.rel_err(gg, rg[n]))
    al, ties = O.grad_allowance(os_, ref, sc.means3D, dpix, parts=True, **kw)
    G.assert_grads_elementwise(f"backward_{name}_{variant}", names, grads, rg, sc, cam, ref, allow=al, ties=ties)
    # the autograd wrappers' binding: the same bits, colour / covariance
    # gradients only when their precomputed input was given
    lean = C.rasterize_gaussians_backward_lean(s.bg, t["means3D"], radii, colt, scales, rots, s.scale_modifier, covt,
                                               s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy,
                                               torch.from_numpy(dpix).cuda(), sh, s.sh_degree, s.campos, geom, K,
                                               binning, img, False)
    for n, g, gl in zip(names, grads, lean):
        if (n == "dL_dcolors" and colors is None) or (n == "dL_dcov3D" and cov is None):
            assert gl.numel() == 0, n
        else:
            assert G.rel_err(gl.cpu().numpy(), g.cpu().numpy()) < 1e-5, n  # (float atomics: run-order noise)


def test_backward_parity_without_forward_zeroing():
    """fwd_zero 0: the forward leaves the accumulator rows alone and the
    backward zeroes them itself (the path a forward under the forward-only
    hint takes): gradients against the oracle."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    C.set_thread_option("fwd_zero", 0)
    try:
        test_backward_parity("cfg1_10k_256", 10000, 256, 256, 0, "sh")
        test_backward_parity("ragged_3k_250x130", 3000, 250, 130, 7, "colors_precomp")
    finally:
        C.set_thread_option("fwd_zero", 1)


def test_backward_parity_gauss_forms():
    """bwd_gauss's two SH16 kernels against the oracle: the drgb-known kernel
    (the forward stored d(rgb)/d(dir), dL_dsh in two half-size LDS rounds: the
    default) and the coefficient kernel (sh_drgb 0: the SH rows staged
    through LDS); the forward-only hint's path is
    test_backward_without_stored_sh_derivatives."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    for drgb in (1, 0):
        C.set_thread_option("sh_drgb", drgb)
        try:
            test_backward_parity("cfg1_10k_256", 10000, 256, 256, 0, "sh")
            test_backward_parity("ragged_3k_250x130", 3000, 250, 130, 7, "sh")
            test_backward_parity("g1_64_32x32", 64, 32, 32, 3, "sh")
        finally:
            C.set_thread_option("sh_drgb", 1)


@pytest.mark.parametrize("P,W,H", [(20000, 128, 128), (2_100_000, 160, 96), (20000, 1000, 40), (20000, 16400, 16)])
def test_binning_forms_bit_exact(P, W, H):
    """The binning's size-dependent forms against the oracle, bit for bit:
    the row-banded duplicate (binning.hip band_stage_kernel /
    band_split_kernel: 1024 x 1 below 2M Gaussians, 512 x 2 sources and 8
    sub-bucket count slots from 2M), a wide grid (few rows, many split
    workgroups per row) and a grid wider than one append round's 1024 bins
    (16400 px: the direct LDS duplicate); each forward twice (the second runs
    the duplicate speculatively)."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(P, W, H, 12)
    _gpu_forward(sc, cam)
    _, _, (K, color, radii, geom, binning, img) = _gpu_forward(sc, cam)
    _, ref, _ = _oracle_forward(sc, cam)
    assert K == ref.num_rendered
    d = C.parse_buffers(geom, binning, img, P, K, W, H, 16)
    np.testing.assert_array_equal(d["ranges"].cpu().numpy().astype(np.uint32), ref.ranges)
    np.testing.assert_array_equal(d["point_list"].cpu().numpy().astype(np.uint32), ref.point_list)
    assert G.image_l1(color.cpu().numpy(), ref.color) < G.IMAGE_L1_TOL


def _clustered_scene(P, cam, seed, kind):
    """Depth distributions that stress the per-tile sort: 'ties' -- a third of
    the Gaussians are exact copies (same mean, so the same depth bits: the
    order falls to the index, as after clone densification); 'cluster' -- 90 %
    of the depths within 0.1 % of each other plus a few far outliers (the
    bucket map's range is wide, its buckets crowded: the bitonic fallback);
    'two' -- two depth planes."""
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    sc = S.make_scene(P, cam, seed=seed)
    rng = np.random.default_rng(seed + 99)
    m = sc.means3D.copy()
    f = np.where(rng.random(P) < 0.5, 1.0, rng.random(P))  # half uniform, half towards the centre
    m[:, :2] *= f[:, None].astype(np.float32)  # (tiles of every size class)
    if kind == "ties":
        src = rng.integers(0, P // 20, P // 3)
        dst = rng.choice(np.arange(P // 20, P), P // 3, replace=False)
        m[dst] = m[src]
    elif kind == "cluster":
        z = np.where(rng.random(P) < 0.9, 5.0 + 0.005 * rng.random(P), 2.0 + 18.0 * rng.random(P)).astype(np.float32)
        m[:, :2] *= (z / m[:, 2])[:, None]
        m[:, 2] = z
    else:
        z = np.where(rng.random(P) < 0.5, 4.0, 9.0).astype(np.float32)
        m[:, :2] *= (z / m[:, 2])[:, None]
        m[:, 2] = z
    sc.means3D = m.astype(np.float32)
    return sc


@pytest.mark.parametrize("kind", ["ties", "cluster", "two"])
@pytest.mark.parametrize("sort_algo", [0, 1])
def test_tile_sort_adversarial_depths(kind, sort_algo):
    """point_list / ranges bit-exact against the oracle's stable (depth, idx)
    order for both tile sorts (bucket sort, bitonic networks) on tiles of
    every size class (<= 1024, <= 2048, <= 4096 and the merge path)."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H = 100000, 256, 192
    cam = S.make_camera(W, H)
    sc = _clustered_scene(P, cam, 5, kind)
    C.set_tuning("sort_algo", sort_algo)
    try:
        _, _, (K, color, radii, geom, binning, img) = _gpu_forward(sc, cam)
    finally:
        C.set_tuning("sort_algo", 1)
    _, ref, _ = _oracle_forward(sc, cam)
    assert K == ref.num_rendered
    n = ref.ranges[:, 1] - ref.ranges[:, 0]
    assert all(((n > a) & (n <= b)).any() for a, b in ((1, 1024), (1024, 2048), (2048, 4096), (4096, 1 << 30)))
    d = C.parse_buffers(geom, binning, img, P, K, W, H, 16)
    np.testing.assert_array_equal(d["ranges"].cpu().numpy().astype(np.uint32), ref.ranges)
    np.testing.assert_array_equal(d["point_list"].cpu().numpy().astype(np.uint32), ref.point_list)
    np.testing.assert_array_equal(d["point_list_keys"].cpu().numpy().view(np.uint64), ref.point_list_keys)


def test_backward_with_unfilled_work_buckets():
    """render_bwd takes its heaviest-first order from the work buckets the
    base forward render fills.  An image buffer whose buckets do not cover
    the grid (zeroed here, as after a forward that never rendered) must not
    drop tiles: every block falls back to the identity order and the
    gradients are unchanged (atomic-order noise only)."""
    import ctypes
    import os
    import gaussian_splatting_with_eye_tracking_amd as pkg
    import gaussian_splatting_with_eye_tracking_amd._C as C
    P, W, H, seed = 3000, 250, 130, 7
    sc, cam = G.scene_and_camera(P, W, H, seed)
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    dpix = torch.from_numpy(S.make_cotangent(H, W, seed + 1)).cuda()
    lib = ctypes.CDLL(os.path.join(os.path.dirname(pkg.__file__), "libgsplat_amd.so"))
    view = (ctypes.c_void_p * 19)()  # gs_image_view: 19 pointers
    base = 1 << 20
    assert lib.gs_image_view_of(ctypes.c_void_p(base), W, H, 16, ctypes.byref(view)) == 0
    off = view[15] - base  # bucket_count
    e = torch.Tensor([])
    out = []
    for corrupt in (False, True):
        s, t, (K, color, radii, geom, binning, img) = _gpu_forward(sc, cam)
        if corrupt:
            img[off:off + 1024].zero_()
        g = C.rasterize_gaussians_backward(s.bg, t["means3D"], radii, e, t["scales"], t["rotations"],
                                           s.scale_modifier, e, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy,
                                           dpix, t["shs"], s.sh_degree, s.campos, geom, K, binning, img, False)
        out.append([x.cpu().numpy() for x in g])
    for a, b in zip(*out):
        assert np.all(np.isfinite(b))
        assert G.rel_err(b, a) < 1e-5


def _psnr(img, gt):
    """utils/image_utils.py:19-21 (per leading row, then the mean as
    metrics.py / train.py report it), on images clamped to [0, 1] as saved."""
    img = np.clip(img, 0.0, 1.0).astype(np.float64)
    gt = np.clip(gt, 0.0, 1.0).astype(np.float64)
    mse = ((img - gt) ** 2).reshape(img.shape[0], -1).mean(1)
    return float(np.mean(20.0 * np.log10(1.0 / np.sqrt(mse))))


def test_config2_full_size_parity_and_psnr():
    """BASELINE config 2 at full size (1M Gaussians, 1920x1080, seed 0):
    the tile keys / point_list / ranges bit-exact, the image within the L1
    bar, PSNR against a target within 0.01 dB of the oracle's (the
    north_star's PSNR bar), and every gradient within 1e-4 relative."""
    import oracle as O
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H = 1_000_000, 1920, 1080
    sc, cam = G.scene_and_camera(P, W, H, 0)
    s, t, (K, color, radii, geom, binning, img) = _gpu_forward(sc, cam)
    os_, ref, kw = _oracle_forward(sc, cam)
    assert K == ref.num_rendered
    d = C.parse_buffers(geom, binning, img, P, K, W, H, 16)
    np.testing.assert_array_equal(radii.cpu().numpy(), ref.radii)
    np.testing.assert_array_equal(d["ranges"].cpu().numpy().astype(np.uint32), ref.ranges)
    np.testing.assert_array_equal(d["point_list"].cpu().numpy().astype(np.uint32), ref.point_list)
    np.testing.assert_array_equal(d["point_list_keys"].cpu().numpy().view(np.uint64), ref.point_list_keys)
    got = color.cpu().numpy()
    assert G.image_l1(got, ref.color) < G.IMAGE_L1_TOL
    gt = np.clip(ref.color + np.random.default_rng(3).normal(0, 0.05, ref.color.shape), 0, 1).astype(np.float32)
    assert abs(_psnr(got, gt) - _psnr(ref.color, gt)) < 0.01
    assert _psnr(got, ref.color) > 80.0
    dpix = S.make_cotangent(H, W, 1)
    e = torch.Tensor([])
    grads = C.rasterize_gaussians_backward(s.bg, t["means3D"], radii, e, t["scales"], t["rotations"],
                                           s.scale_modifier, e, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy,
                                           torch.from_numpy(dpix).cuda(), t["shs"], s.sh_degree, s.campos, geom, K,
                                           binning, img, False)
    rg = O.backward(os_, ref, sc.means3D, dpix, **kw)
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    for n, g in zip(names, grads):
        assert G.rel_err(g.cpu().numpy(), rg[n]) < G.GRAD_REL_TOL, (n, G.rel_err(g.cpu().numpy(), rg[n]))
    al, ties = O.grad_allowance(os_, ref, sc.means3D, dpix, parts=True, **kw)
    G.assert_grads_elementwise("config2", names, grads, rg, sc, cam, ref, allow=al, ties=ties)


@pytest.mark.parametrize("bwd_variant", [0, 1])  # the fallback and the default (opacity-scaled sums)
@pytest.mark.parametrize("fwd_variant", [0, 1])
def test_blend_geometries_match_oracle(fwd_variant, bwd_variant):
    """The default and the fallback forward / backward blends (gs_set_tuning),
    every pairing, against the oracle (the fallback forward leaves no hit
    codes: the backward then culls by geometry)."""
    import oracle as O
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H, seed = 10000, 256, 256, 0
    sc, cam = G.scene_and_camera(P, W, H, seed)
    try:
        C.set_tuning("fwd_variant", fwd_variant)
        C.set_tuning("bwd_variant", bwd_variant)
        s, t, (K, color, radii, geom, binning, img) = _gpu_forward(sc, cam, bg=(0.2, 0.1, 0.05))
        dpix = S.make_cotangent(H, W, seed + 1)
        e = torch.Tensor([])
        grads = C.rasterize_gaussians_backward(s.bg, t["means3D"], radii, e, t["scales"], t["rotations"],
                                               s.scale_modifier, e, s.viewmatrix, s.projmatrix, s.tanfovx,
                                               s.tanfovy, torch.from_numpy(dpix).cuda(), t["shs"], s.sh_degree,
                                               s.campos, geom, K, binning, img, False)
        torch.cuda.synchronize()
    finally:
        C.set_tuning("fwd_variant", -1)
        C.set_tuning("bwd_variant", -1)
    os_, ref, kw = _oracle_forward(sc, cam, bg=(0.2, 0.1, 0.05))
    assert G.image_l1(color.cpu().numpy(), ref.color) < G.IMAGE_L1_TOL
    rg = O.backward(os_, ref, sc.means3D, dpix, **kw)
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    for n, g in zip(names, grads):
        assert G.rel_err(g.cpu().numpy(), rg[n]) < G.GRAD_REL_TOL, (n, fwd_variant, bwd_variant)


def test_autograd_dropin_matches_direct_call():
    """The drop-in GaussianRasterizer (autograd) returns the same image and
    gradients as the raw _C calls, in the reference's gradient order."""
    from diff_gaussian_rasterization import GaussianRasterizer
    sc, cam = G.scene_and_camera(2000, 96, 64, 2)
    s = G.torch_settings(cam)
    t = G.scene_tensors(sc, requires_grad=True)
    means2D = torch.zeros_like(t["means3D"], requires_grad=True)
    ras = GaussianRasterizer(s)
    color, radii = ras(means3D=t["means3D"], means2D=means2D, opacities=t["opacities"], shs=t["shs"],
                       scales=t["scales"], rotations=t["rotations"])
    dpix = torch.randn_like(color)
    (color * dpix).sum().backward()
    assert means2D.grad is not None and torch.all(means2D.grad[:, 2] == 0)
    for k in ("means3D", "opacities", "shs", "scales", "rotations"):
        assert t[k].grad is not None and torch.isfinite(t[k].grad).all(), k
    vis = ras.markVisible(t["means3D"].detach())
    import oracle as O
    np.testing.assert_array_equal(vis.cpu().numpy(),
                                  O.mark_visible(sc.means3D, cam.world_view_transform, cam.full_proj_transform))


def test_second_backward_of_one_forward_rezeroes():
    """The forward render zeroes the backward's accumulator rows (the first
    backward skips its memset); a second backward of the same forward
    (retain_graph) must zero them itself: equal gradients both times, and the
    radii / unused-image cases hand autograd no materialised zeros."""
    from diff_gaussian_rasterization import GaussianRasterizer
    sc, cam = G.scene_and_camera(10000, 256, 256, 0)
    s = G.torch_settings(cam)
    t = G.scene_tensors(sc, requires_grad=True)
    means2D = torch.zeros_like(t["means3D"], requires_grad=True)
    color, radii = GaussianRasterizer(s)(means3D=t["means3D"], means2D=means2D, opacities=t["opacities"],
                                         shs=t["shs"], scales=t["scales"], rotations=t["rotations"])
    dpix = torch.randn_like(color)
    keys = ("means3D", "opacities", "shs", "scales", "rotations")
    g1 = torch.autograd.grad((color * dpix).sum(), [t[k] for k in keys] + [means2D], retain_graph=True)
    g2 = torch.autograd.grad((color * dpix).sum(), [t[k] for k in keys] + [means2D])
    for k, a, b in zip(keys + ("means2D",), g1, g2):
        assert float((a - b).abs().max()) <= 1e-5 * max(float(a.abs().max()), 1e-30), k
    # a loss on the radii alone: no gradient reaches the Gaussians
    color, radii = GaussianRasterizer(s)(means3D=t["means3D"], means2D=means2D, opacities=t["opacities"],
                                         shs=t["shs"], scales=t["scales"], rotations=t["rotations"])
    gz = torch.autograd.grad(color.sum() * 0 + radii.float().sum() * 0, [t["means3D"]], allow_unused=True)
    assert gz[0] is None or float(gz[0].abs().max()) == 0.0


def test_speculative_duplicate_matches_synchronous():
    """The base forward launches the duplicate before K is on the host, into
    a binning buffer sized by the previous call's K (+1/8): a call whose K
    exceeds that capacity must relaunch it (here the 30k scene after the
    10k one), a call within it must keep it; images and gradients are
    bit-identical to the synchronous path (tuning "spec_dup" 0)."""
    from diff_gaussian_rasterization import GaussianRasterizer
    import gaussian_splatting_with_eye_tracking_amd._C as C
    scenes = [G.scene_and_camera(P, 256, 192, seed) for P, seed in ((10000, 0), (30000, 1), (30000, 1), (8000, 2))]

    def run():
        out = []
        for sc, cam in scenes:
            s = G.torch_settings(cam)
            t = G.scene_tensors(sc, requires_grad=True)
            m2 = torch.zeros_like(t["means3D"], requires_grad=True)
            color, radii = GaussianRasterizer(s)(means3D=t["means3D"], means2D=m2, opacities=t["opacities"],
                                                 shs=t["shs"], scales=t["scales"], rotations=t["rotations"])
            g = torch.autograd.grad((color * color).sum(), [t["means3D"], t["opacities"]])
            out.append((color.detach().clone(), radii.clone()) + tuple(x.clone() for x in g))
        return out

    try:
        C.set_tuning("spec_dup", 0)
        ref = run()
        C.set_tuning("spec_dup", 1)
        spec = run()
    finally:
        C.set_tuning("spec_dup", 1)
    for i, (a, b) in enumerate(zip(ref, spec)):
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), i
        for x, y in zip(a[2:], b[2:]):
            assert float((x - y).abs().max()) <= 1e-5 * max(float(x.abs().max()), 1e-30), i


def test_empty_scene():
    from diff_gaussian_rasterization import GaussianRasterizer
    sc, cam = G.scene_and_camera(0, 64, 48)
    s = G.torch_settings(cam)
    t = G.scene_tensors(sc)
    color, radii = GaussianRasterizer(s)(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]),
                                          opacities=t["opacities"], shs=t["shs"], scales=t["scales"],
                                          rotations=t["rotations"])
    assert color.shape == (3, 48, 64) and torch.all(color == 0) and radii.numel() == 0


def test_all_culled():
    """Every Gaussian behind the near plane: K = 0, image = background."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(500, 64, 48)
    sc.means3D[:, 2] = -5.0
    s, t, (K, color, radii, geom, binning, img) = _gpu_forward(sc, cam, bg=(0.5, 0.25, 0.125))
    assert K == 0 and torch.all(radii == 0)
    np.testing.assert_allclose(color.cpu().numpy()[:, 0, 0], [0.5, 0.25, 0.125])


def test_prefiltered_violation_raises():
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(100, 32, 32)
    sc.means3D[0, 2] = -1.0
    s = G.torch_settings(cam)
    t = G.scene_tensors(sc)
    with pytest.raises(RuntimeError, match="prefiltered"):
        C.rasterize_gaussians(s.bg, t["means3D"], torch.Tensor([]), t["opacities"], t["scales"], t["rotations"], 1.0,
                              torch.Tensor([]), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, 32, 32, t["shs"], 3,
                              s.campos, True, False)
    # the header is not zeroed per call: the next calls (the caching allocator
    # hands back the same geometry bytes, stale error word included) must not
    # raise once every point is in front of the camera
    ok = t["means3D"].clone()
    ok[0, 2] = 5.0
    for _ in range(3):
        out = C.rasterize_gaussians(s.bg, ok, torch.Tensor([]), t["opacities"], t["scales"], t["rotations"], 1.0,
                                    torch.Tensor([]), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, 32, 32,
                                    t["shs"], 3, s.campos, True, False)
        assert out[0] > 0


# ---------------------------------------------------------------- AMR ----
def _amr_gpu_steps(sc, cam, interpolate_last=False, bg=(0.0, 0.0, 0.0), after_step0=None):
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    s = G.torch_settings(cam, amr=True, bg=bg)
    t = G.scene_tensors(sc)
    e = torch.Tensor([])
    u8 = torch.Tensor([]).to(torch.uint8)
    means2D = torch.zeros_like(t["means3D"])
    args = (t["means3D"], means2D, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    c0, radii, gb, bb, ib = _RasterizeGaussians.apply(*args, 0, e, u8, u8, u8, False, s)
    if after_step0 is not None:
        after_step0(ib)
    acc = c0
    steps = [c0]
    for k in range(1, 5):
        ck, rk, gb, bb, ib = _RasterizeGaussians.apply(*args, k, acc, gb, bb, ib, interpolate_last and k == 4, s)
        assert rk.shape == radii.shape and not bool(rk.any())  # the steps return zero radii, as the reference
        steps.append(ck)
        acc = acc + ck
    torch.cuda.synchronize()
    return acc, radii, steps, (gb, bb, ib)


@pytest.mark.parametrize("amr_variant", [4, 0])
@pytest.mark.parametrize("name,P,W,H,seed", [("amr_10k_256", 10000, 256, 256, 0), ("amr_ragged", 4000, 200, 120, 3),
                                             # 66 x 33 = 2178 tiles > 2048: the radix-select percentile path
                                             ("amr_big_grid", 3000, 2112, 1056, 8),
                                             # dense: long sub-lists (several 32-entry batches per region)
                                             ("amr_dense", 60000, 160, 96, 4)])
def test_amr_foveated_steps(name, P, W, H, seed, amr_variant):
    """Both AMR blends (4: 8x8-region sub-lists + records, the default; 0:
    full 32-px lists, the fallback) against the oracle: per-step images, and
    per pixel n_contrib / final T of the last step that rendered it (the
    contributor indices of the sub-lists are the positions in the tile
    list)."""
    import oracle as O
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(P, W, H, seed)
    C.set_tuning("amr_variant", amr_variant)
    try:
        acc, radii, steps, (gb, bb, ib) = _amr_gpu_steps(sc, cam, bg=(0.1, 0.1, 0.1))
    finally:
        C.set_tuning("amr_variant", 4)
    s = O.settings_from_camera(cam, bg=(0.1, 0.1, 0.1))
    kw = dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    racc, rradii, st, rsteps = O.amr_render_foveated(s, kw)
    np.testing.assert_array_equal(radii.cpu().numpy(), rradii)
    K = st.fwd.num_rendered
    d = C.parse_buffers(gb, bb, ib, P, K, W, H, 32)
    np.testing.assert_array_equal(d["ranges"].cpu().numpy().astype(np.uint32), st.fwd.ranges)
    np.testing.assert_array_equal(d["point_list"].cpu().numpy().astype(np.uint32), st.fwd.point_list)
    np.testing.assert_array_equal(d["pv"].cpu().numpy()[:3].astype(np.uint32), st.percentile_values)
    np.testing.assert_array_equal(d["levels"].cpu().numpy().astype(np.uint32), st.levels)
    np.testing.assert_array_equal(d["levels_last"].cpu().numpy().astype(np.uint32), st.levels_last)
    np.testing.assert_array_equal(d["levels_current"].cpu().numpy().astype(np.uint32), st.levels_current)
    assert torch.all(steps[0] == 0)
    for k in range(5):
        assert G.image_l1(steps[k].cpu().numpy(), rsteps[k]) < G.IMAGE_L1_TOL, k
    assert G.image_l1(acc.cpu().numpy(), racc) < G.IMAGE_L1_TOL
    # pixels some step rendered (round <= level); the others are never written
    rendered = (O.amr_pixel_rounds(W, H) <= O.amr_tile_levels_per_pixel(st.levels, W, H)).reshape(-1)
    nc = d["n_contrib"].cpu().numpy().astype(np.uint32)[rendered]
    rnc = st.n_contrib[rendered]
    assert np.mean(nc != rnc) < 1e-3  # exp is hardware v_exp_f32 vs libm expf
    same = nc == rnc
    np.testing.assert_allclose(d["accum_alpha"].cpu().numpy()[rendered][same], st.final_T[rendered][same],
                               rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("name,P,W,H,seed", [("amr_10k_256", 10000, 256, 256, 0), ("amr_big_grid", 3000, 2112, 1056, 8),
                                             ("amr_dense", 60000, 160, 96, 4),
                                             # tile counts >= 2^16: the LDS sort of the counts
                                             ("amr_huge_counts", 150000, 64, 64, 6),
                                             # ... on a grid > 2048 tiles: the radix select
                                             ("amr_huge_counts_big_grid", 150000, 2112, 1056, 6)])
def test_amr_level_percentiles(name, P, W, H, seed):
    """The AMR percentiles and levels against the oracle: by the two-pass
    histogram select (every tile count < 2^16), the LDS sort of the counts
    and the radix select (a count >= 2^16 on grids of <= / > 2048 tiles)."""
    import oracle as O
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(P, W, H, seed)
    if name.startswith("amr_huge_counts"):  # most Gaussians piled onto one spot
        sc.means3D[: P - P // 8, :2] *= np.float32(1e-3)
        sc.scales[: P - P // 8] = np.float32(0.003)
    acc, radii, steps, (gb, bb, ib) = _amr_gpu_steps(sc, cam, bg=(0.1, 0.1, 0.1))
    s = O.settings_from_camera(cam, bg=(0.1, 0.1, 0.1))
    kw = dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    _, _, st, _ = O.amr_render_foveated(s, kw)
    d = C.parse_buffers(gb, bb, ib, P, st.fwd.num_rendered, W, H, 32)
    if name.startswith("amr_huge_counts"):
        n = st.fwd.ranges[:, 1] - st.fwd.ranges[:, 0]
        assert n.max() >= 1 << 16
    np.testing.assert_array_equal(d["pv"].cpu().numpy()[:3].astype(np.uint32), st.percentile_values)
    np.testing.assert_array_equal(d["levels"].cpu().numpy().astype(np.uint32), st.levels)


@pytest.mark.parametrize("P,W,H,seed", [(10000, 256, 256, 0), (60000, 160, 96, 4), (3000, 2112, 1056, 8)])
def test_amr_variants_bit_identical(P, W, H, seed):
    """The region sub-lists (default) and the full-list blocks (fallback)
    evaluate the same operations on the same operands for every (pixel,
    entry) pair the reference blends -- the sub-lists drop only entries whose
    alpha < 1/255 at every pixel of the region: n_contrib and final T are
    bit-identical.  The step images differ only in the final compose
    C + T bg (one fused multiply-add in the region kernel, a rounded product
    and a sum in the fallback): within 1 ulp, written here as 1e-6."""
    import oracle as O
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(P, W, H, seed)
    out = {}
    for v in (4, 0):
        C.set_tuning("amr_variant", v)
        try:
            acc, radii, steps, (gb, bb, ib) = _amr_gpu_steps(sc, cam, bg=(0.1, 0.2, 0.3))
        finally:
            C.set_tuning("amr_variant", 4)
        d = C.parse_buffers(gb, bb, ib, P, 0, W, H, 32)
        K = int(d["hdr"][0].item())
        d = C.parse_buffers(gb, bb, ib, P, K, W, H, 32)
        # pixels some step rendered (the others are never written)
        lv = d["levels"].cpu().numpy().astype(np.uint32)
        rendered = torch.from_numpy((O.amr_pixel_rounds(W, H) <= O.amr_tile_levels_per_pixel(lv, W, H)).reshape(-1))
        out[v] = [s_.cpu() for s_ in steps] + [d["n_contrib"].cpu()[rendered], d["accum_alpha"].cpu()[rendered]]
    nst = len(out[4]) - 2
    for i, (a_, b_) in enumerate(zip(out[4], out[0])):
        if i < nst:
            assert float((a_ - b_).abs().max()) <= 1e-6, i
        else:
            assert torch.equal(a_, b_), i


def test_amr_steps_with_nothing_in_front():
    """K = 0 (every Gaussian behind the near plane): the progressive steps run
    on an empty binning buffer and match the oracle (background on the
    rendered sub-lattices)."""
    import oracle as O
    sc, cam = G.scene_and_camera(500, 96, 64, 2)
    sc.means3D[:, 2] = -5.0
    acc, radii, steps, (gb, bb, ib) = _amr_gpu_steps(sc, cam, bg=(0.3, 0.2, 0.1))
    assert bb.numel() == 0 and int((radii > 0).sum()) == 0
    s = O.settings_from_camera(cam, bg=(0.3, 0.2, 0.1))
    kw = dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    racc, _, _, rsteps = O.amr_render_foveated(s, kw)
    for k in range(5):
        np.testing.assert_allclose(steps[k].cpu().numpy(), rsteps[k], atol=1e-6)
    np.testing.assert_allclose(acc.cpu().numpy(), racc, atol=1e-6)


@pytest.mark.parametrize("amr_variant", [4, 0])
def test_amr_render_once_interpolated(amr_variant):
    import oracle as O
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from diff_gaussian_rasterization_amr import GaussianRasterizer
    sc, cam = G.scene_and_camera(8000, 224, 160, 5)
    s = G.torch_settings(cam, amr=True)
    t = G.scene_tensors(sc)
    C.set_tuning("amr_variant", amr_variant)
    try:
        color, radii, gb, bb, ib = GaussianRasterizer(s)(
            means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"], shs=t["shs"],
            scales=t["scales"], rotations=t["rotations"], foveaStep=-2, interpolate_image=True)
    finally:
        C.set_tuning("amr_variant", 4)
    os_ = O.settings_from_camera(cam)
    rcol, rrad, st = O.amr_render_once(os_, dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs,
                                                  scales=sc.scales, rotations=sc.rotations))
    assert G.image_l1(color.cpu().numpy(), rcol) < G.IMAGE_L1_TOL


def test_amr_step4_interpolate():
    """foveaStep 4 with interpolate_image=True (the reference's racy path,
    defined here as precomp-copy-then-neighbour-copy)."""
    import oracle as O
    sc, cam = G.scene_and_camera(6000, 160, 96, 9)
    acc, radii, steps, _ = _amr_gpu_steps(sc, cam, interpolate_last=True)
    s = O.settings_from_camera(cam)
    racc, _, _, rsteps = O.amr_render_foveated(
        s, dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales, rotations=sc.rotations),
        interpolate_image=True)
    assert G.image_l1(steps[4].cpu().numpy(), rsteps[4]) < G.IMAGE_L1_TOL
    assert G.image_l1(acc.cpu().numpy(), racc) < G.IMAGE_L1_TOL


@pytest.mark.parametrize("W,H,centre,min_level,replace", [
    (256, 256, None, 1, False),                 # the reference's discs: image centre, W/2 .. W/16
    (256, 160, (181.0, 99.0), 1, False),        # a tracked fovea off centre
    (200, 120, (20.5, 110.0), 0, False),        # periphery left blank (the TODO read literally)
    (256, 160, (181.0, 99.0), 1, True),         # eccentricity alone decides the level
])
def test_amr_fovea_levels_extension(W, H, centre, min_level, replace):
    """Extension beyond parity: fovea-driven tile
    levels between step 0 and steps 1..4.  Levels bit-exact against the
    oracle's restatement of the rule; every step's image and the sum against
    the oracle's AMR render with the same levels."""
    import oracle as O
    from gaussian_splatting_with_eye_tracking_amd import rasterization_amr as RA
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(6000, W, H, 4)
    centres, radii = RA.reference_foveae(W, H, centre)
    hook = lambda ib: RA.apply_fovea_levels(ib, W, H, centres, radii, min_level, replace)  # noqa: E731
    acc, radii_g, steps, (gb, bb, ib) = _amr_gpu_steps(sc, cam, after_step0=hook)
    s = O.settings_from_camera(cam)
    kw = dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    racc, _, st, rsteps = O.amr_render_foveated(
        s, kw, levels_hook=lambda lv: O.fovea_levels(lv, W, H, centres, radii, min_level, replace))
    d = C.parse_buffers(gb, bb, ib, 6000, st.fwd.num_rendered, W, H, 32)
    got = d["levels"].cpu().numpy().astype(np.uint32)
    np.testing.assert_array_equal(got, st.levels)
    assert got.min() >= min_level and got.max() <= 4
    if not replace:
        assert (got <= O.amr_render_foveated(s, kw)[2].levels).all()
    for k in range(5):
        assert G.image_l1(steps[k].cpu().numpy(), rsteps[k]) < G.IMAGE_L1_TOL, k
    assert G.image_l1(acc.cpu().numpy(), racc) < G.IMAGE_L1_TOL


def test_amr_fovea_levels_rejects_bad_buffer():
    from gaussian_splatting_with_eye_tracking_amd import rasterization_amr as RA
    small = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(RuntimeError, match="too small"):
        RA.apply_fovea_levels(small, 256, 256, *RA.reference_foveae(256, 256))


def _amr_grads_vs_oracle(t, means2D, cam, levels, dpix, mode, interpolate):
    import oracle as O
    sc_np = {k: v.detach().cpu().numpy() for k, v in t.items()}
    s = O.settings_from_camera(cam)
    rg = O.amr_backward(s, dict(means3D=sc_np["means3D"], opacities=sc_np["opacities"], shs=sc_np["shs"],
                                scales=sc_np["scales"], rotations=sc_np["rotations"]), dpix, mode, levels,
                        interpolate_image=interpolate)
    pairs = [(means2D.grad, rg["dL_dmeans2D"]), (t["means3D"].grad, rg["dL_dmeans3D"]),
             (t["shs"].grad, rg["dL_dsh"]), (t["opacities"].grad, rg["dL_dopacity"]),
             (t["scales"].grad, rg["dL_dscales"]), (t["rotations"].grad, rg["dL_drotations"])]
    assert np.abs(rg["dL_dopacity"]).sum() > 0  # the case has gradient at all
    for i, (g, r) in enumerate(pairs):
        assert G.rel_err(g.cpu().numpy(), r) < G.GRAD_REL_TOL, (i, G.rel_err(g.cpu().numpy(), r))


@pytest.mark.parametrize("interpolate", [False, True])
@pytest.mark.parametrize("W,H,seed", [(224, 160, 5), (200, 120, 3)])
def test_amr_backward_render_once(interpolate, W, H, seed):
    """Extension: render_once's image differentiated
    through the pixels it rendered (and the interpolation copies) against
    the oracle's restatement (base backward on the 32-px binning with the
    cotangent kept on the rendered pixels)."""
    from diff_gaussian_rasterization_amr import GaussianRasterizer
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(5000, W, H, seed)
    s = G.torch_settings(cam, amr=True)
    t = G.scene_tensors(sc, requires_grad=True)
    means2D = torch.zeros_like(t["means3D"], requires_grad=True)
    color, radii, gb, bb, ib = GaussianRasterizer(s)(
        means3D=t["means3D"], means2D=means2D, opacities=t["opacities"], shs=t["shs"], scales=t["scales"],
        rotations=t["rotations"], foveaStep=-2, interpolate_image=interpolate)
    dpix = S.make_cotangent(H, W, seed + 1)
    (color * torch.from_numpy(dpix).cuda()).sum().backward()
    torch.cuda.synchronize()
    K = int(C.parse_buffers(gb, bb, ib, 5000, 0, W, H, 32)["hdr"][0].item())
    levels = C.parse_buffers(gb, bb, ib, 5000, K, W, H, 32)["levels"].cpu().numpy().astype(np.uint32)
    _amr_grads_vs_oracle(t, means2D, cam, levels, dpix, -2, interpolate)


def test_amr_backward_five_steps_sum():
    """The 5-step foveated frame (gaussian_renderer_amr.render's sum of the
    step images) back-propagated through autograd: every step's backward
    covers its own round, so the sum equals render_once's (no interpolation)
    -- checked against the oracle; step 0 contributes nothing."""
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    import gaussian_splatting_with_eye_tracking_amd._C as C
    W, H, seed = 224, 160, 6
    sc, cam = G.scene_and_camera(5000, W, H, seed)
    s = G.torch_settings(cam, amr=True)
    t = G.scene_tensors(sc, requires_grad=True)
    means2D = torch.zeros_like(t["means3D"], requires_grad=True)
    e = torch.Tensor([])
    u8 = torch.Tensor([]).to(torch.uint8)
    args = (t["means3D"], means2D, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    acc, radii, gb, bb, ib = _RasterizeGaussians.apply(*args, 0, e, u8, u8, u8, False, s)
    for k in range(1, 5):
        ck, _, gb, bb, ib = _RasterizeGaussians.apply(*args, k, acc, gb, bb, ib, False, s)
        acc = acc + ck
    dpix = S.make_cotangent(H, W, seed + 1)
    (acc * torch.from_numpy(dpix).cuda()).sum().backward()
    torch.cuda.synchronize()
    K = int(C.parse_buffers(gb, bb, ib, 5000, 0, W, H, 32)["hdr"][0].item())
    levels = C.parse_buffers(gb, bb, ib, 5000, K, W, H, 32)["levels"].cpu().numpy().astype(np.uint32)
    _amr_grads_vs_oracle(t, means2D, cam, levels, dpix, -2, False)


def test_amr_backward_rejects_interpolated_steps():
    """foveaStep >= 1 with interpolate_image=True has no backward: it is
    refused in the forward when an input requires grad, and runs normally
    under no_grad."""
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    sc, cam = G.scene_and_camera(500, 64, 64, 1)
    s = G.torch_settings(cam, amr=True)
    t = G.scene_tensors(sc, requires_grad=True)
    e = torch.Tensor([])
    u8 = torch.Tensor([]).to(torch.uint8)
    args = (t["means3D"], torch.zeros_like(t["means3D"]), t["shs"], e, t["opacities"], t["scales"],
            t["rotations"], e)
    c0, _, gb, bb, ib = _RasterizeGaussians.apply(*args, 0, e, u8, u8, u8, False, s)
    with pytest.raises(RuntimeError, match="render_once"):
        _RasterizeGaussians.apply(*args, 1, c0, gb, bb, ib, True, s)
    with torch.no_grad():
        c1, *_ = _RasterizeGaussians.apply(*args, 1, c0, gb, bb, ib, True, s)
    assert c1.shape == c0.shape


def test_fovea_levels_after_forward_invalidates_saved_buffer():
    """apply_fovea_levels rewrites the levels of an image buffer in place: a
    pending backward that saved the buffer raises instead of using them."""
    from diff_gaussian_rasterization_amr import GaussianRasterizer
    from gaussian_splatting_with_eye_tracking_amd import rasterization_amr as RA
    sc, cam = G.scene_and_camera(800, 96, 64, 2)
    s = G.torch_settings(cam, amr=True)
    t = G.scene_tensors(sc, requires_grad=True)
    color, radii, gb, bb, ib = GaussianRasterizer(s)(
        means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"], shs=t["shs"],
        scales=t["scales"], rotations=t["rotations"], foveaStep=-2, interpolate_image=False)
    RA.apply_fovea_levels(ib, 96, 64, *RA.reference_foveae(96, 64))
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        color.sum().backward()


def test_bindings_reject_misplaced_operands():
    """A host tensor, a short array or a wrong dtype raises a Python error in
    the binding instead of reaching a kernel as a raw pointer."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(300, 64, 48, 3)
    s = G.torch_settings(cam)
    t = G.scene_tensors(sc)
    e = torch.Tensor([])

    def fwd(**over):
        a = dict(bg=s.bg, means3D=t["means3D"], colors=e, opacity=t["opacities"], scales=t["scales"],
                 rotations=t["rotations"], cov=e, sh=t["shs"])
        a.update(over)
        return C.rasterize_gaussians(a["bg"], a["means3D"], a["colors"], a["opacity"], a["scales"], a["rotations"],
                                     1.0, a["cov"], s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, 48, 64,
                                     a["sh"], 3, s.campos, False, False)
    with pytest.raises(RuntimeError, match="opacities"):
        fwd(opacity=t["opacities"].cpu())
    with pytest.raises(RuntimeError, match="scales"):
        fwd(scales=t["scales"][:100])
    with pytest.raises(RuntimeError, match="rotations"):
        fwd(rotations=t["rotations"].double())
    K, color, radii, geom, binning, img = fwd()
    dpix = torch.zeros_like(color)
    with pytest.raises(RuntimeError, match="radii"):
        C.rasterize_gaussians_backward(s.bg, t["means3D"], radii.cpu(), e, t["scales"], t["rotations"], 1.0, e,
                                       s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, dpix, t["shs"], 3, s.campos,
                                       geom, K, binning, img, False)
    with pytest.raises(RuntimeError, match="sh"):
        C.rasterize_gaussians_backward(s.bg, t["means3D"], radii, e, t["scales"], t["rotations"], 1.0, e,
                                       s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, dpix, t["shs"][:10], 3,
                                       s.campos, geom, K, binning, img, False)


# ---------------------------------------------------------- simple-knn ----
@pytest.mark.parametrize("P,seed", [(5, 0), (1000, 1), (5000, 2), (70000, 3)])
def test_dist_cuda2_bit_exact(P, seed):
    import oracle as O
    from simple_knn._C import distCUDA2
    pts = np.random.default_rng(seed).normal(0, 3.0, (P, 3)).astype(np.float32)
    got = distCUDA2(torch.from_numpy(pts).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, O.dist_cuda2(pts))


@pytest.mark.parametrize("how", ["sh_drgb_off", "fwd_no_grad_hint"])
def test_backward_without_stored_sh_derivatives(how):
    """The SH backward from the coefficients (no stored d(rgb)/d(dir) rows):
    thread option "sh_drgb" 0, or a forward told it needs no backward (the
    one-shot "fwd_no_grad" hint the autograd wrappers give under no_grad)
    followed by a backward anyway -- the header flag makes bwd_gauss re-read
    the SH rows."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    try:
        if how == "sh_drgb_off":
            C.set_thread_option("sh_drgb", 0)
        else:
            C.set_thread_option("fwd_no_grad", 1)
        test_backward_parity("cfg1_10k_256", 10000, 256, 256, 0, "sh")
    finally:
        C.set_thread_option("sh_drgb", 1)
        C.set_thread_option("fwd_no_grad", 0)


def test_forward_only_hint_from_autograd_wrapper():
    """Under torch.no_grad the AMR wrapper's foveaStep 0 forward skips the
    SH-derivative rows (header word 7 = 0); with inputs requiring a gradient it
    stores them (1); the hint is one-shot (a direct _C forward after it stores
    them again)."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    import bench
    W, H, P = 256, 256, 10000
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=0)
    dev = torch.device("cuda:0")
    st = bench.raster_settings(cam, dev, "diff_gaussian_rasterization_amr")
    t = bench.device_params(sc, dev, False)
    e = torch.empty(0, device=dev)
    u8 = torch.empty(0, dtype=torch.uint8, device=dev)

    def step0(grad):
        tt = {k: v.detach().clone().requires_grad_(grad) for k, v in t.items()}
        a = (tt["means3D"], torch.zeros_like(tt["means3D"]), tt["shs"], e, tt["opacities"], tt["scales"],
             tt["rotations"], e)
        c_, _r, gb, bb, ib = _RasterizeGaussians.apply(*a, 0, e, u8, u8, u8, False, st)
        torch.cuda.synchronize()
        flag = int(C.parse_buffers(gb, bb, ib, P, 0, W, H, 32)["hdr"][7].item())
        # an AMR geometry buffer always carries the optional tail (d(rgb)/d(dir)
        # + cov3D) and then the 64-B AMR blend rows (ABI 6)
        assert gb.numel() == C.amr_geom_bytes(P), (gb.numel(), C.amr_geom_bytes(P), flag)
        return flag

    with torch.no_grad():
        assert step0(False) == 0
    assert step0(True) == 1
    assert step0(False) == 0  # grad mode on, nothing requires a gradient
    s = G.torch_settings(cam)
    tg = G.scene_tensors(sc)
    out = C.rasterize_gaussians(s.bg, tg["means3D"], e, tg["opacities"], tg["scales"], tg["rotations"],
                                s.scale_modifier, e, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy,
                                s.image_height, s.image_width, tg["shs"], s.sh_degree, s.campos, s.prefiltered,
                                s.debug)
    torch.cuda.synchronize()
    geom = out[3]
    assert int(C.parse_buffers(geom, out[4], out[5], P, 0, W, H, 16)["hdr"][7].item()) == 1


def test_forward_only_hint_cleared_when_the_forward_raises():
    """a forward-only call whose native forward raises before it
    consumes the one-shot hint must not leave it for the next (training)
    forward: that forward still stores the SH-derivative rows."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from diff_gaussian_rasterization import GaussianRasterizer
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    W, H, P = 128, 96, 3000
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=1)
    s = G.torch_settings(cam)
    t = G.scene_tensors(sc)
    r = GaussianRasterizer(s)
    with torch.no_grad(), pytest.raises(Exception):
        bad = t["means3D"][:, :2].contiguous()  # not [P, 3]: the native forward refuses it
        r(means3D=bad, means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"], shs=t["shs"],
          scales=t["scales"], rotations=t["rotations"])
    e = torch.empty(0, device="cuda")
    out = C.rasterize_gaussians(s.bg, t["means3D"], e, t["opacities"], t["scales"], t["rotations"],
                                s.scale_modifier, e, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy,
                                s.image_height, s.image_width, t["shs"], s.sh_degree, s.campos, s.prefiltered,
                                s.debug)
    torch.cuda.synchronize()
    assert int(C.parse_buffers(out[3], out[4], out[5], P, 0, W, H, 16)["hdr"][7].item()) == 1


def test_hit_codes_and_point_list_repeatable():
    """The forward render stores its row-group hit codes in the binning
    scratch and says where in header word 6 (gs_layout.h hit_codes_of).
    Twenty forwards of a scene with few, full tiles (96 tiles, some above
    1024 instances) give the bitonic sort's point_list (sort_algo 0) every
    time, and the default backward (reading the codes) matches the fallback
    backward kernel to float-atomic noise."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H = 12000, 192, 128
    sc = S.make_scene(P, S.make_camera(W, H), seed=3)
    cam = S.make_orbit_camera(W, H, 4.0)
    s = G.torch_settings(cam)
    t = G.scene_tensors(sc)
    e = torch.Tensor([])

    def fwd():
        return C.rasterize_gaussians(s.bg, t["means3D"], e, t["opacities"], t["scales"], t["rotations"], 1.0, e,
                                     s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, H, W, t["shs"], 3, s.campos,
                                     False, False)

    C.set_tuning("sort_algo", 0)
    try:
        K0, c0, r0, g0, b0, i0 = fwd()
        want = C.parse_buffers(g0, b0, i0, P, K0, W, H, 16)["point_list"].cpu()
    finally:
        C.set_tuning("sort_algo", 1)
    dpix = torch.from_numpy(S.make_cotangent(H, W, 7)).cuda()
    for _ in range(20):
        K, color, radii, geom, binning, img = fwd()
        assert K == K0
        d = C.parse_buffers(geom, binning, img, P, K, W, H, 16)
        assert torch.equal(d["point_list"].cpu(), want)
        assert torch.equal(color.cpu(), c0.cpu())
        assert int(d["hdr"][6].item()) != 0 and "hit_codes" in d
    g = C.rasterize_gaussians_backward(s.bg, t["means3D"], radii, e, t["scales"], t["rotations"], 1.0, e,
                                       s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, dpix, t["shs"], 3,
                                       s.campos, geom, K, binning, img, False)
    C.set_tuning("bwd_variant", 0)
    try:
        gf = C.rasterize_gaussians_backward(s.bg, t["means3D"], radii, e, t["scales"], t["rotations"], 1.0, e,
                                            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, dpix, t["shs"], 3,
                                            s.campos, geom, K, binning, img, False)
    finally:
        C.set_tuning("bwd_variant", -1)
    torch.cuda.synchronize()
    for a, b in zip(g[:3], gf[:3]):  # dL_dmeans2D, dL_dcolors, dL_dopacity
        assert G.rel_err(a.cpu().numpy(), b.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("P,W,H,seed", [(10000, 256, 256, 0), (60000, 160, 96, 4), (3000, 2112, 1056, 8)])
def test_amr_fused_tile_sort_matches_separate_sort(P, W, H, seed):
    """The AMR region-list pass sorts the tiles of <= 2048 instances itself
    (render.hip amr_region_lists_kernel kFuse; larger ones by the size-class
    launches): point_list, the records, the region lists and every step image
    equal the separately sorted build's (sort_algo 0: bitonic networks, no
    fusion) bit for bit, repeatedly."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    sc, cam = G.scene_and_camera(P, W, H, seed)
    out = {}
    for algo in (0, 1, 1):
        C.set_tuning("sort_algo", algo)
        try:
            acc, radii, steps, (gb, bb, ib) = _amr_gpu_steps(sc, cam, bg=(0.1, 0.2, 0.3))
        finally:
            C.set_tuning("sort_algo", 1)
        K = int(C.parse_buffers(gb, bb, ib, P, 0, W, H, 32)["hdr"][0].item())
        d = C.parse_buffers(gb, bb, ib, P, K, W, H, 32)
        r = [d["point_list"].cpu(), d["region_count"].cpu()] + [s_.cpu() for s_ in steps]
        if 0 in out:
            for a_, b_ in zip(r, out[0]):
                assert torch.equal(a_, b_)
        else:
            out[0] = r
