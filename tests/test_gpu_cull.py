"""The blend kernels' row-group cull (gs_blend.cuh splat_group_mask) is exact.

A Gaussian is skipped for a 16x4 pixel row group only when a conservative
bounding box of its alpha >= 1/255 ellipse misses the group, i.e. when every
pixel of the group would take the reference's `alpha < 1/255` continue
(base/cr/forward.cu:341-343, base/cr/backward.cu:480-482).  Proof by A/B on
the same kernel: with the cull disabled ("cull" tuning knob = 0) the forward
outputs must be bit-identical, and the gradients identical up to the order of
float atomics (which is not deterministic run to run, cull or not).

Scenes are adversarial for the box: strongly anisotropic Gaussians (the box
of a thin diagonal ellipse is far larger than the ellipse, and Q's rounding
grows with the correlation), opacities just above 1/255 (thresholds near 0),
and a few very large splats.
"""
import numpy as np
import pytest

import gs_helpers as G

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _adversarial_scene(P, W, H, seed):
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=seed, log_scale_mean=np.log(0.02), log_scale_std=1.3)
    rng = np.random.default_rng(seed + 99)
    third = P // 3
    # opacities straddling 1/255 (0.00392...)
    sc.opacities[:third, 0] = rng.uniform(0.0037, 0.0060, third).astype(np.float32)
    # a few very large, very thin splats
    big = rng.choice(P, size=max(1, P // 200), replace=False)
    sc.scales[big] = np.array([0.8, 0.004, 0.004], np.float32)
    return sc, cam


def _forward(sc, cam, fwd_variant):
    import gaussian_splatting_with_eye_tracking_amd._C as C
    C.set_tuning("fwd_variant", fwd_variant)
    s = G.torch_settings(cam)
    t = G.scene_tensors(sc)
    e = torch.Tensor([])
    out = C.rasterize_gaussians(s.bg, t["means3D"], e, t["opacities"], t["scales"], t["rotations"], 1.0, e,
                                s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width,
                                t["shs"], 3, s.campos, False, False)
    K, color, radii, geom, binning, img = out
    bufs = C.parse_buffers(geom, binning, img, sc.P, K, s.image_width, s.image_height, 16)
    torch.cuda.synchronize()
    return s, t, out, {k: bufs[k].clone() for k in ("accum_alpha", "n_contrib", "max_contrib")}


def _backward(s, t, out, dpix, bwd_variant):
    """Returns the 8 reference gradients and the blend kernel's per-Gaussian
    sums grad_accum[P][9] (dL/dcolor 3, dL/dmean2D 2, dL/dconic 3, dL/dopacity)."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    C.set_tuning("bwd_variant", bwd_variant)
    K, color, radii, geom, binning, img = out
    e = torch.Tensor([])
    g = C.rasterize_gaussians_backward(s.bg, t["means3D"], radii, e, t["scales"], t["rotations"], 1.0, e,
                                       s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, dpix, t["shs"], 3,
                                       s.campos, geom, K, binning, img, False)
    torch.cuda.synchronize()
    P = t["means3D"].shape[0]
    acc = C.parse_buffers(geom, binning, img, P, K, s.image_width, s.image_height, 16)["grad_accum"]
    return [x.cpu().numpy() for x in g], acc[:, :9].cpu().numpy()


@pytest.mark.parametrize("P,W,H,seed", [(6000, 256, 192, 1), (30000, 320, 200, 2)])
@pytest.mark.parametrize("variant", [0, 1])  # the fallback and the default blends
def test_cull_is_exact(P, W, H, seed, variant):
    """Forward: bit-identical.  Backward: every per-Gaussian sum the blend
    kernel accumulates (grad_accum) and the screen-space gradients agree to
    float-atomic ordering noise.  (The 3D gradients are per-Gaussian functions
    of those sums; on this scene the Jacobians of the huge thin splats
    amplify the run-to-run atomic noise of dL/dconic to ~1e-3, cull or not,
    so they are compared on the default scene below instead.)"""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    sc, cam = _adversarial_scene(P, W, H, seed)
    dpix = torch.from_numpy(S.make_cotangent(H, W, seed + 1)).cuda()
    res = {}
    try:
        for cull in (0, 1):
            C.set_tuning("cull", cull)
            s, t, out, bufs = _forward(sc, cam, variant)
            grads, acc = _backward(s, t, out, dpix, variant)
            res[cull] = (out[1].cpu().numpy(), {k: v.cpu().numpy() for k, v in bufs.items()}, grads, acc)
    finally:
        C.set_tuning("cull", 1)
        C.set_tuning("fwd_variant", -1)
        C.set_tuning("bwd_variant", -1)
    np.testing.assert_array_equal(res[0][0], res[1][0])  # image, bit-exact
    for k in res[0][1]:
        np.testing.assert_array_equal(res[0][1][k], res[1][1][k], err_msg=k)
    # float-atomic ordering noise only: observed up to ~1.5e-6
    for i in range(3):  # dL_dmeans2D, dL_dcolors, dL_dopacity
        assert G.rel_err(res[1][2][i], res[0][2][i]) < 5e-6, i
    for c in range(9):  # each accumulated term, column by column
        a, b = res[0][3][:, c], res[1][3][:, c]
        scale = np.abs(a).max() + 1e-30
        assert np.abs(a - b).max() / scale < 1e-5, c


def test_cull_is_exact_default_scene_gradients():
    """On the benchmark's scene distribution every gradient agrees to 1e-5."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    sc, cam = G.scene_and_camera(20000, 320, 200, 3)
    dpix = torch.from_numpy(S.make_cotangent(200, 320, 4)).cuda()
    res = {}
    try:
        for cull in (0, 1):
            C.set_tuning("cull", cull)
            s, t, out, bufs = _forward(sc, cam, 1)
            res[cull] = (out[1].cpu().numpy(), _backward(s, t, out, dpix, 1)[0])
    finally:
        C.set_tuning("cull", 1)
    np.testing.assert_array_equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert G.rel_err(b, a) < 1e-5


def test_cull_is_exact_amr_render_once():
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from diff_gaussian_rasterization_amr import GaussianRasterizer
    sc, cam = _adversarial_scene(12000, 288, 160, 4)
    s = G.torch_settings(cam, amr=True)
    t = G.scene_tensors(sc)
    imgs = {}
    try:
        for cull in (0, 1):
            C.set_tuning("cull", cull)
            color, *_ = GaussianRasterizer(s)(
                means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"],
                shs=t["shs"], scales=t["scales"], rotations=t["rotations"], foveaStep=-2, interpolate_image=True)
            imgs[cull] = color.cpu().numpy()
    finally:
        C.set_tuning("cull", 1)
    np.testing.assert_array_equal(imgs[0], imgs[1])


@pytest.mark.parametrize("fwd", [1, 0])
@pytest.mark.parametrize("P,W,H,seed", [(6000, 256, 192, 1), (30000, 320, 200, 2)])
def test_default_backward_matches_fallback(P, W, H, seed, fwd):
    """The default backward (SGPR-mask selects; the power > 0 test dropped for
    Gaussians whose form is provably negative definite; the contributor test
    dropped in batches every pixel has started; staged sums flushed by the
    staging reduce) against the fallback (predicate form, LDS-row sums) on
    the adversarial scene (huge thin splats, near-degenerate conics), after
    the default forward (hit codes) and the fallback forward (geometric
    cull): the blend sums agree to float-atomic ordering noise."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    sc, cam = _adversarial_scene(P, W, H, seed)
    dpix = torch.from_numpy(S.make_cotangent(H, W, seed + 1)).cuda()
    res = {}
    try:
        for v in (0, 1, 2):
            s, t, out, _bufs = _forward(sc, cam, fwd)
            res[v] = _backward(s, t, out, dpix, v)
    finally:
        C.set_tuning("fwd_variant", -1)
        C.set_tuning("bwd_variant", -1)
    for v in (1, 2):
        for i in range(3):  # dL_dmeans2D, dL_dcolors, dL_dopacity
            assert G.rel_err(res[v][0][i], res[0][0][i]) < 5e-6, (v, i)
        assert G.rel_err(res[v][1], res[0][1]) < 5e-6, v


@pytest.mark.parametrize("P,W,H,seed,adv", [(6000, 256, 192, 1, True), (30000, 320, 200, 2, True),
                                            (10000, 256, 256, 0, False)])
def test_default_forward_bit_identical_to_fallback(P, W, H, seed, adv):
    """The default forward (4 waves x 1 px, select form, no power > 0 test in
    provably negative-definite chunks, per-pair wave exit) against the
    fallback (1 wave x 4 px, predicate form): image, final T, n_contrib and
    max_contrib bit for bit, on the adversarial scene (huge thin splats,
    opacities at 1/255) and the default one; only the default leaves hit
    codes."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    if adv:
        sc, cam = _adversarial_scene(P, W, H, seed)
    else:
        cam = S.make_camera(W, H)
        sc = S.make_scene(P, cam, seed=seed)
    res = {}
    try:
        for v in (0, 1):
            s, t, out, bufs = _forward(sc, cam, v)
            hdr = C.parse_buffers(out[3], out[4], out[5], P, int(out[0]), W, H, 16)["hdr"]
            res[v] = (out[1].cpu().numpy(), {k: b.cpu().numpy() for k, b in bufs.items()}, int(hdr[6].item()))
    finally:
        C.set_tuning("fwd_variant", -1)
    np.testing.assert_array_equal(res[1][0], res[0][0])
    for k in res[1][1]:
        np.testing.assert_array_equal(res[1][1][k], res[0][1][k], err_msg=k)
    assert res[1][2] != 0 and res[0][2] == 0  # header word kHdrHitCodes (where the codes are; 0: none)
