"""GPU parity at BASELINE.json's full configurations and at the reference's
edge cases: the HIP path through the C ABI against the CPU
oracle on the same seeded inputs.

* config 3 (AMR, 1M Gaussians, 1920x1080, 32-px tiles): ranges, point_list,
  percentile values and every level array bit-exact; each of the 5 step
  images, the summed frame and render_once (with and without interpolation)
  within the image bar; one AMR backward (render_once) within the gradient
  bar;
* config 4 (6.1M Gaussians, 1600x1063): K, ranges, point_list and the 64-bit
  keys bit-exact, image, all 8 gradients;
* config 5 on one GPU (1M, 1080p, 8 yawed views): the multi-view kernel equals
  the sum of the 8 per-view backwards, and view 0 matches the oracle;
* the reference's training-time settings: active SH degree 0..2 with M = 16
  coefficients (gaussian_renderer/__init__.py:45, scene/gaussian_model.py:
  120-122), M = 1 and M = 9 models, scale_modifier != 1 (:42) and a white
  background (train.py's white_background).

Bars (north_star): integer buffers bit-exact; image L1 < 1e-5; gradients
within 1e-4 relative (L2 norm).  The oracle runs on the box's host threads
(oracle.set_threads) for the full-size cases.
"""
import numpy as np
import pytest

import gs_helpers as G

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

GRAD_NAMES = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
              "dL_drotations"]


@pytest.fixture
def oracle_threads():
    import oracle as O
    O.set_threads(O.host_threads(16))
    yield O
    O.set_threads(1)


def _c_forward(sc, cam, bg=(0.0, 0.0, 0.0), sh_degree=3, scale_modifier=1.0, shs=None):
    import gaussian_splatting_with_eye_tracking_amd._C as C
    s = G.torch_settings(cam, bg=bg, sh_degree=sh_degree, scale_modifier=scale_modifier)
    t = G.scene_tensors(sc)
    if shs is not None:
        t["shs"] = torch.from_numpy(np.ascontiguousarray(shs)).cuda()
    e = torch.Tensor([])
    out = C.rasterize_gaussians(s.bg, t["means3D"], e, t["opacities"], t["scales"], t["rotations"], s.scale_modifier,
                                e, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width,
                                t["shs"], s.sh_degree, s.campos, s.prefiltered, s.debug)
    torch.cuda.synchronize()
    return s, t, out


def _c_backward(s, t, out, dpix):
    import gaussian_splatting_with_eye_tracking_amd._C as C
    K, color, radii, geom, binning, img = out
    e = torch.Tensor([])
    g = C.rasterize_gaussians_backward(s.bg, t["means3D"], radii, e, t["scales"], t["rotations"], s.scale_modifier, e,
                                       s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy,
                                       torch.from_numpy(dpix).cuda(), t["shs"], s.sh_degree, s.campos, geom, K,
                                       binning, img, False)
    torch.cuda.synchronize()
    return g


def _check_binning(C, out, ref, P, W, H, tile=16):
    K, color, radii, geom, binning, img = out
    assert K == ref.num_rendered
    d = C.parse_buffers(geom, binning, img, P, K, W, H, tile)
    np.testing.assert_array_equal(radii.cpu().numpy(), ref.radii)
    np.testing.assert_array_equal(d["ranges"].cpu().numpy().astype(np.uint32), ref.ranges)
    if K:
        np.testing.assert_array_equal(d["point_list"].cpu().numpy().astype(np.uint32), ref.point_list)
        np.testing.assert_array_equal(d["point_list_keys"].cpu().numpy().view(np.uint64), ref.point_list_keys)
    return d


def _check_grads(grads, rg, skip=(), case=None, sc=None, cam=None, ref=None, allow=None):
    """The norm bar on every gradient, and (with `case`) the element-wise bar
    (allow: (oracle.grad_allowance's allowances, its counts))."""
    for n, g in zip(GRAD_NAMES, grads):
        if n in skip:
            continue
        gg = g.cpu().numpy()
        assert gg.shape == rg[n].shape, n
        assert np.all(np.isfinite(gg)), n
        assert G.rel_err(gg, rg[n]) < G.GRAD_REL_TOL, (n, G.rel_err(gg, rg[n]))
    if case is not None:
        names = [n for n in GRAD_NAMES if n not in skip]
        G.assert_grads_elementwise(case, names, [g for n, g in zip(GRAD_NAMES, grads) if n not in skip], rg,
                                   sc, cam, ref, allow=None if allow is None else allow[0],
                                   ties=None if allow is None else allow[1])


# ------------------------------------------------------------ edge cases ---
EDGE_CASES = [
    # name, sh_degree D, coefficients M, scale_modifier, background
    ("D0_M16", 0, 16, 1.0, (0.0, 0.0, 0.0)),
    ("D1_M16", 1, 16, 1.0, (0.0, 0.0, 0.0)),
    ("D2_M16", 2, 16, 1.0, (0.2, 0.1, 0.05)),
    ("D0_M1", 0, 1, 1.0, (0.0, 0.0, 0.0)),
    ("D1_M9", 1, 9, 1.0, (0.0, 0.0, 0.0)),
    ("D2_M9", 2, 9, 1.0, (0.0, 0.0, 0.0)),
    ("mod_0.5", 3, 16, 0.5, (0.0, 0.0, 0.0)),
    ("mod_1.7", 3, 16, 1.7, (0.0, 0.0, 0.0)),
    ("white_bg", 3, 16, 1.0, (1.0, 1.0, 1.0)),
]


@pytest.mark.parametrize("name,D,M,mod,bg", EDGE_CASES)
def test_edge_case_parity(name, D, M, mod, bg):
    """Forward buffers bit-exact, image and the 8 gradients against the oracle
    with the reference's other settings (SH degree / coefficient count,
    scale_modifier, background)."""
    import oracle as O
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H, seed = 8000, 200, 136, 21
    sc, cam = G.scene_and_camera(P, W, H, seed)
    shs = np.ascontiguousarray(sc.shs[:, :M, :])
    C.set_thread_option("store_cov3d", 1)  # the geometry buffer's cov3D is written on request only
    try:
        s, t, out = _c_forward(sc, cam, bg=bg, sh_degree=D, scale_modifier=mod, shs=shs)
    finally:
        C.set_thread_option("store_cov3d", 0)
    os_ = O.settings_from_camera(cam, bg=bg, sh_degree=D, scale_modifier=mod)
    kw = dict(shs=shs, scales=sc.scales, rotations=sc.rotations)
    ref = O.forward(os_, sc.means3D, sc.opacities, **kw)
    d = _check_binning(C, out, ref, P, W, H)
    vis = ref.radii > 0
    np.testing.assert_array_equal(d["rgb"].cpu().numpy()[vis], ref.rgb[vis])
    np.testing.assert_array_equal(d["cov3D"].cpu().numpy()[vis], ref.cov3D[vis])
    np.testing.assert_array_equal(d["conic_opacity"].cpu().numpy()[vis], ref.conic_opacity[vis])
    assert G.image_l1(out[1].cpu().numpy(), ref.color) < G.IMAGE_L1_TOL
    dpix = S.make_cotangent(H, W, seed + 1)
    grads = _c_backward(s, t, out, dpix)
    assert tuple(grads[5].shape) == (P, M, 3)
    _check_grads(grads, O.backward(os_, ref, sc.means3D, dpix, **kw), case=f"edge_{name}", sc=sc, cam=cam, ref=ref,
                 allow=O.grad_allowance(os_, ref, sc.means3D, dpix, parts=True, **kw))


def test_active_sh_degree_zero_through_autograd():
    """The reference's first training iterations: active_sh_degree 0 with the
    full 16-coefficient features (gaussian_renderer/__init__.py:45-49,
    scene/gaussian_model.py:120-122) through the drop-in autograd API:
    dL/dsh is zero past the DC coefficient and matches the oracle."""
    import oracle as O
    from diff_gaussian_rasterization import GaussianRasterizer
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H, seed = 5000, 160, 96, 4
    sc, cam = G.scene_and_camera(P, W, H, seed)
    s = G.torch_settings(cam, sh_degree=0)
    t = G.scene_tensors(sc, requires_grad=True)
    m2 = torch.zeros_like(t["means3D"], requires_grad=True)
    color, radii = GaussianRasterizer(s)(means3D=t["means3D"], means2D=m2, opacities=t["opacities"], shs=t["shs"],
                                         scales=t["scales"], rotations=t["rotations"])
    dpix = S.make_cotangent(H, W, seed + 1)
    torch.autograd.backward(color, torch.from_numpy(dpix).cuda())
    os_ = O.settings_from_camera(cam, sh_degree=0)
    kw = dict(shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    ref = O.forward(os_, sc.means3D, sc.opacities, **kw)
    assert G.image_l1(color.detach().cpu().numpy(), ref.color) < G.IMAGE_L1_TOL
    rg = O.backward(os_, ref, sc.means3D, dpix, **kw)
    gsh = t["shs"].grad.cpu().numpy()
    assert np.all(gsh[:, 1:, :] == 0)
    for name, got in (("dL_dsh", t["shs"].grad), ("dL_dmeans3D", t["means3D"].grad), ("dL_dmeans2D", m2.grad),
                      ("dL_dscales", t["scales"].grad), ("dL_drotations", t["rotations"].grad),
                      ("dL_dopacity", t["opacities"].grad)):
        assert G.rel_err(got.cpu().numpy(), rg[name]) < G.GRAD_REL_TOL, name


# -------------------------------------------------------------- config 4 ---
@pytest.mark.timeout(600)
def test_config4_full_size(oracle_threads):
    """BASELINE config 4 (6.1M Gaussians, 1600x1063): binning bit-exact, image
    and all 8 gradients."""
    O = oracle_threads
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H = 6_100_000, 1600, 1063
    sc, cam = G.scene_and_camera(P, W, H, 0)
    s, t, out = _c_forward(sc, cam)
    os_ = O.settings_from_camera(cam)
    kw = dict(shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    ref = O.forward(os_, sc.means3D, sc.opacities, **kw)
    _check_binning(C, out, ref, P, W, H)
    assert G.image_l1(out[1].cpu().numpy(), ref.color) < G.IMAGE_L1_TOL
    dpix = S.make_cotangent(H, W, 1)
    grads = _c_backward(s, t, out, dpix)
    del out
    _check_grads(grads, O.backward(os_, ref, sc.means3D, dpix, **kw), case="config4", sc=sc, cam=cam, ref=ref,
                 allow=O.grad_allowance(os_, ref, sc.means3D, dpix, parts=True, **kw))


# -------------------------------------------------------------- config 3 ---
@pytest.mark.timeout(600)
def test_config3_full_size_amr(oracle_threads):
    """BASELINE config 3 (1M Gaussians, 1920x1080, 32-px AMR tiles): the
    5-step foveated frame (gaussian_renderer_amr.render) and render_once with
    and without interpolation."""
    O = oracle_threads
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from diff_gaussian_rasterization_amr import GaussianRasterizer, _RasterizeGaussians
    P, W, H = 1_000_000, 1920, 1080
    sc, cam = G.scene_and_camera(P, W, H, 0)
    s = G.torch_settings(cam, amr=True)
    t = G.scene_tensors(sc)
    e = torch.Tensor([])
    u8 = torch.Tensor([]).to(torch.uint8)
    m2 = torch.zeros_like(t["means3D"])
    args = (t["means3D"], m2, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    with torch.no_grad():
        c0, radii, gb, bb, ib = _RasterizeGaussians.apply(*args, 0, e, u8, u8, u8, False, s)
        acc = c0
        steps = [c0.cpu().numpy()]
        for k in range(1, 5):
            ck, _, gb, bb, ib = _RasterizeGaussians.apply(*args, k, acc, gb, bb, ib, False, s)
            acc = acc + ck
            steps.append(ck.cpu().numpy())
        # the fused driver (renderer_amr.render's sequence): the same frame, bit for bit
        from gaussian_splatting_with_eye_tracking_amd.rasterization_amr import render_steps
        fused, fradii, _, _, _ = render_steps(*args, s)
        torch.cuda.synchronize()
        assert torch.equal(fused, acc) and torch.equal(fradii, radii)
    os_ = O.settings_from_camera(cam)
    kw = dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    racc, rradii, st, rsteps = O.amr_render_foveated(os_, kw)
    np.testing.assert_array_equal(radii.cpu().numpy(), rradii)
    K = st.fwd.num_rendered
    d = C.parse_buffers(gb, bb, ib, P, K, W, H, 32)
    assert int(d["hdr"][0].item()) == K
    np.testing.assert_array_equal(d["ranges"].cpu().numpy().astype(np.uint32), st.fwd.ranges)
    np.testing.assert_array_equal(d["point_list"].cpu().numpy().astype(np.uint32), st.fwd.point_list)
    np.testing.assert_array_equal(d["pv"].cpu().numpy()[:3].astype(np.uint32), st.percentile_values)
    np.testing.assert_array_equal(d["levels"].cpu().numpy().astype(np.uint32), st.levels)
    np.testing.assert_array_equal(d["levels_last"].cpu().numpy().astype(np.uint32), st.levels_last)
    np.testing.assert_array_equal(d["levels_current"].cpu().numpy().astype(np.uint32), st.levels_current)
    assert np.bincount(st.levels, minlength=5)[1:].min() > 0  # every level occurs at this size
    for k in range(5):
        assert G.image_l1(steps[k], rsteps[k]) < G.IMAGE_L1_TOL, k
    assert G.image_l1(acc.cpu().numpy(), racc) < G.IMAGE_L1_TOL
    for interp in (False, True):
        with torch.no_grad():
            col = GaussianRasterizer(s)(means3D=t["means3D"], means2D=m2, opacities=t["opacities"], shs=t["shs"],
                                        scales=t["scales"], rotations=t["rotations"], foveaStep=-2,
                                        interpolate_image=interp)[0]
        rcol, _, _ = O.amr_forward(os_, foveaStep=-2, interpolate_image=interp, **kw)
        assert G.image_l1(col.cpu().numpy(), rcol) < G.IMAGE_L1_TOL, interp


@pytest.mark.timeout(600)
def test_config3_full_size_amr_backward(oracle_threads):
    """Extension beyond parity (the AMR backward) at config 3's
    size: render_once without interpolation, all parameter gradients."""
    O = oracle_threads
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from diff_gaussian_rasterization_amr import GaussianRasterizer
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H = 1_000_000, 1920, 1080
    sc, cam = G.scene_and_camera(P, W, H, 0)
    s = G.torch_settings(cam, amr=True)
    t = G.scene_tensors(sc, requires_grad=True)
    m2 = torch.zeros_like(t["means3D"], requires_grad=True)
    color, radii, gb, bb, ib = GaussianRasterizer(s)(
        means3D=t["means3D"], means2D=m2, opacities=t["opacities"], shs=t["shs"], scales=t["scales"],
        rotations=t["rotations"], foveaStep=-2, interpolate_image=False)
    dpix = S.make_cotangent(H, W, 7)
    torch.autograd.backward(color, torch.from_numpy(dpix).cuda())
    torch.cuda.synchronize()
    K = int(C.parse_buffers(gb, bb, ib, P, 0, W, H, 32)["hdr"][0].item())
    levels = C.parse_buffers(gb, bb, ib, P, K, W, H, 32)["levels"].cpu().numpy().astype(np.uint32)
    os_ = O.settings_from_camera(cam)
    rg = O.amr_backward(os_, dict(means3D=sc.means3D, opacities=sc.opacities, shs=sc.shs, scales=sc.scales,
                                  rotations=sc.rotations), dpix, -2, levels)
    for name, got in (("dL_dmeans2D", m2.grad), ("dL_dmeans3D", t["means3D"].grad), ("dL_dsh", t["shs"].grad),
                      ("dL_dopacity", t["opacities"].grad), ("dL_dscales", t["scales"].grad),
                      ("dL_drotations", t["rotations"].grad)):
        assert G.rel_err(got.cpu().numpy(), rg[name]) < G.GRAD_REL_TOL, name


# -------------------------------------------------------------- config 5 ---
@pytest.mark.timeout(600)
def test_config5_eight_views_one_gpu(oracle_threads):
    """BASELINE config 5's step on one GPU: 8 views yawed -17.5..17.5 degrees
    (SURVEY §8(d) row 5), cotangent seeds 100 + v.  The multi-view parameter
    backward of the 8 view records equals the sum of the 8 per-view reference
    backwards (1e-5 relative: float-atomic order noise), and view 0 alone
    matches the oracle."""
    O = oracle_threads
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H = 1_000_000, 1920, 1080
    sc, _ = G.scene_and_camera(P, W, H, 0)
    t = G.scene_tensors(sc)
    e = torch.Tensor([])
    yaws = S.config5_yaws(8)
    recs = []
    summed = None
    osum = None  # the oracle's 8 per-view backwards, summed in double
    asum = tsum = None  # their near-tie allowances and counts, summed
    pnames = ["dL_dmeans3D", "dL_dsh", "dL_dopacity", "dL_dscales", "dL_drotations"]
    kw = dict(shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    for v, yaw in enumerate(yaws):
        cam = S.make_orbit_camera(W, H, yaw)
        s = G.torch_settings(cam)
        out = C.rasterize_gaussians(s.bg, t["means3D"], e, t["opacities"], t["scales"], t["rotations"], 1.0, e,
                                    s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, H, W, t["shs"], 3, s.campos,
                                    False, False)
        K, color, radii, geom, binning, img = out
        dpix = S.make_cotangent(H, W, 100 + v)
        recs.append(DP.view_record(s, radii, geom, K, binning, img, torch.from_numpy(dpix).cuda()))
        g = _c_backward(s, t, out, dpix)
        per = [g[3], g[5], g[2], g[6], g[7]]  # means3D, sh, opacity, scales, rotations
        summed = [x.double().clone() for x in per] if summed is None else [a + b.double() for a, b in zip(summed, per)]
        del out
        os_ = O.settings_from_camera(cam)
        ref = O.forward(os_, sc.means3D, sc.opacities, **kw)
        rg = O.backward(os_, ref, sc.means3D, dpix, **kw)
        al, ties = O.grad_allowance(os_, ref, sc.means3D, dpix, parts=True, **kw)
        if v == 0:  # one view alone: every gradient, both bars
            _check_grads(g, rg, case="config5_view0", sc=sc, cam=cam, ref=ref, allow=(al, ties))
        osum = ({n: rg[n].astype(np.float64) for n in pnames} if osum is None
                else {n: osum[n] + rg[n] for n in pnames})
        asum = ({k: {n: al[k][n] for n in pnames} for k in al} if asum is None
                else {k: {n: asum[k][n] + al[k][n] for n in pnames} for k in al})
        tsum = ties if tsum is None else {k: tsum[k] + ties[k] for k in ties}
        del ref, rg, g, al
    mv = DP.multiview_param_grads(torch.stack(recs), t["means3D"], t["shs"], 3, t["scales"], t["rotations"])
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(mv, summed)):
        assert G.rel_err(a.cpu().numpy(), b.cpu().numpy()) < 1e-5, i
    # the multi-view kernel's parameter gradients against the oracle's 8-view
    # sum: the norm bar and the element-wise bar (the kernel builds with FMA
    # contraction and reciprocal math, build.py SOURCE_FLAGS)
    for n, a in zip(pnames, mv):
        assert G.rel_err(a.cpu().numpy(), osum[n]) < G.GRAD_REL_TOL, n
    G.assert_grads_elementwise("config5_multiview_sum", pnames, list(mv), osum, sc, S.make_orbit_camera(W, H, yaws[0]),
                               allow=asum, ties=tsum)
