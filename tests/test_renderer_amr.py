"""The foveated renderer glue (gaussian_renderer_amr's render / render_once,
SURVEY §8 row B8) and its fused 5-step driver.

* CPU: sh_utils.eval_sh bit-exact against the reference's utils/sh_utils.py
  outputs (tests/golden/ref_pins.npz, tools/make_golden.py); the fused driver
  refuses an autograd graph.
* GPU: rasterization_amr.render_steps with the steps' image sum fused into
  the kernel (gs_amr_accumulate_step) gives the same bits as the reference's
  literal sequence -- foveaStep 0..4 through _RasterizeGaussians.apply and
  `out_color_precomp + rendered_image_k` in torch -- with the same image
  buffer (levels, final T, n_contrib) and radii, with steps 1..4 launched
  one by one or as one launch (GSPLAT_AMD_AMR_STEPS_1_TO_4, also after the
  fovea-level hook); renderer_amr.render / render_once equal the explicit
  calls.
"""
import math
import os
import types

import numpy as np
import pytest

import gs_helpers as G

torch = pytest.importorskip("torch")
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_eval_sh_matches_reference(deg):
    from gaussian_splatting_with_eye_tracking_amd.sh_utils import eval_sh
    p = np.load(os.path.join(GOLD, "ref_pins.npz"))
    got = eval_sh(deg, torch.from_numpy(p["sh_coeffs"]), torch.from_numpy(p["sh_dirs"])).numpy()
    np.testing.assert_array_equal(got, p[f"eval_sh_deg{deg}"])


@pytest.mark.parametrize("deg", [0, 1, 2, 3, 4])
def test_eval_sh_degree4_matches_reference(deg):
    """Up to the reference's C4 branch (utils/sh_utils.py:70-111), 25
    coefficients per channel, bit for bit (tests/golden/sh4_pins.npz)."""
    from gaussian_splatting_with_eye_tracking_amd.sh_utils import eval_sh
    p = np.load(os.path.join(GOLD, "sh4_pins.npz"))
    got = eval_sh(deg, torch.from_numpy(p["sh_coeffs"]), torch.from_numpy(p["sh_dirs"])).numpy()
    np.testing.assert_array_equal(got, p[f"eval_sh_deg{deg}"])


def test_fused_driver_refuses_autograd():
    from gaussian_splatting_with_eye_tracking_amd.rasterization_amr import render_steps
    x = torch.zeros(4, 3, requires_grad=True)
    e = torch.empty(0)
    with pytest.raises(RuntimeError, match="forward-only"):
        render_steps(x, torch.zeros(4, 3), e, e, torch.ones(4, 1), e, e, e, None, fused=True)
    with torch.no_grad(), pytest.raises(RuntimeError, match="forward-only"):
        render_steps(x, torch.zeros(4, 3), e, e, torch.ones(4, 1), e, e, e, None, fused=True, interpolate_image=True)


def _duck(sc, cam, dev="cuda"):
    t = G.scene_tensors(sc, dev)
    pc = types.SimpleNamespace(get_xyz=t["means3D"], get_opacity=t["opacities"], get_scaling=t["scales"],
                               get_rotation=t["rotations"], get_features=t["shs"], active_sh_degree=3,
                               max_sh_degree=3)
    camera = types.SimpleNamespace(
        FoVx=2.0 * math.atan(cam.tanfovx), FoVy=2.0 * math.atan(cam.tanfovy), image_height=int(cam.image_height),
        image_width=int(cam.image_width), world_view_transform=torch.from_numpy(cam.world_view_transform).to(dev),
        full_proj_transform=torch.from_numpy(cam.full_proj_transform).to(dev),
        camera_center=torch.from_numpy(cam.camera_center).to(dev))
    pipe = types.SimpleNamespace(debug=False, compute_cov3D_python=False, convert_SHs_python=False)
    return t, pc, camera, pipe


def _settings_of(camera, bg):
    from diff_gaussian_rasterization_amr import GaussianRasterizationSettings
    return GaussianRasterizationSettings(
        image_height=camera.image_height, image_width=camera.image_width, tanfovx=math.tan(camera.FoVx * 0.5),
        tanfovy=math.tan(camera.FoVy * 0.5), bg=bg, scale_modifier=1.0, viewmatrix=camera.world_view_transform,
        projmatrix=camera.full_proj_transform, sh_degree=3, campos=camera.camera_center, prefiltered=False,
        debug=False)


def _chain(args, s, interpolate=False, after0=None):
    """The reference's sequence, literally (gaussian_renderer_amr/__init__.py:183-594)."""
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    e = torch.Tensor([])
    u8 = torch.Tensor([]).to(torch.uint8)
    c0, radii, gb, bb, ib = _RasterizeGaussians.apply(*args, 0, e, u8, u8, u8, False, s)
    if after0 is not None:
        after0(ib)
    acc = c0
    for k in range(1, 5):
        ck, _, gb, bb, ib = _RasterizeGaussians.apply(*args, k, acc, gb, bb, ib, interpolate if k == 4 else False, s)
        acc = acc + ck
    return acc, radii, gb, bb, ib


CASES = [  # (P, W, H, seed, bg, colours precomputed)
    (10_000, 256, 256, 0, (0.0, 0.0, 0.0), False),
    (60_000, 1000, 600, 1, (1.0, 1.0, 1.0), False),
    (200_000, 1920, 1080, 2, (0.2, 0.5, 0.9), True),
]


@pytest.mark.gpu
@pytest.mark.parametrize("one_launch", [False, True], ids=["per_step", "one_launch"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"P{c[0]}_{c[1]}x{c[2]}")
def test_fused_steps_bit_identical_to_reference_sequence(case, one_launch):
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd.rasterization_amr import render_steps
    P, W, H, seed, bg, precomp = case
    sc, cam = G.scene_and_camera(P, W, H, seed)
    t, pc, camera, pipe = _duck(sc, cam)
    s = _settings_of(camera, torch.tensor(bg, dtype=torch.float32, device="cuda"))
    e = torch.Tensor([]).cuda()
    cols = torch.rand(P, 3, device="cuda", generator=torch.Generator("cuda").manual_seed(seed)) if precomp else e
    shs = e if precomp else t["shs"]
    m2 = torch.zeros_like(t["means3D"])
    args = (t["means3D"], m2, shs, cols, t["opacities"], t["scales"], t["rotations"], e)
    with torch.no_grad():
        ref, rradii, _, _, rib = _chain(args, s)
        got, radii, gb, bb, ib = render_steps(*args, s, one_launch=one_launch)
        torch.cuda.synchronize()
    assert torch.equal(radii, rradii)
    assert torch.equal(got, ref), float((got - ref).abs().max())
    K = int(C.parse_buffers(gb, bb, ib, P, 0, W, H, 32)["hdr"][0].item())
    d, rd = C.parse_buffers(gb, bb, ib, P, K, W, H, 32), C.parse_buffers(gb, bb, rib, P, K, W, H, 32)
    for k in ("levels", "levels_last", "levels_current"):
        assert torch.equal(d[k], rd[k]), k
    # final T and n_contrib are defined where a step rendered: round r of the
    # stride-2 lattice (offsets (0,0), (1,1), (1,0), (0,1)) in tiles of level >= r
    lv = np.minimum(d["levels"].cpu().numpy(), 4)
    y, x = np.mgrid[0:H, 0:W]
    rnd = np.array([[1, 3], [4, 2]])[y % 2, x % 2]  # [y parity, x parity]
    mask = (rnd <= lv[(y // 32) * ((W + 31) // 32) + x // 32]).ravel()
    assert mask.any()
    for k in ("n_contrib", "accum_alpha"):
        np.testing.assert_array_equal(d[k].cpu().numpy()[mask], rd[k].cpu().numpy()[mask], k)


@pytest.mark.gpu
def test_renderer_render_and_render_once_match_explicit_calls():
    from diff_gaussian_rasterization_amr import GaussianRasterizer
    from gaussian_splatting_with_eye_tracking_amd import rasterization_amr as RA
    from gaussian_splatting_with_eye_tracking_amd import renderer_amr as R
    P, W, H = 50_000, 800, 600
    sc, cam = G.scene_and_camera(P, W, H, 3)
    t, pc, camera, pipe = _duck(sc, cam)
    bg = torch.tensor([0.1, 0.2, 0.3], dtype=torch.float32, device="cuda")
    s = _settings_of(camera, bg)
    e = torch.Tensor([]).cuda()
    m2 = torch.zeros_like(t["means3D"])
    args = (t["means3D"], m2, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    with torch.no_grad():
        ref, rradii, _, _, _ = _chain(args, s)
        out = R.render(camera, pc, pipe, bg)
        assert torch.equal(out["render"], ref)
        assert torch.equal(out["radii"], rradii) and torch.equal(out["visibility_filter"], rradii > 0)
        # step 4 interpolated: the literal sequence (not fused)
        ref_i, _, _, _, _ = _chain(args, s, interpolate=True)
        assert torch.equal(R.render(camera, pc, pipe, bg, interpolate_image=True)["render"], ref_i)
        # the fovea-levels extension between step 0 and step 1
        cen, rad = RA.reference_foveae(W, H, (300.0, 200.0))
        lv = lambda ib: RA.apply_fovea_levels(ib, W, H, cen, rad)  # noqa: E731
        ref_f, _, _, _, _ = _chain(args, s, after0=lv)
        assert torch.equal(R.render(camera, pc, pipe, bg, fovea_levels=lv)["render"], ref_f)
        # render_once: one foveaStep -2 call, interpolated
        once = GaussianRasterizer(s)(means3D=t["means3D"], means2D=m2, opacities=t["opacities"], shs=t["shs"],
                                     scales=t["scales"], rotations=t["rotations"], foveaStep=-2)[0]
        assert torch.equal(R.render_once(camera, pc, pipe, bg)["render"], once)
        # override colours and the convert_SHs_python path (colours from sh_utils.eval_sh)
        ov = torch.rand(P, 3, device="cuda", generator=torch.Generator("cuda").manual_seed(5))
        ref_o, _, _, _, _ = _chain((t["means3D"], m2, e, ov, t["opacities"], t["scales"], t["rotations"], e), s)
        assert torch.equal(R.render(camera, pc, pipe, bg, override_color=ov)["render"], ref_o)
        pipe_py = types.SimpleNamespace(debug=False, compute_cov3D_python=False, convert_SHs_python=True)
        img_py = R.render(camera, pc, pipe_py, bg)["render"]
        assert G.image_l1(img_py.cpu().numpy(), ref.cpu().numpy()) < G.IMAGE_L1_TOL


@pytest.mark.gpu
def test_renderer_render_backward_through_the_step_sum():
    """With an autograd graph the renderer runs the literal sequence, so the
    frame's loss reaches the parameters (and the viewspace points) as with the
    reference's graph; the fused driver gives the same image."""
    from gaussian_splatting_with_eye_tracking_amd import renderer_amr as R
    P, W, H = 20_000, 320, 240
    sc, cam = G.scene_and_camera(P, W, H, 4)
    t, pc, camera, pipe = _duck(sc, cam)
    for k in ("means3D", "opacities", "shs"):
        t[k].requires_grad_(True)
    bg = torch.zeros(3, device="cuda")
    out = R.render(camera, pc, pipe, bg)
    out["render"].sum().backward()
    assert t["means3D"].grad is not None and torch.isfinite(t["means3D"].grad).all()
    assert float(t["opacities"].grad.abs().sum()) > 0
    with torch.no_grad():
        assert torch.equal(R.render(camera, pc, pipe, bg)["render"], out["render"].detach())


@pytest.mark.gpu
def test_base_renderer_matches_explicit_call():
    """gaussian_renderer.render's drop-in (renderer.render) = one
    GaussianRasterizer call with the same operands; the override-colour and
    convert_SHs_python paths too."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from gaussian_splatting_with_eye_tracking_amd import renderer as R
    P, W, H = 30_000, 640, 480
    sc, cam = G.scene_and_camera(P, W, H, 6)
    t, pc, camera, pipe = _duck(sc, cam)
    bg = torch.tensor([0.3, 0.3, 0.3], dtype=torch.float32, device="cuda")
    s = _settings_of(camera, bg)
    m2 = torch.zeros_like(t["means3D"])
    with torch.no_grad():
        ref, rradii = GaussianRasterizer(s)(means3D=t["means3D"], means2D=m2, opacities=t["opacities"], shs=t["shs"],
                                            scales=t["scales"], rotations=t["rotations"])
        out = R.render(camera, pc, pipe, bg)
        assert torch.equal(out["render"], ref) and torch.equal(out["radii"], rradii)
        ov = torch.rand(P, 3, device="cuda", generator=torch.Generator("cuda").manual_seed(7))
        ref_o, _ = GaussianRasterizer(s)(means3D=t["means3D"], means2D=m2, opacities=t["opacities"], colors_precomp=ov,
                                         scales=t["scales"], rotations=t["rotations"])
        assert torch.equal(R.render(camera, pc, pipe, bg, override_color=ov)["render"], ref_o)
        pipe_py = types.SimpleNamespace(debug=False, compute_cov3D_python=False, convert_SHs_python=True)
        img_py = R.render(camera, pc, pipe_py, bg)["render"]
        assert G.image_l1(img_py.cpu().numpy(), ref.cpu().numpy()) < G.IMAGE_L1_TOL


@pytest.mark.gpu
def test_fused_steps_with_nothing_visible():
    """Every Gaussian off-screen (K = 0, empty tile lists, every tile at the
    lowest level): the fused driver's frame equals the literal sequence's
    (the background where the rounds render, zero elsewhere)."""
    from gaussian_splatting_with_eye_tracking_amd.rasterization_amr import render_steps
    P, W, H = 5_000, 320, 240
    sc, cam = G.scene_and_camera(P, W, H, 7)
    t, pc, camera, pipe = _duck(sc, cam)
    t["means3D"][:, 0] += 1.0e4
    s = _settings_of(camera, torch.tensor([0.3, 0.2, 0.1], dtype=torch.float32, device="cuda"))
    e = torch.Tensor([]).cuda()
    m2 = torch.zeros_like(t["means3D"])
    args = (t["means3D"], m2, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    with torch.no_grad():
        ref, rradii, _, _, _ = _chain(args, s)
        got, radii, _, _, _ = render_steps(*args, s)
        torch.cuda.synchronize()
    assert int((rradii > 0).sum()) == 0
    assert torch.equal(got, ref) and torch.equal(radii, rradii)


@pytest.mark.gpu
@pytest.mark.parametrize("replace", [False, True])
def test_one_launch_after_fovea_levels_matches_per_step(replace):
    """Steps 1..4 as one launch after apply_fovea_levels (levels lowered, or
    replaced by the fovea discs alone) leave the frame, radii, level state
    and every rendered pixel's final T / n_contrib of the four launches."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import rasterization_amr as RA
    P, W, H = 80_000, 960, 544
    sc, cam = G.scene_and_camera(P, W, H, 11)
    t, pc, camera, pipe = _duck(sc, cam)
    s = _settings_of(camera, torch.tensor([0.1, 0.2, 0.3], dtype=torch.float32, device="cuda"))
    e = torch.Tensor([]).cuda()
    m2 = torch.zeros_like(t["means3D"])
    args = (t["means3D"], m2, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    centres, radii_f = RA.reference_foveae(W, H, (0.3 * W, 0.6 * H))
    hook = lambda ib: RA.apply_fovea_levels(ib, W, H, centres, radii_f, replace=replace)  # noqa: E731
    out = {}
    with torch.no_grad():
        for one in (False, True):
            img, radii, gb, bb, ib = RA.render_steps(*args, s, after_step0=hook, one_launch=one)
            torch.cuda.synchronize()
            K = int(C.parse_buffers(gb, bb, ib, P, 0, W, H, 32)["hdr"][0].item())
            d = C.parse_buffers(gb, bb, ib, P, K, W, H, 32)
            out[one] = (img.clone(), radii.clone(), {k: d[k].clone() for k in
                        ("levels", "levels_last", "levels_current", "n_contrib", "accum_alpha")})
    (i0, r0, d0), (i1, r1, d1) = out[False], out[True]
    assert torch.equal(i0, i1) and torch.equal(r0, r1)
    for k in ("levels", "levels_last", "levels_current"):
        assert torch.equal(d0[k], d1[k]), k
    lv = np.minimum(d0["levels"].cpu().numpy(), 4)
    assert len(np.unique(lv)) > 1
    y, x = np.mgrid[0:H, 0:W]
    rnd = np.array([[1, 3], [4, 2]])[y % 2, x % 2]
    mask = (rnd <= lv[(y // 32) * ((W + 31) // 32) + x // 32]).ravel()
    for k in ("n_contrib", "accum_alpha"):
        np.testing.assert_array_equal(d0[k].cpu().numpy()[mask], d1[k].cpu().numpy()[mask], k)


@pytest.mark.gpu
def test_unfilled_step0_option_does_not_leak():
    """The one-launch frame skips step 0's zero fill through a one-shot thread
    option; the next standalone step-0 call still returns a zero image."""
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    from gaussian_splatting_with_eye_tracking_amd.rasterization_amr import render_steps
    P, W, H = 20_000, 320, 240
    sc, cam = G.scene_and_camera(P, W, H, 5)
    t, pc, camera, pipe = _duck(sc, cam)
    s = _settings_of(camera, torch.tensor([0.3, 0.2, 0.1], dtype=torch.float32, device="cuda"))
    e = torch.Tensor([]).cuda()
    u8 = torch.empty(0, dtype=torch.uint8, device="cuda")
    m2 = torch.zeros_like(t["means3D"])
    args = (t["means3D"], m2, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    with torch.no_grad():
        ref, _, _, _, _ = _chain(args, s)
        for _ in range(2):
            got, _, _, _, _ = render_steps(*args, s)
            img0 = _RasterizeGaussians.apply(*args, 0, e, u8, u8, u8, False, s)[0]
            torch.cuda.synchronize()
            assert torch.equal(got, ref)
            assert int(torch.count_nonzero(img0)) == 0


@pytest.mark.gpu
def test_renderer_render_under_fallback_amr_variant():
    """set_tuning('amr_variant', 0) (the full-list fallback) is safe to flip
    between calls: renderer_amr.render under no_grad then takes the literal
    per-step sequence (the fused steps exist for the default variant only)
    and gives the frame of the default variant's sequence."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from gaussian_splatting_with_eye_tracking_amd import renderer_amr as R
    P, W, H = 20_000, 400, 300
    sc, cam = G.scene_and_camera(P, W, H, 4)
    t, pc, camera, pipe = _duck(sc, cam)
    bg = torch.tensor([0.0, 0.0, 0.0], dtype=torch.float32, device="cuda")
    with torch.no_grad():
        ref = R.render(camera, pc, pipe, bg)["render"]
        assert C.get_tuning("amr_variant") == 4
        C.set_tuning("amr_variant", 0)
        try:
            assert C.get_tuning("amr_variant") == 0
            got = R.render(camera, pc, pipe, bg)["render"]
        finally:
            C.set_tuning("amr_variant", 4)
        torch.cuda.synchronize()
    assert G.image_l1(got.cpu().numpy(), ref.cpu().numpy()) < G.IMAGE_L1_TOL
