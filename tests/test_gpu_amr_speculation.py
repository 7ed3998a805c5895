"""The speculative AMR steps of the torch binding (torch_ext.cpp SpecSteps):
the reference's literal foveated sequence (gaussian_renderer_amr/__init__.py:
183-594 -- foveaStep 0..4 through _RasterizeGaussians.apply, the caller
adding each step's image) with step 1 rendering all four steps' images in one
launch (GSPLAT_AMD_AMR_STEPS_1_TO_4_SPLIT) and steps 2..4 served from it,
against the same calls with the speculation off (every step its own launch):

* every step's image, the summed frame and the radii bit for bit, the level
  state after step 4, final T and n_contrib where a round rendered;
* the misses fall back to the per-step path with the level state the steps
  served so far leave: a fovea-level change between steps (the image
  buffer's version moves), step 4 with interpolation, a step repeated, and a
  new frame before the last step (a frame left before step 4 keeps the
  level state, final T and n_contrib of all four steps: the one launch
  wrote them).
"""
import numpy as np
import pytest

import gs_helpers as G

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _args(P, W, H, seed, precomp=False):
    sc, cam = G.scene_and_camera(P, W, H, seed)
    s = G.torch_settings(cam, amr=True, bg=(0.2, 0.5, 0.9) if precomp else (0.0, 0.0, 0.0))
    t = G.scene_tensors(sc)
    e = torch.Tensor([]).cuda()
    cols = torch.rand(P, 3, device="cuda", generator=torch.Generator("cuda").manual_seed(seed)) if precomp else e
    shs = e if precomp else t["shs"]
    m2 = torch.zeros_like(t["means3D"])
    return (t["means3D"], m2, shs, cols, t["opacities"], t["scales"], t["rotations"], e), s


def _chain(args, s, spec, hook=None, steps=(1, 2, 3, 4), interp4=False):
    """The literal sequence; hook(k, ib) runs before step k.  Returns the step
    images, the frame, step 0's radii and buffers, the steps' radii."""
    import gaussian_splatting_with_eye_tracking_amd._C as C
    from diff_gaussian_rasterization_amr import _RasterizeGaussians
    e = torch.Tensor([]).cuda()
    u8 = torch.Tensor([]).to(torch.uint8).cuda()
    C.set_amr_speculation(spec)
    try:
        c0, radii, gb, bb, ib = _RasterizeGaussians.apply(*args, 0, e, u8, u8, u8, False, s)
        imgs, rads = [c0.clone()], []
        acc = c0
        for k in steps:
            if hook is not None:
                hook(k, ib)
            ck, rk, gb, bb, ib = _RasterizeGaussians.apply(*args, k, acc, gb, bb, ib, interp4 and k == 4, s)
            imgs.append(ck.clone())
            rads.append(rk.clone())
            acc = acc + ck
        torch.cuda.synchronize()
        return imgs, acc, radii, (gb, bb, ib), rads
    finally:
        C.set_amr_speculation(True)


def _rendered_mask(levels, W, H):
    lv = np.minimum(levels, 4)
    y, x = np.mgrid[0:H, 0:W]
    rnd = np.array([[1, 3], [4, 2]])[y % 2, x % 2]
    return (rnd <= lv[(y // 32) * ((W + 31) // 32) + x // 32]).ravel()


def _same(a, b, P, W, H, state=True):
    import gaussian_splatting_with_eye_tracking_amd._C as C
    ia, fa, ra, bufa, rka = a
    ib_, fb, rb, bufb, rkb = b
    assert len(ia) == len(ib_)
    for k, (x, y) in enumerate(zip(ia, ib_)):
        assert torch.equal(x, y), k
    assert torch.equal(fa, fb)
    assert torch.equal(ra, rb)
    for x, y in zip(rka, rkb):
        assert torch.equal(x, y) and not x.any()
    if not state:
        return
    K = int(C.parse_buffers(*bufa, P, 0, W, H, 32)["hdr"][0].item())
    da, db = C.parse_buffers(*bufa, P, K, W, H, 32), C.parse_buffers(*bufb, P, K, W, H, 32)
    for k in ("levels", "levels_last", "levels_current"):
        assert torch.equal(da[k], db[k]), k
    m = _rendered_mask(da["levels"].cpu().numpy(), W, H)
    for k in ("n_contrib", "accum_alpha"):
        np.testing.assert_array_equal(da[k].cpu().numpy()[m], db[k].cpu().numpy()[m], k)


@pytest.mark.parametrize("case", [(10_000, 256, 256, 0, False), (60_000, 1000, 600, 1, False),
                                  (200_000, 1920, 1080, 2, True)], ids=lambda c: f"P{c[0]}_{c[1]}x{c[2]}")
def test_speculative_steps_equal_per_step_calls(case):
    P, W, H, seed, precomp = case
    args, s = _args(P, W, H, seed, precomp)
    with torch.no_grad():
        on = _chain(args, s, True)
        off = _chain(args, s, False)
    _same(on, off, P, W, H)
    # the fused driver's frame (render_steps) too
    from gaussian_splatting_with_eye_tracking_amd.rasterization_amr import render_steps
    with torch.no_grad():
        fused = render_steps(*args, s)[0]
    torch.cuda.synchronize()
    assert torch.equal(fused, on[1])


def test_speculation_misses_fall_back_to_the_per_step_path():
    from gaussian_splatting_with_eye_tracking_amd import rasterization_amr as RA
    P, W, H = 60_000, 1000, 600
    args, s = _args(P, W, H, 3)
    cen, rad = RA.reference_foveae(W, H, (300.0, 200.0))

    def fovea_before_2(k, ib):  # a level change between steps 1 and 2 (the version moves)
        if k == 2:
            RA.apply_fovea_levels(ib, W, H, cen, rad)

    with torch.no_grad():
        for kw in (dict(hook=fovea_before_2), dict(interp4=True), dict(steps=(1, 2, 2, 3, 4)),
                   dict(steps=(1, 2, 3))):
            on = _chain(args, s, True, **kw)
            off = _chain(args, s, False, **kw)
            # (a frame left before step 4: the buffer's level state, final T
            # and n_contrib are those of all four steps -- documented)
            _same(on, off, P, W, H, state=kw.get("steps", (1, 2, 3, 4))[-1] == 4)
        # a frame left after step 3, then a new one: nothing of the old survives
        _chain(args, s, True, steps=(1, 2, 3))
        on = _chain(args, s, True)
        off = _chain(args, s, False)
    _same(on, off, P, W, H)


def test_speculation_under_autograd_matches_per_step_gradients():
    """With an autograd graph (the renderer's training use) the served step
    images carry the same backward as the per-step ones."""
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    P, W, H = 20_000, 400, 300
    args, s = _args(P, W, H, 5)
    cot = torch.from_numpy(S.make_cotangent(H, W, 9)).cuda()
    grads = []
    for spec in (True, False):
        a = [x.detach().clone().requires_grad_(x.numel() > 0 and i != 7) for i, x in enumerate(args)]
        _imgs, frame, _r, _b, _rk = _chain(tuple(a), s, spec)
        torch.autograd.backward(frame, cot)
        torch.cuda.synchronize()
        grads.append([x.grad.clone() for x in a if x.grad is not None])
    for x, y in zip(*grads):
        assert G.rel_err(x.cpu().numpy(), y.cpu().numpy()) < 1e-5
