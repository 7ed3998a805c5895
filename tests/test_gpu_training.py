"""The training iteration on the GPU (csrc/train.hip + training.py) against
the reference's own optimiser machinery restated in oracle/train_oracle.py
(nn.Parameters + torch.optim.Adam, scene/gaussian_model.py:149-407).

* Adam: the fused kernel against torch.optim.Adam on the same device, over
  several steps with per-group learning rates, a scheduled xyz rate and a
  group skipped (grad None) in the middle.  Tolerance: 2 ulp-ish (rtol 1e-6)
  -- same formula and operation order, f32.
* densification statistics: the kernel against the reference's
  gather / norm / scatter on the rasterizer's own radii and means2D grads
  (rtol 1e-6; denom and max radii exact).
* post-backward lockstep: after our render + loss + backward, the oracle is
  put in the identical state and both run train.py:108-125 at iterations that
  densify, reset opacity and step; structure (P, masks) must match exactly,
  values to Adam's tolerance.
* a short training run fits a target image (loss falls, P changes, no NaN).
"""
import math

import numpy as np
import pytest
import torch

import gs_helpers as G
import train_oracle as TO

pytestmark = pytest.mark.gpu


def _T():
    from gaussian_splatting_with_eye_tracking_amd import training
    return training


def raw_from_scene(sc, device="cuda"):
    from gaussian_splatting_with_eye_tracking_amd import ply
    g = ply.from_activated(sc.means3D, sc.opacities, sc.scales, sc.rotations, sc.shs)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(device)  # noqa: E731
    return {"xyz": t(g.xyz), "f_dc": t(g.features_dc), "f_rest": t(g.features_rest), "opacity": t(g.opacity),
            "scaling": t(g.scaling), "rotation": t(g.rotation)}


def oracle_from(m):
    """An OracleModel in exactly m's state (params, grads, moments, steps, statistics, lrs)."""
    T = _T()
    raw = {g: m.param[g].detach().clone() for g in T.GROUPS}
    o = TO.OracleModel(raw, m.spatial_lr_scale, m.opt, m.device)
    for grp in o.optimizer.param_groups:
        grp["lr"] = m.lr[grp["name"]]
    for g in T.GROUPS:
        if m.steps[g] > 0:
            o.optimizer.state[o.p[g]] = {"step": torch.tensor(float(m.steps[g])),
                                         "exp_avg": m.group_view(m.exp_avg, g).clone(),
                                         "exp_avg_sq": m.group_view(m.exp_avg_sq, g).clone()}
        o.p[g].grad = m.group_view(m.grads, g).clone() if m.has_grad[g] else None
    o.xyz_gradient_accum = m.xyz_gradient_accum.clone()
    o.denom = m.denom.clone()
    o.max_radii2D = m.max_radii2D.clone()
    return o


def _close(a, b, rtol, atol, what):
    a, b = a.detach(), b.detach()
    d = (a - b).abs()
    bad = d > atol + rtol * b.abs()
    if bool(bad.any()):
        i = int(torch.nonzero(bad.flatten())[0])
        raise AssertionError(f"{what}: {int(bad.sum())}/{a.numel()} differ, max abs {float(d.max()):.3e}, "
                             f"first at {i}: {float(a.flatten()[i])!r} vs {float(b.flatten()[i])!r}")


def assert_close_state(m, o, rtol=1e-6, atol=1e-8):
    T = _T()
    assert m.P == o.p["xyz"].shape[0]
    for g in T.GROUPS:
        e1, e2, st = o.moments(g)
        _close(m.group_view(m.exp_avg, g), e1, rtol, 1e-3 * atol, g + " exp_avg")
        _close(m.group_view(m.exp_avg_sq, g), e2, rtol, 1e-6 * atol, g + " exp_avg_sq")
        _close(m.param[g], o.p[g], rtol, atol, g + " param")
        assert m.steps[g] == st, g
    for k in ("xyz_gradient_accum", "denom", "max_radii2D"):
        torch.testing.assert_close(getattr(m, k), getattr(o, k), rtol=1e-6, atol=0, msg=k)


def test_adam_kernel_matches_torch_adam():
    T = _T()
    P = 5003
    gen = torch.Generator().manual_seed(0)
    raw = {g: (torch.randn((P,) + T.group_row_shape(g, 3), generator=gen)).cuda() for g in T.GROUPS}
    m = T.FlatGaussianModel(raw, 3, spatial_lr_scale=2.5, device="cuda")
    o = TO.OracleModel(raw, 2.5, m.opt, "cuda")
    for it in range(1, 7):
        m.update_learning_rate(it * 1000)
        o.set_lr(it * 1000)
        for g in T.GROUPS:
            scale = 10.0 ** float(torch.randint(-9, 1, (1,), generator=gen))
            grad = (torch.randn(m.param[g].shape, generator=gen) * scale).cuda()
            grad[torch.rand(grad.shape, generator=gen).cuda() < 0.05] = 0.0
            m.group_view(m.grads, g).copy_(grad)
            o.p[g].grad = grad.clone()
        m.mark_backward()
        if it == 3:  # opacity was replaced this iteration: no gradient, no step
            m.has_grad["opacity"] = False
            o.p["opacity"].grad = None
        m.optimizer_step()
        o.optimizer.step()
        m.zero_grad()
        o.optimizer.zero_grad(set_to_none=True)
    assert m.steps["opacity"] == 5 and m.steps["xyz"] == 6
    assert_close_state(m, o)
    # same formula, same operation order, same fmas: bit-identical to torch
    for g in T.GROUPS:
        same = (m.param[g].detach() == o.p[g].detach()).float().mean().item()
        assert same == 1.0, (g, same)


def _render_case(P=3000, W=128, H=96, seed=0):
    sc, cam = G.scene_and_camera(P, W, H, seed=seed)
    s = G.torch_settings(cam)
    return sc, cam, s


def test_densify_stats_kernel_matches_reference():
    T = _T()
    sc, cam, s = _render_case()
    m = T.FlatGaussianModel(raw_from_scene(sc), 3, 1.0)
    m.active_sh_degree = 3
    pkg = m.render(s)
    (pkg["render"] * torch.randn_like(pkg["render"])).sum().backward()
    g2d, radii = pkg["viewspace_points"].grad, pkg["radii"]
    assert int((radii > 0).sum()) > 100 and int((radii == 0).sum()) > 0
    o = oracle_from(m)
    for _ in range(3):
        m.add_densification_stats(g2d, radii)
        o.add_stats(g2d, radii)
    torch.testing.assert_close(m.xyz_gradient_accum, o.xyz_gradient_accum, rtol=1e-6, atol=0)
    torch.testing.assert_close(m.denom, o.denom, rtol=0, atol=0)
    torch.testing.assert_close(m.max_radii2D, o.max_radii2D, rtol=0, atol=0)


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("iteration", [2999, 3000, 3100, 4000])
def test_post_backward_lockstep_with_reference(iteration, fused):
    """train.py:108-125 at a plain step (2999), densify + opacity reset
    (3000), densify with the screen-size prune (3100) and a step after
    densification (4000, opacity step count lagging)."""
    T = _T()
    sc, cam, s = _render_case(seed=iteration)
    m = T.FlatGaussianModel(raw_from_scene(sc), 3, spatial_lr_scale=5.0)
    m.active_sh_degree = 3
    gen = torch.Generator().manual_seed(iteration)
    # a state mid-training: moments, step counts (opacity one behind), statistics
    for g in T.GROUPS:
        m.group_view(m.exp_avg, g).copy_(torch.randn(m.param[g].shape, generator=gen) * 1e-4)
        m.group_view(m.exp_avg_sq, g).copy_(torch.rand(m.param[g].shape, generator=gen) * 1e-8)
        m.steps[g] = iteration - (2 if g == "opacity" else 1)
    m.xyz_gradient_accum.copy_(torch.rand(m.P, 1, generator=gen) * 0.002)
    m.denom.copy_(torch.randint(0, 8, (m.P, 1), generator=gen).float())
    gt = torch.rand(3, cam.image_height, cam.image_width, generator=gen).cuda()
    pkg, terms = T.forward_backward(m, iteration, s, gt, fused=fused)
    assert math.isfinite(float(terms["loss"]))
    o = oracle_from(m)
    g2d = pkg["viewspace_grad"].clone()
    radii = pkg["radii"].clone()
    torch.manual_seed(7)
    T.post_backward(m, iteration, pkg, scene_extent=5.0)
    torch.manual_seed(7)
    o.post_backward(iteration, g2d, radii, extent=5.0)
    if iteration in (3000, 3100):
        assert m.P != 3000
    assert_close_state(m, o)


@pytest.mark.parametrize("active_sh", [0, 3])
def test_fused_path_matches_autograd_path(active_sh):
    """render_and_backward (activation kernels, fused loss gradient straight
    into the rasterizer backward, no autograd) against torch activations +
    the drop-in autograd rasterizer + l1_ssim_loss + loss.backward(): image
    and radii identical, raw-parameter gradients within 1e-5 relative."""
    T = _T()
    sc, cam, s = _render_case(P=5000, W=160, H=120, seed=9)
    raw = raw_from_scene(sc)
    raw["rotation"] = raw["rotation"] * torch.linspace(0.5, 2.0, 5000, device="cuda")[:, None]  # unnormalised
    gt = torch.rand(3, 120, 160, device="cuda", generator=torch.Generator("cuda").manual_seed(1))
    out = []
    for fused in (True, False):
        m = T.FlatGaussianModel(raw, 3, spatial_lr_scale=5.0)
        m.active_sh_degree = active_sh
        pkg, terms = T.forward_backward(m, 1, s, gt, fused=fused)
        out.append((m, pkg, terms))
    (mf, pf, tf), (ma, pa, ta) = out
    torch.testing.assert_close(pf["render"], pa["render"].detach(), rtol=0, atol=1e-6)
    assert torch.equal(pf["radii"], pa["radii"])
    assert abs(float(tf["loss"]) - float(ta["loss"])) < 1e-6
    torch.testing.assert_close(pf["viewspace_grad"], pa["viewspace_grad"], rtol=1e-5, atol=1e-9)
    for g in T.GROUPS:
        a, b = mf.group_view(mf.grads, g), ma.group_view(ma.grads, g)
        rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
        assert rel < 1e-5, (g, rel)
        if g == "f_rest" and active_sh == 0:
            assert float(a.abs().max()) == 0.0


def test_training_run_fits_a_target():
    T = _T()
    sc, cam, s = _render_case(P=4000, W=160, H=120, seed=3)
    from gaussian_splatting_with_eye_tracking_amd import GaussianRasterizer
    tgt = G.scene_tensors(sc)
    with torch.no_grad():
        gt, _ = GaussianRasterizer(s)(means3D=tgt["means3D"], means2D=torch.zeros_like(tgt["means3D"]),
                                      opacities=tgt["opacities"], shs=tgt["shs"], scales=tgt["scales"],
                                      rotations=tgt["rotations"])
    sc2, _ = G.scene_and_camera(4000, 160, 120, seed=4)
    opt = T.OptimizationParams(densify_from_iter=20, densification_interval=20, opacity_reset_interval=1000,
                               densify_until_iter=80, iterations=10_000)
    m = T.FlatGaussianModel(raw_from_scene(sc2), 3, spatial_lr_scale=5.0, opt=opt)
    losses, sizes = [], []
    for it in range(1, 121):
        terms = T.training_iteration(m, it, s, gt, scene_extent=5.0)
        losses.append(float(terms["loss"]))
        sizes.append(m.P)
    assert all(math.isfinite(x) for x in losses)
    assert np.mean(losses[-10:]) < 0.85 * np.mean(losses[:10]), (losses[:10], losses[-10:])
    assert len(set(sizes)) > 1
    assert torch.isfinite(m.params).all()


@pytest.mark.parametrize("active_sh", [1, 3])
def test_views_exchange_path_matches_fused_path(active_sh):
    """render_and_backward_views (blend backward -> view record -> gather ->
    multi-view parameter backward), here with one rank, against the fused
    single-view path: same image, raw-parameter gradients within 1e-5
    relative (atomic-order noise), densification statistics as the per-view
    kernel's (accum 1e-5 relative, denom / max radii exact)."""
    T = _T()
    sc, cam, s = _render_case(P=5000, W=160, H=120, seed=4)
    raw = raw_from_scene(sc)
    gt = torch.rand(3, 120, 160, device="cuda", generator=torch.Generator("cuda").manual_seed(2))
    mf = T.FlatGaussianModel(raw, 3, spatial_lr_scale=5.0)
    mv = T.FlatGaussianModel(raw, 3, spatial_lr_scale=5.0)
    for m in (mf, mv):
        m.active_sh_degree = active_sh
    pf, tf = mf.render_and_backward(s, gt, mf.opt.lambda_dssim)
    mf.add_densification_stats(pf["viewspace_grad"], pf["radii"])
    pv, tv = T.render_and_backward_views(mv, s, gt, mv.opt.lambda_dssim, stats=True)
    assert pv["stats_done"]
    torch.testing.assert_close(pv["render"], pf["render"], rtol=0, atol=0)
    assert torch.equal(pv["radii"], pf["radii"])
    for g in T.GROUPS:
        a, b = mv.group_view(mv.grads, g), mf.group_view(mf.grads, g)
        rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
        assert rel < 1e-5, (g, rel)
    rel = float((mv.xyz_gradient_accum - mf.xyz_gradient_accum).norm() / mf.xyz_gradient_accum.norm())
    assert rel < 1e-5
    assert torch.equal(mv.denom, mf.denom)
    assert torch.equal(mv.max_radii2D, mf.max_radii2D)
