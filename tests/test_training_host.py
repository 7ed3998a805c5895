"""Host logic of the training iteration (training.py) against the oracle
restatement of the reference's GaussianModel + torch.optim.Adam
(oracle/train_oracle.py), on CPU.

Covered here without a GPU: the flat-buffer layout and autograd aliasing,
the learning-rate schedule, densify_and_prune (clone + split + prune, with
the same torch.normal samples) and reset_opacity on identical states
including the Adam moments, and the world-size-2 gloo exchange of the
gradient buffer and the densification statistics.  The Adam / statistics
kernels themselves are in tests/test_gpu_training.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gaussian_splatting_with_eye_tracking_amd import training as T
import train_oracle as TO

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def raw_scene(P, seed=0, sh_degree=3):
    g = torch.Generator().manual_seed(seed)
    M = (sh_degree + 1) ** 2
    return {
        "xyz": torch.randn(P, 3, generator=g) * 2,
        "f_dc": torch.randn(P, 1, 3, generator=g) * 0.5,
        "f_rest": torch.randn(P, M - 1, 3, generator=g) * 0.1,
        "opacity": torch.randn(P, 1, generator=g) * 3,
        "scaling": torch.randn(P, 3, generator=g) * 1.0 - 4.0,   # exp: ~0.002 .. 0.15
        "rotation": torch.randn(P, 4, generator=g),
    }


def twin(P=400, seed=0, steps=7, extent=3.0):
    """A FlatGaussianModel and an OracleModel in the same state: parameters,
    Adam moments + step counts, densification statistics."""
    raw = raw_scene(P, seed)
    opt = T.OptimizationParams()
    m = T.FlatGaussianModel(raw, 3, spatial_lr_scale=extent, opt=opt, device="cpu")
    o = TO.OracleModel(raw, extent, opt, "cpu")
    g = torch.Generator().manual_seed(seed + 1)
    for name in T.GROUPS:
        e1 = torch.randn(m.param[name].shape, generator=g) * 1e-3
        e2 = torch.rand(m.param[name].shape, generator=g) * 1e-6
        m.group_view(m.exp_avg, name).copy_(e1)
        m.group_view(m.exp_avg_sq, name).copy_(e2)
        m.steps[name] = steps
        o.optimizer.state[o.p[name]] = {"step": torch.tensor(float(steps)), "exp_avg": e1.clone(),
                                        "exp_avg_sq": e2.clone()}
    accum = torch.rand(P, 1, generator=g) * 0.004
    denom = torch.randint(0, 5, (P, 1), generator=g).float()
    radii = torch.randint(0, 40, (P,), generator=g).float()
    for t in (m, o):
        t.xyz_gradient_accum = accum.clone()
        t.denom = denom.clone()
        t.max_radii2D = radii.clone()
    return m, o


def assert_same(m, o):
    assert m.P == o.p["xyz"].shape[0]
    for name in T.GROUPS:
        torch.testing.assert_close(m.param[name].detach(), o.p[name].detach(), rtol=0, atol=0, msg=name)
        e1, e2, st = o.moments(name)
        torch.testing.assert_close(m.group_view(m.exp_avg, name), e1, rtol=0, atol=0, msg=name)
        torch.testing.assert_close(m.group_view(m.exp_avg_sq, name), e2, rtol=0, atol=0, msg=name)
        assert m.steps[name] == st, name
    for k in ("xyz_gradient_accum", "denom", "max_radii2D"):
        torch.testing.assert_close(getattr(m, k), getattr(o, k), rtol=0, atol=0, msg=k)


def test_flat_layout_and_autograd_aliasing():
    raw = raw_scene(50)
    m = T.FlatGaussianModel(raw, 3, 1.0, device="cpu")
    assert m.params.numel() == 50 * 59 and m.seg_end[-1] == 50 * 59
    for name in T.GROUPS:
        np.testing.assert_array_equal(m.param[name].detach().numpy(), raw[name].numpy())
        p = m.param[name]
        assert m.params.data_ptr() <= p.data_ptr() < m.params.data_ptr() + m.params.numel() * 4
    # autograd accumulates into the flat gradient buffer
    loss = (m.get_xyz ** 2).sum() + m.get_features.sum() + m.get_opacity.sum() + m.get_scaling.sum() + \
        m.get_rotation[:, 0].sum()
    loss.backward()
    g = m.group_view(m.grads, "xyz")
    torch.testing.assert_close(g, 2 * raw["xyz"])
    torch.testing.assert_close(m.group_view(m.grads, "f_rest"), torch.ones(50, 15, 3))
    s = torch.sigmoid(raw["opacity"])
    torch.testing.assert_close(m.group_view(m.grads, "opacity"), s * (1 - s))
    assert m.param["xyz"].grad.data_ptr() == m.grads.data_ptr()
    m.zero_grad()
    assert float(m.grads.abs().sum()) == 0.0


def test_learning_rate_schedule_matches_reference():
    raw = raw_scene(4)
    m = T.FlatGaussianModel(raw, 3, spatial_lr_scale=4.2, device="cpu")
    o = TO.OracleModel(raw, 4.2, m.opt, "cpu")
    for it in (0, 1, 2, 100, 7000, 29999, 30000, 45000):
        o.set_lr(it)
        assert m.update_learning_rate(it) == o.optimizer.param_groups[0]["lr"]
    assert m.lr["f_rest"] == 0.0025 / 20.0 and m.lr["opacity"] == 0.05
    assert T.get_expon_lr_func(1e-3, 1e-5, max_steps=100)(100) == pytest.approx(1e-5)


@pytest.mark.parametrize("max_screen_size", [None, 20])
def test_densify_and_prune_matches_reference(max_screen_size):
    m, o = twin()
    torch.manual_seed(11)
    m.densify_and_prune(0.0002, 0.005, 3.0, max_screen_size)
    torch.manual_seed(11)
    o.densify_and_prune(0.0002, 0.005, 3.0, max_screen_size)
    assert m.P != 400
    assert_same(m, o)
    assert not any(m.has_grad.values())


def test_densify_prunes_everything_and_empty_model():
    m, o = twin(P=30)
    for t in (m, o):
        t.xyz_gradient_accum.zero_()
    m.group_view(m.params, "opacity").fill_(-20.0)
    with torch.no_grad():
        o.p["opacity"].fill_(-20.0)
    m.densify_and_prune(0.0002, 0.005, 3.0, None)
    o.densify_and_prune(0.0002, 0.005, 3.0, None)
    assert m.P == 0
    assert_same(m, o)
    m.optimizer_step()  # a no-op on an empty model, no kernel launch


def test_reset_opacity_matches_reference():
    m, o = twin(P=64)
    m.mark_backward()
    m.reset_opacity()
    o.reset_opacity()
    assert_same(m, o)
    assert m.has_grad["opacity"] is False and m.has_grad["xyz"] is True
    assert float(m.get_opacity.max()) <= 0.01 + 1e-6


def _gloo_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from gaussian_splatting_with_eye_tracking_amd import training as TT
        m = TT.FlatGaussianModel(raw_scene(40), 3, 1.0, device="cpu")
        g = torch.Generator().manual_seed(100 + rank)
        m.grads.copy_(torch.randn(m.grads.shape, generator=g))
        m.xyz_gradient_accum.copy_(torch.rand(40, 1, generator=g))
        m.denom.copy_(torch.randint(0, 3, (40, 1), generator=g).float())
        m.max_radii2D.copy_(torch.randint(0, 30, (40,), generator=g).float())
        TT.allreduce_training_grads(m)
        TT.reduce_densification_stats(m)
        q.put((rank, m.grads.numpy().copy(), m.xyz_gradient_accum.numpy().copy(), m.denom.numpy().copy(),
               m.max_radii2D.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gradient_and_statistics_exchange():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = socket.socket()
    port.bind(("127.0.0.1", 0))
    p = port.getsockname()[1]
    port.close()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, p, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    out = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in range(2)))
    for pr in procs:
        pr.join(60)
        assert pr.exitcode == 0
    exp = []
    for rank in range(2):
        g = torch.Generator().manual_seed(100 + rank)
        n = 40 * 59
        exp.append((torch.randn(n, generator=g), torch.rand(40, 1, generator=g),
                    torch.randint(0, 3, (40, 1), generator=g).float(), torch.randint(0, 30, (40,), generator=g).float()))
    for r in range(2):
        np.testing.assert_array_equal(out[r][0], out[0][0])
        np.testing.assert_allclose(out[r][0], (exp[0][0] + exp[1][0]).numpy(), rtol=1e-6)
        np.testing.assert_allclose(out[r][1], (exp[0][1] + exp[1][1]).numpy(), rtol=1e-6)
        np.testing.assert_array_equal(out[r][2], (exp[0][2] + exp[1][2]).numpy())
        np.testing.assert_array_equal(out[r][3], torch.maximum(exp[0][3], exp[1][3]).numpy())
