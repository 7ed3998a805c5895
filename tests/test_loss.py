"""Fused L1 + D-SSIM training loss (train.py:91-93, utils/loss_utils.py:17-63).

Pinned to tests/golden/loss_pins.npz: values and autograd gradients of the
reference's own loss_utils (tools/make_golden.py imports /root/reference).
CPU: the float64 oracle with the analytic backward (oracle/loss_oracle.py)
against the pins.  GPU: the HIP kernel against the pins and the oracle.
Tolerances: loss 1e-5 absolute, gradient 1e-4 relative (L2), as the
rasterizer's gradients.
"""
import os

import numpy as np
import pytest

import gs_helpers as G
import loss_oracle as L

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["rand_3x37x53", "near_3x64x80", "same_3x16x16", "rand_1x20x30", "tiny_3x7x5"]


def _pins():
    return np.load(os.path.join(GOLD, "loss_pins.npz"))


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_loss_utils(name):
    d = _pins()
    loss, l1, ssim, grad = L.loss_and_grad(d[name + "_img"], d[name + "_gt"], float(d["lambda_dssim"]))
    assert abs(loss - float(d[name + "_f64_loss"])) < 1e-6
    assert abs(l1 - float(d[name + "_f64_l1"])) < 1e-7
    assert abs(ssim - float(d[name + "_f64_ssim"])) < 1e-6
    ref = d[name + "_f64_grad"]
    assert np.abs(grad - ref).max() < 1e-8 + 1e-5 * np.abs(ref).max()


def test_window_is_the_references():
    w = L.window_1d()
    assert w.dtype == np.float32 and abs(float(w.sum()) - 1.0) < 1e-6
    assert np.argmax(w) == 5 and np.allclose(w, w[::-1])


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_kernel_matches_reference_pins(name):
    import torch
    from gaussian_splatting_with_eye_tracking_amd import losses
    d = _pins()
    x = torch.from_numpy(d[name + "_img"]).cuda().requires_grad_(True)
    y = torch.from_numpy(d[name + "_gt"]).cuda()
    loss, l1, ssim = losses.l1_ssim_loss_terms(x, y, float(d["lambda_dssim"]))
    loss.backward()
    assert abs(float(loss.detach()) - float(d[name + "_f64_loss"])) < 1e-5
    assert abs(float(l1) - float(d[name + "_f64_l1"])) < 1e-5
    assert abs(float(ssim) - float(d[name + "_f64_ssim"])) < 1e-5
    ref = d[name + "_f64_grad"]
    g = x.grad.cpu().numpy()
    if np.abs(ref).max() < 1e-12:  # identical images: zero gradient
        assert np.abs(g).max() < 1e-9
    else:
        assert G.rel_err(g, ref) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("C,H,W", [(3, 200, 301), (3, 1080, 1920), (2, 33, 31)])
def test_kernel_matches_oracle_random(C, H, W):
    import torch
    from gaussian_splatting_with_eye_tracking_amd import losses
    rng = np.random.default_rng(H * W)
    img = rng.uniform(0, 1, (C, H, W)).astype(np.float32)
    gt = np.clip(img + rng.normal(0, 0.1, img.shape), 0, 1).astype(np.float32)
    x = torch.from_numpy(img).cuda().requires_grad_(True)
    loss, l1, ssim = losses.l1_ssim_loss_terms(x, torch.from_numpy(gt).cuda(), 0.2)
    (2.0 * loss).backward()  # the incoming gradient scales the result
    if H * W > 100000:  # the oracle's 121-shift correlation is slow: compare a crop of the gradient
        rl, rl1, rs, rg = L.loss_and_grad(img[:, :64, :96], gt[:, :64, :96])
        # the gradient at p depends on pixels within 10 px (5 + 5 window radii):
        # away from the crop's artificial bottom/right edges the crop is exact
        g = x.grad.cpu().numpy()[:, :54, :86]
        assert G.rel_err(g / 2.0 * (img.size / img[:, :64, :96].size), rg[:, :54, :86]) < 1e-4
        assert 0.0 < float(ssim) < 1.0 and float(l1) > 0.0
    else:
        rl, rl1, rs, rg = L.loss_and_grad(img, gt)
        assert abs(float(loss.detach()) - rl) < 1e-5
        assert G.rel_err(x.grad.cpu().numpy() / 2.0, rg) < 1e-4
