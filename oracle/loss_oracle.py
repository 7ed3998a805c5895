"""CPU ORACLE (test infrastructure only): the training loss of the reference,
train.py:91-93,

    loss = (1 - lambda_dssim) * l1_loss(image, gt) + lambda_dssim * (1 - ssim(image, gt))

with utils/loss_utils.py:17-63 (11x11 Gaussian window, sigma 1.5, zero
padding 5, per channel, mean over [C, H, W]), restated in float64 numpy, and
its gradient w.r.t. `image` written out analytically (the reference gets it
from torch autograd):

    map  = A B / (Cd D),  A = 2 mu1 mu2 + C1, B = 2 s12' + C2,
           Cd = mu1^2 + mu2^2 + C1, D = s11' + s22' + C2,
           s11' = W*(x^2) - mu1^2, s12' = W*(x y) - mu1 mu2,  mu1 = W*x, mu2 = W*y
    dmap/dmu1 = (2 mu2 B - 2 mu2 A) / (Cd D) - map (2 mu1 / Cd - 2 mu1 / D)
    dmap/d(W*x^2) = -map / D,   dmap/d(W*xy) = 2 A / (Cd D)
    dL/dx = W^T * G1 + 2 x W^T * G11 + y W^T * G12 + (1 - lambda) sign(x - y) / n

where G* = (-lambda / n) dmap/d*, W^T is the adjoint of the zero-padded
"same" correlation (= the same correlation: the window is symmetric, G is 0
outside the image) and n = C H W.  Pinned by tests/test_loss.py against
tests/golden/loss_pins.npz, made by tools/make_golden.py from the reference's
own loss_utils.
"""
from __future__ import annotations

import math

import numpy as np

C1 = 0.01 ** 2
C2 = 0.03 ** 2
WINDOW = 11
SIGMA = 1.5


def window_1d() -> np.ndarray:
    """utils/loss_utils.py:23-25: float32 (torch.Tensor) values normalised in float32."""
    g = np.array([math.exp(-(x - WINDOW // 2) ** 2 / float(2 * SIGMA ** 2)) for x in range(WINDOW)], np.float32)
    return (g / g.sum(dtype=np.float32)).astype(np.float32)


def window_2d() -> np.ndarray:
    """utils/loss_utils.py:27-31: float32 outer product."""
    g = window_1d()
    return (g[:, None] * g[None, :]).astype(np.float32)


def _corr_same(x: np.ndarray, w: np.ndarray) -> np.ndarray:
    """Per-channel 'same' correlation with zero padding (F.conv2d, padding=5)."""
    C, H, W = x.shape
    r = w.shape[0] // 2
    xp = np.zeros((C, H + 2 * r, W + 2 * r), np.float64)
    xp[:, r:r + H, r:r + W] = x
    out = np.zeros((C, H, W), np.float64)
    for i in range(w.shape[0]):
        for j in range(w.shape[1]):
            out += float(w[i, j]) * xp[:, i:i + H, j:j + W]
    return out


def loss_and_grad(image, gt, lambda_dssim: float = 0.2):
    """Returns (loss, l1, ssim, dloss/dimage) in float64."""
    x = np.asarray(image, np.float64)
    y = np.asarray(gt, np.float64)
    n = x.size
    w = window_2d()
    mu1, mu2 = _corr_same(x, w), _corr_same(y, w)
    e11, e22, e12 = _corr_same(x * x, w), _corr_same(y * y, w), _corr_same(x * y, w)
    s11, s22, s12 = e11 - mu1 * mu1, e22 - mu2 * mu2, e12 - mu1 * mu2
    A = 2 * mu1 * mu2 + C1
    B = 2 * s12 + C2
    Cd = mu1 * mu1 + mu2 * mu2 + C1
    D = s11 + s22 + C2
    m = A * B / (Cd * D)
    ssim = m.mean()
    l1 = np.abs(x - y).mean()
    loss = (1 - lambda_dssim) * l1 + lambda_dssim * (1 - ssim)
    c = -lambda_dssim / n
    G1 = c * ((2 * mu2 * B - 2 * mu2 * A) / (Cd * D) - m * (2 * mu1 / Cd - 2 * mu1 / D))
    G11 = c * (-m / D)
    G12 = c * (2 * A / (Cd * D))
    grad = _corr_same(G1, w) + 2 * x * _corr_same(G11, w) + y * _corr_same(G12, w)
    grad += (1 - lambda_dssim) * np.sign(x - y) / n
    return float(loss), float(l1), float(ssim), grad
