"""Training loss of the reference on the fused HIP kernel (§8(f) rank 2).

train.py:91-93:  loss = (1 - lambda_dssim) * l1_loss(image, gt) + lambda_dssim * (1 - ssim(image, gt))
with utils/loss_utils.py:17-63.  `l1_ssim_loss` computes the value and the
gradient w.r.t. `image` in one pass (csrc/loss.hip); autograd scales the saved
gradient by the incoming one.  `gt` gets no gradient (it is data).
"""
from __future__ import annotations

import torch

from . import _C


class _L1Ssim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, gt, lambda_dssim):
        out3, grad = _C.l1_ssim_loss(image, gt, float(lambda_dssim))
        ctx.save_for_backward(grad)
        ctx.mark_non_differentiable(out3)
        return out3[0], out3

    @staticmethod
    def backward(ctx, g_loss, _g_terms):
        (grad,) = ctx.saved_tensors
        return grad * g_loss, None, None


def l1_ssim_loss_terms(image: torch.Tensor, gt: torch.Tensor, lambda_dssim: float = 0.2):
    """(loss, l1, ssim): loss differentiable w.r.t. image; l1 / ssim for logging."""
    loss, out3 = _L1Ssim.apply(image, gt, lambda_dssim)
    return loss, out3[1], out3[2]


def l1_ssim_loss(image: torch.Tensor, gt: torch.Tensor, lambda_dssim: float = 0.2) -> torch.Tensor:
    """(1 - lambda) * L1 + lambda * (1 - SSIM), as train.py:91-93."""
    return l1_ssim_loss_terms(image, gt, lambda_dssim)[0]
