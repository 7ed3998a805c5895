"""TEST INFRASTRUCTURE ONLY (never imported by the product path).

CPU restatement of RITnet's DenseNet2D forward in eval mode
(RITnet/densenet.py:17-144: down blocks :34-49, up blocks :72-83, network
:130-144; dropout is the identity in eval, BatchNorm uses the running
statistics) with torch.nn.functional on float32 CPU tensors, from a state
dict -- the checker for csrc/ritnet.hip.  Also a seeded random state dict of
the reference's shapes (32 channels, 1 input, 4 classes) for GPU parity
tests that must not depend on the reference's checkpoint.

Pinning: tests/test_eye_tracking_host.py runs this restatement with the
reference's own checkpoint (RITnet/best_model.pkl, loaded weights_only) on
the reference's eye.png through eye_tracking.preprocess and compares the
labels with the prediction the reference saved (eye_seg_pred.png, right
half) -- in this container only, where /root/reference exists.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

DOWN = ("down_block1", "down_block2", "down_block3", "down_block4", "down_block5")
UP = ("up_block1", "up_block2", "up_block3", "up_block4")


def _conv(sd, name, x, pad):
    return F.conv2d(x, sd[name + ".weight"], sd[name + ".bias"], padding=pad)


def _down(sd, blk, x, pool):  # densenet.py:34-49 (dropout=True, eval)
    if pool:
        x = F.avg_pool2d(x, 2)
    x1 = F.leaky_relu(_conv(sd, blk + ".conv1", x, 1))
    x21 = torch.cat((x, x1), dim=1)
    x22 = F.leaky_relu(_conv(sd, blk + ".conv22", _conv(sd, blk + ".conv21", x21, 0), 1))
    x31 = torch.cat((x21, x22), dim=1)
    out = F.leaky_relu(_conv(sd, blk + ".conv32", _conv(sd, blk + ".conv31", x31, 0), 1))
    return F.batch_norm(out, sd[blk + ".bn.running_mean"], sd[blk + ".bn.running_var"], sd[blk + ".bn.weight"],
                        sd[blk + ".bn.bias"], training=False, eps=1e-5)


def _up(sd, blk, skip, x):  # densenet.py:72-83
    x = F.interpolate(x, scale_factor=2, mode="nearest")
    x = torch.cat((x, skip), dim=1)
    x1 = F.leaky_relu(_conv(sd, blk + ".conv12", _conv(sd, blk + ".conv11", x, 0), 1))
    x21 = torch.cat((x, x1), dim=1)
    return F.leaky_relu(_conv(sd, blk + ".conv22", _conv(sd, blk + ".conv21", x21, 0), 1))


@torch.no_grad()
def forward(sd: Dict[str, torch.Tensor], x: np.ndarray) -> np.ndarray:
    """x: [H, W] float32 (the normalised, transposed image) -> logits [4, H, W]."""
    sd = {k: v.detach().to("cpu", torch.float32) for k, v in sd.items()}
    t = torch.from_numpy(np.ascontiguousarray(x, np.float32))[None, None]
    x1 = _down(sd, "down_block1", t, False)
    x2 = _down(sd, "down_block2", x1, True)
    x3 = _down(sd, "down_block3", x2, True)
    x4 = _down(sd, "down_block4", x3, True)
    x5 = _down(sd, "down_block5", x4, True)
    x6 = _up(sd, "up_block1", x4, x5)
    x7 = _up(sd, "up_block2", x3, x6)
    x8 = _up(sd, "up_block3", x2, x7)
    x9 = _up(sd, "up_block4", x1, x8)
    return _conv(sd, "out_conv1", x9, 0)[0].numpy()


def labels(logits: np.ndarray) -> np.ndarray:
    """RITnet/utils.py:186-190 (torch.max over classes: first maximum)."""
    return np.argmax(logits, axis=0).astype(np.uint8)


def random_state_dict(seed: int = 0, channels: int = 32) -> Dict[str, torch.Tensor]:
    """A DenseNet2D(1, 4, 32) state dict with random weights, biases and
    BatchNorm statistics (weights ~ N(0, sqrt(2 / n)) as densenet.py:118-121)."""
    g = torch.Generator().manual_seed(seed)
    sd: Dict[str, torch.Tensor] = {}

    def conv(name, cin, cout, k):
        n = k * k * cout
        sd[name + ".weight"] = torch.randn(cout, cin, k, k, generator=g) * float(np.sqrt(2.0 / n))
        sd[name + ".bias"] = torch.randn(cout, generator=g) * 0.05

    c = channels
    for i, blk in enumerate(DOWN):
        cin = 1 if i == 0 else c
        conv(blk + ".conv1", cin, c, 3)
        conv(blk + ".conv21", cin + c, c, 1)
        conv(blk + ".conv22", c, c, 3)
        conv(blk + ".conv31", cin + 2 * c, c, 1)
        conv(blk + ".conv32", c, c, 3)
        sd[blk + ".bn.weight"] = 1.0 + 0.1 * torch.randn(c, generator=g)
        sd[blk + ".bn.bias"] = 0.1 * torch.randn(c, generator=g)
        sd[blk + ".bn.running_mean"] = 0.2 * torch.randn(c, generator=g)
        sd[blk + ".bn.running_var"] = 0.5 + torch.rand(c, generator=g)
    for blk in UP:
        conv(blk + ".conv11", 2 * c, c, 1)
        conv(blk + ".conv12", c, c, 3)
        conv(blk + ".conv21", 3 * c, c, 1)
        conv(blk + ".conv22", c, c, 3)
    conv("out_conv1", c, 4, 1)
    return sd
