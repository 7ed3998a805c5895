"""Eye-tracking front end: eye image -> RITnet
segmentation -> pupil centroid -> fovea centre on the rendered frame.

Follows track_render.py:50-97 (the reference's demo; its gaze step is a TODO,
so the pupil centroid is the fovea signal, as SURVEY §8(d) config 3 uses it):

* preprocessing (track_render.py:69-80): PIL "L" image, gamma 0.8 table
  through cv2.LUT then truncated to uint8, cv2.createCLAHE(clipLimit=1.5,
  tileGridSize=(8, 8)).apply, torchvision ToTensor + Normalize([0.5], [0.5])
  (RITnet/dataset.py:35-37), and the (0, 1, 3, 2) permute: the network sees
  the TRANSPOSED image.  OpenCV is not a dependency here: ``clahe`` restates
  its 8-bit CLAHE (per-tile histogram, clip limit int(1.5 * tile area / 256),
  batch + stepped-residual redistribution, rounded LUT, bilinear blend of
  the four surrounding tile LUTs).  ``preprocess`` is that host
  restatement (pinned by the reference's saved segmentation); the tracking
  path runs the same arithmetic on the MI355X (``preprocess_device``,
  csrc/eye_preprocess.hip, bit-identical), so a frame crosses PCIe as
  256 KB of bytes and never takes a host pass.
* DenseNet2D (RITnet/densenet.py:17-144, eval mode: dropout off, BatchNorm
  on running statistics) on the MI355X: every convolution, the fused
  LeakyReLU / BatchNorm epilogues, the pooling, the virtual concatenations /
  upsampling and the class argmax are the HIP kernels of csrc/ritnet.hip
  (``_C.ritnet_conv`` / ``avgpool2`` / ``ritnet_head``).  No CPU fallback.
* get_predictions (RITnet/utils.py:186-190): argmax over the 4 classes
  (0 background, 1 sclera, 2 iris, 3 pupil).
* the pupil centroid (``_C.label_moments``) and its mapping onto the render:
  (x / eye_width * W, y / eye_height * H) in the eye image's orientation.

Checkpoints load with ``torch.load(..., weights_only=True)`` (RITnet's
best_model.pkl is a plain state dict).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _C

BN_EPS = 1e-5          # nn.BatchNorm2d default
GAMMA = 0.8            # track_render.py:72
CLAHE_CLIP = 1.5       # track_render.py:75
CLAHE_GRID = (8, 8)
PUPIL = 3


# ----------------------------------------------------------- preprocessing ---
def gamma_table() -> np.ndarray:
    """track_render.py:72: 255 * linspace(0, 1, 256) ** 0.8 (float64)."""
    return 255.0 * (np.linspace(0, 1, 256) ** GAMMA)


def apply_gamma(img: np.ndarray) -> np.ndarray:
    """cv2.LUT(uint8, float64 table) then np.uint8(...) (truncation)."""
    return gamma_table()[np.asarray(img, np.uint8)].astype(np.uint8)


def _round_half_even(x: np.ndarray) -> np.ndarray:
    return np.rint(x)  # cvRound / saturate_cast<uchar>(float): nearest, ties to even


def clahe(img: np.ndarray, clip_limit: float = CLAHE_CLIP, grid: Tuple[int, int] = CLAHE_GRID) -> np.ndarray:
    """OpenCV's 8-bit CLAHE (cv::createCLAHE(clip, grid)->apply), restated.

    Image sizes divisible by the grid are required (the reference's 640x400
    with 8x8 tiles); OpenCV would pad other sizes with BORDER_REFLECT_101."""
    src = np.asarray(img, np.uint8)
    H, W = src.shape
    tx, ty = grid
    if W % tx or H % ty:
        raise ValueError("clahe: image size must be divisible by the tile grid")
    tw, th = W // tx, H // ty
    total = tw * th
    hist_size = 256
    limit = max(int(clip_limit * total / hist_size), 1) if clip_limit > 0 else 0
    lut_scale = np.float32(hist_size - 1) / np.float32(total)
    luts = np.empty((ty, tx, hist_size), np.float32)
    for j in range(ty):
        for i in range(tx):
            tile = src[j * th:(j + 1) * th, i * tw:(i + 1) * tw]
            hist = np.bincount(tile.ravel(), minlength=hist_size).astype(np.int64)
            if limit > 0:
                over = np.maximum(hist - limit, 0)
                clipped = int(over.sum())
                hist = np.minimum(hist, limit)
                batch = clipped // hist_size
                residual = clipped - batch * hist_size
                hist += batch
                if residual:
                    step = max(hist_size // residual, 1)
                    k = 0
                    while k < hist_size and residual > 0:
                        hist[k] += 1
                        k += step
                        residual -= 1
            csum = np.cumsum(hist)
            luts[j, i] = np.clip(_round_half_even(csum.astype(np.float32) * lut_scale), 0, 255)
    inv_tw = np.float32(1.0) / np.float32(tw)
    inv_th = np.float32(1.0) / np.float32(th)
    xs = np.arange(W, dtype=np.float32) * inv_tw - np.float32(0.5)
    ys = np.arange(H, dtype=np.float32) * inv_th - np.float32(0.5)
    tx1 = np.floor(xs).astype(np.int64)
    xa = (xs - tx1.astype(np.float32)).astype(np.float32)
    tx2 = np.minimum(tx1 + 1, tx - 1)
    tx1 = np.maximum(tx1, 0)
    ty1 = np.floor(ys).astype(np.int64)
    ya = (ys - ty1.astype(np.float32)).astype(np.float32)
    ty2 = np.minimum(ty1 + 1, ty - 1)
    ty1 = np.maximum(ty1, 0)
    v = src.astype(np.int64)
    l11 = luts[ty1[:, None], tx1[None, :], v]
    l12 = luts[ty1[:, None], tx2[None, :], v]
    l21 = luts[ty2[:, None], tx1[None, :], v]
    l22 = luts[ty2[:, None], tx2[None, :], v]
    one = np.float32(1.0)
    xa_, ya_ = xa[None, :], ya[:, None]
    res = (l11 * (one - xa_) + l12 * xa_) * (one - ya_) + (l21 * (one - xa_) + l22 * xa_) * ya_
    return np.clip(_round_half_even(res.astype(np.float32)), 0, 255).astype(np.uint8)


def normalize(img: np.ndarray) -> np.ndarray:
    """ToTensor (x / 255 in float32) + Normalize([0.5], [0.5])."""
    x = np.asarray(img, np.uint8).astype(np.float32) / np.float32(255.0)
    return (x - np.float32(0.5)) / np.float32(0.5)


def preprocess(gray: np.ndarray) -> np.ndarray:
    """track_render.py:69-80: the network input [W, H] (transposed), float32."""
    return np.ascontiguousarray(normalize(clahe(apply_gamma(gray))).T)


_GAMMA_DEV: Dict[torch.device, torch.Tensor] = {}


def preprocess_device(gray: torch.Tensor) -> torch.Tensor:
    """``preprocess`` on the device: uint8 [h, w] device tensor -> float32
    [w, h] (gamma table, CLAHE, ToTensor + Normalize, transpose) by the HIP
    kernels of csrc/eye_preprocess.hip; bit-identical to ``preprocess``."""
    if gray.dtype != torch.uint8 or gray.dim() != 2 or not gray.is_cuda:
        raise ValueError("preprocess_device: uint8 [H, W] device tensor required")
    lut = _GAMMA_DEV.get(gray.device)
    if lut is None:
        lut = torch.from_numpy(gamma_table().astype(np.uint8)).to(gray.device)
        _GAMMA_DEV[gray.device] = lut
    return _C.eye_preprocess(gray.contiguous(), lut, CLAHE_CLIP, CLAHE_GRID[0], CLAHE_GRID[1])


# ----------------------------------------------------------------- network ---
_DOWN = ("down_block1", "down_block2", "down_block3", "down_block4", "down_block5")
_UP = ("up_block1", "up_block2", "up_block3", "up_block4")


class RITnet:
    """DenseNet2D(in 1, out 4, 32 channels) inference on the MI355X kernels.

    ``forward(x)`` takes the normalised, transposed image [H, W] (as the
    reference feeds the model) on the device and returns (logits [4, H, W]
    or None, labels [H, W] uint8).  H and W must be multiples of 16."""

    def __init__(self, state_dict: Dict[str, torch.Tensor], device="cuda"):
        self.device = torch.device(device)
        sd = {k: v.detach().to("cpu", torch.float32) for k, v in state_dict.items()}
        self.conv: Dict[str, Tuple[torch.Tensor, torch.Tensor]] = {}
        for k, w in sd.items():
            if not k.endswith(".weight") or w.dim() != 4:
                continue
            name = k[:-len(".weight")]
            co, ci, kh, kw = w.shape
            packed = w.permute(1, 2, 3, 0).reshape(ci, kh * kw, co).contiguous()  # [Cin][tap][Cout]
            self.conv[name] = (packed.to(self.device), sd[name + ".bias"].contiguous().to(self.device))
        self.bn: Dict[str, Tuple[torch.Tensor, torch.Tensor]] = {}
        for blk in _DOWN:
            g, b = sd[blk + ".bn.weight"], sd[blk + ".bn.bias"]
            m, v = sd[blk + ".bn.running_mean"], sd[blk + ".bn.running_var"]
            invstd = 1.0 / torch.sqrt(v + BN_EPS)    # ATen's eval batch norm: x * alpha + beta
            scale = invstd * g
            shift = b - m * scale
            self.bn[blk] = (scale.contiguous().to(self.device), shift.contiguous().to(self.device))
        self._e = torch.empty(0, device=self.device)

    @classmethod
    def from_checkpoint(cls, path: str, device="cuda") -> "RITnet":
        return cls(torch.load(path, map_location="cpu", weights_only=True), device)

    def _conv(self, name, k, ins, up, out_hw, lrelu, bn=None):
        w, b = self.conv[name]
        out = torch.empty((32,) + tuple(out_hw), device=self.device)
        sc, sh = bn if bn is not None else (self._e, self._e)
        _C.ritnet_conv(k, list(ins), list(up), w, b, bool(lrelu), sc, sh, out)
        return out

    def _down(self, blk, x, pool):
        if pool:
            x = _C.avgpool2(x)
        hw = x.shape[1:]
        x1 = self._conv(blk + ".conv1", 3, [x], [0], hw, True)
        t = self._conv(blk + ".conv21", 1, [x, x1], [0, 0], hw, False)
        x22 = self._conv(blk + ".conv22", 3, [t], [0], hw, True)
        t = self._conv(blk + ".conv31", 1, [x, x1, x22], [0, 0, 0], hw, False)
        return self._conv(blk + ".conv32", 3, [t], [0], hw, True, self.bn[blk])

    def _up(self, blk, skip, x):
        hw = skip.shape[1:]  # x is at half resolution, read through the nearest 2x upsampling
        t = self._conv(blk + ".conv11", 1, [x, skip], [1, 0], hw, False)
        x1 = self._conv(blk + ".conv12", 3, [t], [0], hw, True)
        t = self._conv(blk + ".conv21", 1, [x, skip, x1], [1, 0, 0], hw, False)
        return self._conv(blk + ".conv22", 3, [t], [0], hw, True)

    @torch.no_grad()
    def forward(self, x: torch.Tensor, want_logits: bool = False):
        if x.dim() != 2 or x.shape[0] % 16 or x.shape[1] % 16:
            raise ValueError("RITnet input must be [H, W] with H, W multiples of 16")
        x = x.to(self.device, torch.float32).contiguous().unsqueeze(0)
        x1 = self._down("down_block1", x, False)
        x2 = self._down("down_block2", x1, True)
        x3 = self._down("down_block3", x2, True)
        x4 = self._down("down_block4", x3, True)
        x5 = self._down("down_block5", x4, True)
        x6 = self._up("up_block1", x4, x5)
        x7 = self._up("up_block2", x3, x6)
        x8 = self._up("up_block3", x2, x7)
        x9 = self._up("up_block4", x1, x8)
        w, b = self.conv["out_conv1"]
        logits, labels = _C.ritnet_head(x9, w.reshape(32, 4), b, bool(want_logits))
        return (logits if want_logits else None), labels

    __call__ = forward


# ------------------------------------------------------------- pupil -> fovea ---
def pupil_centroid(labels: torch.Tensor, label: int = PUPIL) -> Optional[Tuple[float, float]]:
    """Centroid (column, row) of the pixels labelled `label` (None if none)."""
    m = _C.label_moments(labels.contiguous(), int(label)).cpu().numpy()
    if m[2] == 0:
        return None
    return float(m[0] / m[2]), float(m[1] / m[2])


def fovea_center(pupil_xy: Tuple[float, float], eye_size: Tuple[int, int], screen_size: Tuple[int, int]):
    """Pupil position in the eye image (x, y of an eye_size = (width, height)
    image) -> the fovea centre on a (width, height) render (SURVEY §8(d)
    config 3: (361.74, 248.19) / (640, 400) -> (1085.2, 670.1) at 1080p)."""
    return (pupil_xy[0] / eye_size[0] * screen_size[0], pupil_xy[1] / eye_size[1] * screen_size[1])


def track(model: RITnet, gray: np.ndarray, screen_size: Tuple[int, int]):
    """One frame of the front end: 8-bit eye image [h, w] -> (labels in the
    eye image's orientation [h, w], pupil (x, y), fovea centre on the screen)."""
    g = torch.from_numpy(np.ascontiguousarray(gray, np.uint8)).to(model.device, non_blocking=True)
    x = preprocess_device(g)
    _, labels_t = model(x)            # transposed image in, transposed labels out
    labels = labels_t.t().contiguous()
    pxy = pupil_centroid(labels)
    h, w = gray.shape
    fovea = fovea_center(pxy, (w, h), screen_size) if pxy is not None else None
    return labels, pxy, fovea
