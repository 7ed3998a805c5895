"""The training iteration around the rasterizer.

Mirrors train.py:67-125 and the GaussianModel optimisation state of
scene/gaussian_model.py:149-407, laid out for one MI355X:

* the six raw parameter groups (xyz, f_dc, f_rest, opacity, scaling,
  rotation -- :45-60) live in ONE flat f32 buffer, group after group, and so
  do their gradients and the two Adam moments.  The nn.Parameters the
  rasterizer's autograd sees are views of it, their ``.grad`` views of the
  gradient buffer, so the backward writes straight into the buffer that the
  data-parallel all-reduce (data_parallel.allreduce_) and the fused Adam
  kernel (csrc/train.hip) read;
* torch.optim.Adam (:163, betas (0.9, 0.999), eps 1e-15, per-group learning
  rates :154-161, the xyz exponential schedule :164-175) is one HIP launch
  over all groups, with per-group step counts so a group whose tensor was
  just replaced (densification, opacity reset) is skipped exactly as torch
  skips a parameter whose .grad is None;
* the densification statistics (train.py:111-113) are one HIP launch;
* the loss is the fused L1 + D-SSIM kernel (losses.py, csrc/loss.hip);
* densify_and_prune / reset_opacity (:210-404) are rare (every 100 / 3000
  iterations) index-heavy reshapes: torch gather/cat on the device, after
  which the flat buffers are rebuilt at the new size.  Their order of
  operations, the random split samples (torch.normal with the reference's
  shapes and call order) and the reference's quirks (max_radii2D is zeroed by
  densification_postfix before the prune reads it) are kept.

There is no CPU fallback: the Adam and statistics steps call the HIP
extension, which must be built and loaded.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist
from torch import nn

from . import _C
from .losses import l1_ssim_loss_terms
from .rasterization import GaussianRasterizationSettings, GaussianRasterizer

GROUPS: Tuple[str, ...] = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
BETAS = (0.9, 0.999)
EPS = 1e-15


@dataclass
class OptimizationParams:
    """arguments/__init__.py:71-89 defaults."""
    iterations: int = 30_000
    position_lr_init: float = 0.00016
    position_lr_final: float = 0.0000016
    position_lr_delay_mult: float = 0.01
    position_lr_max_steps: int = 30_000
    feature_lr: float = 0.0025
    opacity_lr: float = 0.05
    scaling_lr: float = 0.005
    rotation_lr: float = 0.001
    percent_dense: float = 0.01
    lambda_dssim: float = 0.2
    densification_interval: int = 100
    opacity_reset_interval: int = 3000
    densify_from_iter: int = 500
    densify_until_iter: int = 15_000
    densify_grad_threshold: float = 0.0002


def get_expon_lr_func(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """utils/general_utils.py:29-62: log-linear decay with optional delay."""

    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
        else:
            delay_rate = 1.0
        t = np.clip(step / max_steps, 0, 1)
        return delay_rate * np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)

    return helper


def inverse_sigmoid(x: torch.Tensor) -> torch.Tensor:
    """utils/general_utils.py:18-19."""
    return torch.log(x / (1 - x))


def build_rotation(r: torch.Tensor) -> torch.Tensor:
    """utils/general_utils.py:78-99: rotation matrices of the normalised quaternions (w, x, y, z)."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], dim=1)
    return R.view(-1, 3, 3)


def group_row_shape(name: str, sh_degree: int) -> Tuple[int, ...]:
    """Per-Gaussian shape of each raw group (scene/gaussian_model.py:45-60)."""
    return {"xyz": (3,), "f_dc": (1, 3), "f_rest": ((sh_degree + 1) ** 2 - 1, 3), "opacity": (1,),
            "scaling": (3,), "rotation": (4,)}[name]


class FlatGaussianModel:
    """GaussianModel's optimisation state (scene/gaussian_model.py:43-175) in
    flat HBM buffers: `params`, `grads`, `exp_avg`, `exp_avg_sq` ([n] f32,
    groups in GROUPS order), nn.Parameter views per group, densification
    statistics, per-group learning rates and Adam step counts."""

    def __init__(self, raw: Dict[str, torch.Tensor], sh_degree: int, spatial_lr_scale: float,
                 opt: Optional[OptimizationParams] = None, device=None):
        self.max_sh_degree = sh_degree
        self.active_sh_degree = 0
        self.spatial_lr_scale = float(spatial_lr_scale)
        self.opt = opt or OptimizationParams()
        self.percent_dense = self.opt.percent_dense
        dev = torch.device(device) if device is not None else raw["xyz"].device
        self.device = dev
        o = self.opt
        # training_setup (:149-167)
        self.lr: Dict[str, float] = {
            "xyz": o.position_lr_init * self.spatial_lr_scale, "f_dc": o.feature_lr, "f_rest": o.feature_lr / 20.0,
            "opacity": o.opacity_lr, "scaling": o.scaling_lr, "rotation": o.rotation_lr}
        self.xyz_scheduler_args = get_expon_lr_func(
            lr_init=o.position_lr_init * self.spatial_lr_scale, lr_final=o.position_lr_final * self.spatial_lr_scale,
            lr_delay_mult=o.position_lr_delay_mult, max_steps=o.position_lr_max_steps)
        self.steps: Dict[str, int] = {g: 0 for g in GROUPS}
        self._layout(int(raw["xyz"].shape[0]), {g: raw[g].to(dev, torch.float32) for g in GROUPS}, moments=None)

    # ------------------------------------------------------------ layout ---
    def _layout(self, P: int, values: Dict[str, torch.Tensor],
                moments: Optional[Tuple[Dict[str, torch.Tensor], Dict[str, torch.Tensor]]]) -> None:
        """(Re)build the flat buffers at size P from per-group tensors."""
        self.P = P
        sizes = [P * int(np.prod(group_row_shape(g, self.max_sh_degree))) for g in GROUPS]
        self.seg_end: List[int] = list(np.cumsum(sizes).astype(np.int64).tolist())
        n = self.seg_end[-1] if P > 0 else 0
        dev = self.device
        self.params = torch.empty(n, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.param: Dict[str, nn.Parameter] = {}
        self._gview: Dict[str, torch.Tensor] = {}
        off = 0
        for g, end in zip(GROUPS, self.seg_end if P > 0 else [0] * len(GROUPS)):
            shape = (P,) + group_row_shape(g, self.max_sh_degree)
            pv = self.params[off:end].view(shape)
            pv.copy_(values[g].reshape(shape))
            if moments is not None:
                self.exp_avg[off:end].view(shape).copy_(moments[0][g].reshape(shape))
                self.exp_avg_sq[off:end].view(shape).copy_(moments[1][g].reshape(shape))
            p = nn.Parameter(torch.empty(0, device=dev))
            p.data = pv
            self.param[g] = p
            self._gview[g] = self.grads[off:end].view(shape)
            off = end
        M = (self.max_sh_degree + 1) ** 2
        self._act = {"shs": torch.empty((P, M, 3), device=dev), "opacities": torch.empty((P, 1), device=dev),
                     "scales": torch.empty((P, 3), device=dev), "rotations": torch.empty((P, 4), device=dev)}
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros((P,), device=dev)
        self.has_grad: Dict[str, bool] = {g: False for g in GROUPS}
        self.zero_grad()

    def group_view(self, buf: torch.Tensor, g: str) -> torch.Tensor:
        i = GROUPS.index(g)
        lo = self.seg_end[i - 1] if i > 0 else 0
        return buf[lo:self.seg_end[i]].view((self.P,) + group_row_shape(g, self.max_sh_degree))

    # ----------------------------------------------------------- getters ---
    @property
    def get_xyz(self):
        return self.param["xyz"]

    @property
    def get_scaling(self):
        return torch.exp(self.param["scaling"])

    @property
    def get_rotation(self):
        return torch.nn.functional.normalize(self.param["rotation"])

    @property
    def get_opacity(self):
        return torch.sigmoid(self.param["opacity"])

    @property
    def get_features(self):
        return torch.cat((self.param["f_dc"], self.param["f_rest"]), dim=1)

    def oneupSHdegree(self):
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    def update_learning_rate(self, iteration: int) -> float:
        """:169-175 (xyz only)."""
        self.lr["xyz"] = float(self.xyz_scheduler_args(iteration))
        return self.lr["xyz"]

    # --------------------------------------------------------- optimiser ---
    def zero_grad(self, memset: bool = True) -> None:
        """optimizer.zero_grad(set_to_none=True): the buffer is zeroed and
        re-attached (autograd accumulates into an existing .grad in place).
        memset=False defers the zeroing: the fused backward overwrites every
        gradient, and the paths that accumulate zero a stale buffer first."""
        if memset:
            self.grads.zero_()
        self._grads_stale = not memset
        for g in GROUPS:
            self.param[g].grad = self._gview[g]
            self.has_grad[g] = False

    def _fresh_grads(self) -> None:
        if self._grads_stale:
            self.grads.zero_()
            self._grads_stale = False

    def mark_backward(self) -> None:
        """Every group reaches the loss through the renderer, so after a
        backward every parameter has a gradient."""
        for g in GROUPS:
            self.has_grad[g] = True

    def optimizer_step(self) -> None:
        """torch.optim.Adam.step() over the groups that have a gradient."""
        if self.P == 0:
            return
        steps = []
        for g in GROUPS:
            if self.has_grad[g]:
                self.steps[g] += 1
                steps.append(self.steps[g])
            else:
                steps.append(0)
        _C.adam_step(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.seg_end,
                     [float(self.lr[g]) for g in GROUPS], steps, BETAS[0], BETAS[1], EPS)

    # ------------------------------------------------------ densification ---
    def add_densification_stats(self, grad_means2D: torch.Tensor, radii: torch.Tensor) -> None:
        """train.py:111-113 + :405-407 for the visible (radii > 0) Gaussians."""
        _C.densify_stats(radii.contiguous(), grad_means2D, self.xyz_gradient_accum, self.denom, self.max_radii2D)

    def _raw(self) -> Dict[str, torch.Tensor]:
        return {g: self.param[g].detach() for g in GROUPS}

    def _moments(self):
        return ({g: self.group_view(self.exp_avg, g) for g in GROUPS},
                {g: self.group_view(self.exp_avg_sq, g) for g in GROUPS})

    def _rebuild(self, values, m1, m2) -> None:
        steps = dict(self.steps)
        P = int(values["xyz"].shape[0])
        self._layout(P, values, (m1, m2))
        self.steps = steps  # Adam's per-parameter step survives the tensor swaps (:262-268, :314-318)

    def _postfix(self, state, new: Dict[str, torch.Tensor]):
        """densification_postfix (:329-347) on the (values, m1, m2) triple."""
        values, m1, m2 = state
        values = {g: torch.cat((values[g], new[g]), dim=0) for g in GROUPS}
        m1 = {g: torch.cat((m1[g], torch.zeros_like(new[g])), dim=0) for g in GROUPS}
        m2 = {g: torch.cat((m2[g], torch.zeros_like(new[g])), dim=0) for g in GROUPS}
        return values, m1, m2

    @staticmethod
    def _prune(state, valid: torch.Tensor):
        values, m1, m2 = state
        return ({g: values[g][valid] for g in GROUPS}, {g: m1[g][valid] for g in GROUPS},
                {g: m2[g][valid] for g in GROUPS})

    def densify_and_prune(self, max_grad: float, min_opacity: float, extent: float,
                          max_screen_size: Optional[float]) -> None:
        """:389-403 (densify_and_clone :374-387, densify_and_split :349-372,
        prune_points :291-305), then one rebuild of the flat buffers."""
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        m1, m2 = self._moments()
        state = ({g: v.clone() for g, v in self._raw().items()}, {g: v.clone() for g, v in m1.items()},
                 {g: v.clone() for g, v in m2.items()})
        pd = self.percent_dense * extent
        # clone
        scaling = torch.exp(state[0]["scaling"])
        sel = torch.where(torch.norm(grads, dim=-1) >= max_grad, True, False)
        sel = torch.logical_and(sel, torch.max(scaling, dim=1).values <= pd)
        state = self._postfix(state, {g: state[0][g][sel] for g in GROUPS})
        # split (N = 2)
        N = 2
        values = state[0]
        n_init = values["xyz"].shape[0]
        padded = torch.zeros((n_init,), device=self.device)
        padded[:grads.shape[0]] = grads.squeeze()
        sel = torch.where(padded >= max_grad, True, False)
        scaling = torch.exp(values["scaling"])
        sel = torch.logical_and(sel, torch.max(scaling, dim=1).values > pd)
        stds = scaling[sel].repeat(N, 1)
        samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device=self.device), std=stds)
        rots = build_rotation(values["rotation"][sel]).repeat(N, 1, 1)
        new = {
            "xyz": torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + values["xyz"][sel].repeat(N, 1),
            "scaling": torch.log(scaling[sel].repeat(N, 1) / (0.8 * N)),
            "rotation": values["rotation"][sel].repeat(N, 1),
            "f_dc": values["f_dc"][sel].repeat(N, 1, 1),
            "f_rest": values["f_rest"][sel].repeat(N, 1, 1),
            "opacity": values["opacity"][sel].repeat(N, 1)}
        state = self._postfix(state, new)
        prune_filter = torch.cat((sel, torch.zeros(N * int(sel.sum()), device=self.device, dtype=torch.bool)))
        state = self._prune(state, ~prune_filter)
        # prune (max_radii2D was zeroed by densification_postfix, as in the reference)
        values = state[0]
        prune_mask = (torch.sigmoid(values["opacity"]) < min_opacity).squeeze()
        if max_screen_size:
            big_vs = torch.zeros((values["xyz"].shape[0],), device=self.device) > max_screen_size
            big_ws = torch.exp(values["scaling"]).max(dim=1).values > 0.1 * extent
            prune_mask = torch.logical_or(torch.logical_or(prune_mask, big_vs), big_ws)
        state = self._prune(state, ~prune_mask)
        self._rebuild(*state)
        for g in GROUPS:  # fresh nn.Parameters: no .grad until the next backward
            self.has_grad[g] = False

    def reset_opacity(self) -> None:
        """:210-213 with replace_tensor_to_optimizer (:258-271): opacity
        clamped to <= 0.01, its Adam moments zeroed, no gradient this step."""
        op = self.group_view(self.params, "opacity")
        op.copy_(inverse_sigmoid(torch.min(torch.sigmoid(op), torch.ones_like(op) * 0.01)))
        self.group_view(self.exp_avg, "opacity").zero_()
        self.group_view(self.exp_avg_sq, "opacity").zero_()
        self.has_grad["opacity"] = False

    # -------------------------------------------------------- rendering ---
    def render(self, settings: GaussianRasterizationSettings):
        """gaussian_renderer/__init__.py:18-114 (default pipe: SH and the 3D
        covariance evaluated by the rasterizer)."""
        self._fresh_grads()
        screenspace_points = torch.zeros_like(self.param["xyz"], requires_grad=True) + 0
        screenspace_points.retain_grad()
        s = settings._replace(sh_degree=self.active_sh_degree)
        image, radii = GaussianRasterizer(s)(
            means3D=self.get_xyz, means2D=screenspace_points, shs=self.get_features, opacities=self.get_opacity,
            scales=self.get_scaling, rotations=self.get_rotation)
        return {"render": image, "viewspace_points": screenspace_points, "visibility_filter": radii > 0,
                "radii": radii}


    def render_and_backward(self, settings: GaussianRasterizationSettings, gt_image: torch.Tensor,
                            lambda_dssim: float, accumulate: bool = False):
        """render -> L1 + D-SSIM -> backward without autograd: the activation
        kernel fills the rasterizer inputs from the raw segments, the fused
        loss kernel hands dL/dimage straight to the rasterizer backward, and
        the activation backward writes the raw-parameter gradients into the
        flat gradient buffer (gaussian_renderer/__init__.py:18-114 +
        train.py:89-93 + loss.backward()).  Same results as render() +
        l1_ssim_loss + autograd (tests/test_gpu_training.py)."""
        if accumulate:
            self._fresh_grads()
        s = settings._replace(sh_degree=self.active_sh_degree)
        raw = {g: self.group_view(self.params, g) for g in GROUPS}
        a = self._act
        _C.activate(raw["f_dc"], raw["f_rest"], raw["opacity"], raw["scaling"], raw["rotation"], a["shs"],
                    a["opacities"], a["scales"], a["rotations"])
        e = torch.empty(0, device=self.device)
        xyz = raw["xyz"]
        num_rendered, color, radii, geom, binning, img = _C.rasterize_gaussians(
            s.bg, xyz, e, a["opacities"], a["scales"], a["rotations"], s.scale_modifier, e, s.viewmatrix,
            s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, a["shs"], s.sh_degree, s.campos,
            s.prefiltered, s.debug)
        out3, d_image = _C.l1_ssim_loss(color, gt_image, float(lambda_dssim))
        (d_means2D, _d_colors, d_opac, d_means3D, _d_cov3D, d_shs, d_scales, d_rot) = _C.rasterize_gaussians_backward_lean(
            s.bg, xyz, radii, e, a["scales"], a["rotations"], s.scale_modifier, e, s.viewmatrix, s.projmatrix,
            s.tanfovx, s.tanfovy, d_image, a["shs"], s.sh_degree, s.campos, geom, num_rendered, binning, img,
            s.debug)
        gv = {g: self.group_view(self.grads, g) for g in GROUPS}
        _C.activation_backward(d_shs, d_opac, d_scales, d_rot, d_means3D, raw["opacity"], raw["scaling"],
                               raw["rotation"], gv["xyz"], gv["f_dc"], gv["f_rest"], gv["opacity"], gv["scaling"],
                               gv["rotation"], bool(accumulate))
        self._grads_stale = False
        self.mark_backward()
        pkg = {"render": color, "viewspace_grad": d_means2D, "visibility_filter": radii > 0, "radii": radii}
        return pkg, {"loss": out3[0], "l1": out3[1], "ssim": out3[2]}


def render_and_backward_views(model: FlatGaussianModel, settings: GaussianRasterizationSettings,
                              gt_image: torch.Tensor, lambda_dssim: float, stats: bool, group=None):
    """The data-parallel fused iteration with the "views" exchange
    (data_parallel.py): activate -> forward -> fused loss -> blend backward
    of this rank's view -> all-gather of the view records -> multi-view
    parameter backward (the sum over all ranks' views, identical on every
    rank) -> activation backward into the flat gradient buffer.  With stats
    the densification statistics of every rank's view are accumulated too
    (train.py:111-113), so no statistics all-reduce is needed afterwards."""
    from . import data_parallel as DP
    s = settings._replace(sh_degree=model.active_sh_degree)
    raw = {g: model.group_view(model.params, g) for g in GROUPS}
    a = model._act
    _C.activate(raw["f_dc"], raw["f_rest"], raw["opacity"], raw["scaling"], raw["rotation"], a["shs"],
                a["opacities"], a["scales"], a["rotations"])
    e = torch.empty(0, device=model.device)
    xyz = raw["xyz"]
    fwd = _C.rasterize_gaussians(
        s.bg, xyz, e, a["opacities"], a["scales"], a["rotations"], s.scale_modifier, e, s.viewmatrix,
        s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, a["shs"], s.sh_degree, s.campos,
        s.prefiltered, s.debug)
    num_rendered, color, radii, geom, binning, img = fwd
    out3, d_image = _C.l1_ssim_loss(color, gt_image, float(lambda_dssim))
    st = (model.xyz_gradient_accum, model.denom, model.max_radii2D) if stats else None
    d_means3D, d_shs, d_opac, d_scales, d_rot = DP.exchange_view_grads(
        s, fwd, d_image, xyz, a["shs"], a["scales"], a["rotations"], group=group, stats=st)
    gv = {g: model.group_view(model.grads, g) for g in GROUPS}
    _C.activation_backward(d_shs, d_opac, d_scales, d_rot, d_means3D, raw["opacity"], raw["scaling"],
                           raw["rotation"], gv["xyz"], gv["f_dc"], gv["f_rest"], gv["opacity"], gv["scaling"],
                           gv["rotation"], False)
    model._grads_stale = False
    model.mark_backward()
    pkg = {"render": color, "viewspace_grad": None, "visibility_filter": radii > 0, "radii": radii,
           "stats_done": stats}
    return pkg, {"loss": out3[0], "l1": out3[1], "ssim": out3[2]}


def _world(group=None) -> int:
    return dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1


def allreduce_training_grads(model: FlatGaussianModel, group=None) -> None:
    """the one data-path exchange -- the flat gradient buffer,
    summed over the ranks' views with one RCCL all-reduce."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(model.grads, op=dist.ReduceOp.SUM, group=group)


def reduce_densification_stats(model: FlatGaussianModel, group=None) -> None:
    """Before densify_and_prune: every rank accumulated the statistics of its
    own views; sums (accum, denom) and the max (radii) make them the
    statistics of all views, identical on every rank."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(model.xyz_gradient_accum, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(model.denom, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(model.max_radii2D, op=dist.ReduceOp.MAX, group=group)


def forward_backward(model: FlatGaussianModel, iteration: int, settings: GaussianRasterizationSettings,
                     gt_image: torch.Tensor, group=None, fused: bool = True, exchange: str = "views"):
    """train.py:76-93 + the backward: learning-rate schedule, SH degree step,
    render, fused L1 + D-SSIM loss, backward into the flat gradient buffer,
    all-reduce over the data-parallel ranks.  fused=True runs the
    autograd-free native sequence (render_and_backward); fused=False the
    reference-shaped one (torch activations + the drop-in autograd
    rasterizer + autograd).  Returns (render package, loss terms as device
    tensors); pkg["viewspace_grad"] is dL/dmeans2D.  With more than one rank
    and exchange="views" (fused only) the ranks exchange view records instead
    of all-reducing the gradients (data_parallel.py)."""
    model.update_learning_rate(iteration)
    if iteration % 1000 == 0:
        model.oneupSHdegree()
    if fused and exchange == "views" and _world(group) > 1:
        return render_and_backward_views(model, settings, gt_image, model.opt.lambda_dssim,
                                         stats=iteration < model.opt.densify_until_iter, group=group)
    if fused:
        pkg, terms = model.render_and_backward(settings, gt_image, model.opt.lambda_dssim)
    else:
        pkg = model.render(settings)
        loss, l1, ssim = l1_ssim_loss_terms(pkg["render"], gt_image, model.opt.lambda_dssim)
        loss.backward()
        model.mark_backward()
        pkg["viewspace_grad"] = pkg["viewspace_points"].grad
        terms = {"loss": loss.detach(), "l1": l1, "ssim": ssim}
    allreduce_training_grads(model, group)
    return pkg, terms


@torch.no_grad()
def post_backward(model: FlatGaussianModel, iteration: int, pkg, scene_extent: float, white_background: bool = False,
                  group=None, fused: bool = False) -> None:
    """train.py:108-125: densification statistics, densify / prune / opacity
    reset on the reference's schedule, Adam, zero_grad."""
    o = model.opt
    views_stats = pkg.get("stats_done", False)  # every view's statistics already accumulated on every rank
    if iteration < o.densify_until_iter:
        if not views_stats:
            model.add_densification_stats(pkg["viewspace_grad"], pkg["radii"])
        if iteration > o.densify_from_iter and iteration % o.densification_interval == 0:
            if not views_stats:
                reduce_densification_stats(model, group)
            size_threshold = 20 if iteration > o.opacity_reset_interval else None
            model.densify_and_prune(o.densify_grad_threshold, 0.005, scene_extent, size_threshold)
        if iteration % o.opacity_reset_interval == 0 or (white_background and iteration == o.densify_from_iter):
            model.reset_opacity()
    if iteration < o.iterations:
        model.optimizer_step()
        model.zero_grad(memset=not fused)


def training_iteration(model: FlatGaussianModel, iteration: int, settings: GaussianRasterizationSettings,
                       gt_image: torch.Tensor, scene_extent: float, white_background: bool = False,
                       group=None, fused: bool = True, exchange: str = "views") -> Dict[str, torch.Tensor]:
    """One iteration of train.py:67-125 (minus logging / saving / the GUI).
    Returns the loss terms as device tensors (no host sync)."""
    pkg, terms = forward_backward(model, iteration, settings, gt_image, group, fused, exchange)
    post_backward(model, iteration, pkg, scene_extent, white_background, group, fused)
    return terms
