"""CPU ORACLE (test infrastructure only): the optimisation state of the
reference's GaussianModel restated with what the reference itself uses --
one nn.Parameter per group and torch.optim.Adam -- device-agnostic (the
reference hard-codes device="cuda").

Follows scene/gaussian_model.py:
  training_setup           :149-167  (param groups, lrs, Adam(lr=0, eps=1e-15))
  update_learning_rate     :169-175
  reset_opacity            :210-213, replace_tensor_to_optimizer :258-271
  _prune_optimizer         :273-289, prune_points :291-305
  cat_tensors_to_optimizer :307-327, densification_postfix :329-347
  densify_and_split        :349-372, densify_and_clone :374-387
  densify_and_prune        :389-403, add_densification_stats :405-407
and train.py:108-125 for the order of the post-backward phase.  The tests
compare gaussian_splatting_with_eye_tracking_amd.training.FlatGaussianModel
against this on identical states (same seeds for the split samples).
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn

NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")


def expon_lr(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """utils/general_utils.py:29-62."""

    def f(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        d = 1.0
        if lr_delay_steps > 0:
            d = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
        t = np.clip(step / max_steps, 0, 1)
        return d * np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)

    return f


def rotation_matrices(r):
    """utils/general_utils.py:78-99."""
    n = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / n[:, None]
    R = torch.zeros((q.size(0), 3, 3), device=r.device)
    a, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - a * z)
    R[:, 0, 2] = 2 * (x * z + a * y)
    R[:, 1, 0] = 2 * (x * y + a * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - a * x)
    R[:, 2, 0] = 2 * (x * z - a * y)
    R[:, 2, 1] = 2 * (y * z + a * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


class OracleModel:
    def __init__(self, raw, spatial_lr_scale, opt, device):
        self.dev = torch.device(device)
        self.opt = opt
        self.percent_dense = opt.percent_dense
        self.p = {k: nn.Parameter(raw[k].detach().clone().to(self.dev).requires_grad_(True)) for k in NAMES}
        P = self.p["xyz"].shape[0]
        self.xyz_gradient_accum = torch.zeros((P, 1), device=self.dev)
        self.denom = torch.zeros((P, 1), device=self.dev)
        self.max_radii2D = torch.zeros((P,), device=self.dev)
        lrs = {"xyz": opt.position_lr_init * spatial_lr_scale, "f_dc": opt.feature_lr,
               "f_rest": opt.feature_lr / 20.0, "opacity": opt.opacity_lr, "scaling": opt.scaling_lr,
               "rotation": opt.rotation_lr}
        self.optimizer = torch.optim.Adam([{"params": [self.p[k]], "lr": lrs[k], "name": k} for k in NAMES],
                                          lr=0.0, eps=1e-15)
        self.sched = expon_lr(opt.position_lr_init * spatial_lr_scale, opt.position_lr_final * spatial_lr_scale,
                              lr_delay_mult=opt.position_lr_delay_mult, max_steps=opt.position_lr_max_steps)

    # -- state helpers
    def _swap(self, fn_param, fn_state):
        """Replace every group's parameter by fn_param(old) and its moments by
        fn_state(old moment, name) (the reference's three optimizer surgeries)."""
        for group in self.optimizer.param_groups:
            old = group["params"][0]
            name = group["name"]
            st = self.optimizer.state.get(old, None)
            new = nn.Parameter(fn_param(old, name).requires_grad_(True))
            if st is not None:
                st["exp_avg"] = fn_state(st["exp_avg"], name)
                st["exp_avg_sq"] = fn_state(st["exp_avg_sq"], name)
                del self.optimizer.state[old]
                self.optimizer.state[new] = st
            group["params"][0] = new
            self.p[name] = new

    def set_lr(self, iteration):
        for g in self.optimizer.param_groups:
            if g["name"] == "xyz":
                g["lr"] = self.sched(iteration)

    def scaling(self):
        return torch.exp(self.p["scaling"])

    def opacity(self):
        return torch.sigmoid(self.p["opacity"])

    def add_stats(self, grad_means2D, radii):
        vis = radii > 0
        self.max_radii2D[vis] = torch.max(self.max_radii2D[vis], radii[vis])
        self.xyz_gradient_accum[vis] += torch.norm(grad_means2D[vis, :2], dim=-1, keepdim=True)
        self.denom[vis] += 1

    def _postfix(self, new):
        self._swap(lambda old, k: torch.cat((old, new[k]), dim=0),
                   lambda s, k: torch.cat((s, torch.zeros_like(new[k])), dim=0))
        P = self.p["xyz"].shape[0]
        self.xyz_gradient_accum = torch.zeros((P, 1), device=self.dev)
        self.denom = torch.zeros((P, 1), device=self.dev)
        self.max_radii2D = torch.zeros((P,), device=self.dev)

    def prune(self, mask):
        keep = ~mask
        self._swap(lambda old, k: old[keep], lambda s, k: s[keep])
        self.xyz_gradient_accum = self.xyz_gradient_accum[keep]
        self.denom = self.denom[keep]
        self.max_radii2D = self.max_radii2D[keep]

    def densify_and_clone(self, grads, thr, extent):
        sel = torch.where(torch.norm(grads, dim=-1) >= thr, True, False)
        sel = torch.logical_and(sel, torch.max(self.scaling(), dim=1).values <= self.percent_dense * extent)
        self._postfix({k: self.p[k][sel] for k in NAMES})

    def densify_and_split(self, grads, thr, extent, N=2):
        n0 = self.p["xyz"].shape[0]
        padded = torch.zeros((n0,), device=self.dev)
        padded[:grads.shape[0]] = grads.squeeze()
        sel = torch.where(padded >= thr, True, False)
        sel = torch.logical_and(sel, torch.max(self.scaling(), dim=1).values > self.percent_dense * extent)
        stds = self.scaling()[sel].repeat(N, 1)
        samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device=self.dev), std=stds)
        rots = rotation_matrices(self.p["rotation"][sel]).repeat(N, 1, 1)
        new = {"xyz": torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + self.p["xyz"][sel].repeat(N, 1),
               "scaling": torch.log(self.scaling()[sel].repeat(N, 1) / (0.8 * N)),
               "rotation": self.p["rotation"][sel].repeat(N, 1),
               "f_dc": self.p["f_dc"][sel].repeat(N, 1, 1),
               "f_rest": self.p["f_rest"][sel].repeat(N, 1, 1),
               "opacity": self.p["opacity"][sel].repeat(N, 1)}
        self._postfix({k: v.detach() for k, v in new.items()})
        self.prune(torch.cat((sel, torch.zeros(N * sel.sum(), device=self.dev, dtype=bool))))

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size):
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        with torch.no_grad():
            self.densify_and_clone(grads, max_grad, extent)
            self.densify_and_split(grads, max_grad, extent)
            mask = (self.opacity() < min_opacity).squeeze()
            if max_screen_size:
                mask = torch.logical_or(torch.logical_or(mask, self.max_radii2D > max_screen_size),
                                        self.scaling().max(dim=1).values > 0.1 * extent)
            self.prune(mask)

    def reset_opacity(self):
        with torch.no_grad():
            o = self.opacity()
            new = torch.log(torch.min(o, torch.ones_like(o) * 0.01) / (1 - torch.min(o, torch.ones_like(o) * 0.01)))
        for group in self.optimizer.param_groups:
            if group["name"] != "opacity":
                continue
            old = group["params"][0]
            st = self.optimizer.state.get(old, None)
            st["exp_avg"] = torch.zeros_like(new)
            st["exp_avg_sq"] = torch.zeros_like(new)
            del self.optimizer.state[old]
            group["params"][0] = nn.Parameter(new.requires_grad_(True))
            self.optimizer.state[group["params"][0]] = st
            self.p["opacity"] = group["params"][0]

    def post_backward(self, iteration, grad_means2D, radii, extent, white_background=False):
        """train.py:108-125."""
        o = self.opt
        with torch.no_grad():
            if iteration < o.densify_until_iter:
                self.add_stats(grad_means2D, radii)
                if iteration > o.densify_from_iter and iteration % o.densification_interval == 0:
                    size_threshold = 20 if iteration > o.opacity_reset_interval else None
                    self.densify_and_prune(o.densify_grad_threshold, 0.005, extent, size_threshold)
                if iteration % o.opacity_reset_interval == 0 or (
                        white_background and iteration == o.densify_from_iter):
                    self.reset_opacity()
            if iteration < o.iterations:
                self.optimizer.step()
                self.optimizer.zero_grad(set_to_none=True)

    def moments(self, name):
        st = self.optimizer.state.get(self.p[name], None)
        if st is None:
            z = torch.zeros_like(self.p[name])
            return z, z, 0
        return st["exp_avg"], st["exp_avg_sq"], int(st["step"])
