#!/usr/bin/env python3
"""One training iteration of train.py:67-125 on one GPU (training.py), timed
whole and per phase, next to the same iteration with the reference's PyTorch
pieces swapped back in (torch.optim.Adam over six nn.Parameters, the
loss_utils conv2d SSIM, the gather/norm/scatter statistics).

Workload: config 2 (1M Gaussians, 1920x1080, SH degree 3), synthetic scene
and a random target image; iterations 101.. (statistics on, no densification
-- densify_from_iter is 500).  Fused Adam algorithmic bytes: 28 B per
parameter (p, g, m, v read; p, m, v written), 59 parameters per Gaussian.
"""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gaussian_splatting_with_eye_tracking_amd import ply, synthetic as S, training as T  # noqa: E402
from gaussian_splatting_with_eye_tracking_amd.rasterization import GaussianRasterizationSettings  # noqa: E402
from bench_loss import torch_reference_loss  # noqa: E402


def timed(fn, reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = "cuda"
    cam = S.make_camera(args.W, args.H)
    sc = S.make_scene(args.P, cam, seed=0)
    g = ply.from_activated(sc.means3D, sc.opacities, sc.scales, sc.rotations, sc.shs)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    raw = {"xyz": t(g.xyz), "f_dc": t(g.features_dc), "f_rest": t(g.features_rest), "opacity": t(g.opacity),
           "scaling": t(g.scaling), "rotation": t(g.rotation)}
    st = GaussianRasterizationSettings(
        image_height=args.H, image_width=args.W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.zeros(3, device=dev), scale_modifier=1.0,
        viewmatrix=torch.from_numpy(cam.world_view_transform).to(dev),
        projmatrix=torch.from_numpy(cam.full_proj_transform).to(dev), sh_degree=3,
        campos=torch.from_numpy(cam.camera_center).to(dev), prefiltered=False, debug=False)
    gt = torch.rand(3, args.H, args.W, device=dev, generator=torch.Generator(dev).manual_seed(0))
    m = T.FlatGaussianModel(raw, 3, spatial_lr_scale=5.0)
    m.active_sh_degree = 3
    it = [100]

    def iteration():
        it[0] += 1
        T.training_iteration(m, it[0], st, gt, scene_extent=5.0)

    for _ in range(3):
        iteration()
    t_iter = timed(iteration, args.reps)

    # the reference-shaped sequence: torch activations + drop-in autograd rasterizer + autograd
    def iteration_autograd():
        it[0] += 1
        T.training_iteration(m, it[0], st, gt, scene_extent=5.0, fused=False)

    for _ in range(2):
        iteration_autograd()
    t_iter_autograd = timed(iteration_autograd, args.reps)

    # phases of the fused sequence
    def phases():
        it[0] += 1
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record()
        m.update_learning_rate(it[0])
        pkg, _ = m.render_and_backward(st, gt, 0.2)
        e[1].record()
        with torch.no_grad():
            m.add_densification_stats(pkg["viewspace_grad"], pkg["radii"])
            e[2].record()
            m.optimizer_step()
            m.zero_grad(memset=False)
        e[3].record()
        return e

    for _ in range(2):
        phases()
    acc = np.zeros(3)
    for _ in range(args.reps):
        e = phases()
        torch.cuda.synchronize()
        acc += [e[i].elapsed_time(e[i + 1]) for i in range(3)]
    acc /= args.reps
    names = ["activate+render+loss+backward", "densify_stats", "adam+zero_grad"]

    # the reference's pieces on the same GPU
    o_params = {k: torch.nn.Parameter(m.param[k].detach().clone()) for k in T.GROUPS}
    opt = torch.optim.Adam([{"params": [o_params[k]], "lr": m.lr[k], "name": k} for k in T.GROUPS], lr=0.0,
                           eps=1e-15)
    for k in T.GROUPS:
        o_params[k].grad = torch.randn_like(o_params[k])

    def torch_adam():
        opt.step()

    torch_adam()
    t_torch_adam = timed(torch_adam, args.reps)
    n = m.params.numel()

    def fused_adam():
        m.mark_backward()
        m.optimizer_step()

    fused_adam()
    t_fused_adam = timed(fused_adam, args.reps)

    radii = torch.randint(0, 10, (args.P,), device=dev, dtype=torch.int32)
    g2d = torch.randn(args.P, 3, device=dev)
    mr, acc_, den = torch.zeros(args.P, device=dev), torch.zeros(args.P, 1, device=dev), torch.zeros(args.P, 1,
                                                                                                      device=dev)

    def torch_stats():
        vis = radii > 0
        mr[vis] = torch.max(mr[vis], radii[vis])
        acc_[vis] += torch.norm(g2d[vis, :2], dim=-1, keepdim=True)
        den[vis] += 1

    torch_stats()
    t_torch_stats = timed(torch_stats, args.reps)
    t_fused_stats = timed(lambda: m.add_densification_stats(g2d, radii), args.reps)

    x = torch.rand(3, args.H, args.W, device=dev, requires_grad=True)

    def torch_loss():
        x.grad = None
        torch_reference_loss(x, gt).backward()

    torch_loss()
    t_torch_loss = timed(torch_loss, args.reps)

    out = {
        "workload": f"training iteration (train.py:67-125), {args.P} Gaussians, {args.W}x{args.H}, SH3, "
                    "no densify step; fused native sequence (autograd-path time alongside)", "iteration_ms": round(t_iter, 4),
        "iterations_per_s": round(1000.0 / t_iter, 1),
        "iteration_ms_autograd_path": round(t_iter_autograd, 4),
        "phases_ms": {k: round(float(v), 4) for k, v in zip(names, acc)},
        "adam": {"fused_ms": round(t_fused_adam, 4), "torch_optim_adam_ms": round(t_torch_adam, 4),
                 "speedup": round(t_torch_adam / t_fused_adam, 2), "params": n,
                 "fused_algorithmic_GBps": round(28.0 * n / (t_fused_adam * 1e-3) / 1e9, 1)},
        "densify_stats": {"fused_ms": round(t_fused_stats, 4), "torch_ms": round(t_torch_stats, 4),
                          "speedup": round(t_torch_stats / t_fused_stats, 2)},
        "loss": {"torch_eager_ms": round(t_torch_loss, 4)},
        "num_points": m.P,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
