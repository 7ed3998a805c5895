#!/usr/bin/env python3
"""Interleaved in-process A/B of kernel-geometry variants (guide §5.4 rule
24): N variants x R rounds in ONE process on one device, per-stage HIP-event
times from the library's profiler, median and min reported.

usage: python tools/ab_tuning.py --key fwd_variant --values 0 1 2 --stage render [--backward]
(--stage step: the whole call per run, events around the timed loop)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", default="fwd_variant")
    ap.add_argument("--values", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--stage", default="render")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--backward", action="store_true")
    ap.add_argument("--amr", action="store_true", help="time a 5-step foveated AMR frame instead")
    ap.add_argument("--amr-once", action="store_true", help="time AMR render_once (foveaStep -2, interpolated)")
    ap.add_argument("--per-step", action="store_true", help="--amr: also time each fovea step's apply (events)")
    ap.add_argument("--set", nargs="*", default=[], help="fixed tunings key=value applied before the A/B")
    args = ap.parse_args()

    from gaussian_splatting_with_eye_tracking_amd import _C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    for kv in args.set:
        k, v = kv.split("=")
        _C.set_tuning(k, int(v))
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    dev = torch.device("cuda:0")
    cam = S.make_camera(args.W, args.H)
    sc = S.make_scene(args.P, cam, seed=0)
    st = GaussianRasterizationSettings(
        image_height=args.H, image_width=args.W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.zeros(3, device=dev), scale_modifier=1.0,
        viewmatrix=torch.from_numpy(cam.world_view_transform).to(dev),
        projmatrix=torch.from_numpy(cam.full_proj_transform).to(dev), sh_degree=3,
        campos=torch.from_numpy(cam.camera_center).to(dev), prefiltered=False, debug=False)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(sc, k))).to(dev).requires_grad_(args.backward)
         for k in ("means3D", "opacities", "shs", "scales", "rotations")}
    m2 = torch.zeros_like(t["means3D"], requires_grad=args.backward)
    dpix = torch.from_numpy(S.make_cotangent(args.H, args.W, 1)).to(dev)
    ras = GaussianRasterizer(st)

    def run():
        color, _ = ras(means3D=t["means3D"], means2D=m2, opacities=t["opacities"], shs=t["shs"],
                       scales=t["scales"], rotations=t["rotations"])
        if args.backward:
            torch.autograd.backward(color, dpix)
        return color

    if args.amr or args.amr_once:
        from diff_gaussian_rasterization_amr import GaussianRasterizationSettings as AS, _RasterizeGaussians as AR
        ast = AS(**st._asdict())
        e = torch.empty(0, device=dev)
        u8 = torch.empty(0, dtype=torch.uint8, device=dev)
        a = (t["means3D"], m2, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)

        def run():  # noqa: F811  (gaussian_renderer_amr render(): fovea steps 0..4)
            with torch.no_grad():
                if args.amr_once:
                    return AR.apply(*a, -2, e, u8, u8, u8, True, ast)[0]
                # the bench's frame: rasterization_amr.render_steps (sums fused)
                from gaussian_splatting_with_eye_tracking_amd import rasterization_amr as RA
                st_ev = [evs[2 * k] for k in range(5)] if args.per_step else None
                en_ev = [evs[2 * k + 1] for k in range(5)] if args.per_step else None
                return RA.render_steps(*a, ast, starters=st_ev, enders=en_ev)[0]

        evs = [torch.cuda.Event(enable_timing=True) for _ in range(10)]
    step_ms = {v: [] for v in args.values}

    ref_img = None
    results = {v: [] for v in args.values}
    _C.profile_enable(True)
    for r in range(args.rounds):
        for v in args.values:
            _C.set_tuning(args.key, v)
            if args.backward:
                for x in (*t.values(), m2):
                    x.grad = None
            img = run()  # warm
            torch.cuda.synchronize()
            grads = [x.grad.detach().clone() for x in (*t.values(), m2)] if args.backward else []
            if args.backward:
                for x in (*t.values(), m2):
                    x.grad = None
            if ref_img is None:
                ref_img = img.detach().clone()
                ref_grads = grads
            else:
                d = float((img.detach() - ref_img).abs().max())
                if d > 1e-5:
                    print(f"WARNING variant {v}: max image diff {d}")
                for name, g, g0 in zip((*t.keys(), "means2D"), grads, ref_grads):
                    rel = float((g - g0).abs().max() / g0.abs().max().clamp_min(1e-30))
                    if rel > 1e-5:
                        print(f"WARNING variant {v}: {name} grad max rel diff {rel:.2e}")
            _C.profile_read(True)
            acc_steps = np.zeros(5)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run()
                if args.amr and args.per_step:
                    torch.cuda.synchronize()
                    acc_steps += [evs[2 * k].elapsed_time(evs[2 * k + 1]) for k in range(5)]
            e1.record()
            torch.cuda.synchronize()
            if args.amr and args.per_step:
                step_ms[v].append(acc_steps / args.iters)
            prof = _C.profile_read(True)
            if args.stage == "step":  # the whole forward (+ backward) per call, stream time
                results[v].append(e0.elapsed_time(e1) / args.iters)
                continue
            ms, cnt = prof[args.stage]
            results[v].append(ms / max(cnt, 1))
    _C.profile_enable(False)
    out = {str(v): {"median_ms": float(np.median(x)), "min_ms": float(np.min(x)), "all": [round(a, 4) for a in x]}
           for v, x in results.items()}
    if args.amr and args.per_step:
        for v in args.values:
            out[str(v)]["per_step_median_ms"] = [round(float(x), 4) for x in np.median(np.array(step_ms[v]), 0)]
    print(json.dumps({"key": args.key, "stage": args.stage, "set": args.set, "results": out}))


if __name__ == "__main__":
    main()
