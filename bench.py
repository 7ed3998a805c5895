#!/usr/bin/env python3
"""Headline benchmark: rendered views/sec (forward + backward) of the MI355X
Gaussian rasterizer at 1080p with 1M synthetic Gaussians (BASELINE.json
config 2), N data-parallel ranks (config 5 at N = 8).

One *step* = per rank: one forward + backward through the drop-in API
(``diff_gaussian_rasterization.GaussianRasterizer``, autograd) of one
1920x1080 view of the same 1M-Gaussian scene, with a fixed N(0,1) cotangent.
For N > 1 every rank ends the step holding the parameter gradients (59
floats per Gaussian: means3D 3, SH 48, opacity 1, scales 3, rotations 4)
summed over all N views: by default (--exchange views) each rank runs the
blend backward of its view, the 40-B/Gaussian view records are all-gathered
over RCCL and every rank runs the multi-view parameter backward
(data_parallel.py); --exchange params is the plain alternative, each rank's
full backward + one RCCL all-reduce of the 59-float gradients.  Per-GPU work
is fixed as N grows ("weak").

Inputs are resident in HBM before the timed region.  The timed region is K
steps bracketed by barrier + synchronize; the reported time is the max over
ranks.  ``roofline`` is computed from the HIP events the library records on
its launch stream (gs_profile_*) around the dominant kernel (render_bwd)
inside the timed region -- only that kernel is timed there, since every
event pair adds queue time -- with the algorithmic bytes of DESIGN.md; the
per-stage breakdown (``stages``) comes from a second pass of the same K
steps with every stage timed.
``cpu_baseline`` times the CPU oracle (a scalar port of the reference path)
on one full view on rank 0.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ROOFLINE_STAGE = "render_bwd"  # the dominant kernel of the fwd+bwd step

CONFIGS = {
    # name: (P, W, H)
    "cfg2_1080p_1M": (1_000_000, 1920, 1080),
    "cfg3_amr_1080p_1M": (1_000_000, 1920, 1080),   # forward-only foveated AMR (32-px tiles)
    "cfg4_bicycle_6M": (6_100_000, 1600, 1063),
    "small": (100_000, 640, 360),
}


def algorithmic_bytes(stage: str, P: int, V: int, K: int, Kb: int, N: int, T: int) -> float:
    """Compulsory HBM bytes of one launch of `stage`: the bytes
    the reference algorithm must read or write once, whatever the kernel.
    P Gaussians, V visible, K instances, Kb instances up to each tile's last
    contributor (what any blend must read), N pixels, T tiles."""
    if stage == "preprocess":   # means 12 + radii 4 + tiles_touched 4 per P; per V: scales 12, rot 16,
        return 20.0 * P + 289.0 * V  # opacity 4, SH 192 in; depth 4, xy 8, conic 16, rgb 12, cov 24, clamped 1 out
    if stage == "render":       # per entry: id 4 + xy 8 + conic/opacity 16 + rgb 12; per pixel: colour 12,
        return 40.0 * Kb + 20.0 * N + 12.0 * T  # final T 4, n_contrib 4; per tile: range 8 + max_contrib 4
    if stage == "render_bwd":   # per entry: the same 40 B + 9 accumulated floats 36; per pixel: dL/dpix 12,
        return 76.0 * Kb + 20.0 * N + 12.0 * T  # final T 4, n_contrib 4; per tile 12
    if stage == "bwd_gauss":    # radii 4 + all 75 gradient floats 300 per P; per V: accum 36, means 12,
        return 304.0 * P + 293.0 * V  # cov3D 24, scales 12, rot 16, SH 192, clamped 1
    if stage == "duplicate":    # per V: xy 8, radius 4, depth 4; per instance: one 8-B key
        return 16.0 * V + 8.0 * K
    if stage == "count_tiles":  # radius per P, xy per V in; T counts out
        return 4.0 * P + 8.0 * V + 4.0 * T
    if stage == "sort_tiles":   # per instance: key in 8, point_list out 4; per tile: range 8
        return 12.0 * K + 8.0 * T
    if stage == "zero_accum":   # the 64-B accumulator rows (this design's own buffer)
        return 64.0 * P
    if stage == "tile_scan":    # count in, range + cursor + max_contrib out
        return 28.0 * T
    return 0.0


def load_traffic(stage: str):
    """HBM bytes per launch of `stage` from a committed rocprofv3 PMC summary
    (profiles/*pmc*.json written by tools/pmc_summary.py), or None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
            if stage in d.get("per_launch_hbm_bytes", {}):
                return float(d["per_launch_hbm_bytes"][stage])
        except Exception:
            continue
    return None


# VALU issue peak: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU
# instruction (MI355X_MICROARCH.md, execution model).
VALU_PEAK_WAVE_INSTR_PER_S = 256 * 4 * 2.4e9 / 2


def load_valu_instructions(stage: str):
    """SQ_INSTS_VALU per launch of `stage` from a committed PMC summary, or None."""
    for f in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")))):
        try:
            d = json.load(open(f))
            if stage in d.get("per_launch_valu_instructions", {}):
                return float(d["per_launch_valu_instructions"][stage])
        except Exception:
            continue
    return None


def cpu_baseline_views_per_s(P: int, W: int, H: int, seed: int = 0):
    """The CPU oracle (scalar C port of the reference path) timed on one full
    view, forward + backward, single thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    O.lib()
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=seed)
    s = O.settings_from_camera(cam)
    dpix = S.make_cotangent(H, W, 1)
    kw = dict(shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    t0 = time.perf_counter()
    r = O.forward(s, sc.means3D, sc.opacities, **kw)
    O.backward(s, r, sc.means3D, dpix, **kw)
    dt = time.perf_counter() - t0
    return 1.0 / dt, dt


def cpu_amr_test_path(seed: int = 0):
    """BASELINE.json north_star: the reference's CPU path, AMR_test.py, timed
    on the host (oracle/amr_test_path.py restates it) on config 1: 10k
    Gaussians at 256x256; its input image is the CPU oracle's forward render."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import amr_test_path as A
    import oracle as O
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    W = H = 256
    cam = S.make_camera(W, H)
    sc = S.make_scene(10_000, cam, seed=seed)
    t0 = time.perf_counter()
    r = O.forward(O.settings_from_camera(cam), sc.means3D, sc.opacities, shs=sc.shs, scales=sc.scales,
                  rotations=sc.rotations)
    t_render = time.perf_counter() - t0
    out = A.run(sc.means3D, cam.world_view_transform, cam.full_proj_transform, r.color, W, H)
    sec = {k: round(v, 4) for k, v in out["seconds"].items()}
    sec["render_cpu_oracle"] = round(t_render, 4)
    total = sec["total"] + t_render
    return {"value": 1.0 / total, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": "config 1 (10k Gaussians, 256x256): AMR_test.py CPU section (projection, per-tile count "
                      "loop, log10 levels, stride lattice, 3x scipy griddata linear) + CPU oracle render",
            "seconds": sec}


def amr_algorithmic_bytes(ranges: np.ndarray, levels: np.ndarray) -> float:
    """Compulsory bytes of one 5-step frame's amr_render launches (DESIGN.md
    §4): every rendered (tile, round) block reads its tile's entries (id 4 +
    xy 8 + conic/opacity 16 + rgb 12 B) and writes its 256 sub-lattice pixels
    (colour 12 + final T 4 + n_contrib 4 B); a tile of level L renders L rounds."""
    n = (ranges[:, 1] - ranges[:, 0]).astype(np.float64)
    L = np.minimum(levels.astype(np.float64), 4.0)
    return float((L * (40.0 * n + 20.0 * 256)).sum())


def run_amr(args, world, rank, local_rank, distributed, dev):
    """Config 3: forward-only foveated rendering (gaussian_renderer_amr's
    render(): foveaStep 0..4 through _RasterizeGaussians, summing the step
    images; and render_once(): foveaStep -2 with interpolation).  Per-frame and
    single-GPU: for N > 1 every rank renders its own frames (replicas only)."""
    from diff_gaussian_rasterization_amr import GaussianRasterizationSettings, GaussianRasterizer, _RasterizeGaussians
    from gaussian_splatting_with_eye_tracking_amd import _C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S

    P, W, H = CONFIGS[args.config]
    cam = S.make_camera(W, H)
    sc = S.make_scene(P, cam, seed=args.seed)
    st = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.zeros(3, device=dev), scale_modifier=1.0,
        viewmatrix=torch.from_numpy(cam.world_view_transform).to(dev),
        projmatrix=torch.from_numpy(cam.full_proj_transform).to(dev), sh_degree=3,
        campos=torch.from_numpy(cam.camera_center).to(dev), prefiltered=False, debug=False)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(sc, k))).to(dev)
         for k in ("means3D", "opacities", "shs", "scales", "rotations")}
    e = torch.empty(0, device=dev)
    u8 = torch.empty(0, dtype=torch.uint8, device=dev)
    means2D = torch.zeros_like(t["means3D"])
    a = (t["means3D"], means2D, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]

    from gaussian_splatting_with_eye_tracking_amd import rasterization_amr as RA
    # extension: the tracked fovea centre of config 3
    # (pupil (361.74, 248.19) in the 640x400 eye image -> screen) with the
    # reference's unused fovea radii W/2 .. W/16 restricting the AMR levels
    fov_centres, fov_radii = RA.reference_foveae(W, H, (361.74 / 640 * W, 248.19 / 400 * H))

    def frame_5step(record=False, fovea=False):
        if record:
            ev[0].record()
        c, radii, gb, bb, ib = _RasterizeGaussians.apply(*a, 0, e, u8, u8, u8, False, st)
        if fovea:
            RA.apply_fovea_levels(ib, W, H, fov_centres, fov_radii)
        acc = c
        if record:
            ev[1].record()
        for k in range(1, 5):
            c, _, gb, bb, ib = _RasterizeGaussians.apply(*a, k, acc, gb, bb, ib, False, st)
            acc = acc + c
            if record:
                ev[k + 1].record()
        return acc, gb, bb, ib

    rast = GaussianRasterizer(st)

    def frame_once():
        return rast(means3D=t["means3D"], means2D=means2D, opacities=t["opacities"], shs=t["shs"],
                    scales=t["scales"], rotations=t["rotations"], foveaStep=-2, interpolate_image=True)[0]

    with torch.no_grad():
        for _ in range(args.warmup):
            frame_5step()
            frame_once()
        torch.cuda.synchronize()
        if not args.no_profile:
            _C.profile_enable(True)
            _C.profile_read(True)
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step_ms = np.zeros(5)
        for _ in range(args.steps):
            frame_5step(record=True)
            torch.cuda.synchronize()
            step_ms += np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(5)])
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        el5 = time.perf_counter() - t0
        prof = {}
        if not args.no_profile:
            prof = _C.profile_read(True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            frame_once()
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        el1 = time.perf_counter() - t0
        if not args.no_profile:
            _C.profile_enable(False)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            frame_5step(fovea=True)
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        elf = time.perf_counter() - t0
    # extension: the foveated backward -- render_once (interpolated) forward +
    # backward through the drop-in autograd API with a fixed cotangent
    tg = {k: v.detach().clone().requires_grad_(True) for k, v in t.items()}
    m2 = torch.zeros_like(tg["means3D"], requires_grad=True)
    cot = torch.from_numpy(S.make_cotangent(H, W, 1)).to(dev)

    def frame_once_fwd_bwd():
        img = rast(means3D=tg["means3D"], means2D=m2, opacities=tg["opacities"], shs=tg["shs"],
                   scales=tg["scales"], rotations=tg["rotations"], foveaStep=-2, interpolate_image=True)[0]
        torch.autograd.backward(img, cot)

    for _ in range(max(1, args.warmup)):
        frame_once_fwd_bwd()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame_once_fwd_bwd()
    torch.cuda.synchronize()
    elb = time.perf_counter() - t0
    with torch.no_grad():
        if distributed:
            tt = torch.tensor([el5, el1, elf, elb], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el5, el1, elf, elb = (float(v) for v in tt.tolist())
        result = None
        if rank == 0:
            acc, gb, bb, ib = frame_5step()
            torch.cuda.synchronize()
            K = int(_C.parse_buffers(gb, bb, ib, P, 0, W, H, 32)["hdr"][0].item())
            d = _C.parse_buffers(gb, bb, ib, P, K, W, H, 32)
            rng = d["ranges"].cpu().numpy().astype(np.int64)
            lv = d["levels"].cpu().numpy().astype(np.int64)
            _, _, _, ibf = frame_5step(fovea=True)
            lvf = _C.parse_buffers(gb, bb, ibf, P, K, W, H, 32)["levels"].cpu().numpy().astype(np.int64)
            fovea_hist = np.bincount(lvf, minlength=5)[1:].tolist()
            stages = {n: {"avg_ms": ms / c, "launches": c, "ms_per_frame": ms / args.steps}
                      for n, (ms, c) in prof.items() if c}
            roofline = None
            if "amr_render" in stages:
                by = amr_algorithmic_bytes(rng, lv)
                ms = stages["amr_render"]["ms_per_frame"]
                ach = by / (ms * 1e-3) / 1e9
                roofline = {"kernel": "amr_render", "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": load_traffic("amr_render"),
                            "algorithmic_bytes_per_frame": by, "ms_per_frame": round(ms, 4)}
            cpu = None
            if not args.no_cpu_baseline and world == 1:
                cpu = cpu_amr_test_path(args.seed)
            result = {
                "metric": "foveated AMR frames/sec (forward-only render(), 5 fovea steps) at 1080p, 1M Gaussians",
                "value": world * args.steps / el5, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": 1000.0 * el5 / args.steps, "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
                "data": "synthetic (SURVEY §8(d) generator, seed 0)",
                "config": {"workload": f"{args.config}: {P} Gaussians, {W}x{H}, 32x32 AMR tiles, 5-step foveated "
                                       f"render() per frame" + (", replicas" if world > 1 else ""),
                           "P": P, "width": W, "height": H, "K_instances": K, "parallelism": f"replicas{world}",
                           "levels_hist": np.bincount(lv, minlength=5)[1:].tolist()},
                "render_once_fps": world * args.steps / el1,
                "amr_backward_ext": {"render_once_fwd_bwd_fps": world * args.steps / elb,
                                     "note": "extension beyond parity: interpolated render_once forward + "
                                             "backward through the autograd API"},
                "fovea_levels_ext": {"fps": world * args.steps / elf, "centre": [round(v, 2) for v in fov_centres[0]],
                                     "radii": fov_radii, "levels_hist": fovea_hist,
                                     "note": "extension beyond parity: tracked fovea discs clamp the AMR levels"},
                "per_step_ms": [round(x / args.steps, 4) for x in step_ms],
                "roofline": roofline,
                "cpu_baseline": cpu,
                "stages": stages,
            }
            print(json.dumps(result), flush=True)
    return result


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="cfg2_1080p_1M", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="disable the per-stage event timing")
    ap.add_argument("--exchange", choices=("views", "params"), default="views",
                    help="N > 1 gradient exchange: all-gather of per-view screen-space records (default) or "
                         "all-reduce of the 59-float parameter gradients")
    ap.add_argument("--yaw-spread", type=float, default=0.0,
                    help="rank r renders the camera yawed by (r-(N-1)/2)*spread degrees (config 5 uses 5)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    # GS_BENCH_SHARE_DEVICE=1 / GS_BENCH_BACKEND=gloo only rehearse the N>1 path
    # on a one-GPU box (every rank on device 0); real runs use one GPU per rank
    # and RCCL ("nccl").
    if os.environ.get("GS_BENCH_SHARE_DEVICE") == "1":
        local_rank = local_rank % max(1, torch.cuda.device_count())
    if distributed:
        torch.cuda.set_device(local_rank)
        backend = os.environ.get("GS_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local_rank)
    if args.config.startswith("cfg3"):
        result = run_amr(args, world, rank, local_rank, distributed, dev)
        if distributed:
            dist.barrier()
            dist.destroy_process_group()
        return result

    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from gaussian_splatting_with_eye_tracking_amd import _C
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S

    P, W, H = CONFIGS[args.config]
    cam0 = S.make_camera(W, H)
    sc = S.make_scene(P, cam0, seed=args.seed)
    yaw = (rank - (world - 1) / 2.0) * args.yaw_spread
    cam = cam0 if yaw == 0.0 else S.make_orbit_camera(W, H, yaw)
    settings = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.zeros(3, device=dev), scale_modifier=1.0,
        viewmatrix=torch.from_numpy(cam.world_view_transform).to(dev),
        projmatrix=torch.from_numpy(cam.full_proj_transform).to(dev), sh_degree=3,
        campos=torch.from_numpy(cam.camera_center).to(dev), prefiltered=False, debug=False)
    params = {k: torch.from_numpy(np.ascontiguousarray(getattr(sc, k))).to(dev).requires_grad_(True)
              for k in ("means3D", "opacities", "shs", "scales", "rotations")}
    means2D = torch.zeros_like(params["means3D"], requires_grad=True)
    dpix = torch.from_numpy(S.make_cotangent(H, W, 100 + rank)).to(dev)
    rasterizer = GaussianRasterizer(settings)
    # N > 1, --exchange params: parameter grads are views of one flat buffer (DDP's
    # gradient-as-bucket-view): the backward accumulates straight into it and one
    # RCCL all-reduce sums it.  --exchange views (default): each rank runs the
    # blend backward of its view, one RCCL all-gather of the view records, then
    # every rank forms the summed parameter gradients of all N views
    # (data_parallel.py).
    views_mode = distributed and args.exchange == "views"
    flat = DP.FlatGrads(params) if (distributed and not views_mode) else None
    e0 = torch.empty(0, device=dev)

    def step_views():
        with torch.no_grad():
            fwd = _C.rasterize_gaussians(
                settings.bg, params["means3D"], e0, params["opacities"], params["scales"], params["rotations"],
                1.0, e0, settings.viewmatrix, settings.projmatrix, settings.tanfovx, settings.tanfovy, H, W,
                params["shs"], 3, settings.campos, False, False)
            return DP.exchange_view_grads(settings, fwd, dpix, params["means3D"], params["shs"], params["scales"],
                                          params["rotations"])

    def step():
        if views_mode:
            return step_views()
        if flat is not None:
            flat.flat.zero_()
            flat.attach(params)
        else:
            for p in params.values():
                p.grad = None
        means2D.grad = None
        color, radii = rasterizer(means3D=params["means3D"], means2D=means2D, opacities=params["opacities"],
                                  shs=params["shs"], scales=params["scales"], rotations=params["rotations"])
        torch.autograd.backward(color, dpix)
        if flat is not None:
            DP.allreduce_(flat.flat)
        return color

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # Inside the timed region only the roofline kernel (render_bwd, the
    # dominant stage at every config measured) records its event pair: each
    # timed stage costs two event records per launch (~4 us of queue time).
    if not args.no_profile:
        _C.profile_enable(True)
        _C.profile_stages([ROOFLINE_STAGE])
        _C.profile_read(True)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof_timed = {}
    prof = {}
    if not args.no_profile:
        prof_timed = _C.profile_read(True)
        # Per-stage breakdown: the same K steps again, every stage timed
        # (outside the headline timing).
        _C.profile_stages([])
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        prof = _C.profile_read(True)
        _C.profile_enable(False)
    if distributed:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_per_step = 1000.0 * elapsed / args.steps
    views = world * args.steps
    value = views / elapsed

    result = None
    if rank == 0:
        # Workload statistics (K, V, ...) from one extra forward, outside the timed region.
        with torch.no_grad():
            K, color, radii, geom, binning, img = _C.rasterize_gaussians(
                settings.bg, params["means3D"], torch.Tensor([]), params["opacities"], params["scales"],
                params["rotations"], 1.0, torch.Tensor([]), settings.viewmatrix, settings.projmatrix,
                settings.tanfovx, settings.tanfovy, H, W, params["shs"], 3, settings.campos, False, False)
            bufs = _C.parse_buffers(geom, binning, img, P, K, W, H, 16)
        V = int((radii > 0).sum().item())
        rng = bufs["ranges"].cpu().numpy().astype(np.int64)
        n_t = rng[:, 1] - rng[:, 0]
        Kb = int(np.minimum(n_t, bufs["max_contrib"].cpu().numpy().astype(np.int64)).sum())
        N = W * H
        T = ((W + 15) // 16) * ((H + 15) // 16)
        stages = {}
        for name, (ms, cnt) in prof.items():
            if cnt:
                stages[name] = {"avg_ms": ms / cnt, "launches": cnt, "ms_per_step": ms / args.steps}
        roofline = None
        if stages:
            dom = max(stages, key=lambda n: stages[n]["ms_per_step"])
            ms_t, cnt_t = prof_timed.get(dom, (0.0, 0))
            if cnt_t:  # events recorded inside the timed region
                avg_ms, src = ms_t / cnt_t, "timed region"
            else:
                avg_ms, src = stages[dom]["avg_ms"], "stage-profile pass"
            by = algorithmic_bytes(dom, P, V, K, Kb, N, T)
            ach = by / (avg_ms * 1e-3) / 1e9
            roofline = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": load_traffic(dom),
                        "algorithmic_bytes": by, "avg_ms": round(avg_ms, 4), "events": src}
            vi = load_valu_instructions(dom)
            if vi is not None:  # the blend kernels' real bound
                a_ = vi / (avg_ms * 1e-3)
                roofline["valu_issue"] = {"instructions_per_launch": vi, "achieved": round(a_, 1),
                                          "peak": VALU_PEAK_WAVE_INSTR_PER_S, "unit": "wave-instr/s",
                                          "frac": round(a_ / VALU_PEAK_WAVE_INSTR_PER_S, 4)}
            for n, st in stages.items():
                b = algorithmic_bytes(n, P, V, K, Kb, N, T)
                st["algorithmic_GBps"] = round(b / (st["avg_ms"] * 1e-3) / 1e9, 1) if b else None
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            v, dt = cpu_baseline_views_per_s(P, W, H, args.seed)
            cpu = {"value": v, "unit": "views/s", "cores": 1, "kind": "port",
                   "sample": f"one full {W}x{H} view, {P} Gaussians, fwd+bwd, CPU oracle (C, 1 thread): {dt:.1f} s"}
        result = {
            "metric": "rendered views/sec (fwd+bwd) at 1080p, 1M Gaussians; achieved HBM GB/s %",
            "value": value, "unit": "views/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp32", "data": "synthetic (SURVEY §8(d) generator, seed 0)",
            "config": {"workload": f"{args.config}: {P} Gaussians, {W}x{H}, 16x16 tiles, forward+backward, "
                                   f"1 view per GPU per step" + (
                                       ("" if world == 1 else
                                        " + RCCL all-gather of the 40-B/Gaussian view records and the multi-view "
                                        "parameter backward" if args.exchange == "views" else
                                        " + RCCL all-reduce of 59 f32/Gaussian grads")),
                       "exchange": None if world == 1 else args.exchange,
                       "P": P, "width": W, "height": H, "views_per_gpu_per_step": 1,
                       "parallelism": f"dp{world}", "K_instances": K, "V_visible": V, "K_bwd_entries": Kb},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_amr_test_path": cpu_amr_test_path(args.seed) if (cpu is not None) else None,
            "stages": stages,
        }
        print(json.dumps(result), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
