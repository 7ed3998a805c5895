#!/usr/bin/env python3
"""Headline benchmark: rendered views/sec (forward + backward) of the MI355X
Gaussian rasterizer at 1080p with 1M synthetic Gaussians (BASELINE.json
config 2), and the 1 -> 8 GPU data-parallel curve (config 5).

N = 1 (default): one *step* = one forward + backward through the drop-in API
(``diff_gaussian_rasterization.GaussianRasterizer``, autograd) of one
1920x1080 view of the 1M-Gaussian scene with a fixed N(0,1) cotangent
(config 2).  Rank 0 then adds the other single-GPU configurations as
``sub_results`` (config 3: foveated AMR 5-step frame; config 4: 6.1M
Gaussians at 1600x1063; config 5 on one GPU: the 8-view step), each with its
own roofline, and the CPU baselines.

N > 1 (config 5): a fixed global batch of 8 views per step
(cameras yawed -17.5 .. +17.5 degrees in 5-degree steps, cotangent seeds
100 + v), 8 / N views per rank; every rank ends the step holding the
parameter gradients (59 floats per Gaussian) summed over all 8 views.
Headline exchange ("views"): each rank runs the blend backward of its views,
the 40-B/Gaussian view records are all-gathered over RCCL and every rank
runs the multi-view parameter backward (data_parallel.py).  The line also
carries the north_star's exchange ("params": each rank's full backward +
one RCCL all-reduce of the 59-float gradients) and both collectives timed
alone (ms, bus GB/s, the world size RCCL reports).  views/s = 8 / step time
("strong": the global batch is fixed).

Launch: ``python bench.py --gpus N`` starts N ranks itself when WORLD_SIZE
is unset (before any GPU call); under torchrun WORLD_SIZE must equal N.
Inputs are resident in HBM before the timed region; K steps are bracketed by
barrier + synchronize, the time is the max over ranks.  ``roofline``: HIP
events the library records on its launch stream (gs_profile_*) around the
dominant kernel inside the timed region, with the algorithmic bytes of
DESIGN.md §4; ``traffic`` comes only from a committed PMC summary of the
SAME configuration AND the same build (profiles/*pmc_summary.json, keyed by
P, W, H, tile and the native sources' digest, ``build_digest()``).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU issue peak, measured with exact instruction streams (round 4,
# tools/valu_rate.hip inline-asm bodies, profiles/r04a_valu_rate.log): the
# two-operand VOP1/VOP2 forms (v_mul / v_add / v_fmac / v_mov) issue one wave64
# instruction per 2.3-2.6 SIMD-cycles with >= 2 waves per SIMD -- 2.4 taken as
# the peak; VOP3 fma 2.6-3.9, compares / e64 selects / v_min ~4, exp / rcp 8,
# so a real mix runs below this rate at full issue (the blends' mixes cost
# ~3.3 and ~2.9 cycles per instruction).  (Round 3 priced every
# instruction at a packed-FMA rate of 4.43 cycles: its probe's "v_fma" chain
# had been SLP-packed.)
VALU_PEAK_WAVE_INSTR_PER_S = 256 * 4 * 2.4e9 / 2.4
METRIC = "rendered views/sec (fwd+bwd) at 1080p, 1M Gaussians; achieved HBM GB/s %"

CONFIGS = {
    # name: P, W, H, tile size, kind
    "cfg2_1080p_1M": dict(P=1_000_000, W=1920, H=1080, tile=16, kind="fwd_bwd"),
    "cfg3_amr_1080p_1M": dict(P=1_000_000, W=1920, H=1080, tile=32, kind="amr"),
    "cfg4_bicycle_6M": dict(P=6_100_000, W=1600, H=1063, tile=16, kind="fwd_bwd"),
    "cfg5_8view_1080p_1M": dict(P=1_000_000, W=1920, H=1080, tile=16, kind="multiview", views=8),
    "small": dict(P=100_000, W=640, H=360, tile=16, kind="fwd_bwd"),
}


# ------------------------------------------------------------------ launch ---
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str]) -> int:
    """`bench.py --gpus N` without a launcher: start N ranks of this script
    as child processes (one per GPU, LOCAL_RANK = rank) and return the first
    failing exit code (0 if all succeed).  Runs before anything touches the
    GPU; a rank that fails ends the others (their exact PIDs)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:
                    q.kill()
        time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc


# ------------------------------------------------------------- roofline ---
def algorithmic_bytes(stage: str, P: int, V: int, K: int, Kb: int, N: int, T: int, views: int = 1) -> float:
    """SURVEY.md §8(d)'s algorithmic bytes of the reference stage this kernel
    replaces: the compulsory I/O of that stage, counted once (DESIGN.md §7
    maps kernel -> reference stage).  P Gaussians, V visible, K instances, N
    pixels, T tiles (Kb unused: the survey's blend rows read all K)."""
    if stage == "preprocess":   # fwd preprocess
        return 20.0 * P + 291.0 * V
    if stage == "count_tiles":  # the reference's scan: tiles_touched in, offsets out
        return 8.0 * P
    if stage == "tile_scan":    # identifyTileRanges + the ranges memset
        return 8.0 * K + 16.0 * T
    if stage == "duplicate":    # duplicateWithKeys
        return 4.0 * P + 16.0 * V + 12.0 * K
    if stage == "sort_tiles":   # the radix sort
        return 24.0 * K
    if stage == "render":       # blend fwd
        return 40.0 * K + 20.0 * N + 8.0 * T
    if stage == "render_bwd":   # blend bwd
        return 40.0 * K + 20.0 * N + 8.0 * T + 36.0 * V
    if stage == "bwd_gauss":    # bwd zero-init of outputs 300P + cov2D bwd 4P + 84V + preprocess bwd 4P + 523V
        return 308.0 * P + 607.0 * V
    if stage == "multiview_bwd":  # per view 40-B records; params in (means 12, SH 192, scales 12, rot 16),
        return 40.0 * views * P + 232.0 * P + 236.0 * P  # 59 gradient floats out (no reference stage)
    return 0.0


def design_bytes(stage: str, P: int, V: int, K: int, Kb: int, N: int, T: int):
    """What THIS design's kernel must move once, where it differs from the
    reference stage (algorithmic_bytes), else None:
    the blends read only the Kb entries before each tile's last contributor
    and the render zeroes the backward's 64-B accumulator rows; the
    backward's per-entry 36 B are its 64-B atomic rows; the preprocess also
    writes a 48-B SH-derivative row per visible Gaussian that bwd_gauss reads
    instead of the 192-B coefficients; the binning stages move keys per tile
    bucket (no global radix passes)."""
    if stage == "preprocess":
        return 20.0 * P + 337.0 * V
    if stage == "render":       # per entry: id 4 + xy 8 + conic/opacity 16 + rgb 12; per pixel 20; per tile
        return 40.0 * Kb + 20.0 * N + 12.0 * T + 64.0 * P  # range + max_contrib 12; the 64-B accumulator rows
    if stage == "render_bwd":   # per entry: the same 40 B + 9 accumulated floats 36; per pixel 20; per tile 12
        return 76.0 * Kb + 20.0 * N + 12.0 * T
    if stage == "bwd_gauss":    # radii 4 + all 75 gradient floats 300 per P; per V: accum 36, means 12,
        return 304.0 * P + 149.0 * V  # scales 12, rot 16, SH-derivative row 48, clamped 1, + opacity etc.
    if stage == "duplicate":    # per V: xy 8, radius 4, depth 4; per instance: one 8-B key
        return 16.0 * V + 8.0 * K
    if stage == "count_tiles":  # radius per P, xy per V in; T counts out
        return 4.0 * P + 8.0 * V + 4.0 * T
    if stage == "sort_tiles":   # per instance: key in 8, point_list out 4; per tile: range 8
        return 12.0 * K + 8.0 * T
    if stage == "tile_scan":    # count in, range + cursor + max_contrib out
        return 28.0 * T
    return None


def stream_read_bytes(stage: str, P: int, V: int, K: int, Kb: int, N: int, T: int, views: int = 1):
    """Bytes of one launch of `stage` read as wave-contiguous streams, or None
    when (nearly) all its reads are streams.  profiles/r02n_pmc_calib.json
    (tools/pmc_calib.hip, 1 GiB buffer): FETCH_SIZE tallies a streamed 128-B
    line at 64 B (the guide's x2) but a random 8 / 16 / 64-B gather miss at the
    64-B sector it really moves (x1); scattered stores and 64-B atomic rows are
    counted at their true granule by WRITE_SIZE.  So traffic = FETCH + WRITE +
    (streamed bytes) / 2 for the gather-dominated blend kernels."""
    if stage == "render":      # point_list ids; ranges
        return 4.0 * Kb + 8.0 * T
    if stage == "render_bwd":  # point_list ids; dL/dpix, final T, n_contrib; ranges + max_contrib
        return 4.0 * Kb + 20.0 * N + 12.0 * T
    if stage == "amr_render":  # list positions and tile-local records: 64-B-sector reads, none streamed
        return 0.0
    return None


def config_key(P: int, W: int, H: int, tile: int, views: int = 1) -> dict:
    """What a committed PMC summary must match: the scene, image and tile
    size, and (config 5) the views per step."""
    k = {"P": int(P), "W": int(W), "H": int(H), "tile": int(tile)}
    if views != 1:
        k["views"] = int(views)
    return k


def _pmc_files():
    return sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_summary.json")))


_DIGEST = None


def _build_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_gsamd_build_digest", os.path.join(ROOT, "gaussian_splatting_with_eye_tracking_amd", "build.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def build_digest() -> str:
    """gs_build_digest() of the loaded libgsplat_amd.so, checked against the
    digest of the tree's native sources + flags (build.py source_digest,
    check_loaded_digest): a library built from other sources is refused, so a
    summary or bench line that carries this digest was measured on exactly
    these sources."""
    global _DIGEST
    if _DIGEST is None:
        _DIGEST = _build_module().check_loaded_digest()
    return _DIGEST


def _matching_summaries(key: dict):
    """Committed PMC summaries of THIS configuration and THIS build, newest
    first.  Summaries of another configuration or build -- or with neither
    recorded -- are never used."""
    for f in reversed(_pmc_files()):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("config") != key or d.get("build") != build_digest():
            continue
        yield f, d


def load_pmc(stage: str, key: dict, field: str):
    """`field` ("per_launch_hbm_bytes" or "per_launch_valu_instructions") of
    `stage` (per stage invocation) from the newest matching summary, or None."""
    for f, d in _matching_summaries(key):
        v = d.get(field, {}).get(stage)
        if v is not None:
            return float(v), os.path.relpath(f, ROOT)
    return None


def load_raw_kib(stage: str, key: dict):
    """(FETCH_SIZE, WRITE_SIZE) KiB per invocation of `stage` from the newest
    matching summary, or None."""
    for f, d in _matching_summaries(key):
        v = d.get("raw_kib", {}).get(stage)
        if v is not None:
            return float(v["FETCH_SIZE"]), float(v["WRITE_SIZE"])
    return None


def load_kernel_avg_us(stage: str, key: dict):
    """rocprofv3 --kernel-trace --stats mean duration (us) of one invocation
    of `stage` from the newest summary of this configuration AND build, or
    None."""
    for f, d in _matching_summaries(key):
        v = d.get("kernel_avg_us", {}).get(stage)
        if v is not None:
            return float(v), os.path.relpath(f, ROOT)
    return None


def make_roofline(stage: str, by: float, events_ms: float, key: dict, src: str, per: float = 1.0,
                  stream_read: float | None = None, design_by: float | None = None) -> dict:
    """`by` = SURVEY §8(d) algorithmic bytes (algorithmic_bytes) of `per`
    launches of `stage`.  The duration is the rocprofv3 kernel-trace mean of
    the SAME build and configuration (profiles/*pmc_summary.json
    kernel_avg_us, x per) when one is committed -- so frac = bytes / that
    mean / 8 TB/s can be reproduced from profiles/ alone -- else this run's
    HIP-event mean; both timings are in the line.  `stream_read`: streamed
    read bytes per launch (stream_read_bytes) -- given, traffic uses the
    gather calibration instead of doubling every fetched byte."""
    rp = load_kernel_avg_us(stage, key)
    if rp is not None:
        avg_ms, avg_src = rp[0] * 1e-3 * per, f"rocprofv3 kernel trace, {rp[1]}"
    else:
        avg_ms, avg_src = events_ms, f"HIP events ({src}); no rocprofv3 summary of this build"
    ach = by / (avg_ms * 1e-3) / 1e9
    tr = load_pmc(stage, key, "per_launch_hbm_bytes")
    traffic = tr[0] * per if tr else None
    raw = load_raw_kib(stage, key) if stream_read is not None else None
    calib = None
    if raw is not None:
        calib = (1024.0 * (raw[0] + raw[1]) + 0.5 * stream_read) * per
    r = {"kernel": stage, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": calib if calib is not None else traffic,
         "traffic_source": tr[1] if tr else None, "algorithmic_bytes": by,
         "bytes_definition": "SURVEY.md §8(d) reference-stage bytes", "avg_ms": round(avg_ms, 4),
         "avg_ms_source": avg_src, "avg_ms_events": round(events_ms, 4), "events": src, "build": build_digest()}
    if design_by is not None:  # what this design's kernel must move (design_bytes)
        r["design_bytes"] = design_by
        r["design_frac"] = round(design_by / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    if ach > HBM_PEAK_GBS:
        # The reference stage's bytes / this kernel's time exceed the peak: the
        # kernel does not move those bytes (e.g. bwd_gauss reads the 48-B
        # d(rgb)/d(dir) rows the forward stored, not the 192-B SH rows, and
        # zero-fills nothing), so that figure is not a roofline fraction.  The
        # roofline is then taken on what this kernel must move (design_bytes)
        # -- or, without that, on the measured traffic -- and the reference
        # stage's figure stays in the line as an equivalent rate only.
        r["reference_stage_bytes"] = by
        r["reference_stage_equiv_GBps"] = round(ach, 1)
        r.pop("design_frac", None)  # (= frac below)
        basis = design_by if design_by is not None else r["traffic"]
        r["algorithmic_bytes"] = basis
        if basis is None:
            r["achieved"], r["frac"] = None, None
            r["bytes_definition"] = ("none: the reference-stage bytes exceed the peak at this kernel's time and "
                                     "no design or measured bytes are known")
        else:
            a2 = basis / (avg_ms * 1e-3) / 1e9
            r["achieved"], r["frac"] = round(a2, 1), round(a2 / HBM_PEAK_GBS, 4)
            r["bytes_definition"] = (
                "this design's compulsory bytes (bench.py design_bytes, DESIGN.md §4): the SURVEY.md §8(d) "
                "reference-stage bytes / this time would exceed the HBM peak (reference_stage_equiv_GBps), since "
                "this kernel does not move them" if design_by is not None else
                "measured traffic: the reference-stage bytes / this time would exceed the HBM peak")
    if calib is not None:
        r["traffic_note"] = ("FETCH + WRITE + streamed reads / 2 (gathers counted x1, streams x2: "
                             "profiles/r02n_pmc_calib.json)")
        r["traffic_all_fetch_x2"] = traffic
    vi = load_pmc(stage, key, "per_launch_valu_instructions")
    if vi is not None:  # the blend kernels' real bound
        a_ = vi[0] * per / (avg_ms * 1e-3)
        r["valu_issue"] = {"instructions": vi[0] * per, "achieved": round(a_, 1),
                           "peak": VALU_PEAK_WAVE_INSTR_PER_S, "unit": "wave-instr/s",
                           "frac": round(a_ / VALU_PEAK_WAVE_INSTR_PER_S, 4),
                           "peak_definition": "one VOP2 wave64 instruction per 2.4 SIMD-cycles, 1024 SIMDs, "
                                              "2.4 GHz (profiles/r04a_valu_rate.log)"}
    return r


def step_bytes_fwd_bwd(P: int, V: int, K: int, N: int, T: int) -> float:
    """compulsory bytes of one view's whole forward +
    backward, every reference stage counted once: 340P + 950V + 124K + 40N
    + 32T."""
    return 340.0 * P + 950.0 * V + 124.0 * K + 40.0 * N + 32.0 * T


def step_bytes_amr_frame(P: int, V: int, K: int, T: int, ranges: np.ndarray, levels: np.ndarray) -> float:
    """one forward-only 5-step foveated frame, 32P + 307V +
    44K + 24T + 40 sum_t(K_t rounds_t) + 20 N_rendered, plus the B1-B4 terms
    (16T); amr_algorithmic_bytes holds the last two terms (a tile of level L
    renders L rounds of 256 pixels)."""
    return 32.0 * P + 307.0 * V + 44.0 * K + 24.0 * T + 16.0 * T + amr_algorithmic_bytes(ranges, levels)


def step_roofline(nbytes: float, ms_per_step: float, definition: str) -> dict:
    """The whole step against the HBM roofline: §8(d)'s compulsory bytes of
    every stage of the step / the measured step time (the per-kernel
    `roofline` is the dominant kernel's alone)."""
    ach = nbytes / (ms_per_step * 1e-3) / 1e9
    return {"bytes_per_step": nbytes, "ms_per_step": round(ms_per_step, 4), "achieved": round(ach, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "roofline_equiv_per_s": round(1e3 / (ms_per_step * ach / HBM_PEAK_GBS), 1) if ach else None,
            "definition": definition}


# ------------------------------------------------------------ CPU baselines ---
def cpu_baseline_views_per_s(sc, cam, threads: int):
    """The CPU oracle (a scalar C port of the reference path, OpenMP over
    Gaussians / pixel rows / tile-row bands) on one full view, fwd + bwd."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    O.lib()
    O.set_threads(threads)
    s = O.settings_from_camera(cam)
    dpix = S.make_cotangent(cam.image_height, cam.image_width, 1)
    kw = dict(shs=sc.shs, scales=sc.scales, rotations=sc.rotations)
    try:
        t0 = time.perf_counter()
        r = O.forward(s, sc.means3D, sc.opacities, **kw)
        O.backward(s, r, sc.means3D, dpix, **kw)
        dt = time.perf_counter() - t0
    finally:
        O.set_threads(1)
    return 1.0 / dt, dt


def cpu_share() -> tuple[int, str]:
    """The CPUs this job may use, from evidence: the cgroup CPU quota
    (v2 cpu.max "quota period", v1 cfs_quota_us / cfs_period_us), rounded
    down; without a quota the affinity mask, capped by OMP_NUM_THREADS when
    the environment sets it (the pool's stated per-GPU share).  Returns
    (threads, what was read)."""
    def read(p):
        try:
            with open(p) as f:
                return f.read().split()
        except OSError:
            return None
    v2 = read("/sys/fs/cgroup/cpu.max")
    if v2 and len(v2) == 2 and v2[0] != "max":
        n = int(v2[0]) // int(v2[1])
        if n >= 1:
            return n, f"/sys/fs/cgroup/cpu.max ({v2[0]} {v2[1]})"
    q, p = read("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), read("/sys/fs/cgroup/cpu/cpu.cfs_period_us")
    if q and p and int(q[0]) > 0:
        n = int(q[0]) // int(p[0])
        if n >= 1:
            return n, f"/sys/fs/cgroup/cpu/cpu.cfs_quota_us / cpu.cfs_period_us ({q[0]} / {p[0]})"
    try:
        n, src = len(os.sched_getaffinity(0)), "sched_getaffinity"
    except (AttributeError, OSError):
        n, src = os.cpu_count() or 1, "os.cpu_count()"
    quota_note = "cpu.max: " + " ".join(v2) if v2 else "no cgroup cpu quota file"
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and 0 < int(env) < n:
        return int(env), f"OMP_NUM_THREADS={env} (the pool's per-GPU share; {quota_note}, {src}: {n})"
    return n, f"{src} ({quota_note})"


def cpu_baselines(sc, cam) -> dict:
    n, src = cpu_share()
    v1, dt1 = cpu_baseline_views_per_s(sc, cam, 1)
    vn, dtn = cpu_baseline_views_per_s(sc, cam, n)
    W, H, P = cam.image_width, cam.image_height, sc.P
    return {"value": vn, "unit": "views/s", "cores": n, "kind": "port",
            "sample": f"one full {W}x{H} view, {P} Gaussians, fwd+bwd, CPU oracle (C, OpenMP, {n} threads): "
                      f"{dtn:.2f} s",
            "cores_source": src, "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "single_thread": {"value": v1, "cores": 1, "seconds": round(dt1, 2)}}


def cpu_amr_test_path(seed: int = 0):
    """BASELINE.json north_star: the reference's CPU path, AMR_test.py, timed
    on the host (oracle/amr_test_path.py restates it) on config 1: 10k
    Gaussians at 256x256; its input image is the CPU oracle's forward render.
    Single-threaded by construction (Python loops + Qhull)."""
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


# --------------------------------------------------------------- context ---
class Ctx:
    def __init__(self, world, rank, local_rank, distributed, dev, args):
        self.world, self.rank, self.local_rank, self.distributed, self.dev, self.args = (
            world, rank, local_rank, distributed, dev, args)
        self._scenes = {}

    def scene(self, P: int, W: int, H: int):
        """The SURVEY §8(d) scene (seed args.seed) and the identity camera it is
        generated in (cached: configs 2, 3 and 5 share the 1M scene)."""
        from gaussian_splatting_with_eye_tracking_amd import synthetic as S
        k = (P, W, H)
        if k not in self._scenes:
            cam = S.make_camera(W, H)
            self._scenes[k] = (S.make_scene(P, cam, seed=self.args.seed), cam)
        return self._scenes[k]

    def barrier(self):
        import torch.distributed as dist
        if self.distributed:
            dist.barrier()

    def max_over_ranks(self, *vals):
        import torch
        import torch.distributed as dist
        if not self.distributed:
            return vals
        t = torch.tensor(list(vals), device=self.dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return tuple(float(v) for v in t.tolist())


def settle(fn, warmup: int, ctx: "Ctx") -> int:
    """The W warmup steps, then untimed steps until about --ramp-ms of work
    has run.  The GPU's clocks ramp over the first ~40 ms of sustained load
    (profiles/r05a_launch_ramp_cfg2.txt: render_bwd 360 -> 309 us per launch
    across 45 launches); without this the timed region averages part of the
    ramp.  Every rank runs the same number of extra steps (max over ranks),
    so steps that hold collectives stay matched.  Returns that number."""
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if ctx.args.ramp_ms <= 0:
        return 0
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    (dt,) = ctx.max_over_ranks(time.perf_counter() - t0)
    n = int(min(2000, max(0, np.ceil(ctx.args.ramp_ms * 1e-3 / max(dt, 1e-5)))))
    (n,) = ctx.max_over_ranks(float(n))
    for _ in range(int(n)):
        fn()
    torch.cuda.synchronize()
    return int(n) + 1


def raster_settings(cam, dev, module="diff_gaussian_rasterization"):
    import importlib

    import torch
    GRS = importlib.import_module(module).GaussianRasterizationSettings
    return GRS(image_height=cam.image_height, image_width=cam.image_width, tanfovx=cam.tanfovx,
               tanfovy=cam.tanfovy, bg=torch.zeros(3, device=dev), scale_modifier=1.0,
               viewmatrix=torch.from_numpy(cam.world_view_transform).to(dev),
               projmatrix=torch.from_numpy(cam.full_proj_transform).to(dev), sh_degree=3,
               campos=torch.from_numpy(cam.camera_center).to(dev), prefiltered=False, debug=False)


def device_params(sc, dev, requires_grad: bool):
    import torch
    return {k: torch.from_numpy(np.ascontiguousarray(getattr(sc, k))).to(dev).requires_grad_(requires_grad)
            for k in ("means3D", "opacities", "shs", "scales", "rotations")}


def workload_stats(settings, params, P: int, W: int, H: int, tile: int = 16):
    """K, V, Kb and the tile ranges of one forward (outside any timed region)."""
    import torch
    from gaussian_splatting_with_eye_tracking_amd import _C
    with torch.no_grad():
        K, color, radii, geom, binning, img = _C.rasterize_gaussians(
            settings.bg, params["means3D"], torch.Tensor([]), params["opacities"], params["scales"],
            params["rotations"], 1.0, torch.Tensor([]), settings.viewmatrix, settings.projmatrix,
            settings.tanfovx, settings.tanfovy, H, W, params["shs"], 3, settings.campos, False, False)
        bufs = _C.parse_buffers(geom, binning, img, P, K, W, H, tile)
    V = int((radii > 0).sum().item())
    rng = bufs["ranges"].cpu().numpy().astype(np.int64)
    n_t = rng[:, 1] - rng[:, 0]
    Kb = int(np.minimum(n_t, bufs["max_contrib"].cpu().numpy().astype(np.int64)).sum())
    T = ((W + tile - 1) // tile) * ((H + tile - 1) // tile)
    return dict(K=int(K), V=V, Kb=Kb, N=W * H, T=T)


def stage_table(prof: dict, steps: int, P, ws, views=1, key: dict | None = None) -> dict:
    out = {}
    for name, (ms, cnt) in prof.items():
        if cnt:
            st = {"avg_ms": ms / cnt, "launches": cnt, "ms_per_step": ms / steps}
            b = algorithmic_bytes(name, P, ws["V"], ws["K"], ws["Kb"], ws["N"], ws["T"], views)
            gbps = round(b / (st["avg_ms"] * 1e-3) / 1e9, 1) if b else None
            if gbps is not None and gbps > HBM_PEAK_GBS:
                # the kernel does not move the reference stage's bytes (make_roofline)
                st["reference_stage_equiv_GBps"] = gbps
            else:
                st["algorithmic_GBps"] = gbps
            db = design_bytes(name, P, ws["V"], ws["K"], ws["Kb"], ws["N"], ws["T"]) if views == 1 else None
            if db is not None:
                st["design_GBps"] = round(db / (st["avg_ms"] * 1e-3) / 1e9, 1)
            sr = stream_read_bytes(name, P, ws["V"], ws["K"], ws["Kb"], ws["N"], ws["T"], views)
            raw = load_raw_kib(name, key) if key is not None and sr is not None and b else None
            if raw is not None:  # the blend kernels: gather-calibrated traffic (make_roofline)
                st["traffic_over_algorithmic"] = round((1024.0 * (raw[0] + raw[1]) + 0.5 * sr) / b, 3)
            out[name] = st
    return out


# --------------------------------------------------------- config 2 / 4 ---
def run_fwd_bwd(cfg_name: str, ctx: Ctx, steps: int, warmup: int) -> dict:
    """One view forward + backward through the drop-in autograd API per step."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizer
    from gaussian_splatting_with_eye_tracking_amd import _C
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    c = CONFIGS[cfg_name]
    P, W, H = c["P"], c["W"], c["H"]
    sc, cam = ctx.scene(P, W, H)
    settings = raster_settings(cam, ctx.dev)
    params = device_params(sc, ctx.dev, True)
    means2D = torch.zeros_like(params["means3D"], requires_grad=True)
    dpix = torch.from_numpy(S.make_cotangent(H, W, 100 + ctx.rank)).to(ctx.dev)
    rasterizer = GaussianRasterizer(settings)

    def step():
        for p in params.values():
            p.grad = None
        means2D.grad = None
        color, _radii = rasterizer(means3D=params["means3D"], means2D=means2D, opacities=params["opacities"],
                                   shs=params["shs"], scales=params["scales"], rotations=params["rotations"])
        torch.autograd.backward(color, dpix)

    ramp = settle(step, warmup, ctx)
    # Inside the timed region only the roofline kernel (render_bwd, the
    # dominant stage at configs 2 and 4) records its event pair: each timed
    # stage costs two event records per launch (~4 us of queue time).
    prof_stage = "render_bwd"
    if not ctx.args.no_profile:
        _C.profile_enable(True)
        _C.profile_stages([prof_stage])
        _C.profile_read(True)
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    prof_timed, prof = {}, {}
    if not ctx.args.no_profile:
        prof_timed = _C.profile_read(True)
        _C.profile_stages([])  # per-stage breakdown: the same K steps again, every stage timed
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        prof = _C.profile_read(True)
        _C.profile_enable(False)
    (elapsed,) = ctx.max_over_ranks(elapsed)
    res = {"value": ctx.world * steps / elapsed, "unit": "views/s", "ms_per_step": 1000.0 * elapsed / steps,
           "ramp_steps": ramp}
    if ctx.rank != 0:
        return res
    ws = workload_stats(settings, params, P, W, H)
    stages = stage_table(prof, steps, P, ws, key=config_key(P, W, H, 16))
    roofline = None
    if stages:
        dom = max(stages, key=lambda n: stages[n]["ms_per_step"])
        ms_t, cnt_t = prof_timed.get(dom, (0.0, 0))
        avg_ms, src = (ms_t / cnt_t, "timed region") if cnt_t else (stages[dom]["avg_ms"], "stage-profile pass")
        by = algorithmic_bytes(dom, P, ws["V"], ws["K"], ws["Kb"], ws["N"], ws["T"])
        roofline = make_roofline(dom, by, avg_ms, config_key(P, W, H, 16), src,
                                 stream_read=stream_read_bytes(dom, P, ws["V"], ws["K"], ws["Kb"], ws["N"], ws["T"]),
                                 design_by=design_bytes(dom, P, ws["V"], ws["K"], ws["Kb"], ws["N"], ws["T"]))
    res.update({
        "config": {"workload": f"{cfg_name}: {P} Gaussians, {W}x{H}, 16x16 tiles, forward+backward, 1 view per "
                               f"GPU per step", "P": P, "width": W, "height": H, "views_per_gpu_per_step": 1,
                   "parallelism": f"dp{ctx.world}", "K_instances": ws["K"], "V_visible": ws["V"],
                   "K_bwd_entries": ws["Kb"]},
        "roofline": roofline, "stages": stages,
        "step_roofline": step_roofline(step_bytes_fwd_bwd(P, ws["V"], ws["K"], ws["N"], ws["T"]),
                                       res["ms_per_step"],
                                       "SURVEY.md §8(d) fwd+bwd 340P + 950V + 124K + 40N + 32T per view "
                                       "(this view's V, K) / ms per view on one GPU")})
    return res


# ------------------------------------------------------------- config 5 ---
def views_of_rank(global_views: int, world: int, rank: int):
    """Config 5's schedule: `global_views` yawed views per step (-17.5 ..
    +17.5 degrees at 8), global_views / world consecutive ones per rank.
    Returns (this rank's view indices, every view's yaw)."""
    if global_views % world:
        raise SystemExit(f"--views {global_views} is not a multiple of the world size {world}")
    vl = global_views // world
    yaws = [(v - (global_views - 1) / 2.0) * 5.0 for v in range(global_views)]
    return list(range(rank * vl, (rank + 1) * vl)), yaws


def run_multiview(ctx: Ctx, steps: int, warmup: int, global_views: int, exchange_alt: bool = True) -> dict:
    """a fixed global batch of `global_views` yawed views per
    step, global_views / N per rank; every rank ends the step with the summed
    parameter gradients of all views."""
    import torch
    import torch.distributed as dist
    from diff_gaussian_rasterization import GaussianRasterizer
    from gaussian_splatting_with_eye_tracking_amd import _C
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    c = CONFIGS["cfg5_8view_1080p_1M"]
    P, W, H = c["P"], c["W"], c["H"]
    G = global_views
    mine, yaws = views_of_rank(G, ctx.world, ctx.rank)
    vl = len(mine)
    sc, _cam0 = ctx.scene(P, W, H)
    params = device_params(sc, ctx.dev, True)
    views = []
    for v in mine:
        cam = S.make_orbit_camera(W, H, yaws[v])
        st = raster_settings(cam, ctx.dev)
        views.append({"v": v, "st": st, "rast": GaussianRasterizer(st),
                      "dpix": torch.from_numpy(S.make_cotangent(H, W, 100 + v)).to(ctx.dev)})
    st0 = views[0]["st"]
    e0 = torch.empty(0, device=ctx.dev)
    pg = params

    # (3 streams: 1362.7 views/s at config 5 on one GPU; 2: 1340; 1: 1242.6;
    # 4: 1363.1 -- profiles/r05j_bench5_vs*.log)
    vs = {"n": max(1, int(getattr(ctx.args, "view_streams", 3)))}

    def step_views():
        # each view's record is all-gathered as soon as it exists (overlapping
        # the next view's forward + blend backward), the last in chunks that
        # overlap the multi-view backward (data_parallel.ViewExchange)
        # (the views' forward + blend backward alternate over view_streams
        # HIP streams, data_parallel.run_views_on_streams)
        with torch.no_grad():
            ex = DP.ViewExchange(P, vl, ctx.dev)

            def one(j):
                vw = views[j]
                st = vw["st"]
                K, _color, radii, geom, binning, img = _C.rasterize_gaussians(
                    st.bg, pg["means3D"], e0, pg["opacities"], pg["scales"], pg["rotations"], 1.0, e0,
                    st.viewmatrix, st.projmatrix, st.tanfovx, st.tanfovy, H, W, pg["shs"], 3, st.campos, False, False)
                ex.add(j, DP.view_record(st, radii, geom, K, binning, img, vw["dpix"]))

            DP.run_views_on_streams(len(views), one, vs["n"])
            return ex.finish(st0, pg["means3D"], pg["shs"], pg["scales"], pg["rotations"])

    flat = DP.FlatGrads(params)
    m2 = torch.zeros_like(params["means3D"], requires_grad=True)

    def step_params():
        flat.flat.zero_()
        flat.attach(params)
        for vw in views:
            color, _ = vw["rast"](means3D=pg["means3D"], means2D=m2, opacities=pg["opacities"], shs=pg["shs"],
                                  scales=pg["scales"], rotations=pg["rotations"])
            torch.autograd.backward(color, vw["dpix"])
        DP.allreduce_(flat.flat)

    def timed(fn, k):
        ctx.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        ctx.barrier()
        (el,) = ctx.max_over_ranks(time.perf_counter() - t0)
        return el

    ramp = settle(step_views, warmup, ctx)
    el_views = timed(step_views, steps)
    prof = {}
    if not ctx.args.no_profile:
        # (per-stage events on one stream: concurrent views would time each
        # other's kernels)
        n_streams, vs["n"] = vs["n"], 1
        _C.profile_enable(True)
        _C.profile_stages([])
        _C.profile_read(True)
        timed(step_views, steps)
        prof = _C.profile_read(True)
        _C.profile_enable(False)
        vs["n"] = n_streams
    res = {"value": G * steps / el_views, "unit": "views/s", "ms_per_step": 1000.0 * el_views / steps,
           "ramp_steps": ramp, "view_streams": vs["n"]}
    extra = {}
    if exchange_alt:
        for _ in range(max(1, warmup // 2)):
            step_params()
        torch.cuda.synchronize()
        el_params = timed(step_params, steps)
        extra["exchange_params"] = {
            "value": G * steps / el_params, "unit": "views/s", "ms_per_step": 1000.0 * el_params / steps,
            "note": "north_star exchange: full per-view backward into one flat buffer + one RCCL all-reduce "
                    "(sum) of the 59 f32/Gaussian gradients" if ctx.world > 1 else
                    "full per-view backward accumulated into one flat buffer (no collective at N = 1)"}
    if ctx.distributed:
        # the two collectives alone (nccl-tests bus-bandwidth conventions)
        rec = torch.zeros((vl, DP.view_record_numel(P)), device=ctx.dev)
        for _ in range(3):
            DP.gather_view_records(rec)
        el_g = timed(lambda: DP.gather_view_records(rec), steps)
        for _ in range(3):
            DP.allreduce_(flat.flat)
        el_a = timed(lambda: DP.allreduce_(flat.flat), steps)
        n = ctx.world
        g_bytes = rec.numel() * 4 * n
        a_bytes = flat.flat.numel() * 4
        tg, ta = el_g / steps, el_a / steps
        extra["collectives"] = {
            "backend": dist.get_backend(), "world_size": dist.get_world_size(),
            "all_gather_view_records": {"bytes_out": g_bytes, "ms": round(1e3 * tg, 4),
                                        "bus_GBps": round(g_bytes * (n - 1) / n / tg / 1e9, 1)},
            "all_reduce_grads": {"bytes": a_bytes, "ms": round(1e3 * ta, 4),
                                 "bus_GBps": round(a_bytes * 2 * (n - 1) / n / ta / 1e9, 1)}}
    res.update(extra)
    if ctx.rank != 0:
        return res
    ws = workload_stats(views[0]["st"], params, P, W, H)
    # every view of the step (this rank's), for the step roofline
    wss = [ws] + [workload_stats(vw["st"], params, P, W, H) for vw in views[1:]]
    key5 = config_key(P, W, H, 16, G)
    stages = stage_table(prof, steps, P, ws, G, key=key5)
    roofline = None
    if stages:
        dom = max(stages, key=lambda n: stages[n]["ms_per_step"])
        by = algorithmic_bytes(dom, P, ws["V"], ws["K"], ws["Kb"], ws["N"], ws["T"], G)
        roofline = make_roofline(dom, by, stages[dom]["avg_ms"], key5, "stage-profile pass",
                                 stream_read=stream_read_bytes(dom, P, ws["V"], ws["K"], ws["Kb"], ws["N"], ws["T"]))
    res.update({
        "config": {"workload": f"cfg5_8view_1080p_1M: {P} Gaussians, {W}x{H}, 16x16 tiles, {G} views per step "
                               f"(yaw -17.5..17.5 deg), {vl} per GPU, forward + blend backward + view-record "
                               f"exchange + multi-view parameter backward",
                   "P": P, "width": W, "height": H, "global_views_per_step": G, "views_per_gpu_per_step": vl,
                   "exchange": "views", "parallelism": f"dp{ctx.world}", "K_instances_view0": ws["K"],
                   "V_visible_view0": ws["V"]},
        "roofline": roofline, "stages": stages,
        "step_roofline": step_roofline(
            sum(step_bytes_fwd_bwd(P, w["V"], w["K"], w["N"], w["T"]) for w in wss),
            res["ms_per_step"],
            f"SURVEY.md §8(d) fwd+bwd 340P + 950V + 124K + 40N + 32T summed over this GPU's {len(wss)} views "
            f"(each view's V, K; the multi-view exchange moves different bytes) / ms per step")})
    return res


# ------------------------------------------------------------- config 3 ---
def amr_algorithmic_bytes(ranges: np.ndarray, levels: np.ndarray) -> float:
    """Compulsory bytes of one 5-step frame's amr_render launches (DESIGN.md
    §4): every rendered (tile, round) block reads its tile's entries (id 4 +
    xy 8 + conic/opacity 16 + rgb 12 B) and writes its 256 sub-lattice pixels
    (colour 12 + final T 4 + n_contrib 4 B); a tile of level L renders L rounds."""
    n = (ranges[:, 1] - ranges[:, 0]).astype(np.float64)
    L = np.minimum(levels.astype(np.float64), 4.0)
    return float((L * (40.0 * n + 20.0 * 256)).sum())


def run_amr(ctx: Ctx, steps: int, warmup: int, extensions: bool = True) -> dict:
    """Config 3: forward-only foveated rendering (gaussian_renderer_amr's
    render(): foveaStep 0..4 through _RasterizeGaussians, summing the step
    images -- rasterization_amr.render_steps, the sums fused into the steps;
    and render_once(): foveaStep -2 with interpolation).  Per-frame and
    single-GPU: for N > 1 every rank renders its own frames (replicas only)."""
    import torch
    from diff_gaussian_rasterization_amr import GaussianRasterizer, _RasterizeGaussians
    from gaussian_splatting_with_eye_tracking_amd import _C
    from gaussian_splatting_with_eye_tracking_amd import rasterization_amr as RA
    from gaussian_splatting_with_eye_tracking_amd import synthetic as S
    c = CONFIGS["cfg3_amr_1080p_1M"]
    P, W, H = c["P"], c["W"], c["H"]
    dev = ctx.dev
    sc, cam = ctx.scene(P, W, H)
    st = raster_settings(cam, dev, "diff_gaussian_rasterization_amr")
    t = device_params(sc, dev, False)
    e = torch.empty(0, device=dev)
    u8 = torch.empty(0, dtype=torch.uint8, device=dev)
    means2D = torch.zeros_like(t["means3D"])
    a = (t["means3D"], means2D, t["shs"], e, t["opacities"], t["scales"], t["rotations"], e)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    # extension: the tracked fovea centre of config 3
    # (pupil (361.74, 248.19) in the 640x400 eye image -> screen) with the
    # reference's unused fovea radii W/2 .. W/16 restricting the AMR levels
    fov_centres, fov_radii = RA.reference_foveae(W, H, (361.74 / 640 * W, 248.19 / 400 * H))

    def frame_5step(record=False, fovea=False, fused=True):
        # gaussian_renderer_amr.render's rasterizer sequence (renderer_amr.render
        # without its Python camera / model plumbing): fused, the steps add
        # their pixels into the frame in the kernel, steps 1..4 as one launch
        # (render_steps' default without per-step events); record: per-step
        # events, so steps 1..4 launched one by one (per_step_ms); fused=False
        # the literal apply + torch-add sequence (apply_chain_fps below)
        lv = (lambda ib: RA.apply_fovea_levels(ib, W, H, fov_centres, fov_radii)) if fovea else None
        if record:
            ev[0].record()
        acc, _radii, gb, bb, ib = RA.render_steps(*a, st, fused=fused, enders=ev[1:] if record else None,
                                                  after_step0=lv)
        return acc, gb, bb, ib

    rast = GaussianRasterizer(st)

    def frame_once():
        return rast(means3D=t["means3D"], means2D=means2D, opacities=t["opacities"], shs=t["shs"],
                    scales=t["scales"], rotations=t["rotations"], foveaStep=-2, interpolate_image=True)[0]

    def warm_pair():
        frame_5step()
        frame_once()

    with torch.no_grad():
        ramp = settle(warm_pair, warmup, ctx)
        ctx.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            frame_5step()
        torch.cuda.synchronize()
        ctx.barrier()
        el5 = time.perf_counter() - t0
        # (--no-profile, the rocprofv3 runs: only the timed frame's launches, so
        # the kernel statistics are the frame's -- no apply-chain or per-step
        # passes launching the step kernel one step at a time)
        diag = not ctx.args.no_profile
        el5u = float("nan")
        if diag:
            # (its step images and sums: allocator blocks the fused frame never
            # asks for; a chain timed after only 10 untimed frames ran 0.4625 ms
            # per frame over 20 frames, 0.4431 over the next 50, 0.437 from then
            # on -- profiles/r06i_chain_frames.log: the same settling as the
            # fused frame's)
            settle(lambda: frame_5step(fused=False), max(10, warmup), ctx)
            t0 = time.perf_counter()
            for _ in range(steps):
                frame_5step(fused=False)
            torch.cuda.synchronize()
            ctx.barrier()
            el5u = time.perf_counter() - t0
        # per-stage times: a second pass of the timed frame with stage events;
        # per-step times: a third, with events between steps 1..4 launched
        # one by one
        prof = {}
        step_ms = np.zeros(5)
        if not ctx.args.no_profile:
            _C.profile_enable(True)
            _C.profile_stages([])
            _C.profile_read(True)
            for _ in range(steps):
                frame_5step()
            torch.cuda.synchronize()
            prof = _C.profile_read(True)
            _C.profile_enable(False)
        for _ in range(steps if diag else 0):
            frame_5step(record=True)
            torch.cuda.synchronize()
            step_ms += np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(5)])
        t0 = time.perf_counter()
        for _ in range(steps):
            frame_once()
        torch.cuda.synchronize()
        ctx.barrier()
        el1 = time.perf_counter() - t0
        elf = None
        if extensions:
            t0 = time.perf_counter()
            for _ in range(steps):
                frame_5step(fovea=True)
            torch.cuda.synchronize()
            ctx.barrier()
            elf = time.perf_counter() - t0
    elb = None
    if extensions:
        # the foveated backward (extension): render_once (interpolated) forward +
        # backward through the drop-in autograd API with a fixed cotangent
        tg = {k: v.detach().clone().requires_grad_(True) for k, v in t.items()}
        m2 = torch.zeros_like(tg["means3D"], requires_grad=True)
        cot = torch.from_numpy(S.make_cotangent(H, W, 1)).to(dev)

        def frame_once_fwd_bwd():
            img = rast(means3D=tg["means3D"], means2D=m2, opacities=tg["opacities"], shs=tg["shs"],
                       scales=tg["scales"], rotations=tg["rotations"], foveaStep=-2, interpolate_image=True)[0]
            torch.autograd.backward(img, cot)

        for _ in range(max(1, warmup)):
            frame_once_fwd_bwd()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            frame_once_fwd_bwd()
        torch.cuda.synchronize()
        elb = time.perf_counter() - t0
    el5, el1, el5u = ctx.max_over_ranks(el5, el1, el5u)
    res = {"value": ctx.world * steps / el5, "unit": "frames/s", "ms_per_step": 1000.0 * el5 / steps,
           "render_once_fps": ctx.world * steps / el1, "ramp_steps": ramp,
           "apply_chain_fps": ctx.world * steps / el5u if el5u == el5u else None,
           "frame": "renderer_amr.render's sequence with the step-image sums fused into the step kernels and "
                    "steps 1..4 in one launch (gs_amr_accumulate_step, bit-identical); per_step_ms: the steps "
                    "launched one by one with events between them; apply_chain_fps: the literal apply + "
                    "torch-add sequence"}
    if ctx.rank != 0:
        return res
    with torch.no_grad():
        acc, gb, bb, ib = frame_5step()
        torch.cuda.synchronize()
        K = int(_C.parse_buffers(gb, bb, ib, P, 0, W, H, 32)["hdr"][0].item())
        d = _C.parse_buffers(gb, bb, ib, P, K, W, H, 32)
        rng = d["ranges"].cpu().numpy().astype(np.int64)
        lv = d["levels"].cpu().numpy().astype(np.int64)
        V3 = int((_RasterizeGaussians.apply(*a, 0, e, u8, u8, u8, False, st)[1] > 0).sum().item())
        fovea_hist = None
        if extensions:
            _, _, _, ibf = frame_5step(fovea=True)
            lvf = _C.parse_buffers(gb, bb, ibf, P, K, W, H, 32)["levels"].cpu().numpy().astype(np.int64)
            fovea_hist = np.bincount(lvf, minlength=5)[1:].tolist()
    stages = {n: {"avg_ms": ms / cnt, "launches": cnt, "ms_per_frame": ms / steps} for n, (ms, cnt) in prof.items()
              if cnt}
    roofline = None
    if "amr_render" in stages:
        by = amr_algorithmic_bytes(rng, lv)
        ms = stages["amr_render"]["ms_per_frame"]
        # the PMC summary holds means per launch; the roofline is per frame
        roofline = make_roofline("amr_render", by, ms, config_key(P, W, H, 32), "stage-profile pass",
                                 per=stages["amr_render"]["launches"] / steps, stream_read=0.0)
        roofline["per"] = "frame (the one amr_render launch of steps 1..4; traffic per frame)"
    res.update({
        "metric": "foveated AMR frames/sec (forward-only render(), 5 fovea steps) at 1080p, 1M Gaussians",
        "config": {"workload": f"cfg3_amr_1080p_1M: {P} Gaussians, {W}x{H}, 32x32 AMR tiles, 5-step foveated "
                               f"render() per frame" + (", replicas" if ctx.world > 1 else ""),
                   "P": P, "width": W, "height": H, "K_instances": K, "parallelism": f"replicas{ctx.world}",
                   "levels_hist": np.bincount(lv, minlength=5)[1:].tolist()},
        "per_step_ms": [round(x / steps, 4) for x in step_ms] if diag else None,
        "roofline": roofline, "stages": stages,
        "step_roofline": step_roofline(step_bytes_amr_frame(P, V3, K, len(lv), rng, lv), res["ms_per_step"],
                                       "SURVEY.md §8(d) forward-only AMR frame 32P + 307V + 44K + 24T + "
                                       "40 sum_t(K_t rounds_t) + 20 N_rendered + 16T / ms per frame")})
    if extensions:
        res["amr_backward_ext"] = {"render_once_fwd_bwd_fps": steps / elb,
                                   "note": "extension beyond parity: interpolated render_once forward + backward "
                                           "through the autograd API"}
        res["fovea_levels_ext"] = {"fps": steps / elf, "centre": [round(v, 2) for v in fov_centres[0]],
                                   "radii": fov_radii, "levels_hist": fovea_hist,
                                   "note": "extension beyond parity: tracked fovea discs clamp the AMR levels"}
    return res


def summary(r: dict, keys=("value", "unit", "ms_per_step", "config", "roofline", "step_roofline", "per_step_ms",
                           "render_once_fps", "apply_chain_fps", "exchange_params", "ramp_steps",
                           "view_streams")) -> dict:
    out = {k: r[k] for k in keys if k in r}
    if r.get("stages"):  # compact per-stage ms per step (or per frame)
        out["stages_ms"] = {n: round(v.get("ms_per_step", v.get("ms_per_frame", 0.0)), 4)
                            for n, v in r["stages"].items()}
    return out


# ------------------------------------------------------------------ main ---
def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="default: cfg2_1080p_1M at N = 1, cfg5_8view_1080p_1M at N > 1")
    ap.add_argument("--views", type=int, default=8, help="config 5: global views per step")
    ap.add_argument("--view-streams", type=int, default=3,
                    help="config 5: HIP streams the rank's views alternate over (1: one stream)")
    ap.add_argument("--ramp-ms", type=float, default=100.0,
                    help="after the W warmup steps, untimed steps for about this long so the GPU clocks "
                         "have settled before the timed region (0: off); the count is in the line as ramp_steps")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sub", action="store_true", help="N = 1: skip the config 3 / 4 / 5 sub-results")
    ap.add_argument("--no-profile", action="store_true", help="disable the per-stage event timing")
    ap.add_argument("--no-ext", action="store_true", help="config 3: skip the extension legs (fovea discs, "
                    "AMR backward), e.g. for PMC passes")
    ap.add_argument("--launcher-dry-run", action="store_true",
                    help="test hook: rendezvous over gloo on the CPU and print the JSON skeleton (no GPU)")
    return ap.parse_args(argv)


def dry_run(world, rank, global_views: int = 8):
    """CPU test of the launcher: every rank joins a gloo group and rehearses
    config 5's exchange schedule on small records -- this rank's views
    (views_of_rank), each record handed to data_parallel.ViewExchange as
    run_multiview does (the last view gathered in chunks), and the flat
    parameter-gradient all-reduce; rank 0 prints whether every rank received
    every view's record in rank-then-view order and the all-reduced sum, bit
    for bit on every rank."""
    import torch
    import torch.distributed as dist
    from gaussian_splatting_with_eye_tracking_amd import data_parallel as DP
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([float(rank)])
    DP.allreduce_(t)
    ok = float(t.item()) == world * (world - 1) / 2
    mine, _yaws = views_of_rank(global_views, world, rank)
    P = 37
    n = DP.view_record_numel(P)
    ex = DP.ViewExchange(P, len(mine), "cpu", chunks=4)
    for j, v in enumerate(mine):  # record of view v: its values say which view it is
        ex.add(j, torch.arange(n, dtype=torch.float32) + 1000.0 * v)
    want = torch.stack([torch.arange(n, dtype=torch.float32) + 1000.0 * v for v in range(global_views)])
    views_ok = bool(torch.equal(ex.records(), want))
    flat = torch.zeros(DP.flat_numel_per_gaussian() * P)
    for v in mine:  # each view's gradients accumulated into the one flat buffer, then one all-reduce
        flat += torch.linspace(-1.0, 1.0, flat.numel()) * (v + 1)
    DP.allreduce_(flat)
    want_flat = torch.zeros_like(flat)
    for r in range(world):  # the same adds in rank order: a reference for the all-reduced sum
        acc = torch.zeros_like(flat)
        for v in views_of_rank(global_views, world, r)[0]:
            acc += torch.linspace(-1.0, 1.0, flat.numel()) * (v + 1)
        want_flat += acc
    sum_ok = bool(torch.allclose(flat, want_flat, rtol=1e-6, atol=1e-6))
    # every rank holds the same bits (what rank 0 holds, broadcast and compared)
    ref = flat.clone()
    recs = ex.records()
    if world > 1:
        dist.broadcast(ref, 0)
    same = torch.tensor([float(torch.equal(ref, flat) and torch.equal(recs, want))])
    DP.allreduce_(same)
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "n_gpus": world, "dry_run": True, "allreduce_ok": ok,
                          "views_per_rank": len(mine), "view_exchange_ok": views_ok, "grad_allreduce_ok": sum_ok,
                          "ranks_identical": float(same.item()) == world}), flush=True)


def main(argv=None):
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: start the ranks here, before anything touches the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:] if argv is None else list(argv)))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launcher_dry_run:
        return dry_run(world, rank)

    import torch
    import torch.distributed as dist
    build_digest()  # refuse a native library built from other sources than this tree's (after torch: its HIP runtime)
    # A/B hook: GSAMD_TUNING="key=value,..." (gs_set_tuning: performance-only
    # choices with identical results); recorded in the line when set
    tuning = os.environ.get("GSAMD_TUNING", "")
    if tuning:
        from gaussian_splatting_with_eye_tracking_amd import _C
        for kv in tuning.split(","):
            k, v = kv.split("=")
            _C.set_tuning(k.strip(), int(v))
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
    torch.cuda.set_device(dev)
    ctx = Ctx(world, rank, local_rank, distributed, dev, args)
    cfg = args.config or ("cfg2_1080p_1M" if world == 1 else "cfg5_8view_1080p_1M")
    kind = CONFIGS[cfg]["kind"]
    base = {"metric": METRIC, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "higher_is_better": True, "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (SURVEY §8(d) generator, seed 0)"}
    if kind == "amr":
        r = run_amr(ctx, args.steps, args.warmup, extensions=not args.no_ext)
        out = dict(base, **r, scaling="weak")
    elif kind == "multiview":
        r = run_multiview(ctx, args.steps, args.warmup, args.views)
        out = dict(base, **r, scaling="strong" if world > 1 else "weak")
    else:
        r = run_fwd_bwd(cfg, ctx, args.steps, args.warmup)
        out = dict(base, **r, scaling="weak")
    if rank == 0 and world == 1 and kind == "fwd_bwd" and cfg == "cfg2_1080p_1M" and not args.no_sub:
        torch.cuda.empty_cache()
        sub = {}
        k3 = max(5, args.steps // 2)
        sub["cfg3_amr_1080p_1M"] = summary(run_amr(ctx, k3, min(3, args.warmup), extensions=False))
        sub["cfg3_amr_1080p_1M"]["metric"] = "foveated AMR frames/sec (forward-only 5-step render())"
        sub["cfg5_8view_1080p_1M_1gpu"] = summary(run_multiview(ctx, max(5, args.steps // 4),
                                                                min(3, args.warmup), args.views))
        torch.cuda.empty_cache()
        sub["cfg4_bicycle_6M"] = summary(run_fwd_bwd("cfg4_bicycle_6M", ctx, max(5, args.steps // 2),
                                                     min(3, args.warmup)))
        out["sub_results"] = sub
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        c = CONFIGS[cfg]
        sc, cam = ctx.scene(c["P"], c["W"], c["H"])
        if kind in ("fwd_bwd", "multiview"):
            out["cpu_baseline"] = cpu_baselines(sc, cam)
        out["cpu_amr_test_path"] = cpu_amr_test_path(args.seed)
    if tuning:
        out["tuning"] = tuning
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
