"""tools/pmc_summary.py: counters and durations keyed by full kernel name,
stages as launch-weighted sums over their kernels (never an overwrite or a
mean that mixes kernels), and bench.py attaching only summaries of the same
configuration and build."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

import pmc_summary as PS  # noqa: E402


def test_short_name_strips_arguments_not_template():
    n = "void gsamd::sort_tiles_small_kernel<16>(int, int, unsigned int const*, unsigned long const*, unsigned int*)"
    assert PS.short_name(n) == "gsamd::sort_tiles_small_kernel<16>"
    assert PS.short_name("gsamd::count_tiles_kernel(int, int)") == "gsamd::count_tiles_kernel"


def test_two_kernel_stage_is_summed_per_invocation():
    # config 4's sort: the E = 16 network (460 us) and the wide kernel (5 us),
    # each launched once per forward (14 forwards) -- the stage is their sum
    stats = {"gsamd::sort_tiles_small_kernel<16>": (14, 460_000.0),
             "gsamd::sort_tiles_wide_kernel<512>": (14, 5_000.0),
             "gsamd::sort_tiles_small_kernel<4>": (14, 5_000.0),
             "gsamd::preprocess_kernel<true, true, false>": (14, 422_000.0)}
    fetch = {"gsamd::sort_tiles_small_kernel<16>": [100_000.0] * 5,
             "gsamd::sort_tiles_wide_kernel<512>": [1_000.0] * 5,
             "gsamd::sort_tiles_small_kernel<4>": [2_000.0] * 5}
    write = {"gsamd::sort_tiles_small_kernel<16>": [50_000.0] * 5,
             "gsamd::sort_tiles_wide_kernel<512>": [500.0] * 5,
             "gsamd::sort_tiles_small_kernel<4>": [700.0] * 5}
    r = PS.summarise(fetch, write, None, stats)
    assert abs(r["kernel_avg_us"]["sort_tiles"] - 470.0) < 1e-9
    assert abs(r["kernel_avg_us"]["preprocess"] - 422.0) < 1e-9
    assert r["raw_kib"]["sort_tiles"]["FETCH_SIZE"] == 103_000.0
    assert r["raw_kib"]["sort_tiles"]["WRITE_SIZE"] == 51_200.0
    assert r["per_launch_hbm_bytes"]["sort_tiles"] == (2 * 103_000.0 + 51_200.0) * 1024
    assert set(r["kernels"]) == set(stats)  # every kernel keeps its own row
    assert r["implausible"] == {}


def test_rarer_kernel_is_weighted_by_its_launches():
    # a kernel launched on every other invocation adds half its mean
    stats = {"gsamd::sort_tiles_small_kernel<4>": (10, 100_000.0),
             "gsamd::sort_tiles_wide_kernel<512>": (5, 40_000.0)}
    r = PS.summarise(None, None, None, stats)
    assert abs(r["kernel_avg_us"]["sort_tiles"] - 120.0) < 1e-9


def test_implausible_stage_is_flagged():
    stats = {"gsamd::count_tiles_kernel": (4, 1_000.0)}        # 1 us
    fetch = {"gsamd::count_tiles_kernel": [10_000.0] * 4}      # 20 MB corrected in 1 us
    write = {"gsamd::count_tiles_kernel": [0.0] * 4}
    r = PS.summarise(fetch, write, None, stats)
    assert "count_tiles" in r["implausible"]


def test_bench_attaches_only_same_build(tmp_path, monkeypatch):
    import bench
    key = bench.config_key(10, 20, 30, 16)
    good = {"config": key, "build": bench.build_digest(), "per_launch_hbm_bytes": {"render": 1.0}}
    stale = {"config": key, "build": "0" * 16, "per_launch_hbm_bytes": {"render": 2.0}}
    (tmp_path / "r01_x_pmc_summary.json").write_text(json.dumps(good))
    (tmp_path / "r02_x_pmc_summary.json").write_text(json.dumps(stale))  # newer, other build
    monkeypatch.setattr(bench, "_pmc_files", lambda: sorted(str(p) for p in tmp_path.glob("*pmc_summary.json")))
    v, src = bench.load_pmc("render", key, "per_launch_hbm_bytes")
    assert v == 1.0 and src.endswith("r01_x_pmc_summary.json")
    assert bench.load_pmc("render", bench.config_key(1, 2, 3, 16), "per_launch_hbm_bytes") is None
