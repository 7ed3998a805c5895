"""bench.py's own launcher (no GPU): `bench.py --gpus N` without WORLD_SIZE
starts N ranks itself; under a launcher WORLD_SIZE must equal --gpus."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_starts_its_own_ranks(n):
    """`bench.py --gpus N` (the driver's N = 2, 4, 8 scaling runs) starts N
    ranks, and each rehearses config 5's exchange schedule over gloo: 8 / N
    views per rank, the pipelined view-record gather (at N = 8 one view per
    rank: only the chunked last-view path) and the flat gradient all-reduce,
    bit-identical on every rank."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launcher-dry-run"],
                       capture_output=True, text=True, env=_env(), timeout=280)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    L = lines[0]
    assert L["n_gpus"] == n and L["allreduce_ok"] and L["views_per_rank"] == 8 // n
    assert L["view_exchange_ok"] and L["grad_allreduce_ok"] and L["ranks_identical"]


@pytest.mark.timeout(120)
def test_bench_rejects_world_size_mismatch():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launcher-dry-run"],
                       capture_output=True, text=True, env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       timeout=100)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr


@pytest.mark.timeout(120)
def test_bench_single_rank_dry_run():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--launcher-dry-run"],
                       capture_output=True, text=True, env=_env(), timeout=100)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1
