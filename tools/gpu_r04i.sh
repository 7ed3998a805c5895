#!/usr/bin/env bash
# round 4 session i: AMR percentiles by the two-pass histogram select
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04i] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04i] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04i] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "amr"
run ab_lvl 400 python tools/ab_tuning.py --key amr_levels_hist --values 0 1 0 1 --stage amr_levels --amr --rounds 6
run bench3 400 python bench.py --config cfg3_amr_1080p_1M --steps 20 --warmup 3 --no-cpu-baseline
echo "[r04i] done"
