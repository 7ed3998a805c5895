#!/usr/bin/env bash
# round 4 session ze: multiview backward with the SH rows' loads issued back to back
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04ze
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04ze] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04ze] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04ze] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_multiview.py tests/test_gpu_dist_views.py
run bench5 600 python bench.py --config cfg5_8view_1080p_1M --steps 10 --warmup 3 --no-cpu-baseline
echo "[r04ze] done"
