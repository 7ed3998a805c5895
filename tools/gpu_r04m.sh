#!/usr/bin/env bash
# round 4 session m: backward variants 11 (flush fused into the staging reduce) and 12 (11 at 5 waves/SIMD)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04m] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04m] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04m] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_cull.py -k "(geometries_match_oracle and (10 or 11 or 12)) or sgpr_mask or unfilled_work or backward_parity"
run ab_bwd2 400 python tools/ab_tuning.py --key bwd_variant --values 10 11 12 10 11 12 --stage render_bwd --backward --rounds 6
run ab_bwd4 400 python tools/ab_tuning.py --key bwd_variant --values 10 11 12 10 11 12 --stage render_bwd --backward --P 6100000 --W 1600 --H 1063 --rounds 4
echo "[r04m] done"
