#!/usr/bin/env bash
# round 4 session z3: forward variant 9 (the wave leaves its chunk once every pixel has finished, tested per pair of entries)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04z3
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04z3] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04z3] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04z3] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_cull.py tests/test_gpu_parity.py -k "cull or sgpr_mask_forward or (geometries_match_oracle and (9- or 11-))"
run ab_fwd2 400 python tools/ab_tuning.py --key fwd_variant --values 8 9 8 9 8 9 --stage render --rounds 6
run ab_fwd4 400 python tools/ab_tuning.py --key fwd_variant --values 8 9 8 9 8 9 --stage render --P 6100000 --W 1600 --H 1063 --rounds 4
echo "[r04z3] done"
