#!/usr/bin/env bash
# round 4 session z2: AMR region lists in XCD-compact strips (amr_lists_order 2) against heaviest-first (1) and tile order (0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04z2
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04z2] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04z2] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04z2] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "amr_fold_phases"
run ab_lorder 400 python tools/ab_tuning.py --key amr_lists_order --values 1 2 0 1 2 0 --stage amr_lists --amr --rounds 6
echo "[r04z2] done"
