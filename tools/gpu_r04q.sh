#!/usr/bin/env bash
# round 4 session q: AMR fold without the power test in safe batches (amr_sel 3); region lists in heaviest-first tile order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04q
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04q] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04q] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04q] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "amr"
run ab_sel 400 python tools/ab_tuning.py --key amr_sel --values 1 3 1 3 --stage amr_render --amr --rounds 6
run ab_lorder 400 python tools/ab_tuning.py --key amr_lists_order --values 0 1 0 1 --stage amr_lists --amr --rounds 6
echo "[r04q] done"
