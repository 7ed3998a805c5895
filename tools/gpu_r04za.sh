#!/usr/bin/env bash
# round 4 session za: tile scan with the (slice, wave) totals prefixed by one wave
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04za
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04za] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04za] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04za] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_parity_configs.py -k "bit_exact or scan or amr_foveated or config"
run ab_scan2 400 python tools/ab_tuning.py --key scan_slices --values 0 1 0 1 --stage tile_scan --rounds 6
run ab_scan4 400 python tools/ab_tuning.py --key scan_slices --values 0 1 0 1 --stage tile_scan --P 6100000 --W 1600 --H 1063 --rounds 4
echo "[r04za] done"
