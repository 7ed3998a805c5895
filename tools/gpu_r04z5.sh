#!/usr/bin/env bash
# round 4 session z5: non-temporal stores for the other bwd_gauss outputs (bg_nt 3) and the forward zeroing (zero_nt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04z5
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04z5] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04z5] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04z5] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "gauss_store_forms"
run ab_nt2 400 python tools/ab_tuning.py --key bg_nt --values 1 3 1 3 --stage bwd_gauss --backward --rounds 6
run ab_nt4 600 python tools/ab_tuning.py --key bg_nt --values 1 3 1 3 --stage bwd_gauss --backward --P 6100000 --W 1600 --H 1063 --rounds 6
run ab_znt2 400 python tools/ab_tuning.py --key zero_nt --values 0 1 0 1 --stage step --backward --rounds 6 --set bg_nt=1
run ab_znt4 600 python tools/ab_tuning.py --key zero_nt --values 0 1 0 1 --stage step --backward --P 6100000 --W 1600 --H 1063 --rounds 6 --set bg_nt=1
echo "[r04z5] done"
