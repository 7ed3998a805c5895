#!/usr/bin/env bash
# round 4 session z7: non-temporal geometry loads in the preprocess (pp_nt bit 2) and the Gaussian backward (bg_nt bit 2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04z7
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04z7] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04z7] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04z7] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pp_dma or preprocess_forms or gauss_store_forms"
run ab_pp2 400 python tools/ab_tuning.py --key pp_nt --values 3 7 3 7 --stage preprocess --backward --rounds 6
run ab_pp4 600 python tools/ab_tuning.py --key pp_nt --values 3 7 3 7 --stage preprocess --backward --P 6100000 --W 1600 --H 1063 --rounds 4
run ab_bg2 400 python tools/ab_tuning.py --key bg_nt --values 1 5 1 5 --stage bwd_gauss --backward --rounds 6
run ab_bg4 600 python tools/ab_tuning.py --key bg_nt --values 1 5 1 5 --stage bwd_gauss --backward --P 6100000 --W 1600 --H 1063 --rounds 4
echo "[r04z7] done"
