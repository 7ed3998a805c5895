#!/usr/bin/env bash
# round 4 session z6: preprocess non-temporal SH DMA loads (pp_nt bit 0) and drgb stores (bit 1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04z6
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04z6] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04z6] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04z6] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pp_dma or preprocess_forms"
run ab_pp2 400 python tools/ab_tuning.py --key pp_nt --values 0 1 2 3 0 1 2 3 --stage preprocess --rounds 4
run ab_pp4 600 python tools/ab_tuning.py --key pp_nt --values 0 1 2 3 0 1 2 3 --stage preprocess --P 6100000 --W 1600 --H 1063 --rounds 3
run ab_ppstep4 600 python tools/ab_tuning.py --key pp_nt --values 0 3 0 3 --stage step --backward --P 6100000 --W 1600 --H 1063 --rounds 6
echo "[r04z6] done"
