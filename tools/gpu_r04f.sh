#!/usr/bin/env bash
# round 4 session f: staged preprocess records (pp_dma 3), backward variant 10 default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04f] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04f] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04f] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "forward_buffers_bit_exact or preprocess_forms or staged_preprocess or amr_foveated_steps"
run ab_pp2 400 python tools/ab_tuning.py --key pp_dma --values 1 3 1 3 --stage preprocess --backward --rounds 6
run ab_pp4 400 python tools/ab_tuning.py --key pp_dma --values 1 3 1 3 --stage preprocess --backward --P 6100000 --W 1600 --H 1063 --rounds 4
run ab_pp3 400 python tools/ab_tuning.py --key pp_dma --values 1 3 1 3 --stage preprocess --amr --rounds 6
echo "[r04f] done"
