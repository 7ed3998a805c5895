#!/usr/bin/env bash
# round 4 session e: pipelined preprocess (pp_dma 2) and unrolled-slot backward (variant 10): parity, A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04e] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04e] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04e] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "forward_buffers_bit_exact or preprocess_forms or (geometries_match_oracle and 10)"
run tests_cull 300 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_cull.py -k sgpr_mask
run ab_pp2 400 python tools/ab_tuning.py --key pp_dma --values 1 2 1 2 --stage preprocess --backward --rounds 6
run ab_pp4 400 python tools/ab_tuning.py --key pp_dma --values 1 2 1 2 --stage preprocess --backward --P 6100000 --W 1600 --H 1063 --rounds 4
run ab_pp3 400 python tools/ab_tuning.py --key pp_dma --values 1 2 1 2 --stage preprocess --amr --rounds 6
run ab_bwd2 400 python tools/ab_tuning.py --key bwd_variant --values 9 10 9 10 --stage render_bwd --backward --rounds 6
run ab_bwd4 400 python tools/ab_tuning.py --key bwd_variant --values 9 10 9 10 --stage render_bwd --backward --P 6100000 --W 1600 --H 1063 --rounds 4
echo "[r04e] done"
