#!/usr/bin/env bash
# round 4 session l: binning chunk size A/B (count_tiles + duplicate), configs 2 and 4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04l] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04l] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04l] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "thread_contiguous or forward_buffers or forward_only_hint"
for st in count_tiles duplicate; do
  run ab_chunk4_$st 400 python tools/ab_tuning.py --key bin_chunk --values 4096 8192 16384 2048 4096 8192 16384 2048 --stage $st --P 6100000 --W 1600 --H 1063 --rounds 3
  run ab_chunk2_$st 400 python tools/ab_tuning.py --key bin_chunk --values 4096 8192 2048 1024 4096 8192 2048 1024 --stage $st --rounds 4
done
run tests_m 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_cull.py -k "(geometries_match_oracle and (10 or 11 or 12)) or sgpr_mask or unfilled_work or backward_parity"
run ab_bwd2_m 400 python tools/ab_tuning.py --key bwd_variant --values 10 11 12 10 11 12 --stage render_bwd --backward --rounds 6
run ab_bwd4_m 400 python tools/ab_tuning.py --key bwd_variant --values 10 11 12 10 11 12 --stage render_bwd --backward --P 6100000 --W 1600 --H 1063 --rounds 4
echo "[r04l] done"
