#!/usr/bin/env bash
# round 4 session j: bwd_gauss without scratch + staged 3-float outputs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04j
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04j] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04j] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04j] stop after fault-type exit $rc"; exit "$rc"; fi
}
run tests 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multiview.py -k "backward_parity or gauss_store or multiview or bwd_gauss"
run ab_bg2 400 python tools/ab_tuning.py --key bg_stage_mlp --values 1 2 1 2 --stage bwd_gauss --backward --rounds 6
run ab_bg4 400 python tools/ab_tuning.py --key bg_stage_mlp --values 1 2 1 2 --stage bwd_gauss --backward --P 6100000 --W 1600 --H 1063 --rounds 4
run pmc_w4 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_w4 -o run --output-format csv -- python3 bench.py --config cfg4_bicycle_6M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext
run pmc_f4 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_f4 -o run --output-format csv -- python3 bench.py --config cfg4_bicycle_6M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext
echo "[r04j] done"
