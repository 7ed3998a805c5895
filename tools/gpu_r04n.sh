#!/usr/bin/env bash
# round 4 session k: full GPU suite + bench at the current build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04n
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04n] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04n] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04n] stop after fault-type exit $rc"; exit "$rc"; fi
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run tests 900 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests
run bench 400 python bench.py --steps 20 --warmup 5
run ab_zero2_render 400 python tools/ab_tuning.py --key fwd_zero --values 1 0 1 0 --stage render --backward --rounds 6
run ab_zero2_zero 400 python tools/ab_tuning.py --key fwd_zero --values 1 0 1 0 --stage zero_accum --backward --rounds 6
run ab_zero4_render 400 python tools/ab_tuning.py --key fwd_zero --values 1 0 1 0 --stage render --backward --P 6100000 --W 1600 --H 1063 --rounds 4
run ab_zero4_zero 400 python tools/ab_tuning.py --key fwd_zero --values 1 0 1 0 --stage zero_accum --backward --P 6100000 --W 1600 --H 1063 --rounds 4
run ab_bg2 400 python tools/ab_tuning.py --key bg_stage_mlp --values 2 3 2 3 --stage bwd_gauss --backward --rounds 6
run ab_bg4 400 python tools/ab_tuning.py --key bg_stage_mlp --values 2 3 2 3 --stage bwd_gauss --backward --P 6100000 --W 1600 --H 1063 --rounds 4
echo "[r04n] done"
