#!/usr/bin/env bash
# round 4 session y: bwd_gauss stage 2 vs 3 (drgb-known kernel) at config 4 with 48-B grad rows, more rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04y
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04y] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04y] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04y] stop after fault-type exit $rc"; exit "$rc"; fi
}
run ab_bg4 600 python tools/ab_tuning.py --key bg_stage_mlp --values 2 3 2 3 --stage bwd_gauss --backward --P 6100000 --W 1600 --H 1063 --rounds 8
echo "[r04y] done"
