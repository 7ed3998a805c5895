#!/usr/bin/env bash
# round 4 session s: forward variant 9 vs 8 without hit-code recording (the quadrant cull alone)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04s
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04s] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04s] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04s] stop after fault-type exit $rc"; exit "$rc"; fi
}
run ab_fwd2_nocodes 400 python tools/ab_tuning.py --key fwd_variant --values 8 9 8 9 --stage render --rounds 6 --set hit_codes=0
echo "[r04s] done"
