#!/usr/bin/env bash
# round 4 session u: XCD-compact backward tile order (xcd_map bit 1) against the global heaviest-first bucket order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04u
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04u] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04u] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04u] stop after fault-type exit $rc"; exit "$rc"; fi
}
run ab_xcd2 400 python tools/ab_tuning.py --key xcd_map --values 1 3 1 3 --stage render_bwd --backward --rounds 6
run ab_xcd4 400 python tools/ab_tuning.py --key xcd_map --values 1 3 1 3 --stage render_bwd --backward --P 6100000 --W 1600 --H 1063 --rounds 4
echo "[r04u] done"
