#!/usr/bin/env bash
# round 4 session zh: binning chunk (Gaussians per count / LDS-duplicate workgroup) at configs 2 and 3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04zh
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04zh] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04zh] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04zh] stop after fault-type exit $rc"; exit "$rc"; fi
}
run ab_c2 400 python tools/ab_tuning.py --key bin_chunk --values 4096 2048 1024 4096 2048 1024 --stage count_tiles --rounds 4
run ab_c3 400 python tools/ab_tuning.py --key bin_chunk --values 4096 2048 1024 4096 2048 1024 --stage count_tiles --amr --rounds 4
run ab_d3 400 python tools/ab_tuning.py --key bin_chunk --values 4096 2048 1024 4096 2048 1024 --stage duplicate --amr --rounds 4
echo "[r04zh] done"
