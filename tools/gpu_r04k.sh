#!/usr/bin/env bash
# round 4 session k: full GPU suite + bench at the current build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04k] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04k] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04k] stop after fault-type exit $rc"; exit "$rc"; fi
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run tests 900 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests
run bench 400 python bench.py --steps 20 --warmup 5
echo "[r04k] done"
