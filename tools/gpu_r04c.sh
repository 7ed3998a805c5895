#!/usr/bin/env bash
# round 4 session c: backward variant 9 as default -- smoke, the GPU suite,
# the default bench line, kernel stats and one PMC pass (torch-first load fix)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04c] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04c] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04c] stop after fault-type exit $rc"; exit "$rc"; fi
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pmc_waves 150 rocprofv3 --pmc SQ_WAVES --kernel-trace -d $O/pmc_waves -o run --output-format csv -- python3 bench.py --config cfg2_1080p_1M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext
run tests 900 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests
run bench 400 python bench.py --steps 20 --warmup 5
run prof2 300 rocprofv3 --kernel-trace --stats -d $O/prof2 -o run --output-format csv -- python3 bench.py --config cfg2_1080p_1M --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-sub --no-ext
echo "[r04c] done"
