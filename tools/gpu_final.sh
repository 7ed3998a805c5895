#!/usr/bin/env bash
# End-of-round evidence at the current build: GPU tests, smoke, the default
# bench line, rocprofv3 kernel stats + FETCH/WRITE/VALU counter passes for
# configs 2, 3, 4 and 5, summarised into profiles/ by tools/pmc_summary.py.
# usage: tools/gpu_final.sh <tag>     (e.g. r04z)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r04z}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_session.sh smoke tests bench prof2 pmc2 prof3 pmc3 prof4 pmc4 prof5 pmc5 || exit $?
for c in cfg2_1080p_1M cfg3_amr_1080p_1M cfg4_bicycle_6M cfg5_8view_1080p_1M; do
  python3 tools/pmc_summary.py --tag "$TAG" --config "$c" --out gpurun_out/profiles > "gpurun_out/summary_$c.log" 2>&1 || echo "summary $c failed"
done
echo "[final] done"
