#!/usr/bin/env bash
# round 4 session b: health, VALU probe, variant-8 parity and A/B, PMC read-back check
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04b
mkdir -p $O
export TMPDIR=/tmp
fault() { case "$1" in 0|1|5) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[r04b] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r04b] $name rc=$rc"; grep -v "^W2026\|^E2026" "$O/$name.log" | tail -n 4
  if fault "$rc"; then echo "[r04b] stop after fault-type exit $rc"; exit "$rc"; fi
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run rates 150 ./tools/valu_rate
run tests 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_readback.py tests/test_gpu_cull.py tests/test_gpu_multiview.py -k "readback or sgpr_mask or more_than_64 or cull_is_exact"
run tests_par 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "geometries_match_oracle and (8 or 7 or 9) or hint"
run tests_amr 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "fold_phases or mask_select"
run ab_amr_sel 400 python tools/ab_tuning.py --key amr_sel --values 1 2 1 2 --stage amr_render --amr --rounds 6
run ab_bwd2 400 python tools/ab_tuning.py --key bwd_variant --values 7 8 9 7 8 9 --stage render_bwd --backward --rounds 6
run ab_bwd4 400 python tools/ab_tuning.py --key bwd_variant --values 7 8 9 7 8 9 --stage render_bwd --backward --P 6100000 --W 1600 --H 1063 --rounds 4
run ab_fwd2 400 python tools/ab_tuning.py --key fwd_variant --values 5 7 5 7 --stage render --rounds 6
run ab_fwd4 400 python tools/ab_tuning.py --key fwd_variant --values 5 7 5 7 --stage render --P 6100000 --W 1600 --H 1063 --rounds 4
run pmc_waves 120 rocprofv3 --pmc SQ_WAVES --kernel-trace -d $O/pmc_waves -o run --output-format csv -- python3 bench.py --config cfg2_1080p_1M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext
GSAMD_HDR_MIRROR=1 run pmc_waves_m1 120 rocprofv3 --pmc SQ_WAVES --kernel-trace -d $O/pmc_waves_m1 -o run --output-format csv -- python3 bench.py --config cfg2_1080p_1M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext
run pmcA_cfg2 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d $O/pmcA_cfg2 -o run --output-format csv -- python3 bench.py --config cfg2_1080p_1M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext
for d in $O/pmc*; do [ -d "$d" ] && python3 tools/pmc_kernel.py "$d" --json > "$d.json"; done
echo "[r04b] done"
