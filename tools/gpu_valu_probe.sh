#!/usr/bin/env bash
# Round 4: the VALU issue rate, settled by exact instruction streams
# (tools/valu_rate.hip, inline-asm bodies) and by the SQ utilisation counters
# of the probe itself and of the two blend kernels at config 2.
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/valu
export TMPDIR=/tmp
O=gpurun_out/valu
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[probe] $(date +%T) $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1 || { echo "[probe] $name failed rc=$?"; tail -n 20 "$O/$name.log"; exit 1; }
}
CNT_A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
CNT_B="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
step rates 120 ./tools/valu_rate
cat "$O/rates.log"
for w in 1 8; do
  step "pmcA_fma_w$w" 60 rocprofv3 --pmc $CNT_A --kernel-trace -d "$O/pmcA_fma_w$w" -o run --output-format csv -- ./tools/valu_rate "v_fma_f32 v,v,k,k" $w
  step "pmcB_fma_w$w" 60 rocprofv3 --pmc $CNT_B --kernel-trace -d "$O/pmcB_fma_w$w" -o run --output-format csv -- ./tools/valu_rate "v_fma_f32 v,v,k,k" $w
  step "pmcA_mul_w$w" 60 rocprofv3 --pmc $CNT_A --kernel-trace -d "$O/pmcA_mul_w$w" -o run --output-format csv -- ./tools/valu_rate v_mul_f32 $w
done
step pmcA_exp_w8 60 rocprofv3 --pmc $CNT_A --kernel-trace -d "$O/pmcA_exp_w8" -o run --output-format csv -- ./tools/valu_rate v_exp_f32 8
step pmcA_salu_w8 60 rocprofv3 --pmc $CNT_A --kernel-trace -d "$O/pmcA_salu_w8" -o run --output-format csv -- ./tools/valu_rate "v_mul_f32 + 2 SALU (1:2)" 8
step pmcA_cfg2 300 rocprofv3 --pmc $CNT_A --kernel-trace -d "$O/pmcA_cfg2" -o run --output-format csv -- python3 bench.py --config cfg2_1080p_1M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext
step pmcB_cfg2 300 rocprofv3 --pmc $CNT_B --kernel-trace -d "$O/pmcB_cfg2" -o run --output-format csv -- python3 bench.py --config cfg2_1080p_1M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext
for d in "$O"/pmc*; do
  [ -d "$d" ] && python3 tools/pmc_kernel.py "$d" --json > "$d.json"
done
echo "[probe] done"
