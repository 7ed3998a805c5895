#!/usr/bin/env bash
# Guarded GPU session for gpurun: every GPU step has its own time limit and
# the script stops at the first fault-type exit (abort/segv/timeout).  A
# pytest exit code of 1 (test failures) is not a fault and does not stop it.
# usage: [GS_TAG=r05a] tools/gpu_session.sh <step> [<step> ...]   steps: tests smoke bench prof pmc ...
# logs go to gpurun_out/$GS_TAG/ (default gpurun_out/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${GS_TAG:-}
mkdir -p "$O"
export TMPDIR=/tmp
# the digest of the native sources this session runs (tools/pmc_summary.py records it)
python -c "import bench; print(bench.build_digest())" > gpurun_out/build_digest.txt
cp gpurun_out/build_digest.txt "$O/build_digest.txt"
fault() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[gpu_session] $(date +%T) start $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[gpu_session] $(date +%T) end $name rc=$rc"
  tail -n 5 "$O/$name.log"
  if fault "$rc"; then echo "[gpu_session] stopping after fault-type exit $rc in $name"; exit "$rc"; fi
  return 0
}
cfg_of() { case "$1" in *2) echo cfg2_1080p_1M;; *3) echo cfg3_amr_1080p_1M;; *4) echo cfg4_bicycle_6M;; *5) echo cfg5_8view_1080p_1M;; esac; }
for step in "$@"; do
  case "$step" in
    probe) run probe 60 bash -c 'echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>&1)"; echo "cfs: $(cat /sys/fs/cgroup/cpu/cpu.cfs_quota_us 2>&1) / $(cat /sys/fs/cgroup/cpu/cpu.cfs_period_us 2>&1)"; echo "nproc $(nproc) OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset}"; python3 -c "import bench; print(bench.cpu_share())"' ;;
    gaptrace) run gaptrace 600 rocprofv3 --kernel-trace -d "$O/gaptrace" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub ;;
    benchns) run bench_ns 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub ;;
    ab) run "ab_${AB_NAME:-x}" 600 python tools/ab_tuning.py $AB_ARGS ;;
    ab2) run "ab_${AB_NAME:-x}_2" 600 python tools/ab_tuning.py $AB_ARGS2 ;;
    pytestk) run "pytest_${PT_NAME:-k}" 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -rf -k "$PT_K" ;;
    tests) run pytest_gpu 900 python -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 -rf ;;
    configs) run pytest_configs 1100 python -u -m pytest tests/test_gpu_parity_configs.py tests/test_gpu_parity.py -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread -rf ;;
    amrtests) run pytest_amr 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_configs.py tests/test_gpu_cull.py -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread -rf -k "amr or config3 or cull" ;;
    parity) run pytest_parity 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_cull.py -q -m gpu -p no:cacheprovider --timeout 300 -rf ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5 ;;
    benchdef) run bench_default 600 python bench.py ;;  # the driver's exact command
    bench3) run bench_cfg3 600 python bench.py --config cfg3_amr_1080p_1M --steps 20 --warmup 3 ;;
    bench4) run bench_cfg4 600 python bench.py --config cfg4_bicycle_6M --steps 10 --warmup 3 --no-cpu-baseline ;;
    dist2) GS_BENCH_SHARE_DEVICE=1 GS_BENCH_BACKEND=gloo run bench_dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 ;;
    dist2l) GS_BENCH_SHARE_DEVICE=1 GS_BENCH_BACKEND=gloo run bench_dist2_launcher 600 python bench.py --gpus 2 --steps 5 --warmup 2 ;;
    dist2amr) GS_BENCH_SHARE_DEVICE=1 GS_BENCH_BACKEND=gloo run bench_dist2amr 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --config cfg3_amr_1080p_1M ;;
    benchnp) run bench_np 400 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-profile &&
             run bench_p 400 python bench.py --steps 50 --warmup 5 --no-cpu-baseline ;;
    benchq) run bench 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    prof) run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile ;;
    pmc_issue2) run pmc_issue2 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_issue2 -o run --output-format csv -- python3 bench.py --config cfg2_1080p_1M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext ;;
    pmc_issue4) run pmc_issue4 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_issue4 -o run --output-format csv -- python3 bench.py --config cfg4_bicycle_6M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext ;;
    mv) run pytest_mv 400 python -m pytest tests/test_gpu_multiview.py tests/test_gpu_dist_views.py -q -m gpu -p no:cacheprovider --timeout 300 -rf &&
        run bench_exchange 400 python tools/bench_exchange.py ;;
    eye) run pytest_eye 400 python -m pytest tests/test_gpu_eye_tracking.py -q -m gpu -p no:cacheprovider --timeout 300 -rf &&
         run bench_eye 300 python tools/bench_eye.py ;;
    gputrain) run pytest_gpu_train 600 python -m pytest tests/test_gpu_training.py tests/test_loss.py -q -m gpu -p no:cacheprovider --timeout 300 -rf ;;
    train) run bench_train 600 python tools/bench_train.py ;;
    proftrain) run rocprof_train 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- python3 tools/bench_train.py --reps 10 ;;
    prof2|prof3|prof4|prof5)
      c=$(cfg_of "$step"); run "rocprof_$c" 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$c" -o run --output-format csv -- python3 bench.py --config "$c" --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-sub --no-ext ;;
    pmc2|pmc3|pmc4|pmc5)  # one counter per pass (separate runs), MI355X_MICROARCH.md HBM recipe
      c=$(cfg_of "$step")
      run "pmc_${c}_fetch" 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "gpurun_out/pmc_${c}_fetch" -o run --output-format csv -- python3 bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext &&
      run "pmc_${c}_write" 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "gpurun_out/pmc_${c}_write" -o run --output-format csv -- python3 bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext &&
      run "pmc_${c}_valu" 300 rocprofv3 --pmc SQ_INSTS_VALU --kernel-trace -d "gpurun_out/pmc_${c}_valu" -o run --output-format csv -- python3 bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext ;;
    gaptrace3) run gaptrace3 600 rocprofv3 --kernel-trace -d "$O/gaptrace3" -o run --output-format csv -- python3 bench.py --config cfg3_amr_1080p_1M --steps 20 --warmup 3 --no-cpu-baseline --no-ext ;;
    bench5) run bench_cfg5 600 python bench.py --config cfg5_8view_1080p_1M --steps 10 --warmup 3 --no-cpu-baseline ;;
    trace3) run trace_cfg3 300 rocprofv3 --kernel-trace -d gpurun_out/trace_cfg3 -o run --output-format csv -- python3 bench.py --config cfg3_amr_1080p_1M --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-ext ;;
    sqa2|sqa3|sqa4|sqa5|sqb2|sqb3|sqb4|sqb5)  # SQ issue / wait counters per kernel (two 8-counter sets)
      c=$(cfg_of "$step")
      case "$step" in
        sqa*) cnt="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" ;;
        *) cnt="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" ;;
      esac
      run "${step}_$c" 300 rocprofv3 --pmc $cnt --kernel-trace -d "gpurun_out/${step}_$c" -o run --output-format csv -- python3 bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext ;;
    sqc2|sqc3|sqc4|sqc5|sqd2|sqd3|sqd4|sqd5)  # wave-cycle breakdown (c) and LDS / L2 behaviour (d)
      c=$(cfg_of "$step")
      case "$step" in
        sqc*) cnt="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY" ;;
        *) cnt="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum" ;;
      esac
      run "${step}_$c" 300 rocprofv3 --pmc $cnt --kernel-trace -d "gpurun_out/${step}_$c" -o run --output-format csv -- python3 bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext ;;
    elem) GS_ELEM_SOFT=1 GS_ELEM_REPORT="$O/elem.jsonl" run pytest_elem 900 python -u -m pytest tests/test_gpu_parity_configs.py tests/test_gpu_parity.py -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread -rf -k "config2 or config4 or config5 or backward_parity or edge_case" ;;
    chaintime) run chain_timing 300 python tools/amr_chain_timing.py ;;
    chainframes) run chain_frames 300 python tools/amr_chain_timing.py frames ;;
    mvtests) run pytest_mv2 600 python -u -m pytest tests/test_gpu_multiview.py tests/test_gpu_parity_configs.py -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -rf -k "multiview or config5" ;;
    spec) run pytest_spec 600 python -u -m pytest tests/test_gpu_amr_speculation.py tests/test_gpu_capi_ctypes.py tests/test_renderer_amr.py -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -rf ;;
    chaintrace) run chain_trace 300 rocprofv3 --kernel-trace -d "$O/chain_trace" -o run --output-format csv -- python3 tools/amr_chain_timing.py inline &&
                python tools/frame_gaps.py "$O/chain_trace/run_kernel_trace.csv" > "$O/chain_gaps.txt" 2>&1; cat "$O/chain_gaps.txt" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_session] done"
