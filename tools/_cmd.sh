set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof3t -o run --output-format csv -- python3 bench.py --config cfg3_amr_1080p_1M --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-sub --no-ext > gpurun_out/prof3t.log 2>&1
echo rc=$?
