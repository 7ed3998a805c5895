set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_readback.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/readback.log 2>&1 && \
GSAMD_HDR_MIRROR=0 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-sub --no-profile > gpurun_out/b_m0.log 2>&1 && \
GSAMD_HDR_MIRROR=2 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-sub --no-profile > gpurun_out/b_m2.log 2>&1 && \
GSAMD_HDR_MIRROR=0 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-sub --no-profile > gpurun_out/b_m0b.log 2>&1 && \
GSAMD_HDR_MIRROR=2 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-sub --no-profile > gpurun_out/b_m2b.log 2>&1 && \
GSAMD_HDR_MIRROR=0 timeout -k 10 300 python bench.py --config cfg3_amr_1080p_1M --steps 50 --warmup 5 --no-cpu-baseline --no-sub --no-profile --no-ext > gpurun_out/b3_m0.log 2>&1 && \
GSAMD_HDR_MIRROR=2 timeout -k 10 300 python bench.py --config cfg3_amr_1080p_1M --steps 50 --warmup 5 --no-cpu-baseline --no-sub --no-profile --no-ext > gpurun_out/b3_m2.log 2>&1
echo rc=$?
