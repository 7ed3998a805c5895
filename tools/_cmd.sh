set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_configs.py tests/test_gpu_cull.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/parf.log 2>&1 && \
timeout -k 10 300 python tools/ab_tuning.py --key fwd_variant --values 3 5 --stage render > gpurun_out/abf_cfg2.log 2>&1 && \
timeout -k 10 300 python tools/ab_tuning.py --key fwd_variant --values 3 5 --stage render --P 6100000 --W 1600 --H 1063 --rounds 4 > gpurun_out/abf_cfg4.log 2>&1
echo rc=$?
