set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_configs.py tests/test_gpu_cull.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/par7.log 2>&1 && \
timeout -k 10 300 python tools/ab_tuning.py --key bwd_variant --values 0 7 --stage render_bwd --backward > gpurun_out/ab7_cfg2.log 2>&1 && \
timeout -k 10 300 python tools/ab_tuning.py --key bwd_variant --values 0 7 --stage render_bwd --backward --P 6100000 --W 1600 --H 1063 --rounds 4 > gpurun_out/ab7_cfg4.log 2>&1
echo rc=$?
