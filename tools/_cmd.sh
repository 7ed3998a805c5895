set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_configs.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/par_drgb.log 2>&1 && \
timeout -k 10 300 python tools/ab_tuning.py --key sh_drgb --values 0 1 --stage bwd_gauss --backward --rounds 6 > gpurun_out/ab_drgb_bg2.log 2>&1 && \
timeout -k 10 300 python tools/ab_tuning.py --key sh_drgb --values 0 1 --stage preprocess --backward --rounds 6 > gpurun_out/ab_drgb_pp2.log 2>&1 && \
timeout -k 10 400 python tools/ab_tuning.py --key sh_drgb --values 0 1 --stage bwd_gauss --backward --P 6100000 --W 1600 --H 1063 --rounds 4 > gpurun_out/ab_drgb_bg4.log 2>&1 && \
timeout -k 10 400 python tools/ab_tuning.py --key sh_drgb --values 0 1 --stage preprocess --backward --P 6100000 --W 1600 --H 1063 --rounds 4 > gpurun_out/ab_drgb_pp4.log 2>&1
echo rc=$?
