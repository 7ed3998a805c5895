set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "amr or AMR or config3 or fovea or once" > gpurun_out/para.log 2>&1 && \
timeout -k 10 300 python tools/ab_tuning.py --key amr_sel --values 0 1 --stage amr_render --amr-once > gpurun_out/aba_once.log 2>&1
echo rc=$?
