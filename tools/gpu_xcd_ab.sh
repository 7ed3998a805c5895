set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cull.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_xcd.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_xcd.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/ab_tuning.py --key xcd_map --values 0 1 --stage render > gpurun_out/ab_xcd_fwd.log 2>&1 || exit $?
tail -4 gpurun_out/ab_xcd_fwd.log
timeout -k 10 300 python tools/ab_tuning.py --key xcd_map --values 0 1 --stage render_bwd --backward > gpurun_out/ab_xcd_bwd.log 2>&1 || exit $?
tail -4 gpurun_out/ab_xcd_bwd.log
