set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "xcd or full_size" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_xcd.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_xcd.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/ab_tuning.py --key xcd_map --values 1 3 --stage render_bwd --backward > gpurun_out/ab_xcd_bwd.log 2>&1 || exit $?
tail -1 gpurun_out/ab_xcd_bwd.log
timeout -k 10 300 python tools/ab_tuning.py --key xcd_map --values 1 3 --stage render_bwd --backward --P 6100000 --W 1600 --H 1063 --rounds 4 > gpurun_out/ab_xcd_bwd4.log 2>&1 || exit $?
tail -1 gpurun_out/ab_xcd_bwd4.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_xcd3 -o run --output-format csv -- python3 tools/ab_tuning.py --key xcd_map --values 3 --rounds 1 --iters 3 --stage render_bwd --backward > gpurun_out/pmc_xcd3.log 2>&1 || exit $?
