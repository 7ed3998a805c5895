set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_xcd$v -o run --output-format csv -- python3 tools/ab_tuning.py --key xcd_map --values $v --rounds 1 --iters 3 --stage render_bwd --backward > gpurun_out/pmc_xcd$v.log 2>&1 || exit $?
done
