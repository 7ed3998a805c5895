#!/usr/bin/env bash
# quick health check of the forward path: smoke, read-back tests, a plain bench, one PMC pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
O=gpurun_out/diag
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 $O/smoke.log
timeout -k 10 300 python -c "
import ctypes, torch
lib = ctypes.CDLL('gaussian_splatting_with_eye_tracking_amd/libgsplat_amd.so')
torch.zeros(1, device='cuda')
print('optin', torch.cuda.get_device_properties(0))
" > $O/props.log 2>&1; tail -2 $O/props.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_readback.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/readback.log 2>&1; echo "readback rc=$?"; tail -3 $O/readback.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub > $O/bench.log 2>&1; echo "bench rc=$?"; tail -c 600 $O/bench.log
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES --kernel-trace -d $O/pmc1 -o run --output-format csv -- python3 bench.py --config cfg2_1080p_1M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext > $O/pmc1.log 2>&1; echo "pmc1 rc=$?"; grep -v "^W2026\|^E2026" $O/pmc1.log | tail -3
GSAMD_HDR_MIRROR=1 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES --kernel-trace -d $O/pmc1m -o run --output-format csv -- python3 bench.py --config cfg2_1080p_1M --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-sub --no-ext > $O/pmc1m.log 2>&1; echo "pmc1 mirror1 rc=$?"; grep -v "^W2026\|^E2026" $O/pmc1m.log | tail -3
