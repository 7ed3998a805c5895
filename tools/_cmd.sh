set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_tuning.py --key fwd_hint --values 1 0 1 0 --stage preprocess --amr --rounds 6 > gpurun_out/ab_fwd_hint_cfg3.log 2>&1 || exit $?
tail -8 gpurun_out/ab_fwd_hint_cfg3.log
