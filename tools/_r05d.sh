export GS_TAG=r05d
bash tools/gpu_session.sh tests &&
AB_NAME=bwd2 AB_ARGS="--key bwd_variant --values 1 2 --stage render_bwd --backward" bash tools/gpu_session.sh ab &&
AB_NAME=bwd4 AB_ARGS="--key bwd_variant --values 1 2 --stage render_bwd --backward --P 6100000 --W 1600 --H 1063" bash tools/gpu_session.sh ab &&
bash tools/gpu_session.sh benchq
