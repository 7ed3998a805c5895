export GS_TAG=r05e
bash tools/gpu_session.sh tests smoke bench prof2 prof5
