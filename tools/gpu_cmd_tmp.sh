set -u
cd $GRAFT_REPO_ROOT
STEPS="balance" TAG=r04y BAL_ARGS="--configs C4,C2F --shares 1,4,8 --rounds 3 --variants b0,b1,b1q8,b1q16" bash tools/gpu_r04.sh
