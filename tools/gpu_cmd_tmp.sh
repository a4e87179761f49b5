set -u
cd $GRAFT_REPO_ROOT
STEPS="tests" TAG=r04u PYTEST_K="balance or variants" bash tools/gpu_r04.sh || exit 1
timeout -k 10 900 python3 tools/lib_ab.py --roots ab/r03,.,.:bal0 --configs C2,C2F,C4 --rounds 3 > gpurun_out/lib_ab_r04u.txt 2>&1 || { echo lib_ab failed; tail -20 gpurun_out/lib_ab_r04u.txt; exit 1; }
python3 -c "
import json;t=open('gpurun_out/lib_ab_r04u.txt').read();d=json.loads(t[t.index('{\n'):]);print(json.dumps(d['median_ms']))"
STEPS="balance" TAG=r04u BAL_ARGS="--configs C4,C2F,C2 --shares 1,4,8 --rounds 3 --variants b0,b1" bash tools/gpu_r04.sh
