set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 tools/lib_ab.py --roots ab/r03,.,.:bal0 --configs C2,C2F,C4 --rounds 3 > gpurun_out/lib_ab_final.txt 2>&1 || { echo lib_ab failed; tail -20 gpurun_out/lib_ab_final.txt; exit 1; }
python3 -c "
import json;t=open('gpurun_out/lib_ab_final.txt').read();d=json.loads(t[t.index('{\n'):]);print(json.dumps(d['median_ms']))"
STEPS="strips" TAG=r04final bash tools/gpu_r04.sh
