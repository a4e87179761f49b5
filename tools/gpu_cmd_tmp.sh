set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python3 tools/lib_ab.py --roots .:bal0,ab/ls6:bal0 --configs C2,C2F,C3,C4,C5 --rounds 3 > gpurun_out/lib_ab_ls6.txt 2>&1 || { echo lib_ab failed; tail -20 gpurun_out/lib_ab_ls6.txt; exit 1; }
python3 -c "
import json;t=open('gpurun_out/lib_ab_ls6.txt').read();d=json.loads(t[t.index('{\n'):]);print(json.dumps(d['median_ms']))"
