set -o pipefail
L=realtimeraytracing_gradproject_amd/lib
V="base=$L/librtamd.so lds21=$L/variants/ldstop21/librtamd.so lds85=$L/variants/ldstop85/librtamd.so near=$L/variants/tlasnear/librtamd.so trim=$L/variants/tlastrim/librtamd.so"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/ab.py --configs C4 --share 4 --rounds 9 --steps 40 $V > gpurun_out/cand_share4_r06l.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --configs C2 --share 8 --rounds 9 --steps 40 $V > gpurun_out/cand_share8_r06l.txt 2>&1 &&
timeout -k 10 400 python3 -u tools/ab.py --configs C2,C2F,C3,C4,REF --rounds 9 --steps 30 $V > gpurun_out/cand_full_r06l.txt 2>&1
