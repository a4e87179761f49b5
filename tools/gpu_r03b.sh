set -u
SKIP_BENCH=1 SKIP_TRACE=1 TAG=r03b bash tools/gpu_session.sh || exit 1
RT_COMM_TIMING=1 timeout -k 10 300 python3 tools/native_strips_cost.py --config C2 > gpurun_out/native_strips_cost_r03b.json 2> gpurun_out/native_strips_cost_r03b.err || { echo cost failed; exit 1; }
timeout -k 10 300 python3 bench.py --mode strips --extra= --no-cpu-baseline > gpurun_out/bench_strips1_r03b.json 2> gpurun_out/bench_strips1_r03b.err || { echo strips bench failed; exit 1; }
V=realtimeraytracing_gradproject_amd/lib
TESTS=0 CONFIGS=C5 ROUNDS=5 AB="base=$V/librtamd.so wide=$V/variants/mswide/librtamd.so" bash tools/gpu_ab.sh || exit 1
LIB=$V/librtamd.so CFG=C5 TAG=base bash tools/pmc_write.sh || exit 1
LIB=$V/variants/mswide/librtamd.so CFG=C5 TAG=wide bash tools/pmc_write.sh || exit 1
echo all-ok
