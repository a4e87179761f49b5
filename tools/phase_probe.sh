set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
for cfg in C2 C4; do for m in 1 2; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/phase_${cfg}_$m -o run --output-format csv -- python3 $R/tools/one_config.py --config $cfg --frames 60 --mode $m > $O/phase_${cfg}_$m.log 2>&1
f=$(find $O/phase_${cfg}_$m -name "*kernel_stats.csv" | head -1); echo "$cfg mode $m"; head -3 $f | cut -c1-200
done; done
