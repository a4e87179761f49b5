#!/bin/bash
# Workgroup-shape variants with frames in flight (3 streams): tools/overlap_probe.py --lib per variant.
set -e
mkdir -p gpurun_out
for cfg in ${CFGS:-C2 C2F C4}; do
  for v in ${VARIANTS:-base wx4 wy2}; do
    timeout -k 10 120 python -u tools/overlap_probe.py --config $cfg --shares 1 --streams 3 --frames 100 --rounds 3 \
      --lib realtimeraytracing_gradproject_amd/lib/variants/$v/librtamd.so > gpurun_out/wg_${cfg}_$v.json 2>>gpurun_out/wg.err
  done
done
