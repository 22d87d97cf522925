#!/bin/bash
# k_r2c_fused timing probes (HSFFT_R2C_PROBE bits: 1 twiddle2, 2 stage-2 twiddles, 4 stores, 8 data loads off)
export TMPDIR=/tmp
for p in ${PROBES:-0 16 32 4}; do
  HSFFT_R2C_PROBE=$p timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/r2cp_$p -o kt --output-format csv -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs > gpurun_out/r2cp_$p.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r2cp_$p/kt_kernel_stats.csv')):
    if 'r2c_fused' in r['Name']: print('probe $p', r['Name'][:40], round(float(r['AverageNs'])/1e6,3))"
done
