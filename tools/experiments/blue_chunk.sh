#!/bin/bash
# c4 per-kernel times vs Bluestein chunk size (does a MALL-resident intermediate speed the kernels?)
export TMPDIR=/tmp
for c in 32 64 128 4096; do
  HSFFT_BLUE_T=${BT:-1} HSFFT_BLUE_CHUNK_MB=$c timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/bc$c -o kt --output-format csv -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bc$c.log 2>&1 || exit 1
done
