#!/bin/bash
# c4 kernel times with the Bluestein intermediates aliased on die (HSFFT_DEV_ALIAS=2, timing only)
export TMPDIR=/tmp
for al in 2 0; do
  HSFFT_DEV_ALIAS=$al timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/ba$al -o kt --output-format csv -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ba$al.log 2>&1 || exit 1
done
