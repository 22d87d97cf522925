#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for wt in 32 8 16 64 128 256 32; do
  HSFFT_R2C_WT=$wt timeout -k 10 120 python3 bench.py --config c5 --no-cpu-baseline --no-other-configs --steps 3 --warmup 1 > gpurun_out/c5_wt$wt.json 2>gpurun_out/c5_err.log
  echo "wt=$wt $(python3 -c "import json;d=json.load(open('gpurun_out/c5_wt$wt.json'));print(d['value'])")"
done
