#!/bin/bash
# c1 latency: blocking stream wait vs event polling (HSFFT_SMALL_SPIN), alternated
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for s in 0 1 0 1; do
  HSFFT_SMALL_SPIN=$s timeout -k 10 120 python3 bench.py --config c1 --no-cpu-baseline --no-other-configs > gpurun_out/c1_spin$s.json 2>gpurun_out/c1_err.log
  echo "spin=$s $(python3 -c "import json;d=json.load(open('gpurun_out/c1_spin$s.json'));print(d['value'], d.get('latency_us'))")"
done
