#!/bin/bash
# bench.py once per environment setting: tools/sweep_env.sh "VAR=a VAR2=b" "VAR=c" ...
set -e
cd "$GRAFT_REPO_ROOT"
for cfg in "$@"; do
  tag=$(echo "$cfg" | tr ' =' '_-')
  env $cfg timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sw_$tag.json 2> gpurun_out/sw_err.log
  echo "$cfg $(python3 -c "import json;d=json.load(open('gpurun_out/sw_$tag.json'));print(d['value'],d['roofline']['pass_ms'])")"
done
