#!/bin/bash
# round-3 GPU session H: c5 pass-A column groups per workgroup (HSFFT_PFP), c4 poll sleep
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'])"; }
for q in 4 2 8 16 1 4; do
  HSFFT_PFP=$q timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/h_c5_pfp$q.log 2>&1 || exit $?
  one gpurun_out/h_c5_pfp$q.log "c5 PFP=$q"
done
for sl in 1 0 4 1; do
  HSFFT_BX_SLEEP=$sl timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 10 > gpurun_out/h_c4_s$sl.log 2>&1 || exit $?
  one gpurun_out/h_c4_s$sl.log "c4 sleep=$sl"
done
exit 0
