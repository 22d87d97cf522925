#!/bin/bash
# round-3 GPU session R: bench.py with the output-placement probe (placement records in the
# JSON line); c5 first-pass walk length 4 vs 1 (HSFFT_PFP) three times interleaved
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('pass_ms'), d.get('stream_copy_gbs'), d.get('placement'))"; }
for pass in 1 2 3; do
  timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-other-configs --steps 5 --warmup 2 > gpurun_out/r_c2_$pass.log 2>&1 || exit $?
  one gpurun_out/r_c2_$pass.log "c2 pass=$pass"
  for q in 4 1; do
    HSFFT_PFP=$q timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r_c5_pfp${q}_$pass.log 2>&1 || exit $?
    one gpurun_out/r_c5_pfp${q}_$pass.log "c5 PFP=$q pass=$pass"
  done
done
exit 0
