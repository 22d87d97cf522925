#!/bin/bash
# round-3 GPU session AA: kernel trace + FETCH / WRITE of c2, c3, c4, c5 with the final code and
# placement-checked bench buffers (profiles/r03b_*; pmc_traffic.json)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r3b_c2 --config c2 --no-other-configs --steps 5 --warmup 2 || exit $?
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r3b_c3 --config c3 --steps 10 --warmup 2 || exit $?
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r3b_c4 --config c4 --steps 3 --warmup 1 || exit $?
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r3b_c5 --config c5 --steps 2 --warmup 1 || exit $?
for c in c2 c3 c4 c5; do
  python3 tools/prof_summary.py gpurun_out/prof_r3b_$c --json gpurun_out/prof_r3b_$c/summary.json > gpurun_out/prof_r3b_$c/summary.txt
  echo "== $c"; grep '^{' gpurun_out/prof_r3b_$c/kt.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r.get('pass_ms'), d.get('placement',{}).get('copy_gbs'))"
  python3 -c "
import json; s=json.load(open('gpurun_out/prof_r3b_$c/summary.json'))
for k,v in s.items():
    if v.get('calls',0) > 1: print('  ', k[:60], round(v.get('avg_ms',0),3), v.get('calls'), round(v.get('hbm_bytes_corrected',0)/1e9,2))"
done
exit 0
