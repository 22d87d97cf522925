#!/bin/bash
# round-3 GPU session AH: c3's last stage reading a transposed copy of its twiddles (coalesced
# loads; HSFFT_ROW_TWL=0 reads the plan's table as is): parity subset, then c3 TWL 1 / 0
# interleaved x3, then kernel traces of c3 (both) and c5 (PFG 1 / 2)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "stop rc=$1"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "12600 or config3 or mixed_whole or dropin_repeated or paired_load" > gpurun_out/pytest_r3ah.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_r3ah.log; stop $rc
for rep in 1 2 3; do
  for t in 1 0; do
    HSFFT_ROW_TWL=$t timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-other-configs --steps 20 > gpurun_out/c3_twl${t}_$rep.log 2>&1; stop $?
    grep '^{' gpurun_out/c3_twl${t}_$rep.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.readline())
print('c3 TWL=$t rep $rep', d['value'], 'ms', d['ms_per_step'], 'place', (d.get('placement') or {}).get('copy_gbs'))
"
  done
done
for t in 1 0; do
  HSFFT_ROW_TWL=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_twl$t -o kt --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline --no-other-configs > gpurun_out/prof_c3_twl$t.log 2>&1; stop $?
done
for g in 1 2; do
  HSFFT_PFG=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_pfg$g -o kt --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --no-other-configs > gpurun_out/prof_c5_pfg$g.log 2>&1; stop $?
done
find gpurun_out/prof_c3_twl* gpurun_out/prof_c5_pfg* -name '*kernel_stats.csv' | while read f; do echo "== $f"; python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:4]: print('  ', x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e6,3),'ms')
"; done
exit 0
