#!/bin/bash
# round-5 GPU session H (records at HEAD): smoke(), the default bench line, then kernel traces +
# FETCH / WRITE of c2, c3, c4 and c5 (tools/profile.sh) and their summaries.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5h_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r5h_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r5h_bench.log 2>&1; rc=$?; tail -c 400 gpurun_out/r5h_bench.log; echo; [ $rc = 0 ] || exit $rc
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r5h_c2 --config c2 --no-other-configs --steps 5 --warmup 2 || exit $?
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r5h_c3 --config c3 --steps 5 --warmup 2 || exit $?
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r5h_c4 --config c4 --steps 3 --warmup 1 || exit $?
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r5h_c5 --config c5 --steps 2 --warmup 1 || exit $?
for c in c2 c3 c4 c5; do
  python3 tools/prof_summary.py gpurun_out/prof_r5h_$c --json gpurun_out/prof_r5h_$c/summary.json > gpurun_out/prof_r5h_$c/summary.txt
  echo "== $c"; head -30 gpurun_out/prof_r5h_$c/summary.txt
done
exit 0
