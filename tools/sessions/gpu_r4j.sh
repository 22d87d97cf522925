#!/bin/bash
# round-4 GPU session J: HEAD with the session-I defaults (c3 F45, 2^20 pass-A non-temporal
# stores, walk1 PFH=1) -- full GPU suite, smoke(), kernel trace + FETCH / WRITE of c2, c3, c5
# (pmc_traffic.json), then the default bench line
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/j_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/j_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/j_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/j_smoke.log; [ $rc = 0 ] || exit $rc
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r4j_c2 --config c2 --no-other-configs --steps 5 --warmup 2 || exit $?
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r4j_c3 --config c3 --steps 10 --warmup 2 || exit $?
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r4j_c5 --config c5 --steps 2 --warmup 1 || exit $?
for c in c2 c3 c5; do
  python3 tools/prof_summary.py gpurun_out/prof_r4j_$c --json gpurun_out/prof_r4j_$c/summary.json > gpurun_out/prof_r4j_$c/summary.txt
  echo "== $c"; head -12 gpurun_out/prof_r4j_$c/summary.txt
done
timeout -k 10 600 python -u bench.py > gpurun_out/j_bench.log 2>&1; rc=$?; tail -c 1500 gpurun_out/j_bench.log; exit $rc
