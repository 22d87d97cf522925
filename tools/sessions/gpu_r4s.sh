#!/bin/bash
# round-4 GPU session S: HEAD with the c3 stage-5 twiddle default -- full GPU suite, smoke(), the
# default bench line on a fresh box (first), then kernel traces + FETCH / WRITE of c3 and c4
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/s_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/s_bench.log 2>&1; rc=$?; tail -c 600 gpurun_out/s_bench.log; [ $rc = 0 ] || exit $rc
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r4s_c3 --config c3 --steps 10 --warmup 2 || exit $?
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r4s_c4 --config c4 --steps 3 --warmup 1 || exit $?
for c in c3 c4; do
  python3 tools/prof_summary.py gpurun_out/prof_r4s_$c --json gpurun_out/prof_r4s_$c/summary.json > gpurun_out/prof_r4s_$c/summary.txt
  echo "== $c"; grep -A6 -E "^void (mr|bxc)" gpurun_out/prof_r4s_$c/summary.txt
done
exit 0
