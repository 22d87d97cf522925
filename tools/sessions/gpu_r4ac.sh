#!/bin/bash
# round-4 GPU session AC (final, with one column group per first-pass workgroup): full GPU suite,
# smoke(), the default bench line, then kernel traces + FETCH / WRITE of c2 and c5
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=10 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ac_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ac_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/ac_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/ac_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/ac_bench.log 2>&1; rc=$?; tail -c 300 gpurun_out/ac_bench.log; [ $rc = 0 ] || exit $rc
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r4ac_c2 --config c2 --no-other-configs --steps 5 --warmup 2 || exit $?
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r4ac_c5 --config c5 --steps 2 --warmup 1 || exit $?
for c in c2 c5; do
  python3 tools/prof_summary.py gpurun_out/prof_r4ac_$c --json gpurun_out/prof_r4ac_$c/summary.json > gpurun_out/prof_r4ac_$c/summary.txt
  echo "== $c"; grep -A6 -E "^void pf" gpurun_out/prof_r4ac_$c/summary.txt
done
exit 0
