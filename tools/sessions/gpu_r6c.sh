#!/bin/bash
# round-6 GPU session C (records at HEAD): GPU suite, smoke(), the default bench line, kernel
# traces + FETCH / WRITE of c2 (the headline) and c4 (k_bxcd changed: census), the
# development-build suite.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6c_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6c_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r6c_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r6c_bench.log 2>&1; rc=$?; tail -c 300 gpurun_out/r6c_bench.log; echo; [ $rc = 0 ] || exit $rc
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r6c_c2 --config c2 --no-other-configs --steps 5 --warmup 2 || exit $?
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r6c_c4 --config c4 --steps 3 --warmup 1 || exit $?
for c in c2 c4; do
  python3 tools/prof_summary.py gpurun_out/prof_r6c_$c --json gpurun_out/prof_r6c_$c/summary.json > gpurun_out/prof_r6c_$c/summary.txt
  echo "== $c"; head -12 gpurun_out/prof_r6c_$c/summary.txt
done
HSFFT_DEV_TESTS=1 HSFFT_LIB_PATH=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so timeout -k 10 600 python -u -m pytest tests/dev -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6c_pytest_dev.log 2>&1
rc=$?; echo "dev pytest rc=$rc"; tail -3 gpurun_out/r6c_pytest_dev.log
exit $rc
