#!/bin/bash
# round-5 GPU session P (final at HEAD, after the thread-exit change): GPU suite, smoke(), the
# default bench line.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5p_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5p_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5p_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r5p_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r5p_bench.log 2>&1; rc=$?; tail -c 300 gpurun_out/r5p_bench.log; echo; [ $rc = 0 ] || exit $rc
exit 0
