#!/bin/bash
# round-4 GPU session Z (final): the driver's round-end steps at HEAD -- full GPU suite, smoke(),
# the default bench line -- on a fresh box
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=10 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/z_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/z_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/z_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/z_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/z_bench.log 2>&1; rc=$?; tail -c 400 gpurun_out/z_bench.log; exit $rc
