#!/bin/bash
# round-6 GPU session G (records at HEAD, after the knob snapshot and the C-loop c1 timing): GPU suite, smoke(), the default bench line, kernel
# (kernels unchanged since session C's profiles), the development-build suite.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6g_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6g_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6g_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r6g_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r6g_bench.log 2>&1; rc=$?; tail -c 300 gpurun_out/r6g_bench.log; echo; [ $rc = 0 ] || exit $rc
HSFFT_DEV_TESTS=1 HSFFT_LIB_PATH=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so timeout -k 10 600 python -u -m pytest tests/dev -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6g_pytest_dev.log 2>&1
rc=$?; echo "dev pytest rc=$rc"; tail -3 gpurun_out/r6g_pytest_dev.log
exit $rc
