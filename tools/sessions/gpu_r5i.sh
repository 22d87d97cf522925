#!/bin/bash
# round-5 GPU session I: the new lifecycle test (hsfft_finalize mid-process, then the same plans
# again) and the development build's parity suite after the round-5 removals.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lifecycle.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5i_pytest_lifecycle.log 2>&1
rc=$?; echo "pytest lifecycle rc=$rc"; tail -3 gpurun_out/r5i_pytest_lifecycle.log; [ $rc = 0 ] || exit $rc
HSFFT_DEV_TESTS=1 HSFFT_LIB_PATH=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so timeout -k 10 600 python -u -m pytest tests/dev -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5i_pytest_dev.log 2>&1
rc=$?; echo "pytest dev rc=$rc"; tail -3 gpurun_out/r5i_pytest_dev.log; [ $rc = 0 ] || exit $rc
exit 0
