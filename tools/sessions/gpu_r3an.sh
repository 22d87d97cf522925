#!/bin/bash
# round-3 GPU session AN: largest-size parity (c2c to 2^26, long single-radix chains, Bluestein
# at M = 2^21 / 2^23, r2c to 2^26)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "largest" > gpurun_out/pytest_r3an.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/pytest_r3an.log | head -30; tail -1 gpurun_out/pytest_r3an.log; exit $rc
