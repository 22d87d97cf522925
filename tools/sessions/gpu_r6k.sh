#!/bin/bash
# round-6 GPU session K (HEAD after the timing helper's error-path fix): GPU suite and smoke().
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=3 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6k_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6k_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6k_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r6k_smoke.log
exit $rc
