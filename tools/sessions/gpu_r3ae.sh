#!/bin/bash
# round-3 GPU session AE: repeated drop-in calls with the completion word (every mode)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "completion_word or dropin" > gpurun_out/pytest_r3ae.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'PASSED|FAILED|passed|failed' gpurun_out/pytest_r3ae.log | tail -12
exit $rc
