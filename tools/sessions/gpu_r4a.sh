#!/bin/bash
# round-4 GPU session A: HEAD check -- full GPU suite, then the default bench line (all configs)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=20 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r4a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4a.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r4a.log 2>&1; rc=$?; tail -c 3000 gpurun_out/bench_r4a.log; exit $rc
