#!/bin/bash
# round-5 GPU session N (final at HEAD): GPU suite, smoke(), the default bench line, and a
# kernel trace of the default run (every config's kernels).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=10 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5n_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5n_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5n_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r5n_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r5n_bench.log 2>&1; rc=$?; tail -c 300 gpurun_out/r5n_bench.log; echo; [ $rc = 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5n_default -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r5n_bench_kt.log 2>&1; rc=$?; echo "kt rc=$rc"; [ $rc = 0 ] || exit $rc
find gpurun_out/prof_r5n_default -name "*kernel_stats.csv" -exec head -12 {} \;
exit 0
