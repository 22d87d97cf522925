#!/bin/bash
# round-6 GPU session H (final at HEAD): GPU suite, smoke(), the default bench
# line, and the default bench under a kernel trace (must exit 0 with every config recorded).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6h_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6h_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6h_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r6h_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r6h_bench.log 2>&1; rc=$?; tail -c 200 gpurun_out/r6h_bench.log; echo; [ $rc = 0 ] || exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6h_default -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r6h_bench_kt.log 2>&1; rc=$?; echo "kt rc=$rc"
grep -c "caught signal" gpurun_out/r6h_bench_kt.log; grep "Check failed" gpurun_out/r6h_bench_kt.log | head -3
find gpurun_out/prof_r6h_default -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 | head -14
exit $rc
