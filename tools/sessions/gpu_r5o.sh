#!/bin/bash
# round-5 GPU session O: thread-exit destructors no longer call HIP (objects of exited threads are
# reaped by a live call) -- the threaded / lifecycle / small-path tests, then the DEFAULT bench
# command under a kernel trace (session N: rocprofv3 aborted the process in a thread-exit
# destructor's HIP call during the c1 threads sample, and lost the c3-c5 kernel records).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_threads.py tests/test_gpu_lifecycle.py tests/test_gpu_parity.py -m gpu -x -q -k "thread or lifecycle or finalize or dropin or config1" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5o_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5o_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5o_default -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r5o_bench_kt.log 2>&1; rc=$?; echo "kt rc=$rc"
grep -c "caught signal" gpurun_out/r5o_bench_kt.log; grep "Check failed" gpurun_out/r5o_bench_kt.log | head -3
find gpurun_out/prof_r5o_default -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160
exit $rc
