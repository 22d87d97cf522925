#!/bin/bash
# round-6 GPU session B: the host pipeline's deferred Bluestein launches -- its
# tests, and c4 host rows with the launches deferred (round 6) vs synchronous per chunk (round 5's
# behaviour, HSFFT_BX_SYNC=1); then the DEFAULT bench command under a kernel trace with the
# recycled per-thread sets (must still exit 0 with every config recorded).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_threads.py -m gpu -x -q -k "host or timeout or generations or concurrent" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6b_pytest.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --host-rows 512 > gpurun_out/r6b_c4_host_deferred_$i.log 2>&1; rc=$?; [ $rc = 0 ] || exit $rc
  grep -o '"host_pipeline": {[^}]*}' gpurun_out/r6b_c4_host_deferred_$i.log | sed 's/^/deferred: /'
  HSFFT_BX_SYNC=1 timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --host-rows 512 > gpurun_out/r6b_c4_host_sync_$i.log 2>&1; rc=$?; [ $rc = 0 ] || exit $rc
  grep -o '"host_pipeline": {[^}]*}' gpurun_out/r6b_c4_host_sync_$i.log | sed 's/^/sync per chunk: /'
done
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6b_default -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r6b_bench_kt.log 2>&1; rc=$?; echo "kt rc=$rc"
grep -c "caught signal" gpurun_out/r6b_bench_kt.log; grep "Check failed" gpurun_out/r6b_bench_kt.log | head -3
find gpurun_out/prof_r6b_default -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160
exit $rc
