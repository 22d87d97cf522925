#!/bin/bash
# round-4 GPU session U: c3 row kernel with the next row's first group loaded before the first
# exchange instead of after it (HSFFT_ROW_PFE=1) -- parity, in-process A/B, phase trace
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "12600_row_kernel_variants" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/u_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/u_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c3 --var HSFFT_ROW_PFE --values 0,1 --rounds 6 --iters 5 > gpurun_out/u_c3_pfe.log 2>&1; rc=$?; grep -E "median" gpurun_out/u_c3_pfe.log; [ $rc = 0 ] || exit $rc
for v in 0 1; do
  HSFFT_ROW_PFE=$v HSFFT_ROW_DEBUG=1 timeout -k 10 200 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/u_c3_trace_$v.log 2>&1; rc=$?; grep "k_row2 per row" gpurun_out/u_c3_trace_$v.log | tail -1; [ $rc = 0 ] || exit $rc
done
exit 0
