#!/bin/bash
# round-5 GPU session J: what c1 would cost without a kernel launch -- a resident one-workgroup
# kernel answering requests through page-locked host words (tools/experiments/c1_resident.hip),
# beside the launch-floor probe (c1_latency) and the product's c1 line on the same box.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 tools/experiments/c1_latency > gpurun_out/r5j_c1_latency.log 2>&1; rc=$?; cat gpurun_out/r5j_c1_latency.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 tools/experiments/c1_resident > gpurun_out/r5j_c1_resident.log 2>&1; rc=$?; cat gpurun_out/r5j_c1_resident.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c1 --no-cpu-baseline > gpurun_out/r5j_c1_bench.log 2>&1; rc=$?; tail -c 300 gpurun_out/r5j_c1_bench.log; [ $rc = 0 ] || exit $rc
exit 0
