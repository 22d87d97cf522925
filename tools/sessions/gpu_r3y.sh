#!/bin/bash
# round-3 GPU session Y: c1 completion paths -- stream wait vs a host-polled word written by
# hipStreamWriteValue32 or by the kernel itself
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 tools/experiments/c1_latency > gpurun_out/y_c1_latency.log 2>&1 || exit $?
cat gpurun_out/y_c1_latency.log
timeout -k 10 120 tools/experiments/c1_latency >> gpurun_out/y_c1_latency.log 2>&1 || exit $?
tail -1 gpurun_out/y_c1_latency.log
exit 0
