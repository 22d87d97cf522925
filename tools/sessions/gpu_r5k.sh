#!/bin/bash
# round-5 GPU session K: the resident-kernel c1 floor with the loads issued together
# (c1_resident r3), and a kernel trace of the product's c1 (the one-workgroup k_pass duration).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 tools/experiments/c1_resident > gpurun_out/r5k_c1_resident.log 2>&1; rc=$?; cat gpurun_out/r5k_c1_resident.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5k_c1 -o kt --output-format csv -- python3 bench.py --config c1 --no-cpu-baseline > gpurun_out/r5k_c1_kt.log 2>&1; rc=$?; tail -c 300 gpurun_out/r5k_c1_kt.log; [ $rc = 0 ] || exit $rc
find gpurun_out/prof_r5k_c1 -name "*kernel_stats.csv" -exec head -5 {} \;
exit 0
