#!/bin/bash
# round-4 GPU session AG: spread of the default bench line -- two back-to-back default runs in
# two processes on one box (each on its own first allocations)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 600 python -u bench.py > gpurun_out/ag_bench_$k.log 2>&1; rc=$?; tail -c 200 gpurun_out/ag_bench_$k.log; [ $rc = 0 ] || exit $rc
done
exit 0
