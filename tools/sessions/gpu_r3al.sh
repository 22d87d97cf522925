#!/bin/bash
# round-3 GPU session AL: c5 step time over fresh placements of the library's scratch pool
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/scratch_lottery.py 12 > gpurun_out/al_1.log 2>&1; rc=$?; cat gpurun_out/al_1.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/scratch_lottery.py 12 > gpurun_out/al_2.log 2>&1; rc=$?; cat gpurun_out/al_2.log; exit $rc
