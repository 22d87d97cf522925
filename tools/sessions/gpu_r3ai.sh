#!/bin/bash
# round-3 GPU session AI: in-process A/B on one set of buffers (tools/ab_env.py): c3 last-stage
# twiddles transposed (HSFFT_ROW_TWL 1 / 0), c5 pass A 64-B segments (HSFFT_PFG 2 / 1)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_env.py --config c3 --var HSFFT_ROW_TWL --values 1,0 --rounds 8 --iters 10 > gpurun_out/ab_c3_twl.log 2>&1; rc=$?; tail -2 gpurun_out/ab_c3_twl.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c5 --var HSFFT_PFG --values 2,1 --rounds 8 --iters 3 > gpurun_out/ab_c5_pfg.log 2>&1; rc=$?; tail -2 gpurun_out/ab_c5_pfg.log; [ $rc = 0 ] || exit $rc
exit 0
