#!/bin/bash
# round-3 GPU session AP: the second split exchange of the first passes swizzled (bank model:
# 8 -> 4 cycles per store): full GPU suite, then c2 / c5 in-process A/B (HSFFT_SW2 1 / 0)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3ap.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error" gpurun_out/pytest_r3ap.log | head -5; tail -1 gpurun_out/pytest_r3ap.log; [ $rc = 0 ] || exit $rc
timeout -k 10 240 python -u tools/ab_env.py --config c2 --var HSFFT_SW2 --values 1,0 --rounds 6 --iters 3 > gpurun_out/ap_c2.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/ap_c2.log; [ $rc = 0 ] || exit $rc
timeout -k 10 240 python -u tools/ab_env.py --config c5 --var HSFFT_SW2 --values 1,0 --rounds 6 --iters 3 > gpurun_out/ap_c5.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/ap_c5.log; [ $rc = 0 ] || exit $rc
timeout -k 10 240 python -u tools/ab_env.py --config c2 --var HSFFT_SW2 --values 1,0 --rounds 6 --iters 3 > gpurun_out/ap_c2b.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/ap_c2b.log; exit $rc
