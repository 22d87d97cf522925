#!/bin/bash
# round-4 GPU session AD: re-sweep around the new defaults in-process -- c5 walk length
# (HSFFT_R2C_WT 32 / 16 / 48 / 24, 8 rotation classes, PFH), c2 pass-B rows per workgroup
# (HSFFT_PFB 8 / 4 / 16) with the one-group first pass
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_env.py --config c5 --var HSFFT_R2C_WT --values 32,16,48,24 --rounds 5 --iters 2 > gpurun_out/ad_c5_wt.log 2>&1; rc=$?; grep -E "median" gpurun_out/ad_c5_wt.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_env.py --config c2 --var HSFFT_PFB --values 8,4,16 --rounds 5 --iters 3 > gpurun_out/ad_c2_pfb.log 2>&1; rc=$?; grep -E "median" gpurun_out/ad_c2_pfb.log; exit $rc
