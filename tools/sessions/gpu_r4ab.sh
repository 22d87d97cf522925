#!/bin/bash
# round-4 GPU session AB: confirmation of session AA on another box -- c5 HSFFT_PFP 4 / 1 and c2
# HSFFT_PFQ 4 / 1, eight alternated rounds each
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_env.py --config c5 --var HSFFT_PFP --values 4,1 --rounds 8 --iters 2 > gpurun_out/ab_c5_pfp.log 2>&1; rc=$?; grep -E "median" gpurun_out/ab_c5_pfp.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_env.py --config c2 --var HSFFT_PFQ --values 4,1 --rounds 8 --iters 3 > gpurun_out/ab_c2_pfq.log 2>&1; rc=$?; grep -E "median" gpurun_out/ab_c2_pfq.log; exit $rc
