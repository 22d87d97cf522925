#!/bin/bash
# round-4 GPU session AA: first-pass column-group walk length in-process (the round-3 sweep was
# across runs, inside the allocation lottery): c5 HSFFT_PFP 4 / 1 / 2, c2 HSFFT_PFQ 4 / 1 / 2
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_env.py --config c5 --var HSFFT_PFP --values 4,1,2 --rounds 5 --iters 2 > gpurun_out/aa_c5_pfp.log 2>&1; rc=$?; grep -E "median" gpurun_out/aa_c5_pfp.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_env.py --config c2 --var HSFFT_PFQ --values 4,1,2 --rounds 5 --iters 3 > gpurun_out/aa_c2_pfq.log 2>&1; rc=$?; grep -E "median" gpurun_out/aa_c2_pfq.log; exit $rc
