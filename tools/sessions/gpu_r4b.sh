#!/bin/bash
# round-4 GPU session B: c2 pass-B rows per workgroup (twiddle re-read 12.5 / 6 / 3 %) in-process
# A/B; c5 bench line with a kernel trace in the same process (reconcile bench vs kernel sum)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_env.py --config c2 --var HSFFT_PFB --values 8,16,32 --rounds 6 --iters 3 > gpurun_out/b_c2_pfb.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/b_c2_pfb.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c2 --var HSFFT_PFQ --values 4,8 --rounds 6 --iters 3 > gpurun_out/b_c2_pfq.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/b_c2_pfq.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 -- python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_c5_bench.log 2>&1; rc=$?; tail -c 1500 gpurun_out/b_c5_bench.log; exit $rc
