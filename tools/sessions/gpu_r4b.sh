#!/bin/bash
# round-4 GPU session B: k_r2c_walk1 parity, c5 split walk1 (2 per CU) vs walk2 in-process A/B;
# c2 pass-B rows per workgroup A/B; c5 bench line under a kernel trace (same process)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "r2c_walk1" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/b_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c5 --var HSFFT_R2C_WALK --values 2,3 --rounds 6 --iters 3 > gpurun_out/b_c5_walk.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/b_c5_walk.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c2 --var HSFFT_PFB --values 8,16,32 --rounds 6 --iters 3 > gpurun_out/b_c2_pfb.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/b_c2_pfb.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 -- python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_c5_bench.log 2>&1; rc=$?; tail -c 1500 gpurun_out/b_c5_bench.log; exit $rc
