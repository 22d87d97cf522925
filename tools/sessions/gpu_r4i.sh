#!/bin/bash
# round-4 GPU session I: parity of the non-temporal pass-A stores and of the c3 row kernel with
# stages 4-5 fused over thread pairs (F45); in-process A/B: c3 F45 1 / 0, c2 pass-A NT (bit 1),
# c5 default (walk1, 8 rotation classes) vs the next-hi-tile prefetch (PFH) vs walk2
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -k "nt_stores or 12600_row_kernel_variants or r2c_walk1" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/i_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/i_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c3 --var HSFFT_ROW_F45 --values 1,0 --rounds 6 --iters 5 > gpurun_out/i_c3_f45.log 2>&1; rc=$?; grep -E "median" gpurun_out/i_c3_f45.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c2 --var HSFFT_PFA_NT --values 1,3 --rounds 6 --iters 3 > gpurun_out/i_c2_nt.log 2>&1; rc=$?; grep -E "median" gpurun_out/i_c2_nt.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c5 --values "HSFFT_R2C_ORDER=9" "HSFFT_R2C_ORDER=9;HSFFT_R2C_PFH=1" "HSFFT_R2C_ORDER=9;HSFFT_R2C_PFH=3" "HSFFT_R2C_ORDER=0;HSFFT_R2C_PFH=3" "HSFFT_R2C_WALK=2" --rounds 5 --iters 2 > gpurun_out/i_c5.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/i_c5.log; exit $rc
