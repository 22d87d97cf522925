#!/bin/bash
# round-4 GPU session K: non-temporal store variants -- parity (k_b512 pass B, k_row2 F45 rows,
# walk1 pairs phase), then in-process A/B: c2 HSFFT_PFB_NT 0 / 1, c3 HSFFT_ROW_NT 0 / 1, c5
# HSFFT_R2C_NTW 0 / 1, c5 pass A / split walk overlapped over sub-chunks (HSFFT_R2C_OVL)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -k "nt_stores or 12600_row_kernel_variants or overlapped_subchunks" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/k_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/k_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c2 --var HSFFT_PFB_NT --values 0,1 --rounds 6 --iters 3 > gpurun_out/k_c2_pfb_nt.log 2>&1; rc=$?; grep -E "median" gpurun_out/k_c2_pfb_nt.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c3 --var HSFFT_ROW_NT --values 0,1 --rounds 6 --iters 5 > gpurun_out/k_c3_row_nt.log 2>&1; rc=$?; grep -E "median" gpurun_out/k_c3_row_nt.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c5 --var HSFFT_R2C_NTW --values 0,1 --rounds 6 --iters 2 > gpurun_out/k_c5_ntw.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/k_c5_ntw.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_env.py --config c5 --var HSFFT_R2C_OVL --values 0,64,128,32 --rounds 5 --iters 2 > gpurun_out/k_c5_ovl.log 2>&1; rc=$?; grep -E "median" gpurun_out/k_c5_ovl.log; exit $rc
