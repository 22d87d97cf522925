#!/bin/bash
# round-4 GPU session Q: c3 F45 with the stage-5 twiddles of steps 1-3 copied into LDS before the
# row's stores (HSFFT_ROW_TWN=3) -- parity, then in-process A/B against the default and the
# constant-twiddle probe (development library)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "12600_row_kernel_variants" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/q_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/q_pytest.log; [ $rc = 0 ] || exit $rc
HSFFT_LIB_PATH=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so timeout -k 10 300 python -u tools/ab_env.py --config c3 --var HSFFT_ROW_TWN --values 0,3,2 --rounds 6 --iters 5 > gpurun_out/q_c3_twn.log 2>&1; rc=$?; grep -E "median" gpurun_out/q_c3_twn.log; exit $rc
