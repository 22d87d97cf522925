#!/bin/bash
# round-4 GPU session R: c3 F45 stage-5 twiddles from a transposed copy of the stage's block
# (coalesced: one 16-B word per lane, lanes on consecutive k; HSFFT_ROW_TWN=4) -- parity, then
# in-process A/B against the default, the LDS copy (3) and the constant-twiddle probe (2,
# development library)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "12600" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r_pytest.log; [ $rc = 0 ] || exit $rc
HSFFT_LIB_PATH=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so timeout -k 10 300 python -u tools/ab_env.py --config c3 --var HSFFT_ROW_TWN --values 0,4,2 --rounds 6 --iters 5 > gpurun_out/r_c3_twn.log 2>&1; rc=$?; grep -E "median" gpurun_out/r_c3_twn.log; exit $rc
