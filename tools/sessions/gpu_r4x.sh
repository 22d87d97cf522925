#!/bin/bash
# round-4 GPU session X: the split walk with a CU's second walk started late (HSFFT_R2C_STAGGER:
# n x ~3.4 us), so that the two walks of a CU run their phases apart -- parity, in-process A/B
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
HSFFT_R2C_STAGGER=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "r2c_walk1 and 4194304" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/x_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/x_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_env.py --config c5 --var HSFFT_R2C_STAGGER --values 0,4,8,2 --rounds 5 --iters 2 > gpurun_out/x_c5_stagger.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/x_c5_stagger.log; exit $rc
