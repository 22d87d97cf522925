#!/bin/bash
# round-4 GPU session V: the split walk as a persistent grid of two workgroups per CU
# (HSFFT_R2C_PERSIST=1) -- every-word parity against the one-workgroup-per-item launch, then the
# in-process A/B
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "persistent_grid" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/v_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/v_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_env.py --config c5 --var HSFFT_R2C_PERSIST --values 0,1 --rounds 6 --iters 2 > gpurun_out/v_c5_persist.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/v_c5_persist.log; exit $rc
