#!/bin/bash
# round-4 GPU session H: non-temporal pass-A stores -- parity (2^20 and 2^21 first passes), c2 A/B
# (bit 1), c5 default (walk1, 8 rotation classes) vs row-major
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -k "nt_stores" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/h_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/h_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c2 --var HSFFT_PFA_NT --values 1,3 --rounds 6 --iters 3 > gpurun_out/h_c2_nt.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/h_c2_nt.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c5 --values "HSFFT_R2C_ORDER=9" "HSFFT_R2C_ORDER=0" "HSFFT_R2C_WALK=2" --rounds 5 --iters 2 > gpurun_out/h_c5.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/h_c5.log; exit $rc
