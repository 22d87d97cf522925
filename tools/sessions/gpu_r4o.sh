#!/bin/bash
# round-4 GPU session O: c5 pass A with 64-B row segments (k_firstq<8,3,2>, 1024 threads, one
# workgroup per CU, non-temporal stores; HSFFT_PFP_G=2) -- parity, then in-process A/B against
# the default 32-B form, with column-group walks of 4 / 2 / 8
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -k "2p21" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/o_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/o_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_env.py --config c5 --values "HSFFT_PFP_G=1" "HSFFT_PFP_G=2" "HSFFT_PFP_G=2;HSFFT_PFP=2" "HSFFT_PFP_G=2;HSFFT_PFP=8" "HSFFT_PFP_G=1;HSFFT_PFP=8" --rounds 5 --iters 2 > gpurun_out/o_c5_pfg.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/o_c5_pfg.log; exit $rc
