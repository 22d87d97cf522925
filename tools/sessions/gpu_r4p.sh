#!/bin/bash
# round-4 GPU session P: does F45's stage-5 twiddle wait (loads issued after the previous
# step's stores wait for them: vmcnt is in order) cost c3 time?  Development library, in-process:
# HSFFT_ROW_TWN 0 (default), 1 (next step's twiddles loaded before the stores; 17 dwords of
# spill), 2 (timing probe: constant twiddles, no loads, results wrong)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
HSFFT_LIB_PATH=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so timeout -k 10 300 python -u tools/ab_env.py --config c3 --var HSFFT_ROW_TWN --values 0,1,2 --rounds 6 --iters 5 > gpurun_out/p_c3_twn.log 2>&1; rc=$?; grep -E "median" gpurun_out/p_c3_twn.log; exit $rc
