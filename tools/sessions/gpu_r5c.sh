#!/bin/bash
# round-5 GPU session C: CU-masked streams with XCD-balanced masks (session B found that a mask
# leaving an XCD empty is ignored), the CU-split r2c pipeline call by call (session B's A/B of it
# stalled), then its in-process A/B against the default if it runs.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
DEV=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so
timeout -k 10 300 tools/experiments/cu_mask > gpurun_out/r5c_cu_mask.log 2>&1; rc=$?; echo "cu_mask rc=$rc"; cat gpurun_out/r5c_cu_mask.log; [ $rc = 0 ] || exit $rc
HSFFT_LIB_PATH=$DEV timeout -k 10 150 python -u tools/experiments/r2c_cusplit_debug.py > gpurun_out/r5c_cusplit_debug.log 2>&1; rc=$?
echo "cusplit debug rc=$rc"; cat gpurun_out/r5c_cusplit_debug.log | tail -15; [ $rc = 0 ] || exit $rc
i=0
ab() {
  i=$((i+1))
  timeout -k 10 400 python -u tools/ab_env.py "$@" > gpurun_out/r5c_ab_$i.log 2>&1; rc=$?
  echo "== $*"; grep -E "median" gpurun_out/r5c_ab_$i.log
  [ $rc = 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/r5c_ab_$i.log; exit $rc; }
}
HSFFT_LIB_PATH=$DEV ab --config c5 --values unset "HSFFT_R2C_CUSPLIT=4;HSFFT_R2C_SUB=64;HSFFT_R2C_WT=16" "HSFFT_R2C_CUSPLIT=4;HSFFT_R2C_SUB=128" "HSFFT_R2C_CUSPLIT=3;HSFFT_R2C_SUB=64;HSFFT_R2C_WT=16" "HSFFT_R2C_CUSPLIT=8;HSFFT_R2C_SUB=64;HSFFT_R2C_WT=16" --rounds 4 --iters 2
ab --config c4 --var HSFFT_BX_COOP --values unset,1 --rounds 5 --iters 3
exit 0
