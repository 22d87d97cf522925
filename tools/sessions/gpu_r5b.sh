#!/bin/bash
# round-5 GPU session B: what CU-masked streams do (tools/experiments/cu_mask), parity of the
# development build's variants (tests/dev: incl. the CU-split r2c pipeline), then in-process A/B
# (tools/ab_env.py, one set of buffers): c3 F45 exchange image with a padded pitch
# (HSFFT_ROW_XP=260, dev build) vs packed; c5 pass A and the split walk on complementary CU
# masks (HSFFT_R2C_CUSPLIT, dev build) vs the default; c4 occupancy-checked launch vs the
# cooperative launch (product).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
DEV=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so
timeout -k 10 300 tools/experiments/cu_mask > gpurun_out/r5b_cu_mask.log 2>&1; rc=$?; echo "cu_mask rc=$rc"; cat gpurun_out/r5b_cu_mask.log; [ $rc = 0 ] || exit $rc
HSFFT_DEV_TESTS=1 HSFFT_LIB_PATH=$DEV timeout -k 10 600 python -u -m pytest tests/dev -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5b_pytest_dev.log 2>&1
rc=$?; echo "pytest dev rc=$rc"; tail -3 gpurun_out/r5b_pytest_dev.log; [ $rc = 0 ] || exit $rc
i=0
ab() {
  i=$((i+1))
  timeout -k 10 400 python -u tools/ab_env.py "$@" > gpurun_out/r5b_ab_$i.log 2>&1; rc=$?
  echo "== $*"; grep -E "median" gpurun_out/r5b_ab_$i.log
  [ $rc = 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/r5b_ab_$i.log; exit $rc; }
}
HSFFT_LIB_PATH=$DEV ab --config c3 --var HSFFT_ROW_XP --values unset,260 --rounds 6 --iters 5
HSFFT_LIB_PATH=$DEV ab --config c5 --values unset "HSFFT_R2C_CUSPLIT=4;HSFFT_R2C_SUB=64;HSFFT_R2C_WT=16" "HSFFT_R2C_CUSPLIT=4;HSFFT_R2C_SUB=128" "HSFFT_R2C_CUSPLIT=3;HSFFT_R2C_SUB=64;HSFFT_R2C_WT=16" "HSFFT_R2C_CUSPLIT=6;HSFFT_R2C_SUB=64;HSFFT_R2C_WT=16" --rounds 5 --iters 2
ab --config c4 --var HSFFT_BX_COOP --values unset,1 --rounds 5 --iters 3
exit 0
