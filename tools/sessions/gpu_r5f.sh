#!/bin/bash
# round-5 GPU session F: the store-burst alignment hypothesis (round-4 verdict item 4) tested by
# a walk built to break it -- a per-CU store token (HSFFT_R2C_STOK, development build): parity,
# the token's statistics, then in-process A/B against the default walk; and c4's unconditional
# P1 / P3 loads (HSFFT_BX_UL) re-measured on a second box.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
DEV=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so
HSFFT_DEV_TESTS=1 HSFFT_LIB_PATH=$DEV timeout -k 10 400 python -u -m pytest tests/dev -m gpu -x -q -k store_token --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5f_pytest_stok.log 2>&1
rc=$?; echo "pytest stok rc=$rc"; tail -3 gpurun_out/r5f_pytest_stok.log; [ $rc = 0 ] || exit $rc
for v in 1 2; do
  HSFFT_LIB_PATH=$DEV HSFFT_R2C_STOK=$v HSFFT_R2C_STOK_STATS=1 timeout -k 10 200 python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-finalize > gpurun_out/r5f_stats_$v.log 2>&1
  rc=$?; echo "stats $v rc=$rc"; grep "store token" gpurun_out/r5f_stats_$v.log | tail -4; [ $rc = 0 ] || exit $rc
done
i=0
ab() {
  i=$((i+1))
  timeout -k 10 400 python -u tools/ab_env.py "$@" > gpurun_out/r5f_ab_$i.log 2>&1; rc=$?
  echo "== $*"; grep -E "median" gpurun_out/r5f_ab_$i.log
  [ $rc = 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/r5f_ab_$i.log; exit $rc; }
}
HSFFT_LIB_PATH=$DEV ab --config c5 --var HSFFT_R2C_STOK --values unset,1,2 --rounds 6 --iters 3
ab --config c4 --var HSFFT_BX_UL --values unset,1 --rounds 6 --iters 3
exit 0
