#!/bin/bash
# round-5 GPU session E: parity of the development build (tests/dev: new c3 row kernel with the
# stage-5 twiddles of steps 1-2 / 1-3 by LDS-DMA, HSFFT_ROW_TWN=5 / 6), then in-process A/B: c3 TWN 5, 6 vs 4;
# c4: P1 / P3 loads unconditional (HSFFT_BX_UL, parity then A/B); with the spill-free k_bxcd,
# one acquire per iteration (HSFFT_BX_MERGE) and the poll sleep (HSFFT_BX_SLEEP) re-checked.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
DEV=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so
HSFFT_DEV_TESTS=1 HSFFT_LIB_PATH=$DEV timeout -k 10 600 python -u -m pytest tests/dev -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5e_pytest_dev.log 2>&1
rc=$?; echo "pytest dev rc=$rc"; tail -3 gpurun_out/r5e_pytest_dev.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q -k "unconditional or persistent_launch" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5e_pytest_ul.log 2>&1
rc=$?; echo "pytest UL rc=$rc"; tail -3 gpurun_out/r5e_pytest_ul.log; [ $rc = 0 ] || exit $rc
i=0
ab() {
  i=$((i+1))
  timeout -k 10 400 python -u tools/ab_env.py "$@" > gpurun_out/r5e_ab_$i.log 2>&1; rc=$?
  echo "== $*"; grep -E "median" gpurun_out/r5e_ab_$i.log
  [ $rc = 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/r5e_ab_$i.log; exit $rc; }
}
HSFFT_LIB_PATH=$DEV ab --config c3 --var HSFFT_ROW_TWN --values unset,5,6 --rounds 8 --iters 5
ab --config c4 --var HSFFT_BX_UL --values unset,1 --rounds 6 --iters 3
ab --config c4 --var HSFFT_BX_MERGE --values unset,1 --rounds 5 --iters 3
ab --config c4 --var HSFFT_BX_SLEEP --values unset,0,4 --rounds 5 --iters 3
exit 0
