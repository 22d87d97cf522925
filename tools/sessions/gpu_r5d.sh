#!/bin/bash
# round-5 GPU session D: the CU-masked streams once more, each experiment in its own process
# under its own time limit and line-buffered (session C's run stalled with nothing printed),
# then the CU-split r2c pipeline call by call; last, the GPU suite at HEAD.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
DEV=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5d_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5d_pytest.log; [ $rc = 0 ] || exit $rc
for m in layout copy concurrent; do
  timeout -k 5 60 tools/experiments/cu_mask $m > gpurun_out/r5d_cu_mask_$m.log 2>&1; rc=$?
  echo "cu_mask $m rc=$rc"; cat gpurun_out/r5d_cu_mask_$m.log
  [ $rc = 0 ] || exit $rc
done
HSFFT_LIB_PATH=$DEV timeout -k 10 150 python -u tools/experiments/r2c_cusplit_debug.py > gpurun_out/r5d_cusplit_debug.log 2>&1; rc=$?
echo "cusplit debug rc=$rc"; cat gpurun_out/r5d_cusplit_debug.log | tail -15
exit $rc
