#!/bin/bash
# round-5 GPU session M: second box for the small path's twiddles-ahead first pass (now up to
# 2048 points): the drop-in tests, then c1 in-process A/B at N = 1024, 2048, 512.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_threads.py tests/test_gpu_c_caller.py -m gpu -x -q -k "dropin or config1 or fixtures or thread or caller" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5m_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5m_pytest.log; [ $rc = 0 ] || exit $rc
for n in 1024 2048 512; do
  timeout -k 10 200 python -u tools/ab_c1.py --var HSFFT_SMALL_TWA --values 0,1 --rounds 8 --calls 1000 --n $n > gpurun_out/r5m_ab_c1_$n.log 2>&1; rc=$?
  echo "== n=$n"; grep median gpurun_out/r5m_ab_c1_$n.log; [ $rc = 0 ] || { tail -5 gpurun_out/r5m_ab_c1_$n.log; exit $rc; }
done
exit 0
