#!/bin/bash
# round-5 GPU session A: the GPU suite and the development build's variants (tests/dev; new: the asynchronous Bluestein error contract with
# forced timeouts, `bench.py --gpus 2` starting its own ranks for c2 and c5), then the c4 exit
# crash of round 4: (1) c4 under a kernel trace + FETCH + WRITE with the round-5 defaults
# (occupancy-checked launch, hsfft_finalize before exit); (2) the round-4 cooperative launch
# (HSFFT_BX_COOP=1) with finalize; (3) the cooperative launch without finalize -- last, as it
# may crash at exit; the in-process crash trace (HSFFT_CRASH_TRACE=1) names the frames.  Before
# it: tools/experiments/cu_mask (what CU-masked streams do: layout and copy rates).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=10 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5a_pytest.log; [ $rc = 0 ] || exit $rc
HSFFT_DEV_TESTS=1 HSFFT_LIB_PATH=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so timeout -k 10 600 python -u -m pytest tests/dev -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5a_pytest_dev.log 2>&1
rc=$?; echo "pytest dev rc=$rc"; tail -3 gpurun_out/r5a_pytest_dev.log; [ $rc = 0 ] || exit $rc
export HSFFT_CRASH_TRACE=1
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r5a_c4 --config c4 --steps 3 --warmup 1 || exit $?
HSFFT_BX_COOP=1 NO_PMC=1 tools/profile.sh r5a_c4coop --config c4 --steps 3 --warmup 1 || exit $?
timeout -k 10 300 tools/experiments/cu_mask > gpurun_out/r5a_cu_mask.log 2>&1; rc=$?; echo "cu_mask rc=$rc"; cat gpurun_out/r5a_cu_mask.log; [ $rc = 0 ] || exit $rc
HSFFT_BX_COOP=1 NO_PMC=1 tools/profile.sh r5a_c4coopnf --config c4 --steps 3 --warmup 1 --no-finalize; rc=$?
echo "cooperative launch without finalize: rc=$rc"
grep -n -A100 "hsfft crash trace" gpurun_out/prof_r5a_c4coopnf/kt.log > gpurun_out/r5a_crash_excerpt.txt || true
exit 0
