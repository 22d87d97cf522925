#!/bin/bash
# round-6 GPU session A: the recycled per-thread sets, the per-group arrival
# census of the persistent Bluestein launch (item 5 + ADVICE r5 medium), the N>1 bench fields
# (item 3) -- GPU suite; c1 one-thread / eight-thread numbers; c4 within spread; the c5 walk
# occupancy replica (item 2).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=8 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/r6a_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u - > gpurun_out/r6a_c1.log 2>&1 <<'PY'
import sys, statistics
sys.argv = ["bench.py"]
import bench, hsfft
hsfft.lib().hsfft_set_device(0)
for r in range(3):
    lat = bench.c1_latency()
    t8 = [bench.c1_threads() for _ in range(3)]
    print(f"round {r}: c1 median {lat[len(lat)//2]*1e6:.2f} us, threads8 us/transform {[round(x, 2) for x in t8]}, "
          f"streams created {hsfft.lib().hsfft_thread_streams_created()}", flush=True)
PY
rc=$?; cat gpurun_out/r6a_c1.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r6a_c4.log 2>&1; rc=$?; tail -c 400 gpurun_out/r6a_c4.log; echo; [ $rc = 0 ] || exit $rc
timeout -k 10 300 ./tools/experiments/r2c_occ 512 > gpurun_out/r6a_r2c_occ.txt 2>&1; rc=$?; cat gpurun_out/r6a_r2c_occ.txt; [ $rc = 0 ] || exit $rc
exit 0
