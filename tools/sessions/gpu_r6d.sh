#!/bin/bash
# round-6 GPU session D: hsfft_time_exec_host (c1 timed in a C loop) -- its test, c1 one-thread
# and eight-thread numbers in C vs through ctypes, and the same with 500 extra environment
# variables (what the per-call getenv lookups of the small path cost).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_threads.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r6d_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6d_pytest.log; [ $rc = 0 ] || exit $rc
cat > /tmp/c1d.py <<'PY'
import os, sys
sys.path.insert(0, os.getcwd())
sys.argv = ["bench.py"]
import bench, hsfft
hsfft.lib().hsfft_set_device(0)
for r in range(3):
    one = bench.c1_c_loop(1, 3000, 50)
    eight = bench.c1_c_loop(8, 500, 20)
    lat = bench.c1_latency(1000, 20)
    print(f"round {r}: C loop median {one[0]:.2f} p10 {one[1]:.2f} p90 {one[2]:.2f} mean {one[3]:.2f} us | "
          f"8 C threads {eight[3]:.2f} us/transform | ctypes median {lat[len(lat)//2]*1e6:.2f} | "
          f"python threads8 {bench.c1_threads():.2f}", flush=True)
PY
timeout -k 10 300 python -u /tmp/c1d.py > gpurun_out/r6d_c1.log 2>&1; rc=$?; cat gpurun_out/r6d_c1.log; [ $rc = 0 ] || exit $rc
( for i in $(seq 1 500); do export HSFFT_ZZ_DUMMY_$i=$i; done; timeout -k 10 300 python -u /tmp/c1d.py ) > gpurun_out/r6d_c1_bigenv.log 2>&1; rc=$?; echo "with 500 more env vars:"; cat gpurun_out/r6d_c1_bigenv.log
exit $rc
