#!/bin/bash
# round-3 GPU session G: full suite (per-thread-stream small fft_exec), c1 latency and 8-thread
# throughput with and without the lock-free small path
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3g.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3g.log
case $rc in 0) ;; *) exit $rc;; esac
for c in 1 0 1 0; do
  HSFFT_SMALL_CONCURRENT=$c timeout -k 10 120 python -c "
import bench, hsfft
hsfft.lib().hsfft_set_device(0)
lat = bench.c1_latency()
print('concurrent=$c', 'median_us', round(lat[len(lat)//2]*1e6, 2), 'threads8_us_per_transform', round(bench.c1_threads(), 2), 'threads16', round(bench.c1_threads(16), 2))
" || exit $?
done
exit 0
