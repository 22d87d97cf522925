#!/bin/bash
# round-6 GPU session E: c1 after the per-call knob snapshot (default env and +500 variables),
# the small-path tests, and where c1's 11.6 vs 14.3 us bimodality comes from (NUMA placement of
# the calling thread / the page-locked slots vs the GPU's node).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_threads.py tests/test_gpu_parity.py -m gpu -x -q -k "thread or small or flag or config1 or dropin or exec_host" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r6e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6e_pytest.log; [ $rc = 0 ] || exit $rc
echo "nodes: $(ls /sys/devices/system/node | grep node | tr '\n' ' ')"
for n in /sys/devices/system/node/node*; do echo "$(basename $n) cpus $(cat $n/cpulist)"; done
for d in /sys/class/drm/card*/device; do [ -f $d/numa_node ] && echo "$d numa_node $(cat $d/numa_node)"; done 2>/dev/null | head -4
echo "env vars: $(env | wc -l); nproc $(nproc); affinity $(python3 -c 'import os;print(len(os.sched_getaffinity(0)))')"
cat > /tmp/c1e.py <<'PY'
import os, sys
sys.path.insert(0, os.getcwd())
sys.argv = ["bench.py"]
import bench, hsfft
hsfft.lib().hsfft_set_device(0)
med = []
for r in range(8):
    one = bench.c1_c_loop(1, 2000, 50)
    med.append(round(one[0], 2))
eight = bench.c1_c_loop(8, 500, 20)
print(f"C loop medians {med} | 8 C threads {eight[3]:.2f} us/transform", flush=True)
PY
timeout -k 10 300 python -u /tmp/c1e.py > gpurun_out/r6e_c1.log 2>&1; rc=$?; echo "default env:"; cat gpurun_out/r6e_c1.log; [ $rc = 0 ] || exit $rc
( for i in $(seq 1 500); do export HSFFT_ZZ_DUMMY_$i=$i; done; timeout -k 10 300 python -u /tmp/c1e.py ) > gpurun_out/r6e_c1_bigenv.log 2>&1; rc=$?; echo "with 500 more env vars:"; cat gpurun_out/r6e_c1_bigenv.log; [ $rc = 0 ] || exit $rc
node_of_gpu=$(cat /sys/class/drm/card*/device/numa_node 2>/dev/null | grep -v -- -1 | head -1)
for n in /sys/devices/system/node/node*; do
  cpus=$(cat $n/cpulist)
  timeout -k 10 300 taskset -c $cpus python -u /tmp/c1e.py > gpurun_out/r6e_c1_$(basename $n).log 2>&1; rc=$?
  echo "pinned to $(basename $n) (gpu node ${node_of_gpu:-?}): $(cat gpurun_out/r6e_c1_$(basename $n).log)"; [ $rc = 0 ] || exit $rc
done
exit 0
