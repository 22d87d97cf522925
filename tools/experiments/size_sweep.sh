#!/bin/bash
# c2c GSamples/s across transform lengths at ~4 GiB per direction (what a caller of other
# sizes gets): powers of two, 3/5/7-smooth, Bluestein lengths
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for n in 64 256 1024 4096 16384 65536 262144 1048576 4194304 16777216 67108864 1000 3000 10000 100000 1000000 6561 15625 16807 10368 44100 4097 65521 1000003; do
  b=$(( (1 << 28) / n )); [ $b -lt 1 ] && b=1
  timeout -k 10 120 python bench.py --config c3 --n $n --batch $b --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sz_$n.log 2>&1; rc=$?
  echo "N=$n batch=$b rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/sz_$n.log) $(grep -o '"passes": [0-9]*' gpurun_out/sz_$n.log) $(grep -o '"frac": [0-9.]*' gpurun_out/sz_$n.log | head -1)"
  case $rc in 124|137|134|139) exit $rc;; esac
done
