#!/bin/bash
# 1024-thread generic passes for tiles >= 2048 points (HSFFT_GNT): parity, GSamples/s
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "whole_row or c2c_batched or dropin_host or odd or divergences" > gpurun_out/gnt_pytest.log 2>&1 || { tail -30 gpurun_out/gnt_pytest.log; exit 1; }
tail -1 gpurun_out/gnt_pytest.log
for n in 2000 3000 5000 4913 6561 10000 15625 44100 100000; do
  for w in 1024 256; do
    b=$(( (1 << 28) / n ))
    HSFFT_GNT=$w timeout -k 10 120 python bench.py --config c3 --n $n --batch $b --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/gnt_${n}_$w.log 2>&1 || exit 1
    echo "N=$n nt=$w $(grep -o '"value": [0-9.]*' gpurun_out/gnt_${n}_$w.log) $(grep -o '"passes": [0-9]*' gpurun_out/gnt_${n}_$w.log)"
  done
done
