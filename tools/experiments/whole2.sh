#!/bin/bash
# whole-row generic pass for mixed sizes <= 5120 (HSFFT_WHOLE): parity, then GSamples/s vs passes of <= 512
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "whole_row or c2c_batched or dropin_host or odd" > gpurun_out/whole2_pytest.log 2>&1 || { tail -30 gpurun_out/whole2_pytest.log; exit 1; }
tail -1 gpurun_out/whole2_pytest.log
for n in 1000 2000 3000 5000 243 625 1001 1680; do
  for w in 1 0; do
    b=$(( (1 << 28) / n ))
    HSFFT_WHOLE=$w timeout -k 10 120 python bench.py --config c3 --n $n --batch $b --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/whole2_${n}_$w.log 2>&1 || exit 1
    echo "N=$n whole=$w $(grep -o '"value": [0-9.]*' gpurun_out/whole2_${n}_$w.log) $(grep -o '"passes": [0-9]*' gpurun_out/whole2_${n}_$w.log)"
  done
done
