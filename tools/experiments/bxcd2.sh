#!/bin/bash
# persistent Bluestein: parity, per-phase trace (HSFFT_BX_DEBUG), timing vs three launches
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused.py -k "persistent" > gpurun_out/bxcd_pytest.log 2>&1 || { tail -30 gpurun_out/bxcd_pytest.log; exit 1; }
tail -1 gpurun_out/bxcd_pytest.log
for m in 1; do
  HSFFT_BX_MAP=$m timeout -k 10 120 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bxt_$m.log 2>&1 || exit 1
  HSFFT_BX_DEBUG=1 HSFFT_BX_MAP=$m timeout -k 10 120 python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bxd_$m.log 2>&1 || exit 1
  echo "map=$m $(grep -o '"value": [0-9.]*' gpurun_out/bxt_$m.log) $(grep bxcd gpurun_out/bxd_$m.log | tail -1)"
done
