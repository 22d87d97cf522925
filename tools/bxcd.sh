#!/bin/bash
# persistent Bluestein launch: parity, then c4 timing (persistent vs three launches)
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused.py -k "persistent or row_looped" > gpurun_out/bxcd_pytest.log 2>&1 || { tail -30 gpurun_out/bxcd_pytest.log; exit 1; }
tail -3 gpurun_out/bxcd_pytest.log
for x in 8 0; do
  HSFFT_BLUE_XCD=$x timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/bx$x -o kt --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bx$x.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*' gpurun_out/bx$x.log
done
