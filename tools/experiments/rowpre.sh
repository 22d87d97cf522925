#!/bin/bash
# k_row2 LDS-DMA next-row prefetch (HSFFT_ROW_PRE=1): parity, phase trace, c3 timing
export TMPDIR=/tmp
HSFFT_ROW_PRE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "12600" > gpurun_out/rowpre_pytest.log 2>&1 || { tail -30 gpurun_out/rowpre_pytest.log; exit 1; }
tail -1 gpurun_out/rowpre_pytest.log
for p in 1 0; do
  HSFFT_ROW_PRE=$p timeout -k 10 120 python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rowpre_$p.log 2>&1 || exit 1
  HSFFT_ROW_DEBUG=1 HSFFT_ROW_PRE=$p timeout -k 10 120 python3 bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/rowpre_d$p.log 2>&1 || exit 1
  echo "pre=$p $(grep -o '"value": [0-9.]*' gpurun_out/rowpre_$p.log) $(grep 'k_row2 per row' gpurun_out/rowpre_d$p.log | tail -1)"
done
