#!/bin/bash
export TMPDIR=/tmp
HSFFT_BX_DEBUG=1 timeout -k 10 120 python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bxd3.log 2>&1 || exit 1
grep bxcd gpurun_out/bxd3.log | tail -2
