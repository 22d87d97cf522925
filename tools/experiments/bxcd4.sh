#!/bin/bash
# persistent Bluestein (default): parity (fused + parity suites' Bluestein cases), c4 bench + kernel stats
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_threads.py -k "luestein or persistent or 99991 or threads or golden" > gpurun_out/bxcd4_pytest.log 2>&1 || { tail -30 gpurun_out/bxcd4_pytest.log; exit 1; }
tail -1 gpurun_out/bxcd4_pytest.log
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/bx4 -o kt --output-format csv -- python3 bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bx4.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/bx4.log
timeout -k 10 150 python3 bench.py --config c4 --steps 10 --warmup 2 > gpurun_out/bx4b.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/bx4b.log
