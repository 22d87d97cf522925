#!/bin/bash
# round-4 GPU session L: where k_r2c_walk1's 13.6 ms per 512 rows goes -- timing probes of the
# development library (HSFFT_R2C_W1PROBE, results wrong): 3 no twiddle loads, 4 no stage
# arithmetic, 8 no exchanges, 12 neither, 15 loads + stores only (plus twiddle2), 16 no stores,
# 31 row loads only; in-process on one set of buffers; then c3's row-kernel phase trace (F45 1 / 0)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
HSFFT_LIB_PATH=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so timeout -k 10 500 python -u tools/ab_env.py --config c5 --var HSFFT_R2C_W1PROBE --values 0,3,4,8,12,15,16,31 --rounds 4 --iters 2 > gpurun_out/l_c5_probe.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/l_c5_probe.log; [ $rc = 0 ] || exit $rc
# c3 row-kernel phase trace (wave 0's clock per row and CU): F45 default, then F45=0
for f in 1 0; do
  HSFFT_ROW_F45=$f HSFFT_ROW_DEBUG=1 timeout -k 10 200 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/l_c3_trace_f45_$f.log 2>&1; rc=$?; grep "k_row2 per row" gpurun_out/l_c3_trace_f45_$f.log | tail -2; [ $rc = 0 ] || exit $rc
done
exit 0
