#!/bin/bash
# round-4 GPU session L: where k_r2c_walk1's 13.6 ms per 512 rows goes -- timing probes of the
# development library (HSFFT_R2C_W1PROBE, results wrong): 3 no twiddle loads, 4 no stage
# arithmetic, 8 no exchanges, 12 neither, 15 loads + stores only (plus twiddle2), 16 no stores,
# 31 row loads only; in-process on one set of buffers
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
HSFFT_LIB_PATH=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so timeout -k 10 500 python -u tools/ab_env.py --config c5 --var HSFFT_R2C_W1PROBE --values 0,3,4,8,12,15,16,31 --rounds 4 --iters 2 > gpurun_out/l_c5_probe.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/l_c5_probe.log; exit $rc
