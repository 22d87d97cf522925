#!/bin/bash
# round-4 GPU session C: k_r2c_walk1 without spills (twiddle runs loaded after the exchanges):
# parity, in-process A/B vs walk2 and walk-length / order variants; the c3 replica (one row per
# CU vs half a row per workgroup); the c5 bench line with 512-row output chunks and the
# per-slice placement probe
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "r2c_walk1" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/c_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c5 --values "HSFFT_R2C_WALK=2" "HSFFT_R2C_WALK=3" "HSFFT_R2C_WALK=3;HSFFT_R2C_WT=4" "HSFFT_R2C_WALK=3;HSFFT_R2C_WT=16" "HSFFT_R2C_WALK=3;HSFFT_R2C_ORDER=0" --rounds 5 --iters 3 > gpurun_out/c_c5_walk.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/c_c5_walk.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 ./tools/experiments/c3_replica 65536 > gpurun_out/c_c3_replica.log 2>&1; rc=$?; cat gpurun_out/c_c3_replica.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c_c5_bench.log 2>&1; rc=$?; tail -c 1200 gpurun_out/c_c5_bench.log; exit $rc
