#!/bin/bash
# round-4 GPU session N: c3 row kernel with the next row's remaining groups copied into LDS by
# LDS-DMA before the stores (HSFFT_ROW_DMA): parity, in-process A/B, phase trace; c5 walk1
# rotation-class count / walk length around the default (the walk is contention-bound: its
# probes run slower without arithmetic, session L)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "12600_row_kernel_variants" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/n_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/n_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_env.py --config c3 --var HSFFT_ROW_DMA --values 0,1 --rounds 6 --iters 5 > gpurun_out/n_c3_dma.log 2>&1; rc=$?; grep -E "median" gpurun_out/n_c3_dma.log; [ $rc = 0 ] || exit $rc
HSFFT_ROW_DMA=1 HSFFT_ROW_DEBUG=1 timeout -k 10 200 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/n_c3_trace_dma.log 2>&1; rc=$?; grep "k_row2 per row" gpurun_out/n_c3_trace_dma.log | tail -2; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_env.py --config c5 --values "HSFFT_R2C_ORDER=9" "HSFFT_R2C_ORDER=17" "HSFFT_R2C_ORDER=33" "HSFFT_R2C_ORDER=5" "HSFFT_R2C_ORDER=2" "HSFFT_R2C_ORDER=9;HSFFT_R2C_WT=64" "HSFFT_R2C_ORDER=17;HSFFT_R2C_WT=16" --rounds 4 --iters 2 > gpurun_out/n_c5_order.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/n_c5_order.log; exit $rc
