#!/bin/bash
# round-4 GPU session F: c5 split walk1 long walks vs walk2 on FIRST allocations (no placement
# selection), two processes
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V='HSFFT_R2C_WALK=2 HSFFT_R2C_WALK=2;HSFFT_R2C_WT=32;HSFFT_R2C_ORDER=0 HSFFT_R2C_WALK=3;HSFFT_R2C_WT=32;HSFFT_R2C_ORDER=0 HSFFT_R2C_WALK=3;HSFFT_R2C_WT=64;HSFFT_R2C_ORDER=0 HSFFT_R2C_WALK=3;HSFFT_R2C_WT=32 HSFFT_R2C_WALK=3;HSFFT_R2C_WT=16;HSFFT_R2C_ORDER=2 HSFFT_R2C_WALK=3;HSFFT_R2C_WT=128;HSFFT_R2C_ORDER=0'
for a in 1 2; do
timeout -k 10 400 python -u tools/ab_env.py --config c5 --values $V --rounds 4 --iters 2 > gpurun_out/f_c5_walk_$a.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/f_c5_walk_$a.log; [ $rc = 0 ] || exit $rc
done
