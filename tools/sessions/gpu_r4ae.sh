#!/bin/bash
# round-4 GPU session AE: c2 pass-B rows per workgroup 8 / 4 (HSFFT_PFB), eight alternated rounds,
# twice (two sets of buffers in two processes)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 1 2; do
timeout -k 10 400 python -u tools/ab_env.py --config c2 --var HSFFT_PFB --values 8,4 --rounds 8 --iters 3 > gpurun_out/ae_c2_pfb_$k.log 2>&1; rc=$?; grep -E "median" gpurun_out/ae_c2_pfb_$k.log; [ $rc = 0 ] || exit $rc
done
exit 0
