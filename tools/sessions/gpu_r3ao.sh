#!/bin/bash
# round-3 GPU session AO: in-process A/B of the persistent Bluestein's merged acquire
# (HSFFT_BX_MERGE), measured slower across runs in the first session
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/ab_env.py --config c4 --var HSFFT_BX_MERGE --values unset,1 --rounds 6 --iters 3 > gpurun_out/ao_1.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/ao_1.log; exit $rc
