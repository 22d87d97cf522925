#!/bin/bash
# round-4 GPU session G: c5 pass A with non-temporal output stores (HSFFT_PFA_NT): parity, in-process
# A/B beside walk1, and FETCH_SIZE of pass A both ways
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -k "2p21" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/g_pytest.log; [ $rc = 0 ] || exit $rc
V='HSFFT_R2C_WALK=3;HSFFT_R2C_WT=32;HSFFT_R2C_ORDER=0 HSFFT_R2C_WALK=3;HSFFT_R2C_WT=32;HSFFT_R2C_ORDER=0;HSFFT_PFA_NT=1 HSFFT_R2C_WALK=2 HSFFT_R2C_WALK=2;HSFFT_PFA_NT=1'
timeout -k 10 400 python -u tools/ab_env.py --config c5 --values $V --rounds 4 --iters 2 > gpurun_out/g_c5_nt.log 2>&1; rc=$?; grep -E "placement|median" gpurun_out/g_c5_nt.log; [ $rc = 0 ] || exit $rc
for nt in 0 1; do
HSFFT_PFA_NT=$nt HSFFT_R2C_WALK=3 HSFFT_R2C_WT=32 HSFFT_R2C_ORDER=0 COUNTER_SETS="FETCH_SIZE" tools/profile.sh r4g_nt$nt --config c5 --batch 512 --steps 2 --warmup 1 || exit $?
python3 tools/prof_summary.py gpurun_out/prof_r4g_nt$nt > gpurun_out/prof_r4g_nt$nt/summary.txt; cat gpurun_out/prof_r4g_nt$nt/summary.txt | head -20
done
exit 0
