#!/bin/bash
# round-3 GPU session U: where c5's first pass (pf::k_firstq<8,3,1>) over-fetches -- kernel
# time, FETCH / WRITE and L2 hit rate with the product library, and the same with the L = 512
# stage's global twiddles redirected to one 7-entry run (development library, results WRONG)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
COUNTER_SETS="FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum" tools/profile.sh r3u_prod --config c5 --steps 1 --warmup 0 || exit $?
python3 tools/prof_summary.py gpurun_out/prof_r3u_prod > gpurun_out/prof_r3u_prod/summary.txt
HSFFT_LIB_PATH=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so HSFFT_PFA_PROBE=1 COUNTER_SETS="FETCH_SIZE|TCC_HIT_sum TCC_MISS_sum" tools/profile.sh r3u_probe --config c5 --steps 1 --warmup 0 || exit $?
python3 tools/prof_summary.py gpurun_out/prof_r3u_probe > gpurun_out/prof_r3u_probe/summary.txt
for t in prod probe; do echo "== $t"; grep -A8 'k_firstq' gpurun_out/prof_r3u_$t/summary.txt; done
exit 0
