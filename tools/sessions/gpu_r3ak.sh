#!/bin/bash
# round-3 GPU session AK: c5 split-walk knobs in-process with placement-checked buffers, two
# independent allocations; c2 PFQ 4 / 6
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
ab() {
  i=$((i+1))
  timeout -k 10 240 python -u tools/ab_env.py "$@" > gpurun_out/ak_$i.log 2>&1; rc=$?
  echo "== $*"; grep -E "placement|median" gpurun_out/ak_$i.log
  [ $rc = 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/ak_$i.log; exit $rc; }
}
for rep in 1 2; do
ab --config c5 --rounds 4 --iters 3 --values unset "HSFFT_R2C_WT=16" "HSFFT_R2C_ORDER=0" "HSFFT_R2C_WT=16;HSFFT_R2C_ORDER=0" "HSFFT_R2C_WT=32;HSFFT_R2C_ORDER=0" "HSFFT_R2C_WT=16;HSFFT_R2C_ORDER=2" "HSFFT_R2C_WT=16;HSFFT_R2C_ORDER=9"
done
ab --config c2 --var HSFFT_PFQ --values 4,6,5 --rounds 4 --iters 3
exit 0
