#!/bin/bash
# round-3 GPU session AJ: in-process re-sweeps of the existing launch knobs on one set of
# buffers per config (tools/ab_env.py), free of the allocation lottery that blurred the
# earlier cross-run sweeps
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
ab() {
  i=$((i+1))
  timeout -k 10 240 python -u tools/ab_env.py "$@" > gpurun_out/aj_$i.log 2>&1; rc=$?
  echo "== $*"; grep -E "median" gpurun_out/aj_$i.log
  [ $rc = 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/aj_$i.log; exit $rc; }
}
ab --config c5 --var HSFFT_R2C_WT --values 8,4,6,12,16 --rounds 4 --iters 3
ab --config c5 --var HSFFT_R2C_ORDER --values 9,2,0,17 --rounds 4 --iters 3
ab --config c5 --var HSFFT_PFP --values 4,1,2,8 --rounds 4 --iters 3
ab --config c3 --var HSFFT_MR_XCD --values 1,0 --rounds 4 --iters 10
ab --config c2 --var HSFFT_PFQ --values 4,2,3,6,8 --rounds 3 --iters 3
ab --config c2 --var HSFFT_PFB --values 8,4 --rounds 3 --iters 3
ab --config c2 --var HSFFT_XCD --values 1,0 --rounds 3 --iters 3
ab --config c4 --var HSFFT_BX_MAP --values unset,0,1 --rounds 3 --iters 3
ab --config c4 --var HSFFT_BX_SLEEP --values unset,0,1,4 --rounds 3 --iters 3
exit 0
