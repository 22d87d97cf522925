#!/bin/bash
# round-4 GPU session AH: every round-4 default change against its predecessor, in-process on
# one more box -- c3 F45 1/0, c3 stage-5 twiddles 4/0; c2 pass-A NT 3/1, c2 first-pass walk 1/4;
# c5 walk1 prefetch 1/0, c5 pass-A NT 3/2, c5 first-pass walk 1/4
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
ab() {
  i=$((i+1))
  timeout -k 10 300 python -u tools/ab_env.py "$@" > gpurun_out/ah_$i.log 2>&1; rc=$?
  echo "== $*"; grep -E "median" gpurun_out/ah_$i.log
  [ $rc = 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/ah_$i.log; exit $rc; }
}
ab --config c3 --var HSFFT_ROW_F45 --values 1,0 --rounds 6 --iters 5
ab --config c3 --var HSFFT_ROW_TWN --values 4,0 --rounds 6 --iters 5
ab --config c2 --var HSFFT_PFA_NT --values 3,1 --rounds 5 --iters 3
ab --config c2 --var HSFFT_PFQ --values 1,4 --rounds 5 --iters 3
ab --config c5 --var HSFFT_R2C_PFH --values 1,0 --rounds 5 --iters 2
ab --config c5 --var HSFFT_PFA_NT --values 3,2 --rounds 5 --iters 2
ab --config c5 --var HSFFT_PFP --values 1,4 --rounds 5 --iters 2
exit 0
