#!/bin/bash
# round-5 GPU session G: the GPU suite at HEAD (k_bxcd's unconditional loads now the only form,
# c3's measured-slower variants removed), then in-process A/B: the three-launch Bluestein path's
# last kernel with unconditional chirp loads (HSFFT_BLAST_UL) and k_bxcd's poll sleep 4 vs 1
# (session E: -0.3 %).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5g_pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 gpurun_out/r5g_pytest_gpu.log; [ $rc = 0 ] || exit $rc
i=0
ab() {
  i=$((i+1))
  timeout -k 10 400 python -u tools/ab_env.py "$@" > gpurun_out/r5g_ab_$i.log 2>&1; rc=$?
  echo "== $*"; grep -E "median" gpurun_out/r5g_ab_$i.log
  [ $rc = 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/r5g_ab_$i.log; exit $rc; }
}
ab --config c4 --values "HSFFT_BLUE_XCD=0" "HSFFT_BLUE_XCD=0;HSFFT_BLAST_UL=1" --rounds 6 --iters 3
ab --config c4 --var HSFFT_BX_SLEEP --values unset,4 --rounds 6 --iters 3
exit 0
