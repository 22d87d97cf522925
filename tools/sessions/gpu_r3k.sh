#!/bin/bash
# round-3 GPU session K: c5 split-walk variants (non-temporal data loads / stores) and phase
# trace; c4 persistent Bluestein with the upper half of the groups started late (de-phases
# the two workgroups of every CU), interleaved twice
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'])"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "r2c_walk or bluestein_persistent" > gpurun_out/pytest_r3k.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3k.log
case $rc in 0) ;; *) exit $rc;; esac
HSFFT_R2C_DEBUG=1 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/k_c5_trace.log 2>&1 || exit $?
grep 'r2c_walk2:' gpurun_out/k_c5_trace.log | tail -3
HSFFT_BX_DEBUG=1 timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/k_c4_trace0.log 2>&1 || exit $?
grep 'bxcd:' gpurun_out/k_c4_trace0.log | tail -2
HSFFT_BX_DEBUG=1 HSFFT_BX_SKEW=300 timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/k_c4_trace300.log 2>&1 || exit $?
grep 'bxcd:' gpurun_out/k_c4_trace300.log | tail -2
for pass in 1 2; do
  for nt in 0 1 2 3; do
    HSFFT_R2C_NT=$nt timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/k_c5_nt${nt}_$pass.log 2>&1 || exit $?
    one gpurun_out/k_c5_nt${nt}_$pass.log "c5 nt=$nt pass=$pass"
  done
  for sk in 0 150 300 450; do
    HSFFT_BX_SKEW=$sk timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/k_c4_sk${sk}_$pass.log 2>&1 || exit $?
    one gpurun_out/k_c4_sk${sk}_$pass.log "c4 skew=$sk pass=$pass"
  done
done
exit 0
