#!/bin/bash
# round-3 GPU session L: what the c5 split walk's twiddle streams cost -- timing probes of the
# development library (twiddle2 / stage-2 twiddles read from cache-resident lines: results
# WRONG, timing only) -- and the twiddle2-prefetching walk (HSFFT_R2C_TW2=1): parity, then
# interleaved timing twice, plus phase traces
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'])"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "r2c_walk" > gpurun_out/pytest_r3l.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3l.log
case $rc in 0) ;; *) exit $rc;; esac
for tw in 0 1; do
  HSFFT_R2C_TW2=$tw HSFFT_R2C_DEBUG=1 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/l_c5_trace_tw$tw.log 2>&1 || exit $?
  echo "tw2 prefetch $tw: $(grep 'r2c_walk2:' gpurun_out/l_c5_trace_tw$tw.log | tail -1)"
done
DEV=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so
for pass in 1 2; do
  for tw in 0 1; do
    HSFFT_R2C_TW2=$tw timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/l_c5_tw${tw}_$pass.log 2>&1 || exit $?
    one gpurun_out/l_c5_tw${tw}_$pass.log "c5 tw2-prefetch=$tw pass=$pass"
  done
  for pr in 1 2 3; do
    HSFFT_LIB_PATH=$DEV HSFFT_R2C_PROBE=$pr timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/l_c5_p${pr}_$pass.log 2>&1 || exit $?
    one gpurun_out/l_c5_p${pr}_$pass.log "c5 probe=$pr pass=$pass (dev lib, wrong results)"
  done
done
exit 0
