#!/bin/bash
# round-3 GPU session V: r2c split walk with one output stream parked in LDS and stored during
# the next tile (HSFFT_R2C_PARK=1): parity, phase trace, three interleaved timing passes
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], d.get('stream_copy_gbs'), d.get('placement',{}).get('copy_gbs'))"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "r2c_walk" > gpurun_out/pytest_r3v.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3v.log
case $rc in 0) ;; *) exit $rc;; esac
HSFFT_R2C_PARK=1 HSFFT_R2C_DEBUG=1 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/v_c5_trace.log 2>&1 || exit $?
grep 'r2c_walk2:' gpurun_out/v_c5_trace.log | tail -1
for pass in 1 2 3; do
  for pk in 0 1; do
    HSFFT_R2C_PARK=$pk timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/v_c5_park${pk}_$pass.log 2>&1 || exit $?
    one gpurun_out/v_c5_park${pk}_$pass.log "c5 park=$pk pass=$pass"
  done
done
exit 0
