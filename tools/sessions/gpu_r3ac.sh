#!/bin/bash
# round-3 GPU session AC: c2 passes with the first column group / row loaded before the
# workgroup's twiddle set-up (HSFFT_F0 bit 0: pass A, bit 1: pass B) -- parity of the 2^20
# paths with both on, then F0 = 0 / 1 / 2 / 3 interleaved three times
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('pass_ms'), d.get('stream_copy_gbs'), d.get('placement',{}).get('copy_gbs'))"; }
HSFFT_F0=3 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "config2 or full_size_config2 or power_of_two_sweep or pow2_whole or two_pass or config4 or bluestein" > gpurun_out/pytest_r3ac.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3ac.log
case $rc in 0) ;; *) exit $rc;; esac
for pass in 1 2 3; do
  for f in 0 3 1 2; do
    HSFFT_F0=$f timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-other-configs --steps 10 --warmup 3 > gpurun_out/ac_c2_f${f}_$pass.log 2>&1 || exit $?
    one gpurun_out/ac_c2_f${f}_$pass.log "c2 F0=$f pass=$pass"
  done
done
exit 0
