#!/bin/bash
# round-3 GPU session S: scratch-pool placement probe (HSFFT_PLACE_DEBUG prints the rates);
# c5 first-pass walk length 4 vs 1 three times interleaved, now with both the bench output
# buffer and the library's intermediate placement-checked
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], d.get('stream_copy_gbs'), d.get('placement',{}).get('copy_gbs'))"; grep 'hsfft scratch' "$1" | tr '\n' ';'; echo; }
export HSFFT_PLACE_DEBUG=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "r2c or 12600 or bluestein_persistent_full" > gpurun_out/pytest_r3s.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3s.log
case $rc in 0) ;; *) exit $rc;; esac
for pass in 1 2 3; do
  for q in 4 1; do
    HSFFT_PFP=$q timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/s_c5_pfp${q}_$pass.log 2>&1 || exit $?
    one gpurun_out/s_c5_pfp${q}_$pass.log "c5 PFP=$q pass=$pass"
  done
done
exit 0
