#!/bin/bash
# round-3 GPU session M: first-pass walk length of the column passes (HSFFT_PFP: c5's
# [8,8,8,8] pass, HSFFT_PFQ: c2's [4,8,8,8] pass) -- shorter walks keep the workgroups that
# share a 128-B line closer in time -- interleaved twice, with pass times
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('pass_ms'))"; }
for pass in 1 2; do
  for q in 4 1 2 8; do
    HSFFT_PFP=$q timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/m_c5_pfp${q}_$pass.log 2>&1 || exit $?
    one gpurun_out/m_c5_pfp${q}_$pass.log "c5 PFP=$q pass=$pass"
  done
  for q in 4 1 2; do
    HSFFT_PFQ=$q timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-other-configs --steps 5 --warmup 2 > gpurun_out/m_c2_pfq${q}_$pass.log 2>&1 || exit $?
    one gpurun_out/m_c2_pfq${q}_$pass.log "c2 PFQ=$q pass=$pass"
  done
done
exit 0
