#!/bin/bash
# round-3 GPU session N: c2 pass-A walk length 4 vs 1 (and c5's 4 vs 1), three interleaved
# passes each, plus a kernel trace of both c2 settings
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('pass_ms'), d.get('stream_copy_gbs'))"; }
for pass in 1 2 3; do
  for q in 4 1; do
    HSFFT_PFQ=$q timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-other-configs --steps 5 --warmup 2 > gpurun_out/n_c2_pfq${q}_$pass.log 2>&1 || exit $?
    one gpurun_out/n_c2_pfq${q}_$pass.log "c2 PFQ=$q pass=$pass"
  done
  for q in 4 1; do
    HSFFT_PFP=$q timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/n_c5_pfp${q}_$pass.log 2>&1 || exit $?
    one gpurun_out/n_c5_pfp${q}_$pass.log "c5 PFP=$q pass=$pass"
  done
done
for q in 4 1; do
  HSFFT_PFQ=$q timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/n_prof_pfq$q -o run --output-format csv -- python3 bench.py --config c2 --no-cpu-baseline --no-other-configs --steps 3 --warmup 1 > gpurun_out/n_prof_pfq$q.log 2>&1 || exit $?
  f=$(find gpurun_out/n_prof_pfq$q -name '*kernel_stats.csv' | head -1); echo "PFQ=$q"; cut -d, -f1-4 "$f" | head -6
done
exit 0
