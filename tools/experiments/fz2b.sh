set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
i=0
for spec in "HSFFT_FZ_SPIN=100000 HSFFT_FZ_LAG=6" "HSFFT_FZ_SPIN=100000 HSFFT_FZ_LAG=3 HSFFT_FZ2_NT=3" "HSFFT_FZ_SPIN=100000 HSFFT_FZ_LAG=6 HSFFT_FZ2_NT=3" "HSFFT_FZ_SPIN=100000 HSFFT_FZ_LAG=6 HSFFT_FZ2_NT=1" "HSFFT_FZ_SPIN=100000 HSFFT_FZ_LAG=6 HSFFT_FZ2_NT=2"; do
  i=$((i+1))
  env HSFFT_FUSED=2 HSFFT_FZ_DEBUG=1 $spec timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --batch 1024 > gpurun_out/fz2b_$i.log 2>&1; rc=$?
  echo "== $spec rc=$rc"; grep "fz2" gpurun_out/fz2b_$i.log | tail -2; python3 -c "
import json
for l in open('gpurun_out/fz2b_$i.log'):
    if l.startswith('{'): d=json.loads(l); print('  value', d['value'], 'ms', d['ms_per_step'])"
  case $rc in 124|137|134|139) exit $rc;; esac
done
