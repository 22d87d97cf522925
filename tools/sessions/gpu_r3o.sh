#!/bin/bash
# round-3 GPU session O: copy rate vs allocation (plain / contiguous / one split allocation),
# on a fresh box, then after a c5 bench run and after a c2 bench run (the sequence in which
# session M saw 5.3-5.4 TB/s runs)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 tools/experiments/alloc_rate 64 4 > gpurun_out/o_alloc_fresh.log 2>&1 || exit $?
cat gpurun_out/o_alloc_fresh.log
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/o_c5.log 2>&1 || exit $?
timeout -k 10 300 tools/experiments/alloc_rate 64 4 > gpurun_out/o_alloc_after_c5.log 2>&1 || exit $?
cat gpurun_out/o_alloc_after_c5.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-other-configs --steps 3 --warmup 1 > gpurun_out/o_c2_$i.log 2>&1 || exit $?
  grep '^{' gpurun_out/o_c2_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['stream_copy_gbs'])"
done
timeout -k 10 300 tools/experiments/alloc_rate 64 4 > gpurun_out/o_alloc_after_c2.log 2>&1 || exit $?
cat gpurun_out/o_alloc_after_c2.log
exit 0
