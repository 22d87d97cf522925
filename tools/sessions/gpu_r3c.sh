#!/bin/bash
# round-3 GPU session C: kernel traces + FETCH/WRITE passes of the default c2/c3/c4/c5
# schedules (the bench line's traffic entries), the c3 row-kernel phase trace and the
# persistent-Bluestein phase trace.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
HSFFT_ROW_DEBUG=1 timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/c3_trace.log 2>&1 || exit $?
grep k_row2 gpurun_out/c3_trace.log | tail -2
HSFFT_BX_DEBUG=1 timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/c4_trace.log 2>&1 || exit $?
grep '^bxcd' gpurun_out/c4_trace.log | tail -1
for c in c3 c4 c5 c2; do
  args="--config $c --steps 2 --warmup 1"; [ $c = c2 ] && args="--steps 2 --warmup 1 --no-other-configs"
  COUNTER_SETS="FETCH_SIZE|WRITE_SIZE" tools/profile.sh r03$c $args || exit $?
  python3 tools/prof_summary.py gpurun_out/prof_r03$c --json gpurun_out/prof_r03$c/summary.json > gpurun_out/prof_r03$c/summary.txt || exit $?
done
exit 0
