#!/bin/bash
# round-3 GPU session D: full suite with the split-exchange swizzle, c2 / c5 against the
# round-2-swizzle build (interleaved), then session C's profiles (kernel traces + FETCH /
# WRITE of the default c2/c3/c4/c5 schedules, c3 and c4 phase traces).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('pass_ms'))"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3d.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3d.log
case $rc in 0) ;; *) exit $rc;; esac
L2=mixed-radix-fast-fourier-transform_amd/lib/libhsfft_swz2.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-configs > gpurun_out/d_c2_new$i.log 2>&1 || exit $?; one gpurun_out/d_c2_new$i.log "c2 new"
  HSFFT_LIB_PATH=$L2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-configs > gpurun_out/d_c2_old$i.log 2>&1 || exit $?; one gpurun_out/d_c2_old$i.log "c2 r2swz"
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/d_c5_new$i.log 2>&1 || exit $?; one gpurun_out/d_c5_new$i.log "c5 new"
  HSFFT_LIB_PATH=$L2 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/d_c5_old$i.log 2>&1 || exit $?; one gpurun_out/d_c5_old$i.log "c5 r2swz"
done
HSFFT_ROW_DEBUG=1 timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/c3_trace.log 2>&1 || exit $?
grep k_row2 gpurun_out/c3_trace.log | tail -1
for c in c3 c4 c5 c2; do
  args="--config $c --steps 2 --warmup 1"; [ $c = c2 ] && args="--steps 2 --warmup 1 --no-other-configs"
  COUNTER_SETS="FETCH_SIZE|WRITE_SIZE|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" tools/profile.sh r03$c $args || exit $?
  python3 tools/prof_summary.py gpurun_out/prof_r03$c --json gpurun_out/prof_r03$c/summary.json > gpurun_out/prof_r03$c/summary.txt || exit $?
done
exit 0
