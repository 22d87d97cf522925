#!/bin/bash
# round-3 GPU session A: full GPU suite, config-4 bench (persistent Bluestein with the
# agent-scope acquire) with and without the phase trace, config-3 (row kernel with fused
# [5,5]) against the unfused kernel, the default c2 line, the c2 data-movement replica, and a
# c5 split-order / walk-length sweep.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('pass_ms'))"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3a.log
case $rc in 0|1) ;; *) exit $rc;; esac
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 10 > gpurun_out/b_c4_$i.log 2>&1 || exit $?
  one gpurun_out/b_c4_$i.log c4
done
HSFFT_BX_DEBUG=1 timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/b_c4_dbg.log 2>&1 || exit $?
grep bxcd gpurun_out/b_c4_dbg.log | tail -1
for f in 1 0 1 0; do
  HSFFT_ROW_F23=$f timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 10 > gpurun_out/b_c3_f$f.log 2>&1 || exit $?
  one gpurun_out/b_c3_f$f.log "c3 F23=$f"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-configs > gpurun_out/b_c2.log 2>&1 || exit $?
one gpurun_out/b_c2.log c2
timeout -k 10 300 tools/experiments/c2_replica > gpurun_out/c2_replica.log 2>&1 || exit $?
cat gpurun_out/c2_replica.log
for o in 0 1; do for wt in 8 32; do
  HSFFT_R2C_ORDER=$o HSFFT_R2C_WT=$wt timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/b_c5_o${o}_w$wt.log 2>&1 || exit $?
  one gpurun_out/b_c5_o${o}_w$wt.log "c5 order=$o wt=$wt"
done; done
exit $rc
