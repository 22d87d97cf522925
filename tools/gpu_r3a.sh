#!/bin/bash
# round-3 GPU session A: full GPU suite, then config-4 bench (persistent Bluestein with the
# agent-scope acquire) with and without the phase trace, then the default c2 line.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3a.log
case $rc in 0|1) ;; *) exit $rc;; esac
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 10 > gpurun_out/b_c4_$i.log 2>&1 || exit $?
  grep '^{' gpurun_out/b_c4_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
HSFFT_BX_DEBUG=1 timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/b_c4_dbg.log 2>&1 || exit $?
grep bxcd gpurun_out/b_c4_dbg.log | tail -2
timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-configs > gpurun_out/b_c2.log 2>&1 || exit $?
grep '^{' gpurun_out/b_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], d['roofline'].get('pass_ms'))"
exit $rc
