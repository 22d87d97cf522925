#!/bin/bash
# GPU-box session: parity tests, then bench variants given as "ENV=..;ENV=.." strings.
# Stops at the first fault-class exit (timeout/abort/segfault), per the pool rules.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
stop() { case $1 in 124|137|134|139) echo "fault-class exit $1: stopping"; exit $1;; esac; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; stop $rc
fi
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=$(echo "$spec" | cut -d'|' -f1); bargs=$(echo "$spec" | cut -s -d'|' -f2)
  echo "=== [$i] env: $envs args: ${bargs:-default}"
  env $(echo "$envs" | tr ';' ' ') timeout -k 10 300 python bench.py ${CPU_BASE:---no-cpu-baseline --no-other-configs} ${bargs:---steps 5 --warmup 2} > gpurun_out/bench_$i.log 2>&1
  rc=$?; echo "rc=$rc"; python3 -c "
import json,sys
for l in open('gpurun_out/bench_$i.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline',{})
        print('  value', d['value'], d['unit'], ' ms/step', d['ms_per_step'], ' hbm GB/s', d.get('achieved_hbm_gbs'), ' passes', d['config'].get('passes'), ' pass_ms', r.get('pass_ms'), ' frac', r.get('frac'), ' cpu', d.get('cpu_baseline',{}).get('value'))
" 2>/dev/null || tail -5 gpurun_out/bench_$i.log
  stop $rc
done
exit 0
