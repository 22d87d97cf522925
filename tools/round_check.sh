#!/bin/bash
# full GPU suite, then the default bench exactly as the driver runs it (all configs + CPU baseline)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"
grep '^{' gpurun_out/bench_default.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']
    print('value', d['value'], 'frac', r['frac'], 'cpu', d['cpu_baseline']['value'])
    for k,v in d.get('other_configs',{}).items(): print(' ', k, v.get('value'), v.get('unit'), v.get('roofline',{}).get('frac'))
"
exit $rc
