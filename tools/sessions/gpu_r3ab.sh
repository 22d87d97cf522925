#!/bin/bash
# round-3 GPU session AB (final): full GPU suite + the default bench line (placement-checked buffers)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3ab.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py > gpurun_out/bench_default_r3ab.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_default_r3ab.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']
    print('value', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'pass_ms', r.get('pass_ms'), 'cpu', d['cpu_baseline']['value'], 'copy', d.get('stream_copy_gbs'), 'place', d.get('placement'))
    for k,v in d.get('other_configs',{}).items(): print(' ', k, v.get('value'), v.get('unit'), v.get('frac'), (v.get('cpu_baseline') or {}).get('value'), (v.get('placement') or {}).get('copy_gbs'))
"
exit 0
