#!/bin/bash
# round-3 GPU session AM (third session, final): the driver's round-end steps at HEAD -- GPU
# suite, smoke(), the default bench line -- plus a kernel trace of the c2 step
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3am.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_r3am.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3am.log 2>&1; rc=$?; cat gpurun_out/smoke_r3am.log | tail -2; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_default_r3am.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_default_r3am.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']
    print('value', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'pass_ms', r.get('pass_ms'), 'cpu', d['cpu_baseline']['value'], 'copy', d.get('stream_copy_gbs'), 'place', d.get('placement'))
    for k,v in d.get('other_configs',{}).items(): print(' ', k, v.get('value'), v.get('unit'), v.get('frac'), (v.get('cpu_baseline') or {}).get('value'), (v.get('placement') or {}).get('copy_gbs'))
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3am_c2 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-other-configs > gpurun_out/prof_r3am_c2.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_r3am_c2.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.readline()); print('profiled c2', d['value'], d['roofline'].get('pass_ms'))"
exit 0
