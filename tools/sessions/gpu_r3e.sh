#!/bin/bash
# round-3 GPU session E: the default bench exactly as the driver runs it
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_default_r3.log 2>&1; rc=$?; echo "bench rc=$rc"
grep '^{' gpurun_out/bench_default_r3.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']
    print('value', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'traffic', r['traffic'], 'cpu', d['cpu_baseline']['value'], 'copy', d.get('stream_copy_gbs'))
    for k,v in d.get('other_configs',{}).items(): print(' ', k, v.get('value'), v.get('unit'), v.get('frac'), (v.get('roofline') or {}).get('traffic'), (v.get('cpu_baseline') or {}).get('value'))
"
exit $rc
