#!/bin/bash
# round-3 GPU session P: is the write-rate drop after long full-bandwidth runs thermal / power?
# rocm-smi telemetry every 2 s beside: alloc_rate (fresh), two c5 bench runs, alloc_rate right
# after, a 90 s idle pause, alloc_rate again
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
( while true; do echo "t=$(date +%s.%N)"; rocm-smi -t -P -c 2>/dev/null | grep -E 'GPU\[0\]' ; sleep 2; done ) > gpurun_out/p_smi.log 2>&1 &
SP=$!
trap 'kill $SP 2>/dev/null' EXIT
mark() { echo "MARK $1 t=$(date +%s.%N)" >> gpurun_out/p_smi.log; echo "== $1"; }
mark fresh; timeout -k 10 300 tools/experiments/alloc_rate 64 2 | grep -v free || exit $?
mark c5a; timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/p_c5a.log 2>&1 || exit $?
mark c5b; timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/p_c5b.log 2>&1 || exit $?
mark after; timeout -k 10 300 tools/experiments/alloc_rate 64 2 | grep -v free || exit $?
mark pause; sleep 90
mark rested; timeout -k 10 300 tools/experiments/alloc_rate 64 2 | grep -v free || exit $?
mark c2; timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-other-configs --steps 5 --warmup 2 > gpurun_out/p_c2.log 2>&1 || exit $?
grep '^{' gpurun_out/p_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['stream_copy_gbs'])"
mark end
exit 0
