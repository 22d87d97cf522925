#!/bin/bash
# round-3 GPU session AD: small host-buffer fft_exec whose one-workgroup kernel stores the host
# completion word itself (HSFFT_SMALL_FLAG=2, default) -- drop-in sweeps and threaded tests,
# then c1 with 2 / 1 (command-processor word) / 0 (stream wait) interleaved three times
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "dropin or threads or c_caller or config1 or host or every_length" > gpurun_out/pytest_r3ad.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3ad.log
case $rc in 0) ;; *) exit $rc;; esac
for pass in 1 2 3; do
  for f in 2 1 0; do
    HSFFT_SMALL_FLAG=$f timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline > gpurun_out/ad_c1_f${f}_$pass.log 2>&1 || exit $?
    echo "c1 flag=$f pass=$pass $(grep '^{' gpurun_out/ad_c1_f${f}_$pass.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("latency_us"))')"
  done
done
exit 0
