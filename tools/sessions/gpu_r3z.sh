#!/bin/bash
# round-3 GPU session Z: small host-buffer fft_exec completing through a host-polled word
# (HSFFT_SMALL_FLAG, default 1) -- the drop-in host-buffer sweeps and the threaded tests, then
# c1 with the word vs the stream wait, interleaved three times
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "dropin or threads or c_caller or smoke or host" > gpurun_out/pytest_r3z.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3z.log
case $rc in 0) ;; *) exit $rc;; esac
for pass in 1 2 3; do
  for f in 1 0; do
    HSFFT_SMALL_FLAG=$f timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline > gpurun_out/z_c1_f${f}_$pass.log 2>&1 || exit $?
    echo "c1 flag=$f pass=$pass $(grep '^{' gpurun_out/z_c1_f${f}_$pass.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("latency_us"), d.get("threads8_us_per_transform"))')"
  done
done
exit 0
