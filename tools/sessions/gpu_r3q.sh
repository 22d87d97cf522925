#!/bin/bash
# round-3 GPU session Q: write-rate timeline of two resident 64 GiB buffers, before and after
# freeing a written 120 GiB buffer (background clearing of freed memory?)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 tools/experiments/alloc_rate w > gpurun_out/q_wipe.log 2>&1 || exit $?
cat gpurun_out/q_wipe.log
exit 0
