#!/bin/bash
# round-4 GPU session W: the r2c walk's four output streams without arithmetic as tiles 8 / 16 /
# 32 / 64 columns wide (tools/experiments/r2c_stride: do wider store segments move the 64-KiB-
# strided output faster?), plus session M's load / store / pitch rows again
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 tools/experiments/r2c_stride 512 > gpurun_out/w_stride.log 2>&1; rc=$?; cat gpurun_out/w_stride.log; exit $rc
