#!/bin/bash
# round-4 GPU session M: the r2c walk's memory pattern without arithmetic (tools/experiments/
# r2c_stride): tile loads at the 64-KiB row stride vs padded pitches, the four output streams,
# both together
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 tools/experiments/r2c_stride 512 > gpurun_out/m_stride.log 2>&1; rc=$?; cat gpurun_out/m_stride.log; exit $rc
