#!/bin/bash
# round-4 GPU session AF: c1 floor with the input written by the host into host-mapped
# fine-grained device memory instead of a page-locked slot (tools/experiments/c1_latency)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 tools/experiments/c1_latency > gpurun_out/af_c1.log 2>&1; rc=$?; cat gpurun_out/af_c1.log; exit $rc
