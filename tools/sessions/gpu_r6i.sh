#!/bin/bash
# round-6 GPU session I: the §8f rows' lines at HEAD -- batched convolution, c2r at scale, the
# compact r2c layout, host-resident c2c rows (PCIe-inclusive).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local tag=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r6i_$tag.log 2>&1; local rc=$?; echo "== $tag rc=$rc"; grep "^{" gpurun_out/r6i_$tag.log | cut -c1-420; [ $rc = 0 ] || exit $rc; }
run convolve --convolve 256 --steps 5 --warmup 2
run c5_c2r --config c5 --c2r --steps 3 --warmup 1 --no-cpu-baseline
run c5_compact --config c5 --r2c-compact --steps 3 --warmup 1 --no-cpu-baseline
run c2_host --config c2 --no-other-configs --steps 3 --warmup 1 --no-cpu-baseline --host-rows 256
exit 0
