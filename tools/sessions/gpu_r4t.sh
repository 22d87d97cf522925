#!/bin/bash
# round-4 GPU session T: the edited-twiddle refresh test through the row kernel's transposed
# last-stage copy, the 12600 row variants, the every-word c3 check at full size
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "12600 or config3_every_word" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/t_pytest.log | tail -5; exit $rc
