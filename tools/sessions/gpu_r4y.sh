#!/bin/bash
# round-4 GPU session Y: where c3's row kernel spends its cycles -- LDS bank conflicts, LDS / VALU
# activity and wave waits of k_row2 (F45, transposed stage-5 twiddles), SQ counters in their own
# passes
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
COUNTER_SETS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS|SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" tools/profile.sh r4y_c3 --config c3 --steps 4 --warmup 1 || exit $?
python3 tools/prof_summary.py gpurun_out/prof_r4y_c3 > gpurun_out/prof_r4y_c3/summary.txt; grep -A14 -E "^void mr" gpurun_out/prof_r4y_c3/summary.txt
exit 0
