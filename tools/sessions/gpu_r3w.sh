#!/bin/bash
# round-3 GPU session W: where the c5 split walk's waves wait (SQ / LDS / TA counters)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
COUNTER_SETS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS|SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE|SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR|TA_BUSY_avr TA_TA_BUSY_sum" NO_KT=0 tools/profile.sh r3w --config c5 --steps 1 --warmup 0 || exit $?
python3 tools/prof_summary.py gpurun_out/prof_r3w > gpurun_out/prof_r3w/summary.txt
grep -A30 'k_r2c_walk2' gpurun_out/prof_r3w/summary.txt | head -32
grep -A30 'k_firstq' gpurun_out/prof_r3w/summary.txt | head -32
exit 0
