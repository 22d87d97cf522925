#!/bin/bash
# rocprofv3 passes over one bench command: kernel trace + stats, then PMC counters in their
# own runs (gfx950: FETCH_SIZE and WRITE_SIZE cannot share a pass).  Usage:
#   tools/profile.sh <tag> <bench args...>
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/prof_$tag; mkdir -p $out
stop() { case $1 in 124|137|134|139) echo "fault-class exit $1: stopping"; exit $1;; esac; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $out/kt.log 2>&1; rc=$?; echo "kt rc=$rc"; stop $rc
[ "${NO_PMC:-0}" = 1 ] && exit 0
SETS=${COUNTER_SETS:-"FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS|SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"}
IFS='|' read -ra SETARR <<< "$SETS"
for set in "${SETARR[@]}"; do
  n=$(echo $set | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 150 rocprofv3 --pmc $set -d $out/pmc_$n -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $out/pmc_$n.log 2>&1; rc=$?; echo "pmc $n rc=$rc"; stop $rc
done
exit 0
