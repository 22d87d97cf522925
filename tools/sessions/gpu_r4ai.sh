#!/bin/bash
# round-4 GPU session AI: FETCH / WRITE of c4 (the cooperative persistent Bluestein launch) in
# their own passes, without the kernel-trace pass whose process crashed in exit() in session S
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/prof_r4ai_c4; mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d $out/pmc_$c -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --config c4 --steps 3 --warmup 1 > $out/pmc_$c.log 2>&1; rc=$?; echo "pmc $c rc=$rc"
  case $rc in 0) ;; *) tail -5 $out/pmc_$c.log; exit $rc;; esac
done
python3 tools/prof_summary.py $out > $out/summary.txt; grep -A6 "k_bxcd" $out/summary.txt
exit 0
