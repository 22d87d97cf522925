#!/bin/bash
# round-3 GPU session B: parity of the rotated r2c walk and the merged-acquire Bluestein launch,
# c4 merged vs per-wait acquire, c5 walk orders (+ FETCH_SIZE of the split kernel), and the
# c2 replica with the B-role row prefetch.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('pass_ms'))"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "r2c_walk or persistent" > gpurun_out/pytest_r3b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3b.log
case $rc in 0) ;; *) exit $rc;; esac
for m in 1 0 1 0; do
  HSFFT_BX_MERGE=$m timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 10 > gpurun_out/b_c4_m$m.log 2>&1 || exit $?
  one gpurun_out/b_c4_m$m.log "c4 merge=$m"
done
for spec in "0 32" "2 8" "2 16" "2 32" "0 32"; do
  set -- $spec
  HSFFT_R2C_ORDER=$1 HSFFT_R2C_WT=$2 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/b_c5_o$1_w$2.log 2>&1 || exit $?
  one gpurun_out/b_c5_o$1_w$2.log "c5 order=$1 wt=$2"
done
for spec in "0 32" "1 8" "2 16"; do
  set -- $spec
  HSFFT_R2C_ORDER=$1 HSFFT_R2C_WT=$2 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c5_o$1_w$2 -o pmc --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/pmc_c5_o$1_w$2.log 2>&1 || exit $?
  echo "pmc c5 order=$1 wt=$2 done"
done
timeout -k 10 300 tools/experiments/c2_replica > gpurun_out/c2_replica_b.log 2>&1 || exit $?
cat gpurun_out/c2_replica_b.log
exit 0
