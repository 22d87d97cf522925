#!/bin/bash
# round-3 GPU session I: r2c walk parity incl. rotation classes, then c5 order sweep (twice,
# interleaved) and FETCH of the split kernel for the class variants
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'])"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "r2c_walk" > gpurun_out/pytest_r3i.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3i.log
case $rc in 0) ;; *) exit $rc;; esac
for pass in 1 2; do for spec in "2 16" "3 16" "5 16" "9 8" "5 8" "0 32"; do
  set -- $spec
  HSFFT_R2C_ORDER=$1 HSFFT_R2C_WT=$2 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/i_c5_o$1_w$2_$pass.log 2>&1 || exit $?
  one gpurun_out/i_c5_o$1_w$2_$pass.log "c5 order=$1 wt=$2 pass=$pass"
done; done
for spec in "3 16" "5 16" "9 8"; do
  set -- $spec
  HSFFT_R2C_ORDER=$1 HSFFT_R2C_WT=$2 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ipmc_o$1_w$2 -o pmc --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/ipmc_o$1_w$2.log 2>&1 || exit $?
  python3 - "$1" "$2" <<'PY'
import csv,sys,collections
o,w=sys.argv[1:3]
agg=collections.defaultdict(list)
for r in csv.DictReader(open(f"gpurun_out/ipmc_o{o}_w{w}/pmc_counter_collection.csv")):
    agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
for k,v in agg.items():
    if "walk2" in k: print(f"FETCH order={o} wt={w}: {2*sum(v)/len(v)*1024/1e9:.2f} GB per launch (x2 corrected)")
PY
done
exit 0
