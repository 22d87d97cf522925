#!/bin/bash
# round-3 GPU session F: c5 split walk length / order sweep with FETCH_SIZE per setting
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
one() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'])"; }
for spec in "2 16" "2 8" "2 6" "2 12" "2 24" "0 32" "2 16"; do
  set -- $spec
  HSFFT_R2C_ORDER=$1 HSFFT_R2C_WT=$2 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/f_c5_o$1_w$2.log 2>&1 || exit $?
  one gpurun_out/f_c5_o$1_w$2.log "c5 order=$1 wt=$2"
done
for spec in "2 8" "2 12" "2 16" "0 32"; do
  set -- $spec
  HSFFT_R2C_ORDER=$1 HSFFT_R2C_WT=$2 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fpmc_o$1_w$2 -o pmc --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/fpmc_o$1_w$2.log 2>&1 || exit $?
  python3 - "$1" "$2" <<'PY'
import csv,sys,collections
o,w=sys.argv[1:3]
agg=collections.defaultdict(list)
for r in csv.DictReader(open(f"gpurun_out/fpmc_o{o}_w{w}/pmc_counter_collection.csv")):
    agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
for k,v in agg.items():
    if "walk2" in k: print(f"FETCH order={o} wt={w}: {2*sum(v)/len(v)*1024/1e9:.2f} GB per launch (x2 corrected), {len(v)} launches")
PY
done
exit 0
