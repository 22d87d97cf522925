# kernel-trace profiles of c3, c4, c5 (round 2 baseline)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in c5 c4 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$cfg -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --config $cfg --steps 3 --warmup 1 > gpurun_out/kt_$cfg.log 2>&1; rc=$?; echo "$cfg rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/kt_$cfg.log
  case $rc in 124|137|134|139) exit $rc;; esac
done
