set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/experiments/fz2b.sh || exit $?
export HSFFT_FUSED=2 HSFFT_FZ_SPIN=100000 HSFFT_FZ_LAG=6
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/pmc_fz2_$c -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --batch 1024 > gpurun_out/pmc_fz2_$c.log 2>&1; rc=$?; echo "pmc $c rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done
