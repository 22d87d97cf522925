set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for sp in 1 3; do
HSFFT_BLUE_SPLIT=$sp timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "bluestein or config4 or 99991" -p no:cacheprovider > gpurun_out/bs_test_$sp.log 2>&1; rc=$?; echo "split=$sp test rc=$rc"; tail -1 gpurun_out/bs_test_$sp.log
case $rc in 124|137|134|139) exit $rc;; esac
done
SKIP_TESTS=1 bash tools/gpu_check.sh "|--config c4 --steps 5 --warmup 2" "HSFFT_BLUE_SPLIT=1|--config c4 --steps 5 --warmup 2" "HSFFT_BLUE_SPLIT=2|--config c4 --steps 5 --warmup 2" "HSFFT_BLUE_SPLIT=3|--config c4 --steps 5 --warmup 2"
