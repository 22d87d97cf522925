set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 120 --timeout-method thread -k "roles or large_batch" -p no:cacheprovider > gpurun_out/fz2_test.log 2>&1; rc=$?; echo "test rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/fz2_test.log | tail -12
case $rc in 124|137|134|139) exit $rc;; esac
[ $rc = 0 ] || exit 1
SKIP_TESTS=1 bash tools/gpu_check.sh "HSFFT_FUSED=2|--steps 5 --warmup 2" "HSFFT_FUSED=2;HSFFT_FZ_LAG=2|--steps 5 --warmup 2" "HSFFT_FUSED=2;HSFFT_FZ_LAG=6|--steps 5 --warmup 2" "HSFFT_FUSED=2;HSFFT_FZ_SPIN=0|--steps 5 --warmup 2" "HSFFT_FUSED=2;HSFFT_FZ2_NA=320;HSFFT_FZ2_NB=256|--steps 5 --warmup 2"
