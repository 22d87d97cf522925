set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for wl in 3; do
HSFFT_WL=$wl timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "config2 or power_of_two or two_pass or c2c_batched_device" -p no:cacheprovider > gpurun_out/wl_test_$wl.log 2>&1; rc=$?; echo "wl=$wl test rc=$rc"; tail -2 gpurun_out/wl_test_$wl.log
case $rc in 124|137|134|139) exit $rc;; esac
done
SKIP_TESTS=1 bash tools/gpu_check.sh "HSFFT_WL=1|--steps 5 --warmup 2" "HSFFT_WL=2|--steps 5 --warmup 2" "HSFFT_WL=3|--steps 5 --warmup 2" "HSFFT_WL=3;HSFFT_DEV_ALIAS=1|--steps 5 --warmup 2" "HSFFT_WL=1;HSFFT_WL_PREF=1|--steps 5 --warmup 2" "HSFFT_WL=1;HSFFT_WL_T=8|--steps 5 --warmup 2" "HSFFT_WL=1;HSFFT_WL_T=2|--steps 5 --warmup 2"
