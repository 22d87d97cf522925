set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "odd or divergences or c2c_batched_device or dropin_host or fixtures" -p no:cacheprovider > gpurun_out/odd_test.log 2>&1; rc=$?; echo "test rc=$rc"; tail -1 gpurun_out/odd_test.log
case $rc in 124|137|134|139) exit $rc;; esac
[ $rc = 0 ] || exit 1
bash tools/oddradix.sh
