set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
# generic odd-radix sizes at ~8 GiB per direction: 11^4, 13^3*8, 17*4096, 23*8^3, 31*8^3, 53*4096
for nb in "14641 36000" "17576 30000" "69632 7700" "11776 45000" "15872 34000" "217088 2500" "16384 32768"; do
  set -- $nb
  timeout -k 10 120 python bench.py --config c3 --n $1 --batch $2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/odd_$1.log 2>&1; rc=$?
  echo "N=$1 batch=$2 rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/odd_$1.log) $(grep -o '"passes": [0-9]*' gpurun_out/odd_$1.log)"
  case $rc in 124|137|134|139) exit $rc;; esac
done
