# episodes-per-step sweep of the default 5w5s bench (weak-scaling batch choice)
set -o pipefail
OUT=${1:-gpurun_out/sweep}
mkdir -p $OUT
for B in ${SWEEP:-6144 8192 12288 16384 24576 8192 12288 16384}; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --episodes-per-gpu $B >> $OUT/b.log 2>&1 || exit 1
done
