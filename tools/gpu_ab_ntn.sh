# A/B: NTN workgroup of 4 episodes (variants/_ina_kernels_ntn4.so) vs 8 (in-tree library)
OUT=${1:-gpurun_out/ab_ntn}
ROOT=$PWD
V=$ROOT/variants/_ina_kernels_ntn4.so
mkdir -p $OUT
INA_KERNEL_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "head" -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $OUT/base$i.log 2>&1 || exit $?
  INA_KERNEL_LIB=$V timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $OUT/var$i.log 2>&1 || exit $?
  echo "base $(grep -o '"value": [0-9.]*' $OUT/base$i.log)  ntn4 $(grep -o '"value": [0-9.]*' $OUT/var$i.log)"
done
(cd /tmp && export TMPDIR=/tmp && INA_KERNEL_LIB=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/prof.log 2>&1) || exit $?
python tools/rocpd_summary.py $OUT/prof/run_results.db --steps 25 --top 14 > $OUT/sum.txt 2>&1
grep -E "total|ntn" $OUT/sum.txt
