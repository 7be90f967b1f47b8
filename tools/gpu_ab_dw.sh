# A/B on one box: NTN reference-head dw summed per workgroup in LDS (in-tree) vs per-episode slab rows
# (the baseline library was built from the previous commit in a temporary git worktree)
# (variants/_ina_kernels_dwold.so, built from the previous commit): kernel times, two rounds
OUT=${1:-gpurun_out/ab_dw}
ROOT=$PWD
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/new$i -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/new$i.log 2>&1 || exit $?
  INA_KERNEL_LIB=$ROOT/variants/_ina_kernels_dwold.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/old$i -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/old$i.log 2>&1 || exit $?
done
cd $ROOT
for v in new1 old1 new2 old2; do python tools/rocpd_summary.py $OUT/$v/run_results.db --steps 25 --top 30 > $OUT/$v.txt 2>&1; echo "$v $(grep total $OUT/$v.txt) | $(grep ntn_bwd $OUT/$v.txt | awk '{print $4}') | slab $(grep slab_partial $OUT/$v.txt | awk '{print $4}')"; done
