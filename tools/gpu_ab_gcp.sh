# A/B on one box: lstm_bwd dG image stride (in-tree) vs GT*16+4 (variants/_ina_kernels_gcp0.so), kernel times
# (historical: the stride knob INA_LSTM_GCP_PLAIN was removed after this neutral A/B)
OUT=${1:-gpurun_out/ab_gcp}
ROOT=$PWD
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/new$i -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/new$i.log 2>&1 || exit $?
  INA_KERNEL_LIB=$ROOT/variants/_ina_kernels_gcp0.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/old$i -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/old$i.log 2>&1 || exit $?
done
cd $ROOT
for v in new1 old1 new2 old2; do echo "$v $(python tools/rocpd_summary.py $OUT/$v/run_results.db --steps 25 --top 3 2>&1 | grep lstm_bwd)"; done
