# A/B on one box: rec_attn_bwd at 3 waves/SIMD (in-tree, 19 VGPRs spilled) vs 2 (variants/_ina_kernels_ra2.so,
# no spills): kernel times from rocprofv3, two rounds.  Variant: INA_BUILD_TAG=ra2 INA_VARIANT_FLAGS=-DINA_RA_BWD_WAVES=2
OUT=${1:-gpurun_out/ab_ra}
ROOT=$PWD
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/w3_$i -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/w3_$i.log 2>&1 || exit $?
  INA_KERNEL_LIB=$ROOT/variants/_ina_kernels_ra2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/w2_$i -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/w2_$i.log 2>&1 || exit $?
done
cd $ROOT
for v in w3_1 w2_1 w3_2 w2_2; do echo "$v $(python tools/rocpd_summary.py $OUT/$v/run_results.db --steps 25 --top 4 2>&1 | grep rec_attn_bwd)"; done
