# BERT bench with PyTorch TunableOp GEMM autotuning (hipBLASLt / rocBLAS solutions per shape); the tuned
# table lands in $OUT/tunableop_results0.csv.  usage (on the box): bash tools/gpu_tunable.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/tunable}
mkdir -p $OUT
timeout -k 10 300 python bench.py --encoder bert --steps 5 --warmup 2 > $OUT/base.log 2>&1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_results%d.csv \
timeout -k 10 900 python bench.py --encoder bert --steps 5 --warmup 3 > $OUT/tune.log 2>&1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_results%d.csv \
timeout -k 10 300 python bench.py --encoder bert --steps 5 --warmup 2 > $OUT/tuned.log 2>&1
exit 0
