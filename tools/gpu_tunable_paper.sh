# Paper configuration with PyTorch TunableOp GEMM autotuning: base, tune (writes the table), tuned.
OUT=${1:-gpurun_out/tunable_paper}
mkdir -p $OUT
A="--hidden 128 --word-dim 300 --query 20 --episodes-per-gpu 256"
timeout -k 10 300 python bench.py $A --steps 10 --warmup 3 > $OUT/base.log 2>&1 || exit $?
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_results%d.csv \
timeout -k 10 700 python bench.py $A --steps 3 --warmup 3 > $OUT/tune.log 2>&1 || exit $?
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_results%d.csv \
timeout -k 10 300 python bench.py $A --steps 10 --warmup 3 > $OUT/tuned.log 2>&1
