# Paper configuration (u=128, 300-d words, 5-way 5-shot, Q=20): wide path throughput + kernel stats.
set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_wide_gpu.py -x -q --timeout 150 --timeout-method thread > ${1:-gpurun_out/paper}.tests.log 2>&1 || exit 1
OUT=${1:-gpurun_out/paper}
ROOT=$PWD
mkdir -p $OUT
timeout -k 10 300 python bench.py --hidden 128 --word-dim 300 --query 20 --episodes-per-gpu 256 --steps 5 --warmup 2 > $OUT/b256.log 2>&1 && \
timeout -k 10 300 python bench.py --hidden 128 --word-dim 300 --query 20 --episodes-per-gpu 1024 --steps 5 --warmup 2 > $OUT/b1024.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_pp -o run --output-format rocpd -- python3 $ROOT/bench.py --hidden 128 --word-dim 300 --query 20 --episodes-per-gpu 256 --steps 5 --warmup 2 > $ROOT/$OUT/pb.log 2>&1 && \
cd $ROOT && python tools/rocpd_summary.py $(ls /tmp/prof_pp/*/*.db /tmp/prof_pp/*.db 2>/dev/null | head -1) --steps 7 > $OUT/sum.txt 2>&1
