# Quick GPU check after a kernel change: encoder/attention GPU tests, 5w5s + 5w1s bench, rocprofv3 kernel stats.
# usage (on the box): bash tools/gpu_quick.sh OUTDIR [pytest -k expr]
set -o pipefail
OUT=${1:-gpurun_out/quick}
K=${2:-"attention or fused or encoder or full_model or glue"}
ROOT=$PWD
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $OUT/b5.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --shot 1 > $OUT/b1.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_q -o run --output-format rocpd -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/pb.log 2>&1 && \
cd $ROOT && python tools/rocpd_summary.py $(ls /tmp/prof_q/*/*.db /tmp/prof_q/*.db 2>/dev/null | head -1) --steps 25 --md $OUT/stats.md --csv $OUT/stats.csv > $OUT/sum.txt 2>&1
