# GPU check used during kernel work: tests, kernel bench, 5w5s bench, rocprofv3 kernel stats.
# usage (on the box): bash tools/gpu_check.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/check}
ROOT=$PWD
mkdir -p $OUT
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_wide_gpu.py -x -q > $OUT/t.log 2>&1 && \
timeout -k 10 200 python tools/kbench.py > $OUT/kb.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $OUT/b.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_chk -o run --output-format rocpd -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/pb.log 2>&1 && \
cd $ROOT && python tools/rocpd_summary.py $(ls /tmp/prof_chk/*/*.db /tmp/prof_chk/*.db 2>/dev/null | head -1) --steps 25 --md $OUT/stats.md --csv $OUT/stats.csv > $OUT/sum.txt 2>&1
