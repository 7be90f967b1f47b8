# Round check on the GPU box: all GPU tests, smoke, benches (eager/graph, 5w5s/5w1s), rocprofv3 kernel stats.
# usage (on the box): bash tools/gpu_round.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/round}
ROOT=$PWD
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $OUT/b5.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --graph 1 > $OUT/b5g.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --shot 1 > $OUT/b1.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --shot 1 --graph 1 > $OUT/b1g.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --episodes-per-gpu 2048 > $OUT/b5_2048.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --mode eval > $OUT/beval.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --mode eval --shot 1 > $OUT/beval1.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --mode eval --nota 0.5 > $OUT/bevaln.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --encoder bert > $OUT/bbert.log 2>&1 && \
timeout -k 10 300 python bench.py --hidden 128 --word-dim 300 --query 20 --episodes-per-gpu 256 --steps 10 --warmup 3 > $OUT/bpaper.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rd -o run --output-format rocpd -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/pb.log 2>&1 && \
cd $ROOT && python tools/rocpd_summary.py $(ls /tmp/prof_rd/*/*.db /tmp/prof_rd/*.db 2>/dev/null | head -1) --steps 25 --md $OUT/stats.md --csv $OUT/stats.csv > $OUT/sum.txt 2>&1
