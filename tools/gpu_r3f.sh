# wide BiLSTM v3 (prefetch, tile-major stash, contiguous unit ownership): tests, bench, kernel stats + step sequence
set -o pipefail
OUT=${1:-gpurun_out/r3_f}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $OUT/tests.log; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --hidden 128 --word-dim 300 --query 20 --episodes-per-gpu 256 --steps 5 --warmup 2 > $OUT/bpaper.log 2>&1 && \
PSTEPS=5 PWARM=2 bash tools/gpu_prof.sh $OUT/prof --hidden 128 --word-dim 300 --query 20 --episodes-per-gpu 256 && \
python tools/rocpd_summary.py $(ls /tmp/prof_p/*/*.db /tmp/prof_p/*.db 2>/dev/null | head -1) --sequence adam_kernel > $OUT/prof/seq.txt 2>&1
