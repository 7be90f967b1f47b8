# wide x gather with prefetched position ids: wide / head tests, paper bench, profile
OUT=${1:-gpurun_out/r3q}
ROOT=$PWD
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_wide_gpu.py tests/test_head_wide_gpu.py -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --hidden 128 --word-dim 300 --query 20 --episodes-per-gpu 256 --steps 10 --warmup 3 > $OUT/bpaper.log 2>&1 || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_pj -o run --output-format rocpd -- python3 $ROOT/bench.py --hidden 128 --word-dim 300 --query 20 --episodes-per-gpu 256 --steps 5 --warmup 2 > $ROOT/$OUT/pb.log 2>&1) || exit $?
DB=$(ls /tmp/prof_pj/*/*.db /tmp/prof_pj/*.db 2>/dev/null | head -1)
python tools/rocpd_summary.py $DB --steps 7 --top 60 > $OUT/sum_paper.txt 2>&1
python tools/rocpd_summary.py $DB --sequence sample_episodes > $OUT/seq_paper.txt 2>&1
grep -E "total|wide_x_gather" $OUT/sum_paper.txt; grep -o "\"value\": [0-9.]*" $OUT/bpaper.log
