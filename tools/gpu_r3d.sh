# Round-3 check: all GPU tests, then the bench configurations (default / 1-episode steps graph+eager / 5w1s).
set -o pipefail
OUT=gpurun_out/r3_d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $OUT/tests.log; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $OUT/b5.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --shot 1 > $OUT/b1.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 300 --warmup 20 --episodes-per-gpu 1 > $OUT/b_ep1_graph.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 300 --warmup 20 --episodes-per-gpu 1 --graph 0 > $OUT/b_ep1_eager.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --skip-padding 1 > $OUT/b5_skip.log 2>&1
