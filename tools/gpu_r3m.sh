# BERT with the gradient slabs on the step glue: BERT GPU tests + bench + DP rehearsal on one card
OUT=${1:-gpurun_out/r3m}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bert_gpu.py tests/test_dp_gpu.py -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --encoder bert --steps 5 --warmup 2 > $OUT/bbert.log 2>&1
