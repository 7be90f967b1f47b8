# BERT attention backward with row-major LDS images + hardware-transposed reads: BERT GPU tests,
# bench, and a kernel-trace profile of the bench
OUT=${1:-gpurun_out/r3n}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bert_gpu.py -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --encoder bert --steps 5 --warmup 2 > $OUT/bbert.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' $OUT/bbert.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --encoder bert --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
