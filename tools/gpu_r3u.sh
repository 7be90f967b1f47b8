# device sampler with the class scopes loaded at once: kernel / ragged tests, headline bench, profile
OUT=${1:-gpurun_out/r3u}
ROOT=$PWD
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ragged_gpu.py tests/test_kernels_gpu.py -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $OUT/b5.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' $OUT/b5.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/prof.log 2>&1) || exit $?
python tools/rocpd_summary.py $OUT/prof/run_results.db --steps 25 --top 40 > $OUT/sum.txt 2>&1
grep -E "total|sample_episodes|ragged" $OUT/sum.txt
