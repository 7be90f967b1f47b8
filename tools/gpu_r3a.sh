# Round-3 first GPU check: GPU tests, default bench, roofline passes.
set -o pipefail
OUT=gpurun_out/r3_a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $OUT/tests.log
# 0 = pass, 1 = test failures: carry on; anything else (timeout / abort / crash) ends the call
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $OUT/b5.log 2>&1 && \
bash tools/pmc_roofline.sh $OUT/roofline
