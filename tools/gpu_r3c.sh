# Round-3 check of the lean BPTT step + ragged tiles: all GPU tests, A/B, kernel stats.
set -o pipefail
OUT=gpurun_out/r3_c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $OUT/tests.log; if [ $rc -gt 1 ]; then exit $rc; fi
REPS=2 bash tools/ab_configs.sh $OUT/ab "variants/_ina_kernels_oldbwd.so|--ragged 0" "-|--ragged 0" \
  "variants/_ina_kernels_noslp.so|--ragged 0" "-|--ragged 1" "-|--skip-padding 1" > $OUT/ab.txt 2>&1 && \
bash tools/gpu_prof.sh $OUT/prof
