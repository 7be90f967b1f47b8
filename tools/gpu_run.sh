# One parametrised GPU-box script (replaces the round-3 one-off lease scripts).
# usage (on the box, from the repo root):
#   TESTS="<pytest paths / args>"              GPU tests (empty: none); TESTS_K="<-k expression>" (may hold spaces)
#   BENCH="name|ENV=V ...|bench args;..."      bench.py runs, each with its own env assignments (empty: none)
#   PROF="name|ENV=V ...|bench args;..."       rocprofv3 --kernel-trace --stats runs of bench.py, summarised by
#                                              tools/rocpd_summary.py into OUT/<name>_sum.txt
#   SEQ="<kernel-name substring>"              also OUT/<name>_seq.txt: the last profiled step's kernel sequence
#   bash tools/gpu_run.sh OUT
# Every step has its own time limit; the script stops at the first failure (no GPU step after a fault).
set -o pipefail
OUT=${1:-gpurun_out/run}
ROOT=$PWD
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  if [ -n "$TESTS_K" ]; then
    timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -k "$TESTS_K" -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1
  else
    timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1
  fi
  rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
  [ $rc -ne 0 ] && exit $rc
fi
IFS=';' read -ra RUNS <<< "$BENCH"
for r in "${RUNS[@]}"; do
  [ -z "$r" ] && continue
  IFS='|' read -r name envs args <<< "$r"
  env $envs timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py $args > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $OUT/$name.log)"
  [ $rc -ne 0 ] && { tail -5 $OUT/$name.log; exit $rc; }
done
IFS=';' read -ra PRUNS <<< "$PROF"
for r in "${PRUNS[@]}"; do
  [ -z "$r" ] && continue
  IFS='|' read -r name envs args <<< "$r"
  (cd /tmp && export TMPDIR=/tmp && env $envs timeout -k 10 ${BENCH_TIMEOUT:-300} rocprofv3 --kernel-trace --stats \
     -d /tmp/prof_$name -o run --output-format rocpd -- python3 $ROOT/bench.py $args > $ROOT/$OUT/${name}_prof.log 2>&1)
  rc=$?; echo "prof $name rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/${name}_prof.log; exit $rc; }
  db=$(ls /tmp/prof_$name/*/*.db /tmp/prof_$name/*.db 2>/dev/null | head -1)
  python tools/rocpd_summary.py $db --steps ${PROF_STEPS:-25} --top 30 > $OUT/${name}_sum.txt 2>&1
  [ -n "$SEQ" ] && python tools/rocpd_summary.py $db --sequence "$SEQ" > $OUT/${name}_seq.txt 2>&1
  head -14 $OUT/${name}_sum.txt
done
