# rocprofv3 kernel stats of a short bench.py run.  usage (on the box): bash tools/gpu_prof.sh OUTDIR [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/prof}; shift
ROOT=$PWD
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_p -o run --output-format rocpd -- python3 $ROOT/bench.py --steps ${PSTEPS:-20} --warmup ${PWARM:-5} "$@" > $ROOT/$OUT/pb.log 2>&1 && \
cd $ROOT && python tools/rocpd_summary.py $(ls /tmp/prof_p/*/*.db /tmp/prof_p/*.db 2>/dev/null | head -1) --steps $(( ${PSTEPS:-20} + ${PWARM:-5} )) --md $OUT/stats.md --csv $OUT/stats.csv > $OUT/sum.txt 2>&1
