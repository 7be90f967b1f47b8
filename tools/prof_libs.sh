# Same-box per-kernel A/B of kernel libraries: one rocprofv3 kernel-trace run of bench.py per library,
# summarised to OUTDIR/<n>.txt (top kernels).  usage (on the box):
#   bash tools/prof_libs.sh OUTDIR "libA libB ..." [bench args...]     (paths relative to the repo root)
set -o pipefail
OUT=${1:-gpurun_out/pab}; LIBS=$2; shift 2
ROOT=$PWD
mkdir -p $OUT
i=0
for lib in $LIBS; do
  i=$((i + 1))
  export INA_KERNEL_LIB=$ROOT/$lib
  (cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/prof_ab$i && \
   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ab$i -o run --output-format rocpd -- \
     python3 $ROOT/bench.py --steps 20 --warmup 5 "$@" > $ROOT/$OUT/pb$i.log 2>&1) || exit 1
  echo "$lib" > $OUT/$i.txt
  python tools/rocpd_summary.py $(ls /tmp/prof_ab$i/*/*.db /tmp/prof_ab$i/*.db 2>/dev/null | head -1) --steps 25 --top 12 \
    >> $OUT/$i.txt 2>&1 || exit 1
done
