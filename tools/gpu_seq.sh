# Kernel sequence of one train step (start order, duration, gap) from a rocprofv3 kernel trace.
# usage (on the box): bash tools/gpu_seq.sh OUTDIR [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/seq}; shift
ROOT=$PWD
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/pseq -o run --output-format rocpd -- python3 $ROOT/bench.py "$@" > $ROOT/$OUT/b.log 2>&1 || exit 1
cd $ROOT
DB=$(ls /tmp/pseq/*/*.db /tmp/pseq/*.db 2>/dev/null | head -1)
python3 tools/rocpd_summary.py $DB --sequence adam_kernel > $OUT/seq.txt 2>&1
python3 tools/rocpd_summary.py $DB --top 40 > $OUT/sum.txt 2>&1
