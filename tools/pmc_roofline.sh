# Roofline evidence for one bench configuration (on the GPU box):
#   1. un-profiled kernel times: rocprofv3 --kernel-trace --stats -> stats.csv (tools/rocpd_summary.py)
#   2. four rocprofv3 --pmc passes (counters only with --kernel-trace, never with sys/runtime traces),
#      each within the per-block counter limits (8 SQ, FETCH_SIZE / WRITE_SIZE alone in TCC, 1 GRBM)
#   3. tools/roofline.py -> roofline.md (bytes, TB/s, MFMA / VALU busy, occupancy per kernel)
# usage: bash tools/pmc_roofline.sh OUTDIR [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/roofline}; shift
ROOT=$PWD
mkdir -p $OUT/csv
cd /tmp && export TMPDIR=/tmp
B="--steps 3 --warmup 2 $*"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/rl_stats -o run --output-format rocpd -- python3 $ROOT/bench.py $B > $ROOT/$OUT/stats_run.log 2>&1 && \
python3 $ROOT/tools/rocpd_summary.py $(ls /tmp/rl_stats/*/*.db /tmp/rl_stats/*.db 2>/dev/null | head -1) --steps 5 --csv $ROOT/$OUT/stats.csv > $ROOT/$OUT/sum.txt 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -d /tmp/rlA -o run --output-format csv -- python3 $ROOT/bench.py $B > $ROOT/$OUT/passA.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  -d /tmp/rlB -o run --output-format csv -- python3 $ROOT/bench.py $B > $ROOT/$OUT/passB.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  -d /tmp/rlC -o run --output-format csv -- python3 $ROOT/bench.py $B > $ROOT/$OUT/passC.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE \
  -d /tmp/rlD -o run --output-format csv -- python3 $ROOT/bench.py $B > $ROOT/$OUT/passD.log 2>&1 && \
for p in A B C D; do cp $(find /tmp/rl$p -name '*counter_collection.csv' | head -1) $ROOT/$OUT/csv/${p}_counter_collection.csv || exit 1; done && \
cd $ROOT && python3 tools/roofline.py $OUT/csv --stats $OUT/stats.csv --steps 5 --md $OUT/roofline.md > $OUT/roofline.txt 2>&1
