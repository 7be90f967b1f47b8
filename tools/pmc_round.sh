# Two rocprofv3 PMC passes over a short bench.py run (counters only with --kernel-trace/--stats, never
# with sys/runtime traces), summarised per kernel by tools/pmc_summary.py.
# usage (on the box): bash tools/pmc_round.sh OUTDIR [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
ROOT=$PWD
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS \
  -d /tmp/pmcA -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 2 "$@" > $ROOT/$OUT/passA.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  -d /tmp/pmcB -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 2 "$@" > $ROOT/$OUT/passB.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE \
  -d /tmp/pmcC -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 2 "$@" > $ROOT/$OUT/passC.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE \
  -d /tmp/pmcD -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 2 "$@" > $ROOT/$OUT/passD.log 2>&1 && \
mkdir -p $ROOT/$OUT/csv && cp $(find /tmp/pmcA -name '*counter_collection.csv' | head -1) $ROOT/$OUT/csv/A_counter_collection.csv && \
cp $(find /tmp/pmcB -name '*counter_collection.csv' | head -1) $ROOT/$OUT/csv/B_counter_collection.csv && \
cp $(find /tmp/pmcC -name '*counter_collection.csv' | head -1) $ROOT/$OUT/csv/C_counter_collection.csv && \
cp $(find /tmp/pmcD -name '*counter_collection.csv' | head -1) $ROOT/$OUT/csv/D_counter_collection.csv && \
cd $ROOT && python tools/pmc_summary.py $OUT/csv > $OUT/summary.txt 2>&1
