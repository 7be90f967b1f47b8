# Counter passes (one rocprofv3 --pmc run each, no traces) over tools/gemm_pmc.py: own GEMM vs hipBLASLt.
# usage (on the box): bash tools/gemm_pmc.sh OUTDIR [N K epi]
set -o pipefail
OUT=${1:-gpurun_out/gpmc}; shift
ROOT=$PWD
mkdir -p $OUT/csv
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d /tmp/gpmc$i -o run --output-format csv -- python3 $ROOT/tools/gemm_pmc.py "$@" \
    > $ROOT/$OUT/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $ROOT/$OUT/pass$i.log; exit 1; }
  cp $(find /tmp/gpmc$i -name '*counter_collection.csv' | head -1) $ROOT/$OUT/csv/p${i}_counter_collection.csv
done
cd $ROOT && python tools/pmc_summary.py $OUT/csv > $OUT/summary.txt 2>&1; head -8 $OUT/summary.txt
