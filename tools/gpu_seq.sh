set -o pipefail
ROOT=$PWD
mkdir -p gpurun_out/seq
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/pseq -o run --output-format rocpd -- python3 $ROOT/bench.py --steps 10 --warmup 3 > $ROOT/gpurun_out/seq/b.log 2>&1 || exit 1
cd $ROOT
DB=$(ls /tmp/pseq/*/*.db /tmp/pseq/*.db 2>/dev/null | head -1)
python3 -c "import sqlite3;c=sqlite3.connect('$DB');print([r[1] for r in c.execute('pragma table_info(kernels)')])" > gpurun_out/seq/cols.txt 2>&1
python3 tools/rocpd_summary.py $DB --sequence adam_kernel > gpurun_out/seq/seq.txt 2>&1
