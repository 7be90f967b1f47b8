# reference-mode (1 episode / step) kernel profile, then accuracy sweep part 2
ROOT=$PWD
mkdir -p gpurun_out/acc3 gpurun_out/ep1
timeout -k 10 120 python bench.py --episodes-per-gpu 1 --steps 300 --warmup 20 > gpurun_out/ep1/b_ep1_graph.log 2>&1 || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_ep1 -o run --output-format rocpd -- python3 $ROOT/bench.py --episodes-per-gpu 1 --steps 50 --warmup 10 > $ROOT/gpurun_out/ep1/pb.log 2>&1) || exit $?
DB=$(ls /tmp/prof_ep1/*/*.db /tmp/prof_ep1/*.db 2>/dev/null | head -1)
python tools/rocpd_summary.py $DB --steps 60 > gpurun_out/ep1/sum.txt 2>&1
python tools/rocpd_summary.py $DB --sequence sample_episodes > gpurun_out/ep1/seq.txt 2>&1
PAR=6 bash tools/accuracy_sweep.sh gpurun_out/acc3 "0 1 2" "1 5" "^(ce_paper_t50|ce_paper_f50_d5|ce_paper_u128)$"
