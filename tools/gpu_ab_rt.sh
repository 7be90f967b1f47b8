set -o pipefail
mkdir -p gpurun_out/ab_hl
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "head or glue or full_model or routing or hip_graph" > gpurun_out/ab_hl/tests.log 2>&1 && \
bash tools/ab_libs.sh gpurun_out/ab_hl "variants/_ina_kernels_head.so induction_network_on_fewrel_amd/_ina_kernels.so" > gpurun_out/ab_hl/ab.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rd -o run --output-format rocpd -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/ab_hl/pb.log 2>&1 && \
cd $GRAFT_REPO_ROOT && python tools/rocpd_summary.py $(ls /tmp/prof_rd/*/*.db /tmp/prof_rd/*.db 2>/dev/null | head -1) --steps 25 > gpurun_out/ab_hl/sum.txt 2>&1
timeout -k 10 200 python -u -m pytest tests/test_bert_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/ab_hl/bert_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --mode eval > gpurun_out/ab_hl/beval.log 2>&1
