set -o pipefail
mkdir -p gpurun_out/bert_ab
timeout -k 10 300 python -u -m pytest tests/test_bert_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/bert_ab/tests.log 2>&1 && \
timeout -k 10 300 python bench.py --encoder bert --steps 5 --warmup 2 > gpurun_out/bert_ab/b1.log 2>&1 && \
timeout -k 10 300 python bench.py --encoder bert --steps 5 --warmup 2 > gpurun_out/bert_ab/b2.log 2>&1
