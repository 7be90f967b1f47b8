set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 && \
for lib in variants/_ina_kernels_head.so variants/_ina_kernels_pipe0.so induction_network_on_fewrel_amd/_ina_kernels.so; do
  INA_KERNEL_LIB=$PWD/$lib timeout -k 10 300 python tools/kbench.py >> gpurun_out/kbench.log 2>&1 || exit 1
done && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
