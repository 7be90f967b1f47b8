# End-to-end A/B of two kernel libraries with the same Python (bench.py 5w5s), alternating.
set -o pipefail
mkdir -p gpurun_out/ab10
for i in 1 2 3; do for lib in induction_network_on_fewrel_amd/_ina_kernels.so variants/_ina_kernels_head.so; do
  echo "$lib" >> gpurun_out/ab10/b.log
  INA_KERNEL_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 30 --warmup 5 >> gpurun_out/ab10/b.log 2>&1 || exit 1
done; done
