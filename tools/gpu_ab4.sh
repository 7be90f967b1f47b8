# x_gather A/B: xg-fed forward vs in-kernel-gather forward (+x_gather for the bwd) vs no x_gather.
set -o pipefail
mkdir -p gpurun_out/ab4
for i in 1 2; do for lib in induction_network_on_fewrel_amd/_ina_kernels.so variants/_ina_kernels_fg.so variants/_ina_kernels_fgskip.so; do
  INA_KERNEL_LIB=$PWD/$lib timeout -k 10 200 python tools/kbench.py --reps 30 >> gpurun_out/ab4/kb.log 2>&1 || exit 1
done; done
