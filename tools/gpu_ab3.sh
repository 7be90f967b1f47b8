# LSTM forward bottleneck A/B: default vs VALU-only activations vs no x gathers vs both (kbench).
set -o pipefail
mkdir -p gpurun_out/ab3
for lib in induction_network_on_fewrel_amd/_ina_kernels.so variants/_ina_kernels_act.so variants/_ina_kernels_nox.so variants/_ina_kernels_both.so; do
  INA_KERNEL_LIB=$PWD/$lib timeout -k 10 200 python tools/kbench.py --reps 30 >> gpurun_out/ab3/kb.log 2>&1 || exit 1
done
