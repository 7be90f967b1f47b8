# LSTM backward decomposition (kbench): stash loads, dH loads, dW accumulation.
set -o pipefail
mkdir -p gpurun_out/ab9
for lib in induction_network_on_fewrel_amd/_ina_kernels.so variants/_ina_kernels_nostash.so variants/_ina_kernels_nodh.so variants/_ina_kernels_nodw.so variants/_ina_kernels_allb.so; do
  INA_KERNEL_LIB=$PWD/$lib timeout -k 10 200 python tools/kbench.py --reps 30 >> gpurun_out/ab9/kb.log 2>&1 || exit 1
done
