# LSTM backward: cost of the natural-layout dH reads and of the pos-feature gradient stores (kbench).
set -o pipefail
mkdir -p gpurun_out/ab7
for i in 1 2; do for lib in induction_network_on_fewrel_amd/_ina_kernels.so variants/_ina_kernels_dhlane.so variants/_ina_kernels_nodxp.so; do
  INA_KERNEL_LIB=$PWD/$lib timeout -k 10 200 python tools/kbench.py --reps 30 >> gpurun_out/ab7/kb.log 2>&1 || exit 1
done; done
