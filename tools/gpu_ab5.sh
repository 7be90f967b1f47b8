# LSTM forward bottleneck decomposition (kbench): stores (hnat / stash), dropout hash, activations.
set -o pipefail
mkdir -p gpurun_out/ab5
for lib in induction_network_on_fewrel_amd/_ina_kernels.so variants/_ina_kernels_nohnat.so variants/_ina_kernels_nostash.so variants/_ina_kernels_nohash.so variants/_ina_kernels_act.so variants/_ina_kernels_allx.so; do
  INA_KERNEL_LIB=$PWD/$lib timeout -k 10 200 python tools/kbench.py --reps 30 >> gpurun_out/ab5/kb.log 2>&1 || exit 1
done
