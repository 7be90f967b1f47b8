# LSTM forward: cost of the hnat store layout (natural [seq][t][2U] vs direction planes vs lane layout).
set -o pipefail
mkdir -p gpurun_out/ab6
for i in 1 2; do for lib in induction_network_on_fewrel_amd/_ina_kernels.so variants/_ina_kernels_planes.so variants/_ina_kernels_lanes.so; do
  INA_KERNEL_LIB=$PWD/$lib timeout -k 10 200 python tools/kbench.py --reps 30 >> gpurun_out/ab6/kb.log 2>&1 || exit 1
done; done
