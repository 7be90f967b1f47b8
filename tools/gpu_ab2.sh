set -o pipefail
mkdir -p gpurun_out/ab
for i in 1 2; do for lib in variants/_ina_kernels_selA.so variants/_ina_kernels_nopos.so; do
  INA_KERNEL_LIB=$PWD/$lib timeout -k 10 200 python tools/kbench.py --reps 50 >> gpurun_out/ab/kb.log 2>&1 || exit 1
done; done
