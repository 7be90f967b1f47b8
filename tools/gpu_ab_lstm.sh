# lstm_bwd lean-step check: gradient A/B vs the base build, encoder tests, same-box bench A/B.
set -o pipefail
OUT=gpurun_out/r3_b
mkdir -p $OUT
INA_KERNEL_LIB=$PWD/variants/_ina_kernels_base.so timeout -k 10 120 python tools/grad_dump.py $OUT/g_base.pt > $OUT/gd.log 2>&1 && \
timeout -k 10 120 python tools/grad_dump.py $OUT/g_new.pt >> $OUT/gd.log 2>&1 && \
python tools/grad_dump.py --cmp $OUT/g_new.pt $OUT/g_base.pt > $OUT/gcmp.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_optim.py -m gpu -v -s --timeout 120 --timeout-method thread \
  -k "rec_attention or encoder or lstm or full_model or glue or hip_graph or guard or adam" > $OUT/tests.log 2>&1
rc=$?; if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/ab_libs.sh $OUT "variants/_ina_kernels_base.so induction_network_on_fewrel_amd/_ina_kernels.so variants/_ina_kernels_noslp.so" > $OUT/ab.txt 2>&1
