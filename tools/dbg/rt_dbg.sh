mkdir -p gpurun_out/rt_dbg3
timeout -k 10 120 python tools/dbg/rt_cmp3.py > gpurun_out/rt_dbg3/new.txt 2>&1
INA_KERNEL_LIB=$PWD/variants/_ina_kernels_head.so timeout -k 10 120 python tools/dbg/rt_cmp3.py > gpurun_out/rt_dbg3/old.txt 2>&1
exit 0
