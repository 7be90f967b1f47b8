# native-comm + ragged-sort GPU tests, then accuracy sweep part 1 (plain test failures do not stop the sweep)
mkdir -p gpurun_out/acc3
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py tests/test_ragged_gpu.py -v --timeout 120 --timeout-method thread -k "native or ragged" > gpurun_out/acc3/native_tests.log 2>&1
rc=$?
echo "native/ragged tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/acc3/b5.log 2>&1 || exit $?
PAR=6 bash tools/accuracy_sweep.sh gpurun_out/acc3 "0 1 2" "1 5" "^(ce_paper_f50|ce_paper_f300|ce_ref_f50|mse_paper_f50)$"
