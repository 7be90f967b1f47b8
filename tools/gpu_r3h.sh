# GPU tests (NTN slice split covered by the small-E kernel tests), reference-mode + headline benches,
# hipBLASLt epilogue probe, and a kernel profile of the trainable-word-table training path.
OUT=${1:-gpurun_out/r3h}
ROOT=$PWD
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python bench.py --episodes-per-gpu 1 --steps 300 --warmup 20 > $OUT/b_ep1.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --episodes-per-gpu 64 --steps 100 --warmup 10 > $OUT/b_ep64.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $OUT/b5.log 2>&1 || exit $?
timeout -k 10 120 ./variants/blaslt_probe > $OUT/blaslt_probe.log 2>&1 || exit $?
mkdir -p /tmp/t50
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_t50 -o run --output-format rocpd -- python3 $ROOT/train.py induction 5 5 --val_file $ROOT/gpudata/val.json --split_val true --vocab_from_data true --device cuda --train_iter 40 --episodes_per_step 256 --lr_schedule constant --val_step 1000 --val_iter 10 --test_iter 10 --log_every 20 --relation_head paper --loss_type ce --synthetic_word_dim 50 --train_word_embedding true --fold 0 --processed_dir /tmp/t50/_proc --model_dir /tmp/t50/run > $ROOT/$OUT/t50.log 2>&1) || exit $?
DB=$(ls /tmp/prof_t50/*/*.db /tmp/prof_t50/*.db 2>/dev/null | head -1)
python tools/rocpd_summary.py $DB --steps 40 > $OUT/sum_t50.txt 2>&1
