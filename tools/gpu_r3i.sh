# trained-word-table path: GPU test vs the oracle + training speed (train.py, 256 episodes / step)
OUT=${1:-gpurun_out/r3i}
ROOT=$PWD
mkdir -p $OUT /tmp/t50
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -v --timeout 120 --timeout-method thread -k "trained_words or encoder_backward" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python train.py induction 5 5 --val_file $ROOT/gpudata/val.json --split_val true --vocab_from_data true --device cuda --train_iter 300 --episodes_per_step 256 --lr_schedule constant --val_step 1000 --val_iter 10 --test_iter 10 --log_every 100 --relation_head paper --loss_type ce --synthetic_word_dim 50 --train_word_embedding true --fold 0 --processed_dir /tmp/t50/_proc --model_dir /tmp/t50/run > $OUT/t50.log 2>&1
