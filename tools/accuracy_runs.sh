#!/bin/bash
# FewRel accuracy on a relation-disjoint split of the reference's data/val.json (train.json is not
# shipped): the first 8 relations train, the other 8 validate/test.  No GloVe file is available, so
# the word table is built from the data's own tokens (random init).  Two protocols:
#   parity : the reference schedule (1 episode/step, 30k steps, lr 1e-3 * 0.9^(step/100) staircase,
#            frozen 5-d word table, keep_prob 0.9)
#   tuned  : 64 episodes/step, 3k steps, constant lr 1e-3, trainable 50-d word table
# usage: bash tools/accuracy_runs.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/acc}
mkdir -p "$OUT"
VAL=${VAL:-gpudata/val.json}
[ -f "$VAL" ] || VAL=/root/reference/data/val.json
run() {  # name, K, extra args...
  local name=$1 K=$2; shift 2
  timeout -k 10 900 python train.py induction 5 $K --val_file "$VAL" --split_val true --vocab_from_data true \
    --device cuda --processed_dir "/tmp/acc/_processed_$name" --model_dir "/tmp/acc/$name" "$@" > "$OUT/$name.log" 2>&1
}
run parity_5w1s 1 --train_iter 30000 --synthetic_word_dim 5 && \
run parity_5w5s 5 --train_iter 30000 --synthetic_word_dim 5 && \
run tuned_5w1s 1 --train_iter 3000 --episodes_per_step 64 --lr_schedule constant --synthetic_word_dim 50 \
    --train_word_embedding true --val_step 500 --val_iter 2000 --test_iter 3000 && \
run tuned_5w5s 5 --train_iter 3000 --episodes_per_step 64 --lr_schedule constant --synthetic_word_dim 50 \
    --train_word_embedding true --val_step 500 --val_iter 2000 --test_iter 3000
rc=$?
grep -H "Test accuracy" "$OUT"/*.log
exit $rc
