#!/bin/bash
# FewRel accuracy on relation-disjoint splits of the reference's data/val.json (train.json is not
# shipped).  No GloVe file is available: the word table is built from the data's own tokens (random
# init).  Protocols:
#   parity_*      : reference schedule (1 episode/step, 30k steps, lr 1e-3 * 0.9^floor(step/100),
#                   frozen 5-d word table, keep_prob 0.9, reference head); 8 train / 8 test relations
#   tuned_{ref,paper}_* : 64 episodes/step, 2k steps, constant lr 1e-3, trainable 50-d word table;
#                   11 train / 5 test relations (more relations to learn a relation-agnostic matcher)
#   ce_rel_*      : as tuned_paper but loss_type=ce (softmax cross-entropy over the relation scores:
#                   the MSE-on-sigmoid loss collapses to constant 1/N outputs for hundreds of steps),
#                   frozen 50-d word table, test from the best-val checkpoint
#   ce_inst_* / mse_inst_* : instance-disjoint split (all 16 relations, first 70% of each
#                   relation's sentences train, the rest test): within-relation generalisation
# Only logs are written under <outdir>; checkpoints go to /tmp.
# usage: bash tools/accuracy_runs.sh <outdir> [name-regex]
set -o pipefail
OUT=${1:-gpurun_out/acc}
FILT=${2:-}
mkdir -p "$OUT"
VAL=${VAL:-gpudata/val.json}
[ -f "$VAL" ] || VAL=/root/reference/data/val.json
run() {  # name, K, extra args...
  local name=$1 K=$2; shift 2
  if [ -n "$FILT" ] && ! [[ "$name" =~ $FILT ]]; then return 0; fi   # FILT: bash regex
  timeout -k 10 900 python train.py induction 5 $K --val_file "$VAL" --split_val true --vocab_from_data true \
    --device cuda --processed_dir "/tmp/acc/_processed_$name" --model_dir "/tmp/acc/$name" "$@" > "$OUT/$name.log" 2>&1
}
TUNED="--train_iter 2000 --episodes_per_step 64 --lr_schedule constant --synthetic_word_dim 50 --train_word_embedding true --val_step 500 --val_iter 2000 --test_iter 3000 --train_relations 11"
CE="--train_iter 2000 --episodes_per_step 64 --lr_schedule constant --synthetic_word_dim 50 --val_step 250 --val_iter 2000 --test_iter 3000 --relation_head paper --loss_type ce --test_best true"
INST="--split_mode instance --train_fraction 0.7"
run ce_rel_5w1s 1 $CE --train_relations 11 && \
run ce_rel_5w5s 5 $CE --train_relations 11 && \
run ce_inst_5w1s 1 $CE $INST && \
run ce_inst_5w5s 5 $CE $INST && \
run mse_inst_5w5s 5 $CE $INST --loss_type mse && \
run parity_5w1s 1 --train_iter 30000 --synthetic_word_dim 5 && \
run parity_5w5s 5 --train_iter 30000 --synthetic_word_dim 5 && \
run tuned_ref_5w1s 1 $TUNED && \
run tuned_ref_5w5s 5 $TUNED && \
run tuned_paper_5w1s 1 $TUNED --relation_head paper && \
run tuned_paper_5w5s 5 $TUNED --relation_head paper
rc=$?
grep -H "Test accuracy" "$OUT"/*.log
exit $rc
