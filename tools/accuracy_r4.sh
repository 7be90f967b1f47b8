#!/bin/bash
# Round-4 accuracy protocol on the reference's data/val.json (train.json / GloVe are not shipped; random word
# table from the data's tokens): THREE relation-disjoint blocks per fold --
#   test = relations 5k .. 5k+4 (JSON order), val = the next 5 (wrapping), train = the remaining 6;
#   the checkpoint is selected on the VAL relations (best [EVAL] accuracy, --test_best, as the reference's
#   best-val Saver, model/base.py:168-178) and only then tested on 3,000 episodes of the test relations.
# Configuration: the round-3 best (paper head, softmax-CE, frozen random 300-d words, u = 20).
# usage (GPU box): bash tools/accuracy_r4.sh OUTDIR ["0 1 2"] ["1 5"]
set -o pipefail
OUT=${1:-gpurun_out/acc4}
FOLDS=${2:-"0 1 2"}
KS=${3:-"1 5"}
STEPS=${STEPS:-5000}
mkdir -p "$OUT"
VAL=gpudata/val.json
BASE="--val_file $VAL --split_val true --vocab_from_data true --device cuda --train_iter $STEPS --episodes_per_step 256 \
--lr_schedule constant --val_step 500 --val_iter 1000 --test_iter 3000 --log_every 500 --val_relations 5 --test_best true \
--relation_head paper --loss_type ce --synthetic_word_dim 300"
pids=()
for f in $FOLDS; do
  for k in $KS; do
    name=ce_paper_f300_3way_fold${f}_5w${k}s
    timeout -k 10 1100 python -u train.py induction 5 $k $BASE --fold $f --model_dir /tmp/acc4_$name \
      --processed_dir /tmp/acc4_proc_$name > $OUT/$name.log 2>&1 &
    pids+=($!)
  done
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -h 'Test accuracy' $f) best-val $(grep -h 'Best checkpoint' $f | tail -1)"; done
exit $rc
