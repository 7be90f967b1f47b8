#!/bin/bash
# Few-shot RELATION TRANSFER on the synthetic transfer task (data/synthetic.py::make_transfer_splits; verdict r4
# #5): 48 training relations, 8 validation relations (select the checkpoint, --test_best, as the reference's
# best-val Saver, model/base.py:168-178), 8 held-out test relations whose trigger tokens never occur in training.
# Control: tools/control_baseline.py --task transfer (mean-pooled frozen word vectors -> nearest prototype,
# no training) on the same generated splits.
# usage (GPU box): bash tools/accuracy_transfer.sh OUTDIR ["reference paper"] ["1 5"]
set -o pipefail
OUT=${1:-gpurun_out/transfer}
HEADS=${2:-"reference paper"}
KS=${3:-"1 5"}
STEPS=${STEPS:-3000}
mkdir -p "$OUT"
BASE="--synthetic true --synthetic_task transfer --synthetic_relations 48 --synthetic_instances 300 \
--synthetic_vocab 20000 --synthetic_word_dim 50 --device cuda --train_iter $STEPS --episodes_per_step 64 \
--lr_schedule constant --val_step 250 --val_iter 500 --test_iter 3000 --log_every 250 --test_best true \
--loss_type ce"
pids=()
for h in $HEADS; do
  for k in $KS; do
    name=transfer_${h}_5w${k}s
    timeout -k 10 1000 python -u train.py induction 5 $k $BASE --relation_head $h --model_dir /tmp/tr_$name \
      > $OUT/$name.log 2>&1 &
    pids+=($!)
  done
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
python tools/control_baseline.py --task transfer --dims 50 --episodes 3000 --out $OUT/control.jsonl > $OUT/control.log 2>&1 || rc=$?
for f in $OUT/transfer_*.log; do echo "$(basename $f) $(grep -h 'Test accuracy' $f) best-val $(grep -h 'Best checkpoint' $f | tail -1)"; done
exit $rc
