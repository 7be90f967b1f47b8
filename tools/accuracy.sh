#!/bin/bash
# Accuracy protocols (GPU box), one parametrised script (replaces the round-3..5 accuracy_*.sh one-offs).
#   bash tools/accuracy.sh MODE OUTDIR [args]
#
# MODE folds [FOLDS] [KS] [CONFIG-REGEX]   relation-disjoint folds of the reference's data/val.json (train.json and
#      GloVe are not shipped: word table from the data's own tokens).  Fold k holds out relations 5k .. 5k+4 and
#      trains on the other 11; FINAL weights tested on 3,000 held-out episodes (STEPS=10000 x 256 episodes).
# MODE folds3 [FOLDS] [KS]                 three relation-disjoint blocks per fold (test 5k .. 5k+4, val the next 5,
#      train the remaining 6); checkpoint chosen on the VAL relations (--test_best, the reference's best-val Saver,
#      model/base.py:168-178), then tested.  Paper head, softmax-CE, frozen 300-d words.
# MODE transfer [HEADS] [KS]               the synthetic relation-transfer task (data/synthetic.py::make_transfer_splits:
#      48 train / 8 val / 8 held-out test relations with unseen trigger tokens), best-val checkpoint, test relations;
#      + the mean-pool nearest-prototype control (tools/control_baseline.py) on the same splits.
# MODE transfer_sweep                      same with 64 training relations (FewRel's train split), SEEDS (default
#      "1 2 3"), LOSSES / SCHEDS arms.
# MODE nota [HEADS] [KS]                   FewRel 2.0 NOTA + domain adaptation (BASELINE.json config 5): transfer-task
#      models trained WITH none-of-the-above queries (NOTA_TRAIN, default 0.3, loss ce_nota: softmax over the N
#      scores + a NOTA class of logit 0; NOTA_TRAIN=0 trains as MODE transfer), evaluated by fewrel_eval.py at NOTA
#      rates NOTA_RATES (default 0,0.15,0.5; threshold tuned on the validation relations) on (a) the held-out test
#      relations and (b) a domain-shifted test set
#      (data/synthetic.py --shifted_test: new relations, wider entity gaps, more distractors, shifted filler words)
#      read through --test_file; the control under the same NOTA rule on both.
# Runs PAR (default 4) trainings at once on the one GPU (small, launch-bound models).  Checkpoints go to /tmp.
set -o pipefail
MODE=${1:?mode}
OUT=${2:-gpurun_out/accuracy_$MODE}
shift 2
mkdir -p "$OUT"
VAL=gpudata/val.json
[ -f "$VAL" ] || VAL=/root/reference/data/val.json
PAR=${PAR:-4}
TRANSFER="--synthetic true --synthetic_task transfer --synthetic_relations ${RELS:-48} --synthetic_instances 300 \
--synthetic_vocab 20000 --synthetic_word_dim 50 --device cuda --episodes_per_step 64 --val_step 250 --val_iter 500 \
--test_iter 3000 --log_every 250 --test_best true"

summary() { for f in "$OUT"/*.log; do echo "$(basename $f .log) $(grep -h 'Test accuracy' $f) best-val $(grep -h 'Best checkpoint' $f | tail -1 | awk '{print $NF}')"; done; }
parallel() { xargs -P "$PAR" -I{} bash -c "{}" < "$1"; }

case $MODE in
folds)
  FOLDS=${1:-"0 1 2"}; KS=${2:-"1 5"}; FILT=${3:-.}
  BASE="--val_file $VAL --split_val true --vocab_from_data true --device cuda --train_iter ${STEPS:-10000} \
--episodes_per_step 256 --lr_schedule constant --val_step 1000 --val_iter 1000 --test_iter 3000 --log_every 500"
  declare -A CFG
  CFG[ce_paper_f50]="--relation_head paper --loss_type ce --synthetic_word_dim 50"
  CFG[ce_paper_f300]="--relation_head paper --loss_type ce --synthetic_word_dim 300"
  CFG[ce_paper_t50]="--relation_head paper --loss_type ce --synthetic_word_dim 50 --train_word_embedding true"
  CFG[ce_paper_f50_d5]="--relation_head paper --loss_type ce --synthetic_word_dim 50 --keep_prob 0.5"
  CFG[ce_ref_f50]="--relation_head reference --loss_type ce --synthetic_word_dim 50"
  CFG[mse_paper_f50]="--relation_head paper --loss_type mse --synthetic_word_dim 50"
  CFG[ce_paper_u128]="--relation_head paper --loss_type ce --synthetic_word_dim 300 --hidden_size 128"
  : > "$OUT/cmds.txt"
  for name in "${!CFG[@]}"; do
    [[ "$name" =~ $FILT ]] || continue
    dim=$(echo "${CFG[$name]}" | sed -E 's/.*--synthetic_word_dim ([0-9]+).*/\1/')
    for f in $FOLDS; do for K in $KS; do
      run=${name}_fold${f}_5w${K}s
      echo "timeout -k 10 1000 python train.py induction 5 $K $BASE ${CFG[$name]} --fold $f --processed_dir /tmp/acc/_proc_d$dim --model_dir /tmp/acc/$run > $OUT/$run.log 2>&1" >> "$OUT/cmds.txt"
    done; done
  done
  # one process builds each word table first (runs sharing a processed_dir must not race on it)
  for dim in $(grep -oE "_proc_d[0-9]+" "$OUT/cmds.txt" | sort -u | sed 's/_proc_d//'); do
    timeout -k 10 300 python -c "
import json, os, sys
sys.path.insert(0, '.')
from induction_network_on_fewrel_amd.data import vocab_from_fewrel, FewRelDataset
d = '/tmp/acc/_proc_d$dim'; os.makedirs(d, exist_ok=True)
wv = os.path.join(d, 'vocab_from_data.json')
if not os.path.exists(wv): json.dump(vocab_from_fewrel('$VAL', dim=$dim, seed=12345), open(wv, 'w'))
FewRelDataset.from_json('$VAL', wv, 37, False, processed_dir=d)
" || exit 1
  done
  parallel "$OUT/cmds.txt"; summary ;;
folds3)
  FOLDS=${1:-"0 1 2"}; KS=${2:-"1 5"}
  BASE="--val_file $VAL --split_val true --vocab_from_data true --device cuda --train_iter ${STEPS:-5000} \
--episodes_per_step 256 --lr_schedule constant --val_step 500 --val_iter 1000 --test_iter 3000 --log_every 500 \
--val_relations 5 --test_best true --relation_head paper --loss_type ce --synthetic_word_dim 300"
  : > "$OUT/cmds.txt"
  for f in $FOLDS; do for k in $KS; do
    name=ce_paper_f300_3way_fold${f}_5w${k}s
    echo "timeout -k 10 1100 python -u train.py induction 5 $k $BASE --fold $f --model_dir /tmp/acc4_$name --processed_dir /tmp/acc4_proc_$name > $OUT/$name.log 2>&1" >> "$OUT/cmds.txt"
  done; done
  parallel "$OUT/cmds.txt"; summary ;;
transfer|nota)
  HEADS=${1:-"reference paper"}; KS=${2:-"1 5"}
  LOSS="--loss_type ce"
  if [ "$MODE" = nota ] && [ "${NOTA_TRAIN:-0.3}" != 0 ]; then
    LOSS="--loss_type ce_nota --nota_rate ${NOTA_TRAIN:-0.3} --nota_threshold 0.5"   # val: NOTA below score 0.5
  fi
  : > "$OUT/cmds.txt"
  for h in $HEADS; do for k in $KS; do
    name=transfer_${h}_5w${k}s
    echo "timeout -k 10 1000 python -u train.py induction 5 $k $TRANSFER --train_iter ${STEPS:-3000} --lr_schedule constant $LOSS --relation_head $h --model_dir /tmp/acc_$name > $OUT/$name.log 2>&1" >> "$OUT/cmds.txt"
  done; done
  parallel "$OUT/cmds.txt"; summary
  if [ "$MODE" = nota ]; then
    RATES=${NOTA_RATES:-0,0.15,0.5}
    SHIFT=$OUT/shifted_test.json
    timeout -k 10 300 python -m induction_network_on_fewrel_amd.data.synthetic --shifted_test $SHIFT > /dev/null || exit 1
    : > "$OUT/eval.jsonl"
    for h in $HEADS; do for k in $KS; do
      name=transfer_${h}_5w${k}s
      for tf in "" "--test_file $SHIFT"; do
        timeout -k 10 600 python -u fewrel_eval.py induction 5 $k $TRANSFER --relation_head $h --model_dir /tmp/acc_$name \
          --settings 5-$k --nota_rates $RATES --nota_threshold -1 --iters 3000 $tf 2> $OUT/eval_${name}.err | grep '^{' >> "$OUT/eval.jsonl" || exit 1
      done
    done; done
    timeout -k 10 900 python tools/control_baseline.py --task transfer --dims 50 --episodes 3000 --shots ${KS// /,} \
      --nota_rates $RATES --test_file $SHIFT --out $OUT/control.jsonl > $OUT/control.log 2>&1 || exit 1
    python tools/accuracy_table.py $OUT/eval.jsonl $OUT/control.jsonl > $OUT/summary.txt && cat $OUT/summary.txt
  else
    timeout -k 10 900 python tools/control_baseline.py --task transfer --dims 50 --episodes 3000 \
      --out $OUT/control.jsonl > $OUT/control.log 2>&1
  fi ;;
transfer_sweep)
  : > "$OUT/cmds.txt"
  for seed in ${SEEDS:-1 2 3}; do for h in reference paper; do for k in 1 5; do
    for lo in ${LOSSES:-ce}; do for sc in ${SCHEDS:-constant}; do
      n=${h}_5w${k}s_${sc}_${lo}_s$seed
      echo "timeout -k 10 900 python -u train.py induction 5 $k ${TRANSFER/--synthetic_relations 48/--synthetic_relations ${RELS:-64}} --train_iter ${STEPS:-3000} --relation_head $h --loss_type $lo --lr_schedule $sc --seed $seed --model_dir /tmp/trs_$n > $OUT/$n.log 2>&1" >> "$OUT/cmds.txt"
    done; done
  done; done; done
  parallel "$OUT/cmds.txt"; summary ;;
*) echo "unknown mode $MODE"; exit 2 ;;
esac
