#!/bin/bash
# Round-3 accuracy study on relation-disjoint folds of the reference's data/val.json (train.json and
# GloVe are not shipped; the word table is built from the data's own tokens, random init).
#   * fold k holds out relations 5k .. 5k+4 (JSON order) and trains on the other 11 (train.py --fold);
#   * 10,000 steps x 256 episodes = 2.56 M training episodes per run (20x the round-2 runs);
#   * the FINAL weights are tested (3,000 episodes of the held-out relations): no checkpoint selection
#     on the test relations; the [EVAL] lines every 1,000 steps are the learning curve only.
# Configurations (all 5-way; K in $KS):
#   ce_paper_f50     paper head, softmax-CE, frozen 50-d words, keep_prob 0.9      (round-2 best)
#   ce_paper_f300    same, frozen 300-d words (near-orthogonal random vectors: lexical identity)
#   ce_paper_t50     same, trainable 50-d words
#   ce_paper_f50_d5  same as ce_paper_f50, keep_prob 0.5
#   ce_ref_f50       reference head (W [h N, N])
#   mse_paper_f50    reference loss (MSE on sigmoid scores)
#   ce_paper_u128    the paper's encoder: u = 128, frozen 300-d words
# usage (GPU box): bash tools/accuracy_sweep.sh OUTDIR "0 1 2" "1 5" [config-regex]
# Runs PAR (default 4) trainings concurrently on the one GPU (each is a small, launch-bound model).
set -o pipefail
OUT=${1:-gpurun_out/acc3}
FOLDS=${2:-"0 1 2"}
KS=${3:-"1 5"}
FILT=${4:-.}
PAR=${PAR:-4}
STEPS=${STEPS:-10000}
mkdir -p "$OUT"
VAL=/root/reference/data/val.json
[ -f gpudata/val.json ] && VAL=gpudata/val.json
BASE="--val_file $VAL --split_val true --vocab_from_data true --device cuda --train_iter $STEPS --episodes_per_step 256 \
--lr_schedule constant --val_step 1000 --val_iter 1000 --test_iter 3000 --log_every 500"
declare -A CFG
CFG[ce_paper_f50]="--relation_head paper --loss_type ce --synthetic_word_dim 50"
CFG[ce_paper_f300]="--relation_head paper --loss_type ce --synthetic_word_dim 300"
CFG[ce_paper_t50]="--relation_head paper --loss_type ce --synthetic_word_dim 50 --train_word_embedding true"
CFG[ce_paper_f50_d5]="--relation_head paper --loss_type ce --synthetic_word_dim 50 --keep_prob 0.5"
CFG[ce_ref_f50]="--relation_head reference --loss_type ce --synthetic_word_dim 50"
CFG[mse_paper_f50]="--relation_head paper --loss_type mse --synthetic_word_dim 50"
CFG[ce_paper_u128]="--relation_head paper --loss_type ce --synthetic_word_dim 300 --hidden_size 128"
cmds=$OUT/cmds.txt
: > "$cmds"
for name in ce_paper_f50 ce_paper_f300 ce_paper_t50 ce_paper_f50_d5 ce_ref_f50 mse_paper_f50 ce_paper_u128; do
  [[ "$name" =~ $FILT ]] || continue
  dim=$(echo "${CFG[$name]}" | sed -E 's/.*--synthetic_word_dim ([0-9]+).*/\1/')
  for f in $FOLDS; do for K in $KS; do
    run=${name}_fold${f}_5w${K}s
    echo "timeout -k 10 1000 python train.py induction 5 $K $BASE ${CFG[$name]} --fold $f --processed_dir /tmp/acc3/_proc_d$dim --model_dir /tmp/acc3/$run > $OUT/$run.log 2>&1; echo \"$run rc=\$?\" >> $OUT/status.txt" >> "$cmds"
  done; done
done
# one process builds each word table first (the runs sharing a processed_dir must not race on it)
for dim in $(grep -oE "_proc_d[0-9]+" "$cmds" | sort -u | sed 's/_proc_d//'); do
  timeout -k 10 300 python -c "
import json, os, sys
sys.path.insert(0, '.')
from induction_network_on_fewrel_amd.data import vocab_from_fewrel, FewRelDataset
d = '/tmp/acc3/_proc_d$dim'; os.makedirs(d, exist_ok=True)
wv = os.path.join(d, 'vocab_from_data.json')
if not os.path.exists(wv): json.dump(vocab_from_fewrel('$VAL', dim=$dim, seed=12345), open(wv, 'w'))
FewRelDataset.from_json('$VAL', wv, 37, False, processed_dir=d)
" || exit 1
done
xargs -P "$PAR" -I{} bash -c "{}" < "$cmds"
grep -H "Test accuracy" "$OUT"/*.log | sort
