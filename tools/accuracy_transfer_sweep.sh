#!/bin/bash
# Transfer-task sweep (data/synthetic.py::make_transfer_splits): 64 training relations (FewRel's train split
# has 64), 8 validation and 8 held-out test relations, three seeds (each seed generates its own relations);
# both heads, 5w1s and 5w5s, best-val checkpoint on the validation relations, test on the held-out relations.
# LOSSES / SCHEDS pick the arms (default: CE on a constant learning rate; the reference's exponential decay
# stops learning by step ~1,500 at 64 episodes per step and MSE with the reference head stays at chance:
# profiles/accuracy/r5_transfer/sweep_exp).
# usage (GPU box): bash tools/accuracy_transfer_sweep.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/transfer_sweep}
mkdir -p "$OUT"
STEPS=${STEPS:-3000}
BASE="--synthetic true --synthetic_task transfer --synthetic_relations ${RELS:-64} --synthetic_instances 300 \
--synthetic_vocab 20000 --synthetic_word_dim 50 --device cuda --train_iter $STEPS --episodes_per_step 64 \
--val_step 250 --val_iter 500 --test_iter 3000 --log_every 250 --test_best true"
run() {   # name, extra args
  timeout -k 10 900 python -u train.py induction $2 $BASE ${@:3} --model_dir /tmp/trs_$1 > $OUT/$1.log 2>&1
}
rc=0
for seed in ${SEEDS:-1 2 3}; do
  for h in reference paper; do
    pids=()
    for k in 1 5; do
      for lo in ${LOSSES:-ce}; do
        for sc in ${SCHEDS:-constant}; do
          run ${h}_5w${k}s_${sc}_${lo}_s$seed "5 $k" --relation_head $h --loss_type $lo --lr_schedule $sc --seed $seed &
          pids+=($!)
        done
      done
    done
    for p in "${pids[@]}"; do wait $p || rc=$?; done
  done
done
for f in $OUT/*.log; do echo "$(basename $f .log) $(grep -h 'Test accuracy' $f) best-val $(grep -h 'Best checkpoint' $f | tail -1 | awk '{print $NF}')"; done
exit $rc
