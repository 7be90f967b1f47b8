# Short accuracy experiment on the relation-disjoint val.json split (CPU or GPU).
# usage: bash tools/acc_exp.sh NAME K OUTDIR [extra train.py flags...]
name=$1; K=$2; out=$3; shift 3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
VAL=${VAL:-/root/reference/data/val.json}
timeout -k 10 ${EXP_TIMEOUT:-1500} python "$ROOT/train.py" induction 5 "$K" --val_file "$VAL" --split_val true \
  --vocab_from_data true --device "${DEVICE:-cpu}" --processed_dir "/tmp/exp/p_$name" --model_dir "/tmp/exp/m_$name" \
  --train_relations 11 --episodes_per_step 16 --lr_schedule constant --val_step 200 --val_iter 300 \
  --test_iter 500 --resume false --log_every 100 --relation_head paper "$@" > "$out/$name.log" 2>&1
