# Same-box A/B of kernel libraries: bench.py alternating between libraries (box-to-box clock
# differences are ~8%, larger than most kernel changes).  usage (on the box):
#   bash tools/ab_libs.sh OUTDIR "libA libB ..." [bench args...]     (paths relative to the repo root)
set -o pipefail
OUT=${1:-gpurun_out/ab}; LIBS=$2; shift 2
mkdir -p $OUT
for i in 1 2 3; do for lib in $LIBS; do
  echo "$lib" >> $OUT/b.log
  INA_KERNEL_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 30 --warmup 5 "$@" >> $OUT/b.log 2>&1 || exit 1
done; done
python - "$OUT/b.log" <<'EOF'
import json, sys, collections
res, lib = collections.defaultdict(list), None
for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("{"):
        res[lib].append(json.loads(line)["value"])
    elif line.endswith(".so"):
        lib = line
for k, v in res.items():
    print(f"{k}: {' '.join(f'{x:.0f}' for x in v)}  best {max(v):.0f}")
EOF
