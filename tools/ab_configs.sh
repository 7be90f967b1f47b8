# Same-box A/B of (kernel library, bench flags) configurations, alternating, REPS rounds each.
# usage (on the box): REPS=2 bash tools/ab_configs.sh OUTDIR "lib1|flags1" "lib2|flags2" ...
#   lib = path relative to the repo root ("-" = the in-tree library); flags = extra bench.py flags
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
for i in $(seq 1 ${REPS:-2}); do for cf in "$@"; do
  lib=${cf%%|*}; flags=${cf#*|}
  echo "CONFIG $cf" >> $OUT/b.log
  if [ "$lib" = "-" ]; then
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 $flags >> $OUT/b.log 2>&1 || exit 1
  else
    INA_KERNEL_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 30 --warmup 5 $flags >> $OUT/b.log 2>&1 || exit 1
  fi
done; done
python - "$OUT/b.log" <<'PY'
import json, sys, collections
res, cf = collections.defaultdict(list), None
for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("CONFIG "):
        cf = line[7:]
    elif line.startswith("{"):
        res[cf].append(json.loads(line)["value"])
for k, v in res.items():
    print(f"{k:60s} {' '.join(f'{x:.0f}' for x in v)}  best {max(v):.0f}")
PY
