"""Summarise rocprofv3 --pmc counter CSVs (one dir per pass) per kernel: derived metrics."""
import csv
import glob
import sys
from collections import defaultdict


def load(root):
    vals = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
            vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
    return vals, cnt


def main(root):
    vals, cnt = load(root)
    print(f"{'kernel':48s} {'VALU/wave':>9s} {'MFMA/w':>7s} {'LDS/w':>6s} {'VMRD/w':>7s} {'VMWR/w':>7s} "
          f"{'wait%':>6s} {'waitI%':>6s} {'valu%':>6s} {'mfma%':>6s} {'ldsconf%':>8s} {'rdMB':>7s} {'wrMB':>7s}")
    for k, v in sorted(vals.items()):
        wc = v.get("SQ_WAVE_CYCLES", 0) or 1
        waves = v.get("SQ_WAVES", 0)
        # per-dispatch average of instruction counts (divide by number of dispatch rows)
        n = max(1, cnt[k].get("SQ_INSTS_VALU", 1))
        row = [v.get("SQ_INSTS_VALU", 0) / n, v.get("SQ_INSTS_MFMA", 0) / n, v.get("SQ_INSTS_LDS", 0) / n,
               v.get("SQ_INSTS_VMEM_RD", 0) / n, v.get("SQ_INSTS_VMEM_WR", 0) / n]
        wait = 100 * v.get("SQ_WAIT_ANY", 0) / wc
        waiti = 100 * v.get("SQ_WAIT_INST_ANY", 0) / wc
        valu = 100 * v.get("SQ_ACTIVE_INST_VALU", 0) / wc
        gui = v.get("GRBM_GUI_ACTIVE", 0) or 1
        mfma = 100 * v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui * 4 * 256 / max(1, cnt[k].get("GRBM_GUI_ACTIVE", 1)) * 1)
        lds = v.get("SQ_LDS_IDX_ACTIVE", 0) or 1
        ldsc = 100 * v.get("SQ_LDS_BANK_CONFLICT", 0) / lds
        # HBM traffic per dispatch (FETCH_SIZE / WRITE_SIZE are KB summed over the dispatch's rows)
        rd = v.get("FETCH_SIZE", 0) / max(1, cnt[k].get("FETCH_SIZE", 1)) / 1024
        wr = v.get("WRITE_SIZE", 0) / max(1, cnt[k].get("WRITE_SIZE", 1)) / 1024
        print(f"{k:48s} {row[0]:9.3g} {row[1]:7.3g} {row[2]:6.3g} {row[3]:7.3g} {row[4]:7.3g} {wait:6.1f} {waiti:6.1f} "
              f"{valu:6.1f} {mfma:6.1f} {ldsc:8.1f} {rd:7.1f} {wr:7.1f}")
    print("\nraw sums per kernel:")
    for k, v in sorted(vals.items()):
        print(k, {c: f"{x:.4g}" for c, x in sorted(v.items())})


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc1")
