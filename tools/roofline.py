#!/usr/bin/env python3
"""Per-kernel roofline table from rocprofv3 PMC passes (+ an un-profiled kernel-time summary).

usage: python tools/roofline.py PMC_DIR [--stats stats.csv] [--steps K] [--min-pct 1.0] [--md out.md]

PMC_DIR holds one ``*counter_collection.csv`` per pass (tools/pmc_roofline.sh).  Counters are
averaged per dispatch of each kernel.  Derived columns (MI355X, 256 CUs = 1024 SIMDs, 8 XCDs):

* clock    effective shader clock = GRBM_GUI_ACTIVE / 8 / dispatch wall time (the sum over XCDs)
* occ      mean resident waves per SIMD = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8) / 1024
           (SQ_WAVE_CYCLES counts quad-cycles per resident wave)
* mfma%    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024): share of SIMD-cycles the matrix
           cores were busy
* valu%    SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: share of a resident wave's time issuing VALU
* wait%    SQ_WAIT_ANY / SQ_WAVE_CYCLES: share parked on s_waitcnt / barriers
* rd / wr  FETCH_SIZE / WRITE_SIZE in MB per dispatch.  gfx950's FETCH_SIZE counts wide streaming
           reads at half their bytes (MI355X_MICROARCH.md, HBM): ``rd_x2`` is the corrected upper
           estimate; TB/s uses (rd_x2 + wr) over the UN-profiled kernel time when --stats is given
* %hbm     that bandwidth over the ~6.3 TB/s achievable HBM3E stream rate
"""
import argparse
import csv
import glob
import re
from collections import defaultdict

HBM_TBS = 6.3
SIMDS = 1024


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name).strip()


def load_pmc(root):
    """kernel -> counter -> (sum, dispatches); kernel -> list of profiled durations (ns)."""
    vals = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    dur = defaultdict(dict)
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            key = (f, r["Dispatch_Id"])
            c = r["Counter_Name"]
            vals[k][c] += float(r["Counter_Value"])
            disp[k][c].add(key)
            dur[k][key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    avg = {k: {c: v / max(1, len(disp[k][c])) for c, v in cs.items()} for k, cs in vals.items()}
    pdur = {k: sum(d.values()) / max(1, len(d)) for k, d in dur.items()}
    return avg, pdur


def load_stats(path, steps):
    """stats.csv of tools/rocpd_summary.py: kernel -> (avg_us, calls per step, pct)."""
    out = {}
    for r in csv.DictReader(open(path)):
        k = short(r["kernel"])
        calls = int(r["calls"])
        out[k] = (float(r["avg_us"]), calls / steps if steps else calls, float(r["pct"]))
    return out


def match(k, stats):
    if k in stats:
        return stats[k]
    for s, v in stats.items():   # rocpd names are truncated at 90 characters
        if s.endswith("...") and k.startswith(s[:-3]):
            return v
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc")
    ap.add_argument("--stats", default="")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--min-pct", type=float, default=1.0)
    ap.add_argument("--md", default="")
    a = ap.parse_args()
    avg, pdur = load_pmc(a.pmc)
    stats = load_stats(a.stats, a.steps) if a.stats else {}
    rows = []
    for k, c in avg.items():
        st = match(k, stats)
        if stats and (st is None or st[2] < a.min_pct):
            continue
        us = st[0] if st else pdur[k] / 1e3
        gui = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        clk = gui / (pdur[k]) if pdur[k] else 0.0          # GHz (cycles per ns)
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        occ = 4 * c.get("SQ_WAVE_CYCLES", 0.0) / gui / SIMDS if gui else 0.0
        mfma = 100 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui * SIMDS) if gui else 0.0
        valu = 100 * c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc
        wait = 100 * c.get("SQ_WAIT_ANY", 0.0) / wc
        ldsc = 100 * c.get("SQ_LDS_BANK_CONFLICT", 0.0) / (c.get("SQ_LDS_IDX_ACTIVE", 0.0) or 1.0)
        rd = c.get("FETCH_SIZE", 0.0) / 1024
        wr = c.get("WRITE_SIZE", 0.0) / 1024
        tbs = (2 * rd + wr) / 1e6 / (us / 1e6) if us else 0.0
        rows.append((st[2] if st else 0.0, k, us, rd, 2 * rd, wr, tbs, 100 * tbs / HBM_TBS, mfma, valu, wait, occ,
                     ldsc, clk))
    rows.sort(key=lambda r: (-r[0], -r[2]))
    hdr = ("| % step | kernel | us | rd MB | rd_x2 MB | wr MB | TB/s | %hbm | mfma% | valu% | wait% | occ w/SIMD "
           "| lds conf% | GHz |")
    lines = [hdr, "|" + "---|" * 14]
    for r in rows:
        lines.append(f"| {r[0]:.1f} | `{r[1][:60]}` | {r[2]:.1f} | {r[3]:.0f} | {r[4]:.0f} | {r[5]:.0f} | {r[6]:.2f} | "
                     f"{r[7]:.0f} | {r[8]:.1f} | {r[9]:.1f} | {r[10]:.1f} | {r[11]:.2f} | {r[12]:.1f} | {r[13]:.2f} |")
    txt = "\n".join(lines)
    print(txt)
    if a.md:
        with open(a.md, "w") as fh:
            fh.write(__doc__.split("\n\n", 1)[1] + "\n\n" + txt + "\n")


if __name__ == "__main__":
    main()
