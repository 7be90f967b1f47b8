#!/usr/bin/env python3
"""Kernel-time summary from a rocprofv3 rocpd SQLite database (``rocprofv3 --kernel-trace --stats -d DIR``).

usage: python tools/rocpd_summary.py DIR/prof_results.db [--top 40] [--csv out.csv] [--md out.md] [--steps K]
Prints name, calls, total ms, avg us, % of GPU kernel time (and per-step ms when --steps is given).
"""
import argparse
import csv
import re
import sqlite3


def short(name: str, n: int = 90) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)          # drop argument lists
    return name if len(name) <= n else name[: n - 3] + "..."


def summary(db: str):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name "
                     "order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [(short(r[0]), r[1], r[2] / 1e6, r[3] / 1e3, 100.0 * r[2] / tot) for r in rows], tot / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--csv", default="")
    ap.add_argument("--md", default="")
    ap.add_argument("--steps", type=int, default=0, help="timed+warmup steps in the trace (per-step column)")
    ap.add_argument("--sequence", default="", help="print the kernel sequence (start order, duration, gap) of the "
                    "last full step delimited by this kernel-name substring (e.g. adam_kernel)")
    a = ap.parse_args()
    if a.sequence:
        c = sqlite3.connect(a.db)
        cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
        grid = [g for g in ("grid_size_x", "grid_size_y", "grid_size_z", "grid_x", "grid_y", "grid_z") if g in cols]
        sel = ", ".join(["name", "start", "end"] + grid)
        ks = c.execute(f"select {sel} from kernels order by start").fetchall()
        marks = [i for i, k in enumerate(ks) if a.sequence in k[0]]
        if len(marks) >= 2:
            lo, hi = marks[-2] + 1, marks[-1] + 1
            span = (ks[hi - 1][2] - ks[lo][1]) / 1e3
            busy = sum(k[2] - k[1] for k in ks[lo:hi]) / 1e3
            print(f"step: {hi - lo} kernels, span {span:.1f} us, kernel-busy {busy:.1f} us")
            prev_end = ks[lo - 1][2]
            for k in ks[lo:hi]:
                g = ("grid " + "x".join(str(v) for v in k[3:]) + "  ") if grid else ""
                print(f"{(k[2] - k[1]) / 1e3:9.2f} us  gap {(k[1] - prev_end) / 1e3:7.2f}  {g}{short(k[0], 110)}")
                prev_end = k[2]
        return
    rows, tot = summary(a.db)
    hdr = ["kernel", "calls", "total_ms", "avg_us", "pct"] + (["ms_per_step"] if a.steps else [])
    lines = [f"total GPU kernel time: {tot:.3f} ms"]
    for r in rows[: a.top]:
        extra = f" {r[2] / a.steps:9.3f}" if a.steps else ""
        lines.append(f"{r[4]:6.2f}% {r[2]:10.3f} ms {r[1]:6d} calls {r[3]:10.2f} us{extra}  {r[0]}")
    print("\n".join(lines))
    if a.csv:
        with open(a.csv, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(hdr)
            for r in rows:
                w.writerow([r[0], r[1], f"{r[2]:.4f}", f"{r[3]:.2f}", f"{r[4]:.2f}"] +
                           ([f"{r[2] / a.steps:.4f}"] if a.steps else []))
    if a.md:
        with open(a.md, "w") as fh:
            fh.write(f"Total GPU kernel time {tot:.3f} ms\n\n| % | total ms | calls | avg us | kernel |\n|---|---|---|---|---|\n")
            for r in rows[: a.top]:
                fh.write(f"| {r[4]:.2f} | {r[2]:.3f} | {r[1]} | {r[3]:.2f} | `{r[0]}` |\n")


if __name__ == "__main__":
    main()
