#!/usr/bin/env python3
"""Table of the FewRel 2.0 NOTA / domain-adaptation evaluation (tools/accuracy.sh nota): one row per (data, N-K,
NOTA rate) with the trained heads' accuracy, in-class accuracy, NOTA precision / recall, and the mean-pool control
under the same NOTA rule.
usage: accuracy_table.py eval.jsonl control.jsonl"""
import json
import sys


def main(ev_path, ctl_path):
    ev = [json.loads(l) for l in open(ev_path) if l.strip()]
    ctl = [json.loads(l) for l in open(ctl_path) if l.strip() and '"nota_rate"' in l]
    name = {"transfer_test": "held-out test relations", "shifted": "domain-shifted test (--test_file)"}
    for e in ev:
        e["data"] = "transfer_test" if e["data"] == "transfer_test" else "shifted"
    print("| data | N-K | NOTA rate | model | accuracy | in-class acc | NOTA precision | NOTA recall | threshold |")
    print("|---|---|---|---|---|---|---|---|---|")
    keys = sorted({(e["data"], e["K"], e["nota_rate"]) for e in ev})
    for data, K, rate in keys:
        rows = [e for e in ev if e["data"] == data and e["K"] == K and e["nota_rate"] == rate]
        for e in sorted(rows, key=lambda x: x.get("head", "")):
            thr = e["threshold"]
            print(f"| {name.get(data, data)} | {e['N']}-{K} | {rate} | {e.get('head', '?')} head | "
                  f"{100 * e['accuracy']:.1f} | {100 * e['in_class_accuracy']:.1f} | {100 * e['nota_precision']:.1f} | "
                  f"{100 * e['nota_recall']:.1f} | {'-' if thr is None else round(thr, 2)} |")
        for c in ctl:
            cd = "transfer_test" if c["split"] == "transfer_test" else "shifted"
            if cd == data and c["K"] == K and c["nota_rate"] == rate:
                print(f"| {name.get(data, data)} | {c['N']}-{K} | {rate} | mean-pool control | {100 * c['accuracy']:.1f} | "
                      f"{100 * c['in_class_accuracy']:.1f} | {100 * c['nota_precision']:.1f} | "
                      f"{100 * c['nota_recall']:.1f} | {c['threshold'] if rate > 0 else '-'} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
