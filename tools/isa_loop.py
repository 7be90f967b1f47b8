#!/usr/bin/env python3
"""Instruction mix of each innermost loop of one kernel in a hipcc -S dump.

usage: python tools/isa_loop.py X.s <kernel-name-substring>
Prints, per loop (label with an "Inner Loop Header" comment closed by a backward conditional branch):
total instructions, VALU (non-MFMA), MFMA, transcendentals, 32-bit integer multiplies, VMEM loads /
stores and LDS instructions -- the per-iteration issue budget of a recurrence loop.
"""
import collections
import sys


def loops(path, name):
    s = open(path).read()
    st = s.find(name)
    if st < 0:
        raise SystemExit(f"{name}: not found")
    body = s[st:s.find(".Lfunc_end", st)].split("\n")
    for h, line in enumerate(body):
        if "Inner Loop Header" not in line:
            continue
        lab = line.split(":")[0].strip()
        if not lab.startswith(".L"):   # nested loops: the label sits on the line before the comment
            lab = body[h - 1].split(":")[0].strip()
        ends = [i for i, l in enumerate(body) if i > h and lab in l and "branch" in l]
        if not ends:
            continue
        seg = [l.strip() for l in body[h + 1:ends[0] + 1]]
        seg = [l for l in seg if l and not l.startswith((";", "."))]
        c = collections.Counter(x.split()[0] for x in seg)
        tr = ("v_exp_f32", "v_rcp_f32", "v_log_f32", "v_sqrt_f32", "v_rsq_f32")
        yield lab, dict(
            instrs=len(seg),
            valu=sum(n for k, n in c.items() if k.startswith("v_") and "mfma" not in k),
            mfma=sum(n for k, n in c.items() if "mfma" in k),
            trans=sum(n for k, n in c.items() if k.startswith(tr)),
            mul_lo=sum(n for k, n in c.items() if k.startswith(("v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64"))),
            vmem_ld=sum(n for k, n in c.items() if k.startswith(("global_load", "buffer_load"))),
            vmem_st=sum(n for k, n in c.items() if k.startswith(("global_store", "buffer_store"))),
            lds=sum(n for k, n in c.items() if k.startswith("ds_")),
            salu=sum(n for k, n in c.items() if k.startswith("s_") and not k.startswith(("s_nop", "s_waitcnt"))),
            nop=c["s_nop"], wait=c["s_waitcnt"])


if __name__ == "__main__":
    for lab, d in loops(sys.argv[1], sys.argv[2]):
        print(lab, " ".join(f"{k}={v}" for k, v in d.items()))
