#!/usr/bin/env python3
"""Register / scratch / LDS usage and instruction count per kernel from a hipcc -S dump.

usage: hipcc --offload-arch=gfx950 -O3 -S --cuda-device-only -Icsrc/include csrc/kernels/X.hip -o X.s
       python tools/isa_stats.py X.s [name-filter]
"""
import re
import sys


def stats(path, filt=""):
    s = open(path).read()
    out = []
    for m in re.finditer(r'^(_Z\S+):\s*(?:;.*)?$', s, re.M):
        kern = m.group(1)
        if filt and filt not in kern:
            continue
        j = s.find('.Lfunc_end', m.start())
        body = [l.strip() for l in s[m.end():j].split('\n')]
        n = sum(1 for l in body if l and not l.startswith(('.', ';')))
        meta = s[j:j + 4000]

        def g(k):
            r = re.search(k + r':\s*(\d+)', meta)
            return int(r.group(1)) if r else -1
        out.append((kern, n, g('NumVgprs'), g('NumAgprs'), g('NumSgprs'), g('ScratchSize'), g('Occupancy')))
    return out


if __name__ == "__main__":
    for k, n, v, a, sg, scr, occ in stats(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""):
        print(f"{k[:70]:70s} instr={n:5d} vgpr={v:3d} agpr={a:3d} sgpr={sg:3d} scratch={scr} occ={occ}")
