"""Instruction mix of one kernel in a hipcc -S listing: python tools/isa_mix.py file.s <kernel substring> [top]"""
import re
import sys
from collections import Counter

src, pat = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
s = open(src).read()
for m in re.finditer(r'^(\S+):\s*;\s*@\S+\n(.*?)\.Lfunc_end', s, re.S | re.M):
    if pat not in m.group(1):
        continue
    c = Counter()
    for line in m.group(2).split('\n'):
        t = line.strip().split()
        if t and not t[0].startswith(('.', ';', '_')) and not t[0].endswith(':'):
            c[t[0]] += 1
    print(m.group(1), sum(c.values()))
    for k, v in sorted(c.items(), key=lambda x: -x[1])[:top]:
        print(f"  {k} {v}")
