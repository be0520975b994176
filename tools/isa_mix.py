"""Instruction mix of one kernel in a hipcc --save-temps .s file (static counts; the tile loop
is fully unrolled, so static ~ dynamic per tile).  Usage: python tools/isa_mix.py file.s <name-substring>"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
m = [x for x in re.finditer(r"^(_Z\S+):\s*;", s, re.M) if pat in x.group(1)]
for mm in m:
    name = mm.group(1)
    i = mm.end()
    j = s.index(".Lfunc_end", i)
    c = collections.Counter()
    for l in s[i:j].split("\n"):
        l = l.strip()
        if not l or l.startswith((".", ";")) or l.endswith(":"):
            continue
        c[l.split()[0]] += 1
    cat = collections.Counter()
    for op, n in c.items():
        k = ("mfma" if op.startswith("v_mfma") else "accvgpr" if op.startswith("v_accvgpr") else
             "v_mov" if op.startswith("v_mov") else "valu" if op.startswith("v_") else
             "ds" if op.startswith("ds_") else "scratch" if op.startswith("scratch_") else
             "vmem" if op.startswith(("buffer_", "global_")) else "s_waitcnt" if op.startswith("s_waitcnt") else
             "s_nop" if op == "s_nop" else "salu" if op.startswith("s_") else op)
        cat[k] += n
    print(name[:90], sum(c.values()), dict(cat))
    if len(sys.argv) > 3:
        for op, n in c.most_common(int(sys.argv[3])):
            print(f"  {n:6d} {op}")
