"""Instruction mix of a kernel's ISA between consecutive s_barrier instructions (debug tool).
Usage: python tools/isa_segments.py <file.s> <kernel symbol substring>"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(\S*" + re.escape(sys.argv[2]) + r"\S*):", s, re.M)
start = m.end()
end = s.index(".Lfunc_end", start)
body = s[start:end].split("\n")


def cls(t):
    ins = t.split()[0]
    if ins.startswith("v_mfma"):
        return "mfma"
    if ins.startswith("ds_read") or ins.startswith("ds_load"):
        return "ds_rd"
    if ins.startswith("ds_"):
        return "ds_oth"
    if ins.startswith("buffer_load") and " lds" in t:
        return "dma"
    if ins.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if ins.startswith("scratch_"):
        return "scratch"
    if ins.startswith("v_accvgpr"):
        return "accmov"
    if ins.startswith("v_writelane") or ins.startswith("v_readlane"):
        return "lanemov"
    if ins.startswith("v_"):
        return "valu"
    if ins.startswith("s_waitcnt"):
        return "wait"
    if ins.startswith("s_nop"):
        return "nop"
    if ins.startswith("s_"):
        return "salu"
    return None


segs, cur = [], collections.Counter()
for line in body:
    t = line.strip()
    if not t or t.startswith((";", ".")) or t.endswith(":"):
        continue
    if t.split()[0] == "s_barrier":
        segs.append(cur)
        cur = collections.Counter()
        continue
    c = cls(t)
    if c:
        cur[c] += 1
segs.append(cur)
keys = ["mfma", "ds_rd", "dma", "valu", "accmov", "lanemov", "salu", "wait", "nop", "vmem", "ds_oth", "scratch"]
print(f"{len(segs)} segments; columns: " + " ".join(keys))
for i, c in enumerate(segs):
    print(f"{i:3d} " + " ".join(f"{c.get(k, 0):5d}" for k in keys))
