"""Scan a gfx950 assembly listing (hipcc -save-temps; the library build keeps one per object as
sg-nerf_amd/csrc/build/<src>.gfx950.s) for inline-asm VALU instructions that write a register an MFMA
wrote or reads as its accumulator input (srcC), or read an MFMA's result, within the previous 16
instructions (with no compiler-visible write of that register in between): the hazard recognizer does
not see inline asm, so such a write may land while the MFMA still reads its accumulator input.
Also an MFMA reading an operand an inline-asm VALU wrote fewer than 2 wait states before.
Usage: python tools/asm_hazards.py <file.s> [...]   (prints the candidates and their count; exit 1 if any)
tests/test_asm_hazards.py runs it on every built object and on a planted hazard."""
import re
import sys


def _regs(tok):
    tok = tok.strip().lstrip('-').strip('|')
    m = re.match(r'([va])\[(\d+):(\d+)\]', tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r'([va])(\d+)$', tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    return set()


def scan(text):
    """Hazard candidates of one listing: a list of one-line descriptions."""
    inasm = False
    hist = []  # recent instructions: (kind, dst, srcs, text)
    found = []
    for ln in text.split('\n'):
        s = ln.strip()
        if s.startswith(';;#ASMSTART'):
            inasm = True
            continue
        if s.startswith(';;#ASMEND'):
            inasm = False
            continue
        if not s or s.startswith(';') or s.endswith(':') or s.startswith('.'):
            continue
        parts = s.split(None, 1)
        op = parts[0]
        ops = parts[1].split(',') if len(parts) > 1 else []
        dst = _regs(ops[0]) if ops else set()
        if op.startswith('v_mfma'):
            # the accumulator input (srcC) is read over the MFMA's passes; srcA / srcB are latched at issue
            srcs = _regs(ops[3]) if len(ops) > 3 else set()
        else:
            srcs = set().union(*[_regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
        if inasm and op.startswith('v_') and not op.startswith('v_mfma'):
            # look back for an MFMA reading / writing the asm's destination, or writing a register the asm
            # reads, with no compiler-visible write of that register in between (such a write already waited
            # out the MFMA: the hazard recognizer saw it, and the asm then reads / overwrites that write)
            wd, rs = set(dst), set(srcs)
            for dist, (k, d2, s2, txt) in enumerate(reversed(hist[-16:])):
                if k == 'other' and not txt.startswith('asm:'):
                    wd -= d2
                    rs -= d2
                    if not wd and not rs:
                        break
                if k == 'mfma' and (wd & s2 or wd & d2 or rs & d2):  # WAR / WAW, or RAW of the MFMA's result
                    found.append(f'asm {s!r} {dist + 1} instrs after {txt!r}')
                    break
        if op.startswith('v_mfma'):
            # RAW: an MFMA reading (srcA / srcB / srcC) a register an inline-asm VALU wrote fewer than 2 wait
            # states before (the hazard recognizer does not pad asm writes; the MFMA would read a stale value)
            ab = set().union(*[_regs(o) for o in ops[1:4]]) if len(ops) > 3 else set()
            states = 0
            for k, d2, s2, txt in reversed(hist[-4:]):
                if states >= 2:
                    break
                if txt.startswith('asm:v_') and not txt.startswith('asm:v_mfma') and ab & d2:
                    found.append(f'mfma {s!r} reads asm {txt!r} after {states} wait states')
                    break
                states += 1
        kind = 'mfma' if op.startswith('v_mfma') else 'other'
        nw = 0
        if op == 's_nop':
            nw = int(ops[0], 0) + 1 if ops else 1
        hist.append((kind, dst, srcs, ('asm:' if inasm else '') + s))
        for _ in range(nw - 1):
            hist.append(('nop', set(), set(), 's_nop'))
    return found


def main(paths):
    total = 0
    for p in paths:
        found = scan(open(p).read())
        for f in found[:12]:
            print(f'{p}: {f}')
        total += len(found)
    print('hazard candidates:', total)
    return 1 if total else 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
