#!/usr/bin/env python3
"""Diagnostic: SGPR-spill traffic of one kernel in an assembly listing (-DPSY_ASM_MARKS builds).

usage: tools/isa_spills.py <file.s> <kernel-symbol>
Prints, per `;@@ROUND <pass>` region, the static count of v_writelane / v_readlane instructions
on the compiler's "SGPR spill to VGPR lane" registers, scratch loads / stores, and VALU / SALU
totals — the static cost the 8-waves-per-SIMD register budget adds.  Not part of the product path."""
import collections
import re
import sys


def main(path, sym):
    lines = open(path).read().splitlines()
    st = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    spill_regs = set()
    for l in lines[st:en]:
        m = re.search(r"implicit-def: \$vgpr(\d+) : SGPR spill to VGPR lane", l)
        if m:
            spill_regs.add("v" + m.group(1))
    region = "prologue"
    c = collections.defaultdict(collections.Counter)
    for l in lines[st:en]:
        m = re.search(r";@@ROUND (\w+)", l)
        if m:
            region = m.group(1)
            continue
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")):
            continue
        op = t[0]
        args = " ".join(t[1:])
        if op.startswith("v_writelane") and t[1].rstrip(",") in spill_regs:
            c[region]["spill_w"] += 1
        elif op.startswith("v_readlane") and len(t) > 2 and t[2].rstrip(",") in spill_regs:
            c[region]["spill_r"] += 1
        elif op.startswith("scratch_"):
            c[region]["scratch"] += 1
        if op.startswith("v_"):
            c[region]["valu"] += 1
        elif op.startswith("s_") and not op.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch", "s_barrier")):
            c[region]["salu"] += 1
    tot = collections.Counter()
    for r, cc in c.items():
        tot.update(cc)
        print("%-9s %s" % (r, dict(cc)))
    print("total     %s  spill VGPRs %s" % (dict(tot), sorted(spill_regs)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
