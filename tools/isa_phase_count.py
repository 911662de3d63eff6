#!/usr/bin/env python3
"""Diagnostic: static instruction mix per pass of one kernel in a -DPSY_ASM_MARKS assembly dump.

usage: tools/isa_phase_count.py <file.s> <kernel-symbol-substring>
Counts VALU / SALU / LDS / VMEM / other instructions from each `;@@ROUND <pass>` marker to the
next marker (static counts along the listing, not executed counts: a marker region that contains
a branchy slow path over-counts).  Not part of the product path.
"""
import collections
import re
import sys


def kind(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt") or op.startswith("s_barrier") or op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "ctl"
    if op.startswith("s_"):
        return "salu"
    return None


def main(path, sym):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) or (sym in l and l.endswith(":") is False and l.split(":")[0].endswith(sym)))
    counts = collections.defaultdict(collections.Counter)
    regions = [["prologue", collections.Counter()]]
    cur = "prologue"
    for l in lines[start + 1:]:
        s = l.strip()
        if s.startswith("s_endpgm"):
            break
        m = re.match(r";@@ROUND (\w+)", s)
        if m:
            cur = m.group(1)
            counts[cur]["marks"] += 1
            regions.append([cur, collections.Counter()])
            continue
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        k = kind(s.split()[0])
        if k:
            counts[cur][k] += 1
            regions[-1][1][k] += 1
    if "-v" in sys.argv:
        for i, (p, c) in enumerate(regions):
            print(f"  region {i:3d} {p:6s} valu {c['valu']:5d} salu {c['salu']:5d} lds {c['lds']:4d} vmem {c['vmem']:4d} ctl {c['ctl']:4d}")
    print(f"{'pass':10s} {'marks':>5s} {'valu':>6s} {'salu':>6s} {'lds':>5s} {'vmem':>5s} {'ctl':>5s}   (per mark)")
    for p, c in counts.items():
        n = max(c["marks"], 1)
        print(f"{p:10s} {c['marks']:5d} {c['valu']:6d} {c['salu']:6d} {c['lds']:5d} {c['vmem']:5d} {c['ctl']:5d}   "
              f"valu {c['valu'] / n:.0f} salu {c['salu'] / n:.0f} lds {c['lds'] / n:.0f} vmem {c['vmem'] / n:.0f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
