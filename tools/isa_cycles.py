#!/usr/bin/env python3
"""Diagnostic: modelled VALU issue cycles per region of a -DPSY_ASM_MARKS kernel listing.

usage: tools/isa_cycles.py <file.s> <kernel-symbol> [-v]
gfx950 issue costs measured by tools/ubench_valu3.hip (profiles/r05_ubench/ubench3.txt): the
e32/e64 forms of v_add/sub/subrev_u32, v_and/or/xor/not_b32, v_mov_b32 and v_lshrrev_b32 issue
in ~2 cycles per wave64 instruction; every other VALU opcode tried (v_perm, v_bfe, v_lshlrev,
v_min/max, 3-operand VOP3 forms, SDWA and DPP forms, packed u16, v_cndmask, carry forms,
compares) in ~4.  Static counts along the listing (not executed counts)."""
import collections
import re
import sys

FAST = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_not_b32",
        "v_mov_b32", "v_lshrrev_b32", "v_ashrrev_i32"}


def cost(op, line):
    base = re.sub(r"_e(32|64)$", "", op)
    if "_sdwa" in op or "_dpp" in op or "row_" in line or "quad_perm" in line:
        return 4
    if base in FAST:
        return 2
    return 4


def main(path, sym, verbose):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    regions = [["prologue", collections.Counter()]]
    for l in lines[start + 1:]:
        s = l.strip()
        if s.startswith("s_endpgm") and "ASM" not in s:
            pass
        if s.startswith(".Lfunc_end"):
            break
        m = re.match(r";@@(ROUND|MARK) (\w+)", s)
        if m:
            regions.append([m.group(2), collections.Counter()])
            continue
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        c = regions[-1][1]
        if op.startswith("v_"):
            c["valu"] += 1
            c["cyc"] += cost(op, s)
            if cost(op, s) == 2:
                c["fast"] += 1
            c[op] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_", "buffer_")):
            c["vmem"] += 1
        elif op.startswith("s_nop"):
            c["nop"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    tot = collections.defaultdict(collections.Counter)
    for i, (p, c) in enumerate(regions):
        tot[p].update(c)
        tot[p]["marks"] += 1
        if verbose:
            print(f"region {i:3d} {p:6s} valu {c['valu']:5d} fast {c['fast']:4d} cyc {c['cyc']:6d} salu {c['salu']:5d} "
                  f"nop {c['nop']:3d} lds {c['lds']:4d} vmem {c['vmem']:4d}")
    for p, c in tot.items():
        print(f"{p:8s} marks {c['marks']:3d} valu {c['valu']:6d} fast {c['fast']:5d} cyc {c['cyc']:7d} "
              f"salu {c['salu']:6d} nop {c['nop']:4d} lds {c['lds']:5d}")
    if "-ops" in sys.argv:
        p = sys.argv[sys.argv.index("-ops") + 1]
        ops = {k: v for k, v in tot[p].items() if k.startswith("v_")}
        for k, v in sorted(ops.items(), key=lambda kv: -kv[1]):
            print(f"   {k:28s} {v:5d}  cost {cost(k, k)}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], "-v" in sys.argv)
