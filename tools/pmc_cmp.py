#!/usr/bin/env python3
"""Diagnostic: side-by-side PMC counters of one kernel across pmc_summary outputs.
usage: tools/pmc_cmp.py "<kernel name prefix>" a.txt b.txt ..."""
import sys


def load(path, kern):
    out, cur = {}, None
    for line in open(path):
        if line.startswith("=="):
            cur = line[3:].strip()
            continue
        if cur and cur.startswith(kern):
            f = line.split()
            if len(f) == 2:
                out.setdefault(f[0], float(f[1]))
    return out


kern = sys.argv[1]
tabs = [(p, load(p, kern)) for p in sys.argv[2:]]
keys = sorted(set().union(*[t.keys() for _, t in tabs]))
print("%-24s" % "counter" + "".join("%16s" % p.split("/")[-1][:15] for p, _ in tabs))
for k in keys:
    print("%-24s" % k + "".join("%16.4g" % t.get(k, float("nan")) for _, t in tabs))
