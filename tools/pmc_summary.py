#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter_collection.csv files per kernel (mean per dispatch)."""
import collections
import csv
import glob
import sys


def main():
    root = sys.argv[1]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "tdt_" not in k:
                continue
            short = k.split("(")[0].replace("void psy::", "")
            per[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
            per[short]["_dur_ns"].append(float(r.get("End_Timestamp", 0)) - float(r.get("Start_Timestamp", 0)))
    for k, d in per.items():
        print("==", k)
        for c, v in sorted(d.items()):
            print("   %-24s %16.4g" % (c, sum(v) / len(v)))


if __name__ == "__main__":
    main()
