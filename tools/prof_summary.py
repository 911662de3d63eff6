#!/usr/bin/env python3
"""Summarise rocprofv3 output (results .db or kernel_stats.csv) into a small markdown table.

usage: python tools/prof_summary.py <rocprof output dir> <out.md> [title]
"""
import csv
import glob
import pathlib
import sqlite3
import sys


def rows_from_db(db):
    c = sqlite3.connect(db)
    # the rocpd top_kernels view reports durations in microseconds; normalise to ns
    return [(r[0], int(r[1]), float(r[2]) * 1e3, float(r[3]) * 1e3, float(r[4]))
            for r in c.execute("select name,total_calls,total_duration,average,percentage from top_kernels")]


def rows_from_csv(p):
    out = []
    with open(p) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                        float(r["Percentage"])))
    return out


def main():
    d, out = pathlib.Path(sys.argv[1]), pathlib.Path(sys.argv[2])
    title = sys.argv[3] if len(sys.argv) > 3 else str(d)
    dbs = glob.glob(str(d / "**" / "*.db"), recursive=True)
    csvs = glob.glob(str(d / "**" / "*kernel_stats.csv"), recursive=True)
    rows = rows_from_csv(csvs[0]) if csvs else rows_from_db(dbs[0])
    lines = ["# " + title, "", "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for name, calls, tot, avg, pct in rows[:12]:
        short = name if len(name) < 90 else name[:87] + "..."
        lines.append("| `%s` | %d | %.3f | %.1f | %.2f |" % (short, calls, tot / 1e6, avg / 1e3, pct))
    out.write_text("\n".join(lines) + "\n")
    print("\n".join(lines[:8]))


if __name__ == "__main__":
    main()
