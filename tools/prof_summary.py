#!/usr/bin/env python3
"""Summarise rocprofv3 output (results .db or kernel_stats.csv) into a small markdown table.

usage: python tools/prof_summary.py <rocprof output dir> <out.md> [title] [--steady K]

The table is rocprofv3's own --stats summary (every call, warm-up calls included).  With
--steady K and a kernel trace present, a second table gives each psy:: kernel's average over
its LAST K calls (the timed steps of the bench command, after its warm-up calls: the first call
of a context runs without a plan history and on untouched output pages).
"""
import collections
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


def steady_rows(trace, k):
    per = collections.defaultdict(list)
    with open(trace) as f:
        for r in csv.DictReader(f):
            if "psy::" not in r["Kernel_Name"]:
                continue
            per[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = []
    for name, v in per.items():
        v.sort()
        last = v[-k:]
        out.append((name, len(last), sum(e - s for s, e in last) / len(last)))
    return sorted(out, key=lambda x: -x[2] * x[1])


def main():
    args = [a for a in sys.argv[1:]]
    steady = 0
    if "--steady" in args:
        i = args.index("--steady")
        steady = int(args[i + 1])
        del args[i:i + 2]
    d, out = pathlib.Path(args[0]), pathlib.Path(args[1])
    title = args[2] if len(args) > 2 else str(d)
    dbs = glob.glob(str(d / "**" / "*.db"), recursive=True)
    csvs = glob.glob(str(d / "**" / "*kernel_stats.csv"), recursive=True)
    rows = rows_from_csv(csvs[0]) if csvs else rows_from_db(dbs[0])
    lines = ["# " + title, "", "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for name, calls, tot, avg, pct in rows[:12]:
        short = name if len(name) < 90 else name[:87] + "..."
        lines.append("| `%s` | %d | %.3f | %.1f | %.2f |" % (short, calls, tot / 1e6, avg / 1e3, pct))
    traces = glob.glob(str(d / "**" / "*kernel_trace.csv"), recursive=True)
    if steady and traces:
        lines += ["", "Steady state: average over each psy:: kernel's last %d calls (the timed steps)." % steady, "",
                  "| kernel | calls | avg us |", "|---|---|---|"]
        for name, n, avg in steady_rows(traces[0], steady)[:12]:
            short = name if len(name) < 90 else name[:87] + "..."
            lines.append("| `%s` | %d | %.1f |" % (short, n, avg / 1e3))
    out.write_text("\n".join(lines) + "\n")
    print("\n".join(lines[:8]))


if __name__ == "__main__":
    main()
