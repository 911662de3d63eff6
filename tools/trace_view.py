"""Print a window of a rocprofv3 kernel + memory-copy trace (csv) as one timeline (µs)."""
import csv
import sys

d = sys.argv[1]
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.8
count = int(sys.argv[3]) if len(sys.argv) > 3 else 200
K = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
M = list(csv.DictReader(open(d + "/run_memory_copy_trace.csv")))
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), "K", k["Kernel_Name"][:48], k["Stream_Id"], k["Grid_Size_X"])
      for k in K]
ev += [(int(m["Start_Timestamp"]), int(m["End_Timestamp"]), "M", m["Direction"].replace("MEMORY_COPY_", ""),
        m["Stream_Id"], "") for m in M]
ev.sort()
start = int(len(ev) * frac)
base = ev[start][0]
for e in ev[start:start + count]:
    print("%9.1f %8.1f %s s%s %-48s %s" % ((e[0] - base) / 1e3, (e[1] - e[0]) / 1e3, e[2], e[4], e[3], e[5]))
