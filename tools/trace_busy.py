"""GPU busy time (union of kernel and copy intervals) over the last `window` ms of a rocprofv3
csv trace, the idle gaps, and the copy engines' busy time."""
import csv
import glob
import sys

d, win = sys.argv[1], float(sys.argv[2]) * 1e6
K = list(csv.DictReader(open(glob.glob(d + "/**/run_kernel_trace.csv", recursive=True)[0])))
M = list(csv.DictReader(open(glob.glob(d + "/**/run_memory_copy_trace.csv", recursive=True)[0])))
iv = sorted([(int(k["Start_Timestamp"]), int(k["End_Timestamp"])) for k in K] +
            [(int(m["Start_Timestamp"]), int(m["End_Timestamp"])) for m in M])
end = max(e for _, e in iv)
t0 = end - win
iv = [(max(s, t0), e) for s, e in iv if e > t0]
busy, gaps, cs, ce = 0, [], None, None
for s, e in iv:
    if ce is None:
        cs, ce = s, e
    elif s > ce:
        busy += ce - cs
        gaps.append(s - ce)
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
gaps.sort()
h2d = sum(int(m["End_Timestamp"]) - int(m["Start_Timestamp"]) for m in M
          if int(m["Start_Timestamp"]) > t0 and "HOST_TO" in m["Direction"])
d2h = sum(int(m["End_Timestamp"]) - int(m["Start_Timestamp"]) for m in M
          if int(m["Start_Timestamp"]) > t0 and "TO_HOST" in m["Direction"])
print("window %.1f ms: busy %.1f ms, %d gaps > 100 us (%.1f ms), largest %s us; H2D %.1f ms, D2H %.1f ms" %
      (win / 1e6, busy / 1e6, sum(1 for g in gaps if g > 1e5), sum(g for g in gaps if g > 1e5) / 1e6,
       [round(g / 1e3) for g in gaps[-6:]], h2d / 1e6, d2h / 1e6))
