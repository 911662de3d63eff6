"""Per-stream kernel timeline of the last encode + decode step in a rocprofv3 trace of
bench.py --workload c4 (times in ms from the step's encode plan kernel)."""
import csv
import glob
import sys

d = sys.argv[1]
K = list(csv.DictReader(open(glob.glob(d + "/**/run_kernel_trace.csv", recursive=True)[0])))
ev = sorted([(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"], k["Stream_Id"], k["Grid_Size_X"])
             for k in K])
i0 = [i for i, e in enumerate(ev) if "tdt_encode_plan" in e[2]][-1]
i1 = [i for i, e in enumerate(ev) if "tdt_decode_plan" in e[2] and i > i0][0]
base = ev[i0][0]
end = max(e[1] for e in ev[i0:i1 + 12])
for e in ev[i0:i1 + 12]:
    if e[0] > end:
        break
    n = e[2].replace("psy::", "").replace("(psy::EncodeArgs)", "").replace("(psy::DecodeArgs)", "")
    print("%8.2f %8.2f s%s %-64s %s" % ((e[0] - base) / 1e6, (e[1] - e[0]) / 1e6, e[3], n[:64], e[4]))
