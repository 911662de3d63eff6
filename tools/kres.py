"""Per-kernel resource usage of the library (one line per kernel: VGPRs, spills, occupancy,
LDS), from hipcc's kernel-resource-usage remarks.  Usage: python tools/kres.py [-DPSY_FAST_BUILD]"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", *sys.argv[1:],
       "-I", "include", "psyne_amd/csrc/tdt_api.hip", "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in err.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    name = name.replace("psy::", "").replace("(psy::EncodeArgs)", "").replace("(psy::DecodeArgs)", "")
    print("%-60s vgpr %3s vspill %3s sspill %3s occ %s lds %s" % (name[:60], r.get("VGPRs"), r.get("VGPRs Spill"),
          r.get("SGPRs Spill"), r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]")))
