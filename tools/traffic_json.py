#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc passes -> profiles/<tag>_traffic.json.

usage: python tools/traffic_json.py <pmc dir> <out.json> <config key> [library .so]

The record carries the sha256 of the HIP library the passes ran (default
psyne_amd/libpsyne_tdt.so); bench.py reports `roofline.traffic` only from a record whose hash
matches the library it is running, so a traffic figure can never describe other code.

FETCH_SIZE / WRITE_SIZE are reported in KB.  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE
reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so it is
doubled; WRITE_SIZE reads the bytes exactly for 16-B-per-lane stores.  Per launch = mean over
the dispatches of the kernel.
"""
import collections
import csv
import glob
import hashlib
import os
import json
import pathlib
import sys


def main():
    root, out, key = sys.argv[1], sys.argv[2], sys.argv[3]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("psy::", "")
            if "tdt_" not in k:
                continue
            short = k.split("(")[0].split("<")[0]
            tmpl = k.split("(")[0]
            per[(short, tmpl)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for (short, tmpl), d in per.items():
        if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
            continue
        fetch = 2.0 * 1024 * sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
        write = 1024.0 * sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
        ent = {"template": tmpl, "fetch_bytes_corrected": fetch, "write_bytes": write,
               "hbm_bytes_per_launch": fetch + write, "dispatches": len(d["FETCH_SIZE"])}
        # the largest instantiation of a kernel name is the main pass (sizes-only passes are tiny)
        if short not in kernels or ent["hbm_bytes_per_launch"] > kernels[short]["hbm_bytes_per_launch"]:
            kernels[short] = ent
    # mixed-class workloads (C4): one encode or decode CALL launches a kernel per message class
    # (plus plan, tile passes, copy lists), so the bench's encode / decode figure is per call:
    # every dispatch of the direction's kernels summed, divided by the calls (plan dispatches)
    if key.startswith("c4"):
        for d in ("encode", "decode"):
            tot, calls = 0.0, 0
            for (short, tmpl), c in per.items():
                if not short.startswith("tdt_" + d) and ("tdt_" + d) not in short:
                    continue
                if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                    tot += 2.0 * 1024 * sum(c["FETCH_SIZE"]) + 1024.0 * sum(c["WRITE_SIZE"])
                if short.endswith("tdt_%s_plan_kernel" % d):
                    calls = len(c.get("FETCH_SIZE", []))
            if calls:
                kernels["tdt_%s_kernel" % d] = {
                    "template": "every %s-path kernel of one call (summed over dispatches / calls)" % d,
                    "hbm_bytes_per_launch": tot / calls, "calls": calls}
    lib = pathlib.Path(sys.argv[4] if len(sys.argv) > 4 else
                       pathlib.Path(__file__).resolve().parent.parent / "psyne_amd" / "libpsyne_tdt.so")
    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent.parent))
    from psyne_amd.srchash import recorded
    res = {"config": key, "kernels": kernels, "lib_sha256": hashlib.sha256(lib.read_bytes()).hexdigest(),
           "src_sha256": recorded(lib),  # (written by the build beside the library; None for variants)
           "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) and WRITE_SIZE in separate passes"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
