#!/usr/bin/env python3
"""Diagnostic (not product): what the GPU box exposes for bench.py's topology helpers.

Prints the visibility variables, the KFD topology nodes that have SIMDs, each node's render
minor and the DRM device's numa_node, and what bench.visible_gpus() / numa_bind() return.
Touches no HIP (safe before any GPU call)."""
import os
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent.parent))

for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"):
    print(f"{v}={os.environ.get(v)!r}")
root = pathlib.Path("/sys/class/kfd/kfd/topology/nodes")
try:
    nodes = sorted(root.iterdir(), key=lambda q: int(q.name) if q.name.isdigit() else 1 << 30)
except OSError as e:
    print("kfd topology unreadable:", e)
    nodes = []
for d in nodes:
    try:
        props = dict(l.split()[:2] for l in (d / "properties").read_text().splitlines() if len(l.split()) >= 2)
    except OSError as e:
        print(d.name, "unreadable", e)
        continue
    keys = ("simd_count", "drm_render_minor", "location_id", "domain", "unique_id", "gpu_id")
    gid = ""
    try:
        gid = (d / "gpu_id").read_text().strip()
    except OSError:
        pass
    print(d.name, {k: props.get(k) for k in keys}, "gpu_id file:", gid)
    minor = props.get("drm_render_minor")
    if minor and minor.lstrip("-").isdigit() and int(minor) >= 0:
        p = pathlib.Path(f"/sys/class/drm/renderD{minor}/device/numa_node")
        try:
            print("   ", p, "=", p.read_text().strip())
        except OSError as e:
            print("   ", p, "unreadable:", e)
for p in sorted(pathlib.Path("/dev/dri").glob("renderD*")) if pathlib.Path("/dev/dri").exists() else []:
    print("dev:", p, os.access(p, os.R_OK | os.W_OK))
try:
    print("node dirs:", sorted(x.name for x in pathlib.Path("/sys/devices/system/node").glob("node*")))
except OSError as e:
    print("node dirs unreadable", e)
print("affinity:", len(os.sched_getaffinity(0)), "cpus")
import bench  # noqa: E402  (bench.py imports no torch at module level)

g = bench.visible_gpus()
print("visible_gpus:", len(g), [x.get("drm_render_minor") for x in g])
print("numa_bind(0):", bench.numa_bind(0))
