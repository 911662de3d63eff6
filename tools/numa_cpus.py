"""Print the CPU list (taskset form) of the NUMA node local to visible GPU 0, or of another node
('remote'), within this process's affinity: for pinning host-path harnesses (tcp_loopback) on
the box.  usage: python3 tools/numa_cpus.py [local|remote]"""
import os
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    want = sys.argv[1] if len(sys.argv) > 1 else "local"
    gpus = bench.visible_gpus()
    minor = gpus[0]["drm_render_minor"]
    node = int(pathlib.Path(bench.SYSFS_DRM, "renderD%d" % minor, "device", "numa_node").read_text())
    nodes = sorted(int(p.name[4:]) for p in pathlib.Path(bench.SYSFS_NODE).glob("node[0-9]*"))
    pick = node if want == "local" else next(n for n in nodes if n != node)
    cpus = bench.parse_cpulist(pathlib.Path(bench.SYSFS_NODE, "node%d" % pick, "cpulist").read_text())
    cpus &= os.sched_getaffinity(0)
    print(",".join(str(c) for c in sorted(cpus)))


if __name__ == "__main__":
    main()
