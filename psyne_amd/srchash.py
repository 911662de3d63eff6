"""Content hash of what determines the HIP library's kernels: the device sources
(psyne_amd/csrc/*), the C ABI header and the build recipe (psyne_amd/build.py: compiler flags),
plus the target architecture and compiler the build used.  hipcc's output is not
byte-reproducible (two builds of the same sources differ), so PMC records under profiles/ are
keyed to this hash as well as to the built library's sha256, and a rebuild of unchanged sources
still finds its traffic record.

The hash is computed by psyne_amd/build.py when it links the library and written next to it
(`libpsyne_tdt.so.srcsha`); bench.py and tools/traffic_json.py read that record instead of
re-hashing the working tree, so a stale library, or one built for another architecture, is never
credited with another build's traffic.  No torch import (used by tools on the box)."""
import hashlib
import json
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]


def src_sha256(arch: str = "gfx950", hipcc: str = "/opt/rocm/bin/hipcc") -> str:
    files = sorted(p for p in (ROOT / "psyne_amd" / "csrc").iterdir() if p.suffix in (".h", ".hip", ".hpp"))
    files += [ROOT / "include" / "psyne_tdt.h", ROOT / "psyne_amd" / "build.py"]
    h = hashlib.sha256()
    for p in files:
        h.update(str(p.relative_to(ROOT)).encode() + b"\0" + p.read_bytes() + b"\0")
    h.update(("arch=%s\0hipcc=%s\0" % (arch, hipcc)).encode())
    return h.hexdigest()


def record_path(lib: pathlib.Path) -> pathlib.Path:
    return lib.with_name(lib.name + ".srcsha")


def write_record(lib: pathlib.Path, arch: str, hipcc: str) -> str:
    """Called by the build right after linking `lib`."""
    sha = src_sha256(arch, hipcc)
    record_path(lib).write_text(json.dumps({"src_sha256": sha, "arch": arch, "hipcc": hipcc}) + "\n")
    return sha


def recorded(lib: pathlib.Path):
    """The source hash recorded when `lib` was built, or None (no record, or a record older than
    the library: the library was rebuilt some other way)."""
    r = record_path(pathlib.Path(lib))
    try:
        if r.stat().st_mtime < pathlib.Path(lib).stat().st_mtime:
            return None
        return json.loads(r.read_text()).get("src_sha256")
    except (OSError, ValueError):
        return None


if __name__ == "__main__":
    print(src_sha256())
