"""Content hash of what determines the HIP library's kernels: the device sources
(psyne_amd/csrc/*), the C ABI header and the build recipe (psyne_amd/build.py: compiler flags).
hipcc's output is not byte-reproducible (two builds of the same sources differ), so PMC records
under profiles/ are keyed to this hash as well as to the built library's sha256, and a rebuild
of unchanged sources still finds its traffic record.  No torch import (used by tools on the box)."""
import hashlib
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]


def src_sha256() -> str:
    files = sorted(p for p in (ROOT / "psyne_amd" / "csrc").iterdir() if p.suffix in (".h", ".hip", ".hpp"))
    files += [ROOT / "include" / "psyne_tdt.h", ROOT / "psyne_amd" / "build.py"]
    h = hashlib.sha256()
    for p in files:
        h.update(str(p.relative_to(ROOT)).encode() + b"\0" + p.read_bytes() + b"\0")
    return h.hexdigest()


if __name__ == "__main__":
    print(src_sha256())
