"""Build the gfx950 shared library in-tree: psyne_amd/libpsyne_tdt.so.

hipcc --offload-arch=gfx950 cross-compiles without a GPU, so this runs in the build
container; the resulting .so travels to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import os
import pathlib
import subprocess
import sys

PKG = pathlib.Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "libpsyne_tdt.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PSYNE_ARCH", "gfx950")

SOURCES = [CSRC / "tdt_api.hip"]  # (diagnostic single-TU builds compile this file alone)
ENC_WS_SRC = CSRC / "tdt_enc_ws.hip"  # the encode kernels of one word size
WORD_SIZES = (1, 2, 4, 8, 16)
# every source and header under csrc/ (tdt_api.hip includes the headers, directly or not)
DEPS = SOURCES + [ENC_WS_SRC] + sorted(CSRC.glob("*.h")) + [ROOT / "include" / "psyne_tdt.h"]
OBJ_DIR = PKG / "build"


def needs_build() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(p.stat().st_mtime > t for p in DEPS)


def build(force: bool = False, verbose: bool = False) -> pathlib.Path:
    """Compile tdt_api.hip and one tdt_enc_ws.hip object per word size in parallel (the encode
    kernels dominate the compile time), then link libpsyne_tdt.so."""
    if force or needs_build():
        OBJ_DIR.mkdir(exist_ok=True)
        base = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-I", str(ROOT / "include")]
        jobs = [(base + ["-c", str(SOURCES[0]), "-o", str(OBJ_DIR / "tdt_api.o")], OBJ_DIR / "tdt_api.o")]
        for ws in WORD_SIZES:
            o = OBJ_DIR / f"tdt_enc_ws{ws}.o"
            jobs.append((base + [f"-DPSY_INST_WS={ws}", "-c", str(ENC_WS_SRC), "-o", str(o)], o))
        procs = []
        for cmd, _ in jobs:
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append(subprocess.Popen(cmd))
        bad = [cmd for (cmd, _), p in zip(jobs, procs) if p.wait() != 0]
        if bad:
            raise subprocess.CalledProcessError(1, bad[0])
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *(str(o) for _, o in jobs), "-o", str(LIB)]
        if verbose:
            print(" ".join(link), flush=True)
        subprocess.check_call(link)
        from psyne_amd.srchash import write_record
        write_record(LIB, ARCH, HIPCC)  # (the key PMC traffic records are matched by)
    return LIB


CPP_TEST_SRC = ROOT / "tests" / "cpp" / "test_protocol.cpp"
CPP_TEST_BIN = ROOT / "tests" / "cpp" / "test_protocol"
LOOPBACK_SRC = ROOT / "tests" / "native" / "tcp_loopback.cpp"
LOOPBACK_BIN = ROOT / "tests" / "native" / "tcp_loopback"
SUBSTRATE_TEST_SRC = ROOT / "tests" / "cpp" / "test_substrate.cpp"
SUBSTRATE_TEST_BIN = ROOT / "tests" / "cpp" / "test_substrate"
SELFTEST_SRC = ROOT / "tests" / "native" / "selftest.hip"
SELFTEST_LIB = ROOT / "tests" / "native" / "libtdt_selftest.so"


def build_tests(verbose: bool = False):
    """Test-only native artefacts: the C++ Protocol drop-in test and the primitives self-test."""
    if not CPP_TEST_BIN.exists() or CPP_TEST_BIN.stat().st_mtime < max(
            CPP_TEST_SRC.stat().st_mtime, (ROOT / "include/psyne_amd/hip_tdt_protocol.hpp").stat().st_mtime,
            (ROOT / "include/psyne_amd/protocol_stack.hpp").stat().st_mtime, LIB.stat().st_mtime):
        cmd = ["g++", "-std=c++20", "-O2", "-I", str(ROOT / "include"), str(CPP_TEST_SRC), "-o", str(CPP_TEST_BIN),
               "-L", str(PKG), "-lpsyne_tdt", "-Wl,-rpath," + str(PKG), "-Wl,-rpath,$ORIGIN/../../psyne_amd"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    hdrs = [ROOT / "include/psyne_amd/hip_tdt_protocol.hpp", ROOT / "include/psyne_amd/tdt_substrate.hpp",
            ROOT / "include/psyne_amd/protocol_stack.hpp"]
    if not LOOPBACK_BIN.exists() or LOOPBACK_BIN.stat().st_mtime < max(
            [LOOPBACK_SRC.stat().st_mtime, LIB.stat().st_mtime] + [h.stat().st_mtime for h in hdrs]):
        cmd = ["g++", "-std=c++20", "-O2", "-I", str(ROOT / "include"), str(LOOPBACK_SRC), "-o", str(LOOPBACK_BIN),
               "-L", str(PKG), "-lpsyne_tdt", "-pthread", "-ldl", "-Wl,-rpath," + str(PKG),
               "-Wl,-rpath,$ORIGIN/../../psyne_amd"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    if not SUBSTRATE_TEST_BIN.exists() or SUBSTRATE_TEST_BIN.stat().st_mtime < max(
            [SUBSTRATE_TEST_SRC.stat().st_mtime, LIB.stat().st_mtime] + [h.stat().st_mtime for h in hdrs]):
        cmd = ["g++", "-std=c++20", "-O2", "-I", str(ROOT / "include"), str(SUBSTRATE_TEST_SRC), "-o",
               str(SUBSTRATE_TEST_BIN), "-L", str(PKG), "-lpsyne_tdt", "-pthread", "-Wl,-rpath," + str(PKG),
               "-Wl,-rpath,$ORIGIN/../../psyne_amd"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    if not SELFTEST_LIB.exists() or SELFTEST_LIB.stat().st_mtime < max(
            SELFTEST_SRC.stat().st_mtime, (CSRC / "tdt_device.h").stat().st_mtime):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-shared", str(SELFTEST_SRC), "-o", str(SELFTEST_LIB)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    build_tests(verbose=True)
    print(LIB)
