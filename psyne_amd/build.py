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

SOURCES = [CSRC / "tdt_api.hip"]
# every header under csrc/ (tdt_api.hip includes them all, directly or not)
DEPS = SOURCES + sorted(CSRC.glob("*.h")) + [ROOT / "include" / "psyne_tdt.h"]


def needs_build() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(p.stat().st_mtime > t for p in DEPS)


def build(force: bool = False, verbose: bool = False) -> pathlib.Path:
    if force or needs_build():
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-I", str(ROOT / "include"), *map(str, SOURCES), "-o", str(LIB)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
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
