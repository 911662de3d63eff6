"""psyne_amd/csrc/tdt_log2.h (the device's restatement of glibc log2 + the contracted
entropy step) against the system libm, bit for bit.  The same header is compiled into the
HIP kernels; here it is compiled for the host with -ffp-contract=off."""
import ctypes as C
import pathlib
import subprocess
import tempfile

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]

SRC = r'''
#include "tdt_log2.h"
#include <math.h>
static const double T[128] = PSY_LOG2_TAB_INIT, T2[128] = PSY_LOG2_TAB2_INIT;
long check_cn(unsigned nlo, unsigned nhi, unsigned step) {
  long bad = 0;
  for (unsigned N = nlo; N <= nhi; N += step) { double d = N;
    for (unsigned c = 1; c <= N; c++) { double p = (double)c / d;
      double a = log2(p), b = psy_log2_glibc(p, T, T2);
      if (psy_as_u64(a) != psy_as_u64(b)) bad++;
      double e1 = fma(-p, a, 3.25), e2 = psy_entropy_step(3.25, c, d, T, T2);
      if (psy_as_u64(e1) != psy_as_u64(e2)) bad++; } }
  return bad; }
long check_bits(const unsigned long long *u, long n) {
  long bad = 0;
  for (long i = 0; i < n; i++) { double x = psy_as_f64(u[i]);
    if (psy_as_u64(log2(x)) != psy_as_u64(psy_log2_glibc(x, T, T2))) bad++; }
  return bad; }
'''


@pytest.fixture(scope="module")
def lib():
    d = pathlib.Path(tempfile.mkdtemp())
    (d / "t.c").write_text(SRC)
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fPIC", "-shared",
                           "-I", str(ROOT / "psyne_amd/csrc"), str(d / "t.c"), "-o", str(d / "t.so"), "-lm"])
    L = C.CDLL(str(d / "t.so"))
    L.check_cn.restype = C.c_long
    L.check_cn.argtypes = [C.c_uint, C.c_uint, C.c_uint]
    L.check_bits.restype = C.c_long
    L.check_bits.argtypes = [C.c_void_p, C.c_long]
    return L


def test_every_probability_small_n(lib):
    # every p = c/N the codec produces for messages up to 16 KiB (ws=4)
    assert lib.check_cn(1, 4096, 1) == 0


def test_sampled_large_n(lib):
    # 64 KiB (N=16384), 1 MiB (N=262144) and a spread in between
    for N in (16384, 16385, 65536, 262144):
        assert lib.check_cn(N, N, 1) == 0
    assert lib.check_cn(4097, 200000, 9973) == 0


def test_random_doubles(lib):
    rng = np.random.default_rng(3)
    u = rng.integers(0, 2**63 - 1, 4_000_000, dtype=np.uint64)
    # keep positive normal finite values
    e = (u >> np.uint64(52)) & np.uint64(0x7FF)
    u = u[(e > 0) & (e < 0x7FF)]
    near1 = (np.float64(1.0) + rng.uniform(-0.05, 0.05, 1_000_000)).view(np.uint64)
    u = np.ascontiguousarray(np.concatenate([u, near1]))
    assert lib.check_bits(u.ctypes.data, u.size) == 0
