"""Runs FIRST among the GPU tests: checks the hardware semantics of the device primitives
the codec kernels are built from (tests/native/selftest.hip) against host expectations."""
import ctypes as C
import pathlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

LIB = pathlib.Path(__file__).resolve().parent / "native" / "libtdt_selftest.so"


def host_perm(hi, lo, sel):
    src = int(lo) | (int(hi) << 32)
    out = 0
    for t in range(4):
        s = (sel >> (8 * t)) & 0xFF
        b = (src >> (8 * s)) & 0xFF if s < 8 else 0
        out |= b << (8 * t)
    return out


def host_mask4(x, below):
    prev = [(below >> 24) & 0xFF] + [(x >> (8 * i)) & 0xFF for i in range(3)]
    cur = [(x >> (8 * i)) & 0xFF for i in range(4)]
    return sum((1 << i) for i in range(4) if cur[i] != prev[i])


def test_primitives():
    assert torch.cuda.is_available()
    lib = C.CDLL(str(LIB))
    rng = np.random.default_rng(5)
    x = rng.integers(0, 1000, 256).astype(np.uint32)
    x[64:128] = rng.integers(0, 4, 64) * 0x01010101  # byte-equal patterns for the mask test
    x[5] = x[69] = 0x11223344
    d_in = torch.from_numpy(x.view(np.int32).copy()).cuda()
    d_out = torch.zeros(1700, dtype=torch.int32, device="cuda")
    assert lib.selftest_run(C.c_void_p(d_in.data_ptr()), C.c_void_p(d_out.data_ptr())) == 0
    o = d_out.cpu().numpy().view(np.uint32)
    xs = x.astype(np.uint64)
    for w in range(4):
        seg = xs[64 * w:64 * w + 64]
        assert np.array_equal(o[64 * w:64 * w + 64], np.cumsum(seg).astype(np.uint32)), "wave add-scan"
        assert np.array_equal(o[256 + 64 * w:256 + 64 * w + 64], np.maximum.accumulate(seg).astype(np.uint32)), "wave max-scan"
    ex = np.concatenate([[0], np.cumsum(xs)[:-1]]).astype(np.uint32)
    assert np.array_equal(o[512:768], ex), "team add-scan"
    assert o[768] == np.uint32(xs.sum())
    exm = np.concatenate([[0], np.maximum.accumulate(xs)[:-1]]).astype(np.uint32)
    assert np.array_equal(o[769:1025], exm), "team max-scan"
    assert o[1025] == x.max()
    assert np.array_equal(o[1026:1090], np.concatenate([[0], np.cumsum(xs[:64])[:-1]]).astype(np.uint32)), "W=1 scan"
    assert o[1090] == np.uint32(xs[:64].sum())
    sels = [0x03020100, 0x07060504, 0x0C0C0C0C, 0x0400070C, 0x01050C02, 0x0C0C0706, 0, 0x07070707]
    for l in range(64):
        assert o[1091 + l] == host_mask4(int(x[l]), int(x[l + 64])), ("mask", l)
        assert o[1155 + l] == host_perm(int(x[l]), int(x[l + 64]), sels[l & 7]), ("perm", l)
        assert o[1219 + l] == (((int(x[l]) << 32 | int(x[l + 64])) >> 24) & 0xFFFFFFFF), ("alignbyte", l)
        assert o[1283 + l] == (x[l - 1] if l else 0), ("shift_up", l)
    for l in range(64):
        assert o[1347 + l] == (x[l - 1] if l else 77), ("wave_shr1", l)
        assert o[1411 + l] == (x[l + 1] if l < 63 else 99), ("wave_shl1", l)
    h = (x[:64].astype(np.uint64) * 2654435761) & 0xFFFFFFFF
    lo = np.maximum.accumulate(h & 0xFFFF)
    hi = np.maximum.accumulate(h >> 16)
    assert np.array_equal(o[1475:1539], (lo | (hi << 16)).astype(np.uint32)), "packed u16 max-scan"
    for l in range(64):
        sh = l % 33
        v = 0 if sh == 32 else int(x[l]) >> sh
        want = 0xFFFFFFFF if v == 0 else 32 - v.bit_length()
        assert o[1539 + l] == want, ("ffbh", l, v)


def test_unaligned_lds():
    """ds_write_b16 at odd LDS addresses (the encode staging window is congruent mod 16 with
    an arbitrary output offset) and 16-byte LDS reads at 4-byte-aligned addresses."""
    lib = C.CDLL(str(LIB))
    d_out = torch.zeros(128, dtype=torch.int32, device="cuda")
    assert lib.selftest_unaligned_lds(C.c_void_p(d_out.data_ptr())) == 0
    o = d_out.cpu().numpy().view(np.uint32)
    buf = bytearray(512)
    for l in range(64):
        v = 0x100 + l
        buf[2 * l + 1] = v & 0xFF
        buf[2 * l + 2] = v >> 8
    want = np.frombuffer(bytes(buf[:256]), np.uint32)
    assert np.array_equal(o[:64], want), "unaligned ds_write_b16"
    words = np.frombuffer(bytes(buf), np.uint32)
    x = np.array([words[l] ^ words[l + 1] ^ words[l + 2] ^ words[l + 3] for l in range(64)], np.uint32)
    assert np.array_equal(o[64:128], x), "ds_read_b128 at 4-byte alignment"


@pytest.mark.parametrize("N", [256, 16384, 262144])
def test_device_log2_sweep(N):
    """Every c/N the entropy pass can form for a message of N words (1 KiB, 64 KiB and 1 MiB
    float32 messages): the device's restated glibc log2 and entropy step fma(-p, log2 p, 0)
    are bit-identical to this host's libm log2 (SURVEY.md §7 hard part (i))."""
    import ctypes.util
    lib = C.CDLL(str(LIB))
    lib.selftest_log2_sweep.argtypes = [C.c_uint32, C.c_void_p]
    out = torch.zeros(2 * N, dtype=torch.float64, device="cuda")
    assert lib.selftest_log2_sweep(N, C.c_void_p(out.data_ptr())) == 0
    got = out.cpu().numpy().reshape(N, 2)
    libm = C.CDLL(ctypes.util.find_library("m"))
    libm.log2.restype = C.c_double
    libm.log2.argtypes = [C.c_double]
    p = np.arange(1, N + 1, dtype=np.float64) / np.float64(N)
    want_l = np.array([libm.log2(float(x)) for x in p])
    assert np.array_equal(got[:, 0].view(np.uint64), want_l.view(np.uint64)), "device log2 != libm log2"
    # fma(-p, L, 0.0) rounds the exact product once and adds +0.0 (so -0.0 becomes +0.0): the
    # same as a rounded double multiply followed by + 0.0
    want_s = (-p) * want_l + 0.0
    assert np.array_equal(got[:, 1].view(np.uint64), want_s.view(np.uint64)), "entropy step"


def test_hw_log2_error_bound():
    """The encode's mapping fast path (psyne_amd/csrc/tdt_encode.h, "E") sums c·log2 c with the
    hardware log2 of (float)c and relies on |error| <= 2^-18 for every count a message can have:
    every c in [1, 2^24] (exact in float), and a sample of larger counts (rounded to float)."""
    lib = C.CDLL(str(LIB))
    lib.selftest_hw_log2.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    rng = np.random.default_rng(7)
    cs = [np.arange(1, (1 << 24) + 1, dtype=np.uint32),
          rng.integers(1 << 24, 1 << 32, 1 << 20, dtype=np.uint64).astype(np.uint32)]
    for c in cs:
        d_c = torch.from_numpy(c.astype(np.int64).astype(np.uint32).view(np.int32)).cuda()
        out = torch.empty(c.size, dtype=torch.float32, device="cuda")
        assert lib.selftest_hw_log2(C.c_void_p(d_c.data_ptr()), c.size, C.c_void_p(out.data_ptr())) == 0
        got = out.cpu().numpy().astype(np.float64)
        err = np.abs(got - np.log2(c.astype(np.float64)))
        assert float(err.max()) <= 2.0 ** -18, "hardware log2 error %.3g > 2^-18" % float(err.max())
