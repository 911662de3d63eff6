"""ctypes bindings for the CPU checkers — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The product package (psyne_amd/) never imports this module.

* ``Oracle``  — oracle/libtdt_oracle.so, the plain-C restatement of the reference codec
  (include/psyne/protocol/tdt_compression.hpp).
* ``Reference`` — oracle/_ref/libtdt_ref.so, the reference header itself compiled where it
  lies (oracle/Makefile).  Absent unless it was built in the container that has
  /root/reference; the built file travels to the GPU box.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
ORACLE_SO = HERE / "libtdt_oracle.so"
REF_SO = HERE / "_ref" / "libtdt_ref.so"

# status codes (same values as include/psyne_tdt.h)
OK, E_SHORT, E_MAGIC, E_TRUNCATED, E_BAD_MAPPING, E_CAPACITY = 0, 1, 2, 3, 4, 5
E_BAD_HEADER, E_CONFIG, E_NONDETERMINISTIC = 7, 8, 9

_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)
_i32p = C.POINTER(C.c_int32)


class OracleConfig(C.Structure):
    _fields_ = [
        ("sample_fraction", C.c_float),
        ("word_size", C.c_int32),
        ("bandwidth_threshold_mbps", C.c_double),
        ("cpu_usage_threshold", C.c_double),
        ("min_tensor_size", C.c_uint64),
    ]


def _ptr(a: np.ndarray, t=_u8p):
    return a.ctypes.data_as(t)


def _bytes(x) -> np.ndarray:
    if isinstance(x, np.ndarray):
        return np.ascontiguousarray(x).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(x), dtype=np.uint8)


def encode_bound(n: int, ws: int = 4) -> int:
    return max(n + 4, 20 + 4 * ws + 8 + 2 * n)


class Oracle:
    def __init__(self, path: os.PathLike | None = None):
        self.lib = C.CDLL(str(path or ORACLE_SO))
        L = self.lib
        L.tdt_oracle_should_transform.restype = C.c_int
        L.tdt_oracle_should_transform.argtypes = [C.c_uint64, C.POINTER(OracleConfig), C.c_double, C.c_double]
        L.tdt_oracle_analyze.restype = C.c_int
        L.tdt_oracle_analyze.argtypes = [_u8p, C.c_uint64, C.c_int32, C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_double), _i32p]
        L.tdt_oracle_encode.restype = C.c_int
        L.tdt_oracle_encode.argtypes = [_u8p, C.c_uint64, C.POINTER(OracleConfig), C.c_double, C.c_double,
                                        _i32p, _u8p, C.c_uint64, _u64p]
        L.tdt_oracle_decode.restype = C.c_int
        L.tdt_oracle_decode.argtypes = [_u8p, C.c_uint64, _u8p, C.c_uint64, _u64p]
        L.tdt_oracle_decoded_size.restype = C.c_int
        L.tdt_oracle_decoded_size.argtypes = [_u8p, C.c_uint64, _u64p]
        L.tdt_oracle_encode_batch_mt.restype = C.c_int
        L.tdt_oracle_encode_batch_mt.argtypes = [_u8p, _u64p, C.c_uint32, C.POINTER(OracleConfig), C.c_double,
                                                 C.c_double, _u8p, _u64p, _u64p, _i32p, C.c_int]

    @staticmethod
    def config(word_size=4, sample_fraction=1.0, bandwidth_threshold_mbps=100.0,
               cpu_usage_threshold=0.8, min_tensor_size=1024) -> OracleConfig:
        return OracleConfig(sample_fraction, word_size, bandwidth_threshold_mbps,
                            cpu_usage_threshold, min_tensor_size)

    def should_transform(self, n, cfg=None, bandwidth=10.0, cpu=0.5) -> bool:
        cfg = cfg or self.config()
        return bool(self.lib.tdt_oracle_should_transform(n, C.byref(cfg), bandwidth, cpu))

    def analyze(self, data, word_size=4):
        d = _bytes(data)
        hist = np.zeros((word_size, 256), np.uint32)
        ent = np.zeros(word_size, np.float64)
        mp = np.zeros(word_size, np.int32)
        st = self.lib.tdt_oracle_analyze(_ptr(d), d.size, word_size,
                                         hist.ctypes.data_as(C.POINTER(C.c_uint32)),
                                         ent.ctypes.data_as(C.POINTER(C.c_double)), _ptr(mp, _i32p))
        if st:
            raise ValueError("analyze status %d" % st)
        return hist, ent, mp

    def encode(self, data, cfg=None, bandwidth=10.0, cpu=0.5, mapping=None) -> bytes:
        cfg = cfg or self.config()
        d = _bytes(data)
        cap = encode_bound(d.size, max(cfg.word_size, 1))
        out = np.empty(cap, np.uint8)
        olen = C.c_uint64(0)
        mp = None
        if mapping is not None:
            mp = np.ascontiguousarray(mapping, dtype=np.int32)
        st = self.lib.tdt_oracle_encode(_ptr(d), d.size, C.byref(cfg), bandwidth, cpu,
                                        _ptr(mp, _i32p) if mp is not None else None,
                                        _ptr(out), cap, C.byref(olen))
        if st:
            raise ValueError("oracle encode status %d" % st)
        return out[: olen.value].tobytes()

    def decoded_size(self, blob) -> tuple[int, int]:
        b = _bytes(blob)
        n = C.c_uint64(0)
        st = self.lib.tdt_oracle_decoded_size(_ptr(b), b.size, C.byref(n))
        return st, n.value

    def decode(self, blob) -> tuple[int, bytes]:
        """Returns (status, bytes)."""
        b = _bytes(blob)
        st, n = self.decoded_size(b)
        if st:
            return st, b""
        out = np.empty(max(n, 1), np.uint8)
        olen = C.c_uint64(0)
        st = self.lib.tdt_oracle_decode(_ptr(b), b.size, _ptr(out), out.size, C.byref(olen))
        return st, out[: olen.value].tobytes() if st == 0 else b""

    # batch conveniences -------------------------------------------------------------
    def encode_slotted(self, data: np.ndarray, offsets: np.ndarray, cfg=None, bandwidth=10.0, cpu=0.5,
                       threads: int = 0):
        """Encode every message into its own slot (slot i = the prefix of tdt_encode_bound),
        on `threads` host threads (0 = all usable cores).  Returns (out, slot_off, lengths)."""
        cfg = cfg or self.config()
        d = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = off.size - 1
        sizes = np.diff(off.astype(np.int64))
        bounds = np.maximum(sizes + 4, 20 + 4 * cfg.word_size + 8 + 2 * sizes)
        slot = np.zeros(n + 1, np.uint64)
        np.cumsum(bounds, out=slot[1:])
        out = np.empty(max(int(slot[-1]), 1), np.uint8)
        lens = np.zeros(max(n, 1), np.uint64)
        st = np.zeros(max(n, 1), np.int32)
        thr = threads or len(os.sched_getaffinity(0))
        r = self.lib.tdt_oracle_encode_batch_mt(_ptr(d) if d.size else _ptr(np.zeros(1, np.uint8)), _ptr(off, _u64p),
                                                n, C.byref(cfg), bandwidth, cpu, _ptr(out), _ptr(slot, _u64p),
                                                _ptr(lens, _u64p), _ptr(st, _i32p), int(thr))
        if r:
            raise ValueError("oracle batch encode: status %d" % int(st[st != 0][0]))
        return out, slot, lens[:n]

    def encode_batch(self, data: np.ndarray, offsets: np.ndarray, **kw) -> tuple[bytes, np.ndarray]:
        """Encode every message; returns (concatenated blobs, blob offsets[n+1])."""
        blobs = [self.encode(data[offsets[i]:offsets[i + 1]], **kw) for i in range(len(offsets) - 1)]
        off = np.zeros(len(blobs) + 1, np.uint64)
        off[1:] = np.cumsum([len(b) for b in blobs])
        return b"".join(blobs), off


class Reference:
    """The reference codec itself (compiled header), for golden generation and timing."""

    def __init__(self, path: os.PathLike | None = None):
        p = pathlib.Path(path or REF_SO)
        if not p.exists():
            raise FileNotFoundError(p)
        self.lib = C.CDLL(str(p))
        L = self.lib
        L.tdt_ref_encode.restype = C.c_int
        L.tdt_ref_encode.argtypes = [_u8p, C.c_size_t, C.c_float, C.c_int, C.c_double, C.c_double,
                                     C.c_size_t, _u8p, C.c_size_t, C.POINTER(C.c_size_t)]
        L.tdt_ref_decode.restype = C.c_int
        L.tdt_ref_decode.argtypes = [_u8p, C.c_size_t, _u8p, C.c_size_t, C.POINTER(C.c_size_t)]
        L.tdt_ref_last_error.restype = C.c_char_p
        L.tdt_ref_should_transform.restype = C.c_int
        L.tdt_ref_should_transform.argtypes = [_u8p, C.c_size_t, C.c_int, C.c_double, C.c_double, C.c_size_t]
        L.tdt_ref_encode_ratio.restype = C.c_int
        L.tdt_ref_encode_ratio.argtypes = [_u8p, C.c_size_t, C.c_float, C.c_int, C.c_double,
                                           C.POINTER(C.c_double), C.POINTER(C.c_int)]
        L.tdt_ref_bench.restype = C.c_double
        L.tdt_ref_bench.argtypes = [_u8p, _u64p, C.c_uint32, C.c_float, C.c_int, C.c_int, C.c_int, _u64p]
        self.has_pinned = hasattr(L, "tdt_ref_bench_pinned")
        if self.has_pinned:
            L.tdt_ref_bench_pinned.restype = C.c_double
            L.tdt_ref_bench_pinned.argtypes = [_u8p, _u64p, C.c_uint32, C.c_float, C.c_int, C.c_int, C.c_int, _u64p,
                                               _i32p]

    @staticmethod
    def available(path=None) -> bool:
        return pathlib.Path(path or REF_SO).exists()

    def encode(self, data, sample_fraction=1.0, word_size=4, bandwidth=10.0, cpu=0.5,
               min_tensor_size=1024) -> bytes:
        d = _bytes(data)
        cap = encode_bound(d.size, max(word_size, 1)) + 64
        out = np.empty(cap, np.uint8)
        olen = C.c_size_t(0)
        dp = _ptr(d) if d.size else _ptr(np.zeros(1, np.uint8))
        st = self.lib.tdt_ref_encode(dp, d.size, sample_fraction, word_size, bandwidth, cpu,
                                     min_tensor_size, _ptr(out), cap, C.byref(olen))
        if st:
            raise RuntimeError("ref encode status %d" % st)
        return out[: olen.value].tobytes()

    def decode(self, blob, cap=None) -> tuple[int, bytes, str]:
        b = _bytes(blob)
        cap = cap if cap is not None else (1 << 22)
        out = np.empty(max(cap, 1), np.uint8)
        olen = C.c_size_t(0)
        bp = _ptr(b) if b.size else _ptr(np.zeros(1, np.uint8))
        st = self.lib.tdt_ref_decode(bp, b.size, _ptr(out), cap, C.byref(olen))
        err = self.lib.tdt_ref_last_error().decode() if st == -1 else ""
        return st, out[: olen.value].tobytes() if st == 0 else b"", err

    def encode_ratio(self, data, sample_fraction=1.0, word_size=4, bandwidth=10.0):
        """(blob length, transformation_ratio(), processing_overhead_ms() changed?) after one encode."""
        d = _bytes(data)
        ratio, upd = C.c_double(0.0), C.c_int(0)
        dp = _ptr(d) if d.size else _ptr(np.zeros(1, np.uint8))
        n = self.lib.tdt_ref_encode_ratio(dp, d.size, sample_fraction, word_size, bandwidth, C.byref(ratio),
                                          C.byref(upd))
        return n, ratio.value, bool(upd.value)

    def should_transform(self, n, word_size=4, bandwidth=10.0, cpu=0.5, min_tensor_size=1024) -> bool:
        d = np.zeros(max(n, 1), np.uint8)
        return bool(self.lib.tdt_ref_should_transform(_ptr(d), n, word_size, bandwidth, cpu, min_tensor_size))

    def bench(self, data: np.ndarray, offsets: np.ndarray, sample_fraction=0.3, word_size=4,
              threads=1, reps=1, cpus=None) -> tuple[float, int]:
        """Wall seconds of `threads` workers (one protocol object each) encoding + decoding every
        message `reps` times; cpus: one CPU per worker to pin it to (None: unpinned)."""
        d = _bytes(data)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        enc = C.c_uint64(0)
        if cpus is not None:
            if not self.has_pinned:
                raise RuntimeError("oracle/_ref/libtdt_ref.so predates tdt_ref_bench_pinned: make -C oracle ref")
            cp = np.ascontiguousarray(cpus, dtype=np.int32)
            if cp.size != threads:
                raise ValueError("one CPU per thread")
            s = self.lib.tdt_ref_bench_pinned(_ptr(d), _ptr(off, _u64p), len(off) - 1, sample_fraction, word_size,
                                              threads, reps, C.byref(enc), _ptr(cp, _i32p))
        else:
            s = self.lib.tdt_ref_bench(_ptr(d), _ptr(off, _u64p), len(off) - 1, sample_fraction, word_size,
                                       threads, reps, C.byref(enc))
        if s < 0:
            raise RuntimeError("reference round trip mismatch in bench")
        return s, enc.value
