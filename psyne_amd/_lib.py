"""ctypes binding of include/psyne_tdt.h (libpsyne_tdt.so, built in-tree).

There is no CPU fallback: if the HIP library is missing or no GPU is present, the codec
raises.  Pointers passed to the batch entry points are device pointers.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

LIB_PATH = pathlib.Path(__file__).resolve().parent / "libpsyne_tdt.so"

TDT_OK, TDT_E_SHORT, TDT_E_MAGIC, TDT_E_TRUNCATED, TDT_E_BAD_MAPPING = 0, 1, 2, 3, 4
TDT_E_CAPACITY, TDT_E_UNSUPPORTED, TDT_E_BAD_HEADER, TDT_E_CONFIG = 5, 6, 7, 8
TDT_E_HIP, TDT_E_ARG, TDT_E_CAPTURE = 10, 11, 12
TDT_OPT_LARGE_MIN, TDT_OPT_TILE_CAP, TDT_OPT_NO_SIDE_STREAM = 1, 2, 3
TDT_OPT_SMALL_ON_CALLER_STREAM, TDT_OPT_NO_TWO_PHASE, TDT_OPT_COPY_THREADS = 4, 5, 6


class TdtConfigC(C.Structure):
    _fields_ = [
        ("sample_fraction", C.c_float),
        ("word_size", C.c_int32),
        ("bandwidth_threshold_mbps", C.c_double),
        ("cpu_usage_threshold", C.c_double),
        ("min_tensor_size", C.c_uint64),
    ]


_vp = C.c_void_p
# name -> (restype, argtypes); every function declared in include/psyne_tdt.h
SIGNATURES = {
    "tdt_default_config": (None, [C.POINTER(TdtConfigC)]),
    "tdt_ctx_create": (C.c_int, [C.c_int, C.POINTER(TdtConfigC), C.POINTER(_vp)]),
    "tdt_ctx_destroy": (None, [_vp]),
    "tdt_ctx_set_metrics": (None, [_vp, C.c_double, C.c_double, C.c_double]),
    "tdt_ctx_get_metrics": (None, [_vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "tdt_ctx_set_size_hint": (None, [_vp, C.c_uint64]),
    "tdt_should_transform": (C.c_int, [_vp, C.c_uint64]),
    "tdt_encode_bound": (C.c_uint64, [C.c_uint64, C.c_int32]),
    "tdt_encode_batch": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, C.c_uint64, _vp, _vp, _vp]),
    "tdt_encode_with_mapping_batch": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, _vp, C.c_uint64, _vp, _vp, _vp]),
    "tdt_decode_batch": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, C.c_uint64, _vp, _vp, _vp]),
    "tdt_decoded_sizes_batch": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, _vp, _vp]),
    "tdt_encode_batch_into": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, _vp, _vp, _vp, _vp]),
    "tdt_decode_batch_into": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32, _vp, _vp, _vp, _vp, _vp]),
    "tdt_encode_slots": (C.c_int, [_vp, _vp, C.c_uint32, _vp, _vp]),
    "tdt_decode_slots": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32, _vp, _vp, _vp]),
    "tdt_analyze_batch": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, _vp, _vp, _vp, _vp]),
    "tdt_encode_host": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, C.c_uint64, _vp, _vp]),
    "tdt_decode_host": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, C.c_uint64, _vp, _vp]),
    "tdt_encode_host_v": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, C.c_uint64, _vp, _vp]),
    "tdt_host_alloc": (C.c_int, [C.c_uint64, C.POINTER(C.c_void_p)]),
    "tdt_host_free": (None, [_vp]),
    "tdt_host_copy": (C.c_int, [_vp, _vp, _vp, C.c_uint64]),
    "tdt_copy_device": (C.c_int, [_vp, _vp, C.c_uint64, _vp]),
    "tdt_analyze_host": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, _vp, _vp]),
    "tdt_ctx_error_flags": (C.c_int, [_vp, _vp, C.POINTER(C.c_uint32)]),
    "tdt_ctx_set_option": (C.c_int, [_vp, C.c_int, C.c_uint64]),
    "tdt_last_error": (C.c_char_p, []),
    "tdt_status_string": (C.c_char_p, [C.c_int]),
}

_lib = None


def load(path: pathlib.Path | None = None) -> C.CDLL:
    """Load libpsyne_tdt.so; raises (never falls back) if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # PSYNE_TDT_LIB: an alternative build of the same HIP library (diagnostic experiments)
    p = pathlib.Path(path or os.environ.get("PSYNE_TDT_LIB") or LIB_PATH)
    if not p.exists():
        raise RuntimeError(f"{p} not built: run `python -m psyne_amd.build` (hipcc --offload-arch=gfx950)")
    lib = C.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = lib
    return lib


class TdtError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"TDT error {code}: {msg}")


def check(code: int):
    if code != TDT_OK:
        lib = load()
        raise TdtError(code, lib.tdt_last_error().decode() or lib.tdt_status_string(code).decode())
