#!/usr/bin/env python3
"""Diagnostic: per-phase wave-cycle breakdown of the encode/decode kernels.

Builds psyne_amd/libpsyne_tdt_prof.so with -DPSY_PROF=1 (when run with --build, on the build
host), then (on a GPU box) runs one C3-shaped batch through it and prints, per phase, the
s_memtime cycles summed over waves (lane 0 of every wave), as a share of each kernel's total.
Not part of the product path; the product library is compiled without PSY_PROF.
"""
import argparse
import ctypes as C
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
PROF_LIB = ROOT / "psyne_amd" / "libpsyne_tdt_prof.so"

ENC = ["setup/ticket", "histogram", "entropy+mapping+desc", "A1 run starts", "A2 chunk starts",
       "look-back+header", "B emit"]
DEC = {8: "header+look-back", 9: "pair rounds", 10: "fill+scatter", 11: "store"}


def build():
    from psyne_amd import build as b
    cmd = [b.HIPCC, f"--offload-arch={b.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-DPSY_PROF=1",
           "-DPSY_FAST_BUILD",
           "-I", str(ROOT / "include"), *map(str, b.SOURCES), "-o", str(PROF_LIB)]
    subprocess.check_call(cmd)


def run(msgs, msg_bytes, seed, uniform=False):
    import torch
    from psyne_amd import _lib
    from psyne_amd.tdt import TdtCodec, TDTConfig
    import bench
    lib = _lib.load(PROF_LIB)
    lib.tdt_prof_read.argtypes = [C.c_void_p]
    lib.tdt_prof_read.restype = C.c_int
    codec = TdtCodec(TDTConfig(sample_fraction=1.0), lib=lib)
    codec.set_metrics(10.0, 1.0, 0.5)
    codec.set_size_hint(msg_bytes)
    dev = torch.device("cuda:0")
    data = (bench.gen_uniform(torch, msgs * msg_bytes, seed, dev) if uniform
            else bench.gen_gradient(torch, msgs, msg_bytes, seed, dev))
    off = torch.arange(msgs + 1, dtype=torch.int64, device=dev) * msg_bytes
    buf = (C.c_uint64 * 32)()
    for it in range(3):
        enc, slots, lens, st = codec.encode_into(data, off)
        torch.cuda.synchronize()
        lib.tdt_prof_read(buf)
        e = list(buf)
        back, bslots, blens, st2 = codec.decode_into(enc, slots, in_lengths=lens)
        torch.cuda.synchronize()
        lib.tdt_prof_read(buf)
        d = list(buf)
    te = sum(e[:7])
    print(f"encode: {te:.4g} wave-cycles over {msgs} msgs")
    for i, name in enumerate(ENC):
        print(f"  {name:24s} {e[i] / te:6.1%}  {e[i] / msgs:12.0f} cyc/msg (sum over waves)")
    print(f"  look-back: {e[18]} calls, {e[19]} waited, {e[16]} spins, {e[17]} windows summed")
    td = sum(d[8:12])
    print(f"decode: {td:.4g} wave-cycles")
    for i, name in DEC.items():
        print(f"  {name:24s} {d[i] / td:6.1%}  {d[i] / msgs:12.0f} cyc/msg")
    print(f"  look-back: {d[18]} calls, {d[19]} waited, {d[16]} spins, {d[17]} windows summed")
    assert torch.equal(back, data), "round trip mismatch"


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--msgs", type=int, default=32768)
    ap.add_argument("--msg-bytes", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=0x5EED0002)
    ap.add_argument("--uniform", action="store_true")
    a = ap.parse_args()
    if a.build:
        build()
    else:
        run(a.msgs, a.msg_bytes, a.seed, a.uniform)
