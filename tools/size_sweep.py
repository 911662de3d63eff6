"""Encode/decode GiB/s of the slotted API per message size (gradient-like content), to see
where a mixed-size batch (BASELINE C4) spends its time.  Usage: python tools/size_sweep.py
[--hint N] [--total-gib G] [--sizes 64,1024,...]"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from psyne_amd import TDTConfig, TdtCodec  # noqa: E402
from psyne_amd._lib import check  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64,512,1024,4096,16384,65536,262144,1048576,16777216")
    ap.add_argument("--total-gib", type=float, default=4.0)
    ap.add_argument("--hint", type=int, default=-1, help="size hint (-1: the message size)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--uniform", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = TdtCodec(TDTConfig(sample_fraction=1.0))
    codec.set_metrics(10.0, 1.0, 0.5)
    lib, h = codec._lib, codec._h
    P = lambda t: C.c_void_p(t.data_ptr())
    for mb in [int(s) for s in a.sizes.split(",")]:
        n = max(1, min(int(a.total_gib * 2**30) // mb, 1 << 23))
        data = (bench.gen_uniform(torch, n * mb, 1, dev) if a.uniform else bench.gen_gradient(torch, n, mb, 2, dev))
        off = torch.arange(n + 1, dtype=torch.int64, device=dev) * mb
        lib.tdt_ctx_set_size_hint(h, C.c_uint64(mb if a.hint < 0 else a.hint))
        eslot = torch.empty(n + 1, dtype=torch.int64, device=dev)
        check(lib.tdt_encode_slots(h, P(off), n, P(eslot), None))
        torch.cuda.synchronize()
        enc = torch.empty(int(eslot[-1].item()), dtype=torch.uint8, device=dev)
        elen = torch.empty(n, dtype=torch.int64, device=dev)
        est = torch.empty(n, dtype=torch.int32, device=dev)
        dec = torch.empty_like(data)
        dslot = torch.empty(n + 1, dtype=torch.int64, device=dev)
        dlen = torch.empty(n, dtype=torch.int64, device=dev)
        dst = torch.empty(n, dtype=torch.int32, device=dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        te = td = 0.0
        for r in range(a.reps + 1):
            ev[0].record()
            check(lib.tdt_encode_batch_into(h, P(data), P(off), n, P(enc), P(eslot), P(elen), P(est), None))
            ev[1].record()
            if r == 0:
                check(lib.tdt_decode_slots(h, P(enc), P(eslot), P(elen), n, P(dslot), P(dst), None))
            check(lib.tdt_decode_batch_into(h, P(enc), P(eslot), P(elen), n, P(dec), P(dslot), P(dlen), P(dst), None))
            ev[2].record()
            torch.cuda.synchronize()
            if r:
                te += ev[0].elapsed_time(ev[1]) / a.reps
                td += ev[1].elapsed_time(ev[2]) / a.reps
        ok = bool(torch.equal(dec, data)) and int(est.abs().sum()) == 0
        E = int(elen.sum().item())
        print(json.dumps({"msg_bytes": mb, "msgs": n, "enc_ms": round(te, 3), "dec_ms": round(td, 3),
                          "enc_GiBps": round(n * mb / te / 1e-3 / 2**30, 1), "dec_GiBps": round(n * mb / td / 1e-3 / 2**30, 1),
                          "ratio": round(n * mb / E, 4), "ok": ok}), flush=True)
        del data, enc, dec
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
