#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE codec.

Run in the container that has /root/reference (after `make -C oracle`):

    python tests/golden/make_golden.py

It drives oracle/_ref/libtdt_ref.so — the reference header
include/psyne/protocol/tdt_compression.hpp compiled where it lies by oracle/Makefile —
and records inputs and the reference's outputs.  The reference has no golden vectors or
known-answer tests of its own, so these are the parity anchor.

Outputs (data only, no reference source):
    golden.npz   inputs / outputs byte blobs (uint8), compressed
    cases.json   one record per case: op, config, slices into the blobs, expected status

Case families (SURVEY.md §8(c) list):
  * encode, parity mode (sample_fraction=1.0, bandwidth 10 Mbps): zeros, runs > 255,
    UNCP routing (1020 B, 1026 B, ws=8 1028 B), ws=8 equal-entropy (incl. all-ones mapping
    with an empty stream 0), 64 x 1 KiB uniform, 8 x 64 KiB gradient, 2 x 1 MiB gradient,
    odd sizes, ws in {1,2,8,16};
  * encode, default mode (sample_fraction=0.3): the blob's own mapping is the parity key;
  * policy: should_transform table (tdt_compression_benchmark.cpp:342-348) + size edges;
  * decode: every encode blob, crafted edge blobs, random valid blobs,
    the reference's two decode errors; blobs on which the reference has undefined
    behaviour are recorded with the status our spec assigns ("ref": "ub").
"""
from __future__ import annotations

import json
import pathlib
import struct
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle.oracle import Reference  # noqa: E402

OUTDIR = pathlib.Path(__file__).resolve().parent
TDT, UNCP = 0x54445444, 0x554E4350

E_SHORT, E_MAGIC, E_TRUNCATED, E_BAD_MAPPING, E_BAD_HEADER = 1, 2, 3, 4, 7


class Store:
    def __init__(self):
        self.inp = bytearray()
        self.out = bytearray()
        self.cases = []

    def add(self, rec, inp: bytes, out: bytes | None):
        rec["in"] = [len(self.inp), len(self.inp) + len(inp)]
        self.inp += inp
        if out is not None:
            rec["out"] = [len(self.out), len(self.out) + len(out)]
            self.out += out
        self.cases.append(rec)


def grad(rng, nfloat):
    # tdt_compression_benchmark.cpp:52-66 distribution: 70% exact 0.0f, else N(0, 0.01)
    x = rng.normal(0.0, 0.01, nfloat).astype(np.float32)
    x[rng.random(nfloat) < 0.7] = 0.0
    return x.view(np.uint8).tobytes()


def blob(orig, ws, mapping, streams, ns=None, msize=None, magic=TDT):
    ns = len(streams) if ns is None else ns
    msize = len(mapping) if msize is None else msize
    b = struct.pack("<IIIII", magic, orig & 0xFFFFFFFF, ns, ws & 0xFFFFFFFF, msize)
    b += b"".join(struct.pack("<i", m) for m in mapping)
    for s in streams:
        b += struct.pack("<I", len(s)) + bytes(s)
    return b


def pairs(*pv):
    return bytes(x for p in pv for x in p)


def main():
    ref = Reference()
    rng = np.random.default_rng(0x5EED0000)
    st = Store()

    def enc(name, data: bytes, ws=4, sf=1.0, bw=10.0, cpu=0.5, mt=1024, family="encode"):
        out = ref.encode(data, sample_fraction=sf, word_size=ws, bandwidth=bw, cpu=cpu, min_tensor_size=mt)
        rec = dict(name=name, op="encode", family=family, ws=ws, sample_fraction=sf, bandwidth=bw,
                   cpu=cpu, min_tensor=mt, status=0, ref="ran")
        st.add(rec, data, out)
        # every encode blob is also a decode case
        dst, dout, derr = ref.decode(out, cap=len(data) + 16)
        assert dst == 0 and dout == data, name
        return out

    # ---- parity-mode encodes -------------------------------------------------------
    enc("zeros_1024", bytes(1024))
    w = np.zeros((512, 4), np.uint8)
    w[:, 0] = rng.integers(0, 256, 512)
    enc("long_runs_2048", w.tobytes())           # mapping [1,0,0,0], stream 0: 1536 zeros
    enc("all_0xAB_65536", bytes([0xAB]) * 65536)
    enc("uncp_1020", rng.integers(0, 256, 1020, dtype=np.uint8).tobytes())
    enc("uncp_1026", rng.integers(0, 256, 1026, dtype=np.uint8).tobytes())
    enc("uncp_ws8_1028", rng.integers(0, 256, 1028, dtype=np.uint8).tobytes(), ws=8)
    enc("uncp_bw100_4096", rng.integers(0, 256, 4096, dtype=np.uint8).tobytes(), bw=100.0)
    enc("uncp_cpu_4096", rng.integers(0, 256, 4096, dtype=np.uint8).tobytes(), cpu=0.9)
    enc("uncp_empty", b"")
    enc("small_mt64_64", rng.integers(0, 256, 64, dtype=np.uint8).tobytes(), mt=0)
    enc("small_mt64_60", rng.integers(0, 256, 60, dtype=np.uint8).tobytes(), mt=0)
    for i in range(64):
        enc("uniform_1k_%02d" % i, rng.integers(0, 256, 1024, dtype=np.uint8).tobytes(), family="c2")
    for i in range(8):
        enc("grad_64k_%d" % i, grad(rng, 16384), family="c3")
    for i in range(2):
        enc("grad_1m_%d" % i, grad(rng, 262144), family="c4")
    for i, n in enumerate([1028, 1032, 1100, 2044, 3000, 4100, 12288, 40000, 65540, 99996]):
        kind = i % 3
        if kind == 0:
            d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            d = grad(rng, n // 4)
        else:  # runs of random lengths (incl. > 255)
            vals = []
            while len(vals) < n:
                vals += [int(rng.integers(0, 4))] * int(rng.integers(1, 700))
            d = bytes(vals[:n])
        enc("odd_%d" % n, d)
    # ws sweep
    for ws in (1, 2, 8, 16):
        for i in range(3):
            n = 2048 * (i + 1)
            d = grad(rng, n // 4) if i % 2 else rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            enc("ws%d_%d" % (ws, n), d, ws=ws)
    # ws=8 equal-entropy constructions: every byte position draws the same multiset of
    # counts over a different random permutation of the values.
    found_all_ones = 0
    for trial in range(400):
        wc = 256
        counts = rng.multinomial(wc, np.ones(24) / 24)
        base = np.repeat(np.arange(24), counts)
        cols = []
        for b in range(8):
            perm = rng.permutation(256)[:24]
            col = perm[base]
            rng.shuffle(col)
            cols.append(col)
        d = np.stack(cols, 1).astype(np.uint8).tobytes()
        out = ref.encode(d, word_size=8)
        mp = struct.unpack_from("<8i", out, 20)
        if all(m == 1 for m in mp) and found_all_ones < 4:
            found_all_ones += 1
            enc("ws8_eq_allones_%d" % trial, d, ws=8)
        elif trial < 6:
            enc("ws8_eq_%d" % trial, d, ws=8)
    assert found_all_ones > 0, "no ws=8 all-ones case found"
    # ws=4 equal entropies (must give mapping all-zero per SURVEY §A.3)
    for trial in range(4):
        counts = rng.multinomial(256, np.ones(16) / 16)
        base = np.repeat(np.arange(16), counts)
        cols = []
        for b in range(4):
            col = rng.permutation(256)[:16][base]
            rng.shuffle(col)
            cols.append(col)
        enc("ws4_eq_%d" % trial, np.stack(cols, 1).astype(np.uint8).tobytes())

    # ---- default-mode encodes (random sampling): parity via the blob's mapping --------
    for i in range(16):
        n = [1024, 4096, 65536, 1 << 18][i % 4]
        d = grad(rng, n // 4) if i % 2 else rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        out = ref.encode(d, sample_fraction=0.3)
        rec = dict(name="default_mode_%d" % i, op="encode_with_mapping", family="default", ws=4,
                   sample_fraction=0.3, bandwidth=10.0, cpu=0.5, min_tensor=1024, status=0, ref="ran",
                   mapping=list(struct.unpack_from("<4i", out, 20)))
        st.add(rec, d, out)

    # ---- policy table ----------------------------------------------------------------
    pol = []
    for name, bw, cpu in [("High-speed network", 1000.0, 0.3), ("Medium network", 100.0, 0.4),
                          ("Slow network", 25.0, 0.4), ("Very slow network", 10.0, 0.5),
                          ("Slow + high CPU", 25.0, 0.9)]:
        pol.append(dict(name=name, n=8 << 20, ws=4, bandwidth=bw, cpu=cpu, min_tensor=1024,
                        expect=ref.should_transform(8 << 20, 4, bw, cpu, 1024)))
    for n in [0, 4, 60, 64, 1020, 1022, 1024, 1026, 1028, 4096]:
        for mt in (0, 1024):
            for ws in (4, 8):
                pol.append(dict(name="size_%d_mt%d_ws%d" % (n, mt, ws), n=n, ws=ws, bandwidth=10.0,
                                cpu=0.5, min_tensor=mt, expect=ref.should_transform(n, ws, 10.0, 0.5, mt)))
    for p in pol:
        st.cases.append(dict(name="policy_" + p["name"], op="policy", **{k: v for k, v in p.items() if k != "name"}))

    # ---- crafted decode blobs (valid under the reference) -----------------------------
    def dec(name, b: bytes, ub_status=None):
        if ub_status is not None:
            st.add(dict(name=name, op="decode", family="crafted_ub", status=ub_status, ref="ub"), b, None)
            return
        s, out, err = ref.decode(b, cap=1 << 21)
        if s == 0:
            st.add(dict(name=name, op="decode", family="crafted", status=0, ref="ran"), b, out)
        else:
            code = {"TDT: Invalid encoded data size": E_SHORT, "Invalid TDT magic number": E_MAGIC}[err]
            st.add(dict(name=name, op="decode", family="crafted", status=code, error=err, ref="ran"), b, None)

    dec("short_stream", blob(16, 4, [0, 0, 0, 1], [pairs((3, 0xAA)), pairs((4, 0xBB))]))
    dec("extra_stream_bytes", blob(16, 4, [0, 0, 0, 1], [pairs((12, 1), (9, 2)), pairs((255, 3))]))
    dec("odd_trailing_byte", blob(16, 4, [0, 1, 0, 1], [pairs((5, 7), (3, 9)) + b"\x05", pairs((8, 4)) + b"\x11"]))
    dec("count_zero_pairs", blob(16, 4, [1, 1, 0, 1], [pairs((0, 5), (2, 6), (0, 7), (2, 8)),
                                                        pairs((0, 1), (6, 2), (0, 3), (6, 4))]))
    dec("orig_tail_bytes", blob(18, 4, [0, 0, 1, 1], [pairs((8, 0x10)), pairs((8, 0x20), (4, 0x30))]))
    dec("three_streams", blob(32, 4, [2, 0, 1, 0], [pairs((16, 1)), pairs((3, 2), (5, 3)), pairs((8, 4))]))
    dec("unused_stream", blob(16, 4, [0, 0, 1, 1], [pairs((8, 1)), pairs((8, 2)), b"\xff\xee\xdd"]))
    dec("mapping_size_gt_ws", blob(16, 4, [1, 0, 1, 0, 7, 9], [pairs((8, 3)), pairs((8, 4))]))
    dec("negative_ws", blob(10, -1, [], [pairs((10, 1))]))
    dec("ws_gt_orig", blob(8, 16, [], [pairs((8, 1))]))
    dec("orig_zero", blob(0, 4, [0, 0, 0, 0], [pairs((4, 1))]))
    dec("no_streams_no_words", blob(3, 4, [0, 0, 0, 0], []))
    dec("trailing_garbage", blob(8, 4, [0, 0, 0, 0], [pairs((8, 0x42))]) + b"garbage!")
    dec("ws1", blob(20, 1, [0], [pairs((7, 1), (13, 2))]))
    dec("ws2", blob(20, 2, [1, 0], [pairs((10, 1)), pairs((4, 2), (6, 3))]))
    dec("ws8", blob(40, 8, [0, 1, 0, 1, 0, 1, 0, 1], [pairs((20, 1)), pairs((19, 2), (1, 3))]))
    dec("runs_overflow", blob(64, 4, [0, 0, 0, 0], [pairs(*[(255, 9)] * 4)]))
    dec("uncp_empty", struct.pack("<I", UNCP))
    dec("uncp_payload", struct.pack("<I", UNCP) + bytes(range(37)))
    for n in range(4):
        dec("err_short_%d" % n, struct.pack("<I", TDT)[:n])
    dec("err_magic", b"ABCD" + bytes(40))
    dec("err_magic_4", b"\x00\x00\x00\x00")
    # random valid blobs
    for i in range(48):
        ws = int(rng.choice([1, 2, 4, 8]))
        ns = int(rng.integers(1, 5))
        wc = int(rng.integers(0, 80))
        orig = wc * ws + int(rng.integers(0, ws))
        mapping = [int(rng.integers(0, ns)) for _ in range(ws)]
        streams = []
        for s in range(ns):
            npairs = int(rng.integers(0, 40))
            body = bytes(int(x) for x in rng.integers(0, 256, 2 * npairs))
            body = bytes((b % 9) if j % 2 == 0 else b for j, b in enumerate(body))
            if rng.random() < 0.3:
                body += bytes([int(rng.integers(0, 256))])
            streams.append(body)
        dec("rand_valid_%02d" % i, blob(orig, ws, mapping, streams))
    # undefined behaviour in the reference → our spec's status (not run through the reference)
    good = blob(16, 4, [0, 0, 0, 1], [pairs((12, 1)), pairs((4, 2))])
    for cut in (5, 12, 19, 24, 35, 40, 43, len(good) - 1):
        dec("ub_truncated_%d" % cut, good[:cut], ub_status=E_TRUNCATED if cut >= 8 else E_TRUNCATED)
    dec("ub_mapping_short", blob(16, 4, [0, 0], [pairs((16, 1))]), ub_status=E_BAD_MAPPING)
    dec("ub_mapping_range", blob(16, 4, [0, 0, 2, 0], [pairs((12, 1)), pairs((4, 2))]), ub_status=E_BAD_MAPPING)
    dec("ub_mapping_negative", blob(16, 4, [0, -1, 0, 0], [pairs((16, 1))]), ub_status=E_BAD_MAPPING)
    dec("ub_ws_zero", blob(16, 0, [], [pairs((16, 1))]), ub_status=E_BAD_HEADER)
    dec("ub_stream_len_past_end", blob(16, 4, [0, 0, 0, 0], [pairs((16, 1))])[:-2],
        ub_status=E_TRUNCATED)

    np.savez_compressed(OUTDIR / "golden.npz", inputs=np.frombuffer(bytes(st.inp), np.uint8),
                        outputs=np.frombuffer(bytes(st.out), np.uint8))
    (OUTDIR / "cases.json").write_text(json.dumps(dict(
        generator="tests/golden/make_golden.py",
        reference="include/psyne/protocol/tdt_compression.hpp via oracle/_ref/libtdt_ref.so",
        cases=st.cases), indent=0))
    print("cases", len(st.cases), "inputs", len(st.inp), "outputs", len(st.out))


if __name__ == "__main__":
    main()
