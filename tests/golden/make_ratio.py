#!/usr/bin/env python3
"""Generate tests/golden/ratio_cases.json: the REFERENCE's own transformation_ratio()
(tdt_compression.hpp:329-331, set by compress_tdt :395-396 from encoded_size() :71-78) and
whether processing_overhead_ms() (:332-334) moved, after encoding each parity-mode golden
input with the reference codec compiled where it lies (oracle/_ref/libtdt_ref.so).

Run in the container that has /root/reference:  python tests/golden/make_ratio.py
Data only (names, blob lengths, ratios as float.hex); no reference source is stored."""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from oracle.oracle import Reference  # noqa: E402
from tests.golden_cases import load_golden  # noqa: E402


def main():
    ref = Reference()
    out = {}
    for c in load_golden():
        if c.op != "encode" or c.sample_fraction < 1.0 or c.min_tensor != 1024 or c.cpu != 0.5:
            continue
        n, ratio, upd = ref.encode_ratio(c.input, sample_fraction=1.0, word_size=c.ws, bandwidth=c.bandwidth)
        assert n == c.expected.size, c.name
        out[c.name] = {"blob_len": n, "ratio": float(ratio).hex(), "overhead_updated": upd,
                       "n": int(c.input.size), "ws": c.ws}
    p = pathlib.Path(__file__).resolve().parent / "ratio_cases.json"
    p.write_text(json.dumps({"generator": "tests/golden/make_ratio.py", "cases": out}, indent=0, sort_keys=True))
    print(len(out), "cases ->", p)


if __name__ == "__main__":
    main()
