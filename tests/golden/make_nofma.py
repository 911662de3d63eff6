#!/usr/bin/env python3
"""Which inputs does the reference's mapping decision flip between an FMA build and a
non-FMA build?  (DESIGN.md §2 "Which build parity targets".)

Both are the reference header compiled where it lies (oracle/Makefile): oracle/_ref/
libtdt_ref.so with -march=x86-64-v3 (GCC contracts `entropy -= prob * log2(prob)` into one
vfnmadd, as SURVEY's reference build command -march=native does on any FMA host) and
oracle/_ref/libtdt_ref_nofma.so with -march=x86-64 (rounded multiply, then rounded subtract).
Near-ties are manufactured by giving byte positions the same multiset of counts in a different
bin order (a relabelling of byte values): the entropies then agree up to summation rounding,
so the decision is made by the last bits — exactly where the two builds differ.

Writes tests/golden/nofma_cases.npz (inputs and both builds' blobs of the divergent cases, plus
near-tie cases where they agree) and prints the divergence rate.  Data only."""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from oracle.oracle import REF_SO, Reference  # noqa: E402


def near_tie(rng, n, ws):
    """n-byte message whose ws byte positions are value relabellings of one random column."""
    w = n // ws
    col = rng.integers(0, int(rng.choice([3, 7, 16, 61, 256])), w, dtype=np.uint16)
    out = np.empty((w, ws), np.uint8)
    for b in range(ws):
        perm = rng.permutation(256).astype(np.uint8)
        out[:, b] = perm[col % 256]
        if b and rng.random() < 0.5:
            out[:, b] = np.roll(out[:, b], int(rng.integers(1, w)))
    return out.reshape(-1)


def main():
    fma = Reference(REF_SO)
    nofma = Reference(REF_SO.parent / "libtdt_ref_nofma.so")
    rng = np.random.default_rng(0x5EED00FA)
    div, same = [], []
    tried = 0
    for k in range(4000):
        ws = int(rng.choice([2, 4]))
        n = int(rng.choice([1024, 4096, 16384]))
        x = near_tie(rng, n, ws)
        a = fma.encode(x, sample_fraction=1.0, word_size=ws)
        b = nofma.encode(x, sample_fraction=1.0, word_size=ws)
        tried += 1
        if a != b:
            div.append((ws, x, a, b))
        elif len(same) < 24 and a[:4] == b"DTDT":
            same.append((ws, x, a, b))
    print("near-tie inputs: %d, mapping differs between FMA and non-FMA builds: %d (%.2f%%)"
          % (tried, len(div), 100.0 * len(div) / tried))
    keep = div[:24] + same
    ins = np.concatenate([c[1] for c in keep])
    io = np.concatenate([[0], np.cumsum([c[1].size for c in keep])]).astype(np.int64)
    fa = np.concatenate([np.frombuffer(c[2], np.uint8) for c in keep])
    fo = np.concatenate([[0], np.cumsum([len(c[2]) for c in keep])]).astype(np.int64)
    nb = np.concatenate([np.frombuffer(c[3], np.uint8) for c in keep])
    no = np.concatenate([[0], np.cumsum([len(c[3]) for c in keep])]).astype(np.int64)
    ws = np.array([c[0] for c in keep], np.int32)
    divergent = np.array([i < min(len(div), 24) for i in range(len(keep))])
    np.savez_compressed(pathlib.Path(__file__).resolve().parent / "nofma_cases.npz", inputs=ins, in_off=io,
                        fma_blobs=fa, fma_off=fo, nofma_blobs=nb, nofma_off=no, word_size=ws, divergent=divergent,
                        tried=np.array([tried]), n_divergent=np.array([len(div)]))


if __name__ == "__main__":
    main()
