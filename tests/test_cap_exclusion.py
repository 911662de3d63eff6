"""The encode kernel's cap-exclusion test (psyne_amd/csrc/tdt_encode.h, pass A1).

The kernel skips pass A2 (the 255-cap of simple_rle_compress, reference
include/psyne/protocol/tdt_compression.hpp:568) when every aligned block of B groups (B = 8 for
Ls <= 8 slots per group and stream, B = 4 above) holds a run start in that stream or reaches
past the message end.  This restates that rule on the CPU and checks the implication it relies
on — "clean" => no run of >= 256 bytes in any stream — on adversarial inputs: runs of every
length around the cap, for every ws = 4 stream split.  (The GPU parity tests cover the capped
path itself through the golden cases with runs > 255.)"""
import numpy as np
import pytest


def _streams(words, mapping):
    """Byte planes of a (n_words, ws) uint8 array: stream c = positions mapped to c, word-major
    (separate_byte_streams, reference :527-549)."""
    out = []
    for c in (0, 1):
        cols = [b for b in range(words.shape[1]) if mapping[b] == c]
        out.append(words[:, cols].reshape(-1) if cols else np.zeros(0, np.uint8))
    return out


def _run_starts(s):
    st = np.ones(s.size, bool)
    st[1:] = s[1:] != s[:-1]
    return st


def _max_run(s):
    if s.size == 0:
        return 0
    idx = np.flatnonzero(_run_starts(s))
    return int(np.max(np.diff(np.append(idx, s.size))))


def _clean(words, mapping, ws=4):
    """The kernel's rule: groups of 16 bytes, Ls = (16 / ws) * k slots of stream c per group."""
    n = words.size
    ngroups = (n + 15) // 16
    wpg = 16 // ws
    for c, s in enumerate(_streams(words, mapping)):
        k = sum(1 for b in range(ws) if mapping[b] == c)
        if k == 0:
            continue
        ls = wpg * k
        blk = 8 if ls < 16 else 4
        st = _run_starts(s)
        has = np.zeros(ngroups, bool)
        has[np.flatnonzero(st) // ls] = True
        nblk = (ngroups + blk - 1) // blk
        padded = np.ones(nblk * blk, bool)  # groups past the end count as starts
        padded[:ngroups] = has
        if not padded.reshape(nblk, blk).any(axis=1).all():
            return False
    return True


def _message(rng, n_words, mean_run, word_level):
    """Words whose byte positions change value after geometric runs of mean `mean_run` words;
    word_level: all positions change together and repeat one byte (zero-word stretches: long
    runs in every stream whatever the split)."""
    ws = 4
    cols = []
    for _ in range(1 if word_level else ws):
        vals = []
        while len(vals) < n_words:
            r = int(rng.geometric(1.0 / mean_run))
            vals.extend([int(rng.integers(0, 256))] * r)
        cols.append(vals[:n_words])
    if word_level:
        cols = cols * ws
    return np.array(cols, np.uint8).T.copy()


MAPPINGS = [(0, 1, 1, 1), (0, 0, 1, 1), (0, 0, 0, 1), (0, 0, 0, 0), (1, 0, 1, 0)]


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_clean_implies_no_capped_run(mapping):
    rng = np.random.default_rng(0xCA9 + sum(m << i for i, m in enumerate(mapping)))
    seen_clean = seen_dirty = 0
    for trial in range(160):
        mean_run = [2, 8, 20, 40, 64, 100, 130][trial % 7]
        n_words = int(rng.integers(64, 6000))
        w = _message(rng, n_words, mean_run, word_level=trial % 2 == 1)
        clean = _clean(w, mapping)
        if clean:
            seen_clean += 1
            for s in _streams(w, mapping):
                assert _max_run(s) <= 255, (mapping, mean_run, n_words)
        else:
            seen_dirty += 1
    assert seen_clean > 10 and seen_dirty > 10


def test_gradient_data_is_clean():
    """The bench's gradient-like tensors (70 % zeros, N(0, 0.01)) nearly always pass the rule,
    which is what makes skipping A2 pay."""
    rng = np.random.default_rng(7)
    clean = 0
    for _ in range(20):
        x = rng.normal(0, 0.01, 16384).astype(np.float32)
        x[rng.random(x.size) < 0.7] = 0
        w = x.view(np.uint8).reshape(-1, 4)
        clean += _clean(w, (0, 0, 1, 1)) and _clean(w, (1, 1, 0, 0))
    assert clean >= 18
