"""The encode kernel's round algorithm, emulated on the CPU (tools/emulate_encode.py), against
the golden vectors: pins the index arithmetic (transposed slot layout, run starts, 255-cap,
pair indices, overwrite order and first-end repair, staging window) without a GPU, and asserts
the invariants the kernel's guards rely on."""
import numpy as np
import pytest

from tools.emulate_encode import encode


def test_emulated_rounds_match_golden(golden):
    n = 0
    for c in golden:
        if c.op != "encode" or c.input.size > 5000:
            continue
        if c.expected[:4].tobytes() != b"DTDT":
            continue
        mp = list(np.frombuffer(c.expected[20:20 + 4 * c.ws].tobytes(), np.int32))
        for team in (64, 256):
            assert encode(c.input.tobytes(), mp, ws=c.ws, team=team) == c.expected.tobytes(), c.name
            n += 1
    assert n > 100


@pytest.mark.parametrize("team", [64, 256])
def test_emulated_long_runs(team):
    rng = np.random.default_rng(4)
    from oracle.oracle import Oracle
    o = Oracle()
    for L in (254, 255, 256, 510, 511, 800, 3000):
        v = rng.integers(0, 256, 8192, dtype=np.uint8)
        v[37:37 + L] = 9
        v[5000:5000 + L] = 0
        want = o.encode(v, cfg=o.config(), bandwidth=10.0)
        mp = list(np.frombuffer(want[20:36], np.int32))
        assert encode(v.tobytes(), mp, team=team) == want, L


def test_emulated_word_sizes_and_tails():
    rng = np.random.default_rng(9)
    from oracle.oracle import Oracle
    o = Oracle()
    for ws in (1, 2, 4, 8, 16):
        for nw in (4, 65, 257, 700):
            x = rng.integers(0, 256, nw * ws, dtype=np.uint8)
            x[rng.random(nw * ws) < 0.5] = 0
            x[: (nw * ws) // 3] = 7
            if x.size < 64 or x.size % 4:
                continue
            want = o.encode(x, cfg=o.config(word_size=ws), bandwidth=10.0)
            if want[:4] != b"DTDT":
                continue
            mp = list(np.frombuffer(want[20:20 + 4 * ws], np.int32))
            assert encode(x.tobytes(), mp, ws=ws, team=64) == want, (ws, nw)
