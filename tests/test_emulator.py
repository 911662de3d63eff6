"""The kernel's round algorithm, emulated on the CPU (tools/emulate_encode.py), against the
golden vectors: pins the index arithmetic (run starts, 255-cap, pair indices, staging window)
without a GPU, and asserts the invariants the kernel's guards rely on."""
import numpy as np

from tools.emulate_encode import encode


def test_emulated_rounds_match_golden(golden):
    n = 0
    for c in golden:
        if c.op != "encode" or c.ws not in (4, 8) or c.input.size > 5000:
            continue
        if c.expected[:4].tobytes() != b"DTDT":
            continue
        mp = list(np.frombuffer(c.expected[20:20 + 4 * c.ws].tobytes(), np.int32))
        for team in (64, 256):
            assert encode(c.input.tobytes(), mp, ws=c.ws, team=team) == c.expected.tobytes(), c.name
            n += 1
    assert n > 100


def test_emulated_long_runs():
    rng = np.random.default_rng(4)
    from oracle.oracle import Oracle
    o = Oracle()
    for L in (254, 255, 256, 510, 511, 800):
        v = rng.integers(0, 256, 4096, dtype=np.uint8)
        v[37:37 + L] = 9
        want = o.encode(v, cfg=o.config(), bandwidth=10.0)
        mp = list(np.frombuffer(want[20:36], np.int32))
        assert encode(v.tobytes(), mp, team=64) == want
