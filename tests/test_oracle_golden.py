"""The CPU oracle (oracle/tdt_oracle.c) against the golden vectors produced by the
reference codec (tests/golden/make_golden.py).  Pins the oracle before anything trusts it."""
import numpy as np
import pytest

from oracle.oracle import Oracle, Reference


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def test_golden_has_every_family(golden):
    fam = {c.get("family") for c in golden}
    for f in ("encode", "c2", "c3", "c4", "default", "crafted", "crafted_ub"):
        assert f in fam
    assert any(c.name.startswith("ws8_eq_allones") for c in golden)


def test_encode_parity_mode(oracle, golden):
    n = 0
    for c in golden:
        if c.op != "encode":
            continue
        cfg = oracle.config(word_size=c.ws, sample_fraction=c.sample_fraction, min_tensor_size=c.min_tensor)
        got = oracle.encode(c.input, cfg=cfg, bandwidth=c.bandwidth, cpu=c.cpu)
        assert got == c.expected.tobytes(), c.name
        n += 1
    assert n > 100


def test_encode_with_blob_mapping(oracle, golden):
    for c in golden:
        if c.op != "encode_with_mapping":
            continue
        got = oracle.encode(c.input, cfg=oracle.config(word_size=4, sample_fraction=0.3),
                            bandwidth=c.bandwidth, cpu=c.cpu, mapping=c.mapping)
        assert got == c.expected.tobytes(), c.name


def test_decode_every_blob(oracle, golden):
    for c in golden:
        if c.op in ("encode", "encode_with_mapping"):
            st, out = oracle.decode(c.expected)
            assert st == 0 and out == c.input.tobytes(), c.name
        elif c.op == "decode":
            st, out = oracle.decode(c.input)
            assert st == c.status, (c.name, st)
            if st == 0:
                assert out == c.expected.tobytes(), c.name


def test_policy_table(oracle, golden):
    for c in golden:
        if c.op != "policy":
            continue
        cfg = oracle.config(word_size=c.ws, min_tensor_size=c.min_tensor)
        assert oracle.should_transform(c.n, cfg, c.bandwidth, c.cpu) == c.expect, c.name


def test_mapping_full_sample_gradient_is_1110(oracle, golden):
    # gradient-like data maps [1,1,1,0]
    for c in golden:
        if c.name.startswith("grad_64k"):
            _, _, mp = oracle.analyze(c.input)
            assert list(mp) == [1, 1, 1, 0]


@pytest.mark.skipif(not Reference.available(), reason="oracle/_ref not built (needs /root/reference at build time)")
def test_oracle_vs_reference_random():
    o, r = Oracle(), Reference()
    rng = np.random.default_rng(7)
    for k in range(60):
        n = int(rng.integers(256, 3000)) * 4
        if k % 2:
            d = rng.integers(0, 256, n, dtype=np.uint8)
        else:
            x = rng.normal(0, 0.01, n // 4).astype(np.float32)
            x[rng.random(n // 4) < 0.7] = 0
            d = x.view(np.uint8)
        for ws in (4, 8):
            assert o.encode(d, cfg=o.config(word_size=ws)) == r.encode(d, word_size=ws)
