"""Identity metrics: transformation_ratio() and processing_overhead_ms()
against the reference's own values (tests/golden/ratio_cases.json, made by
tests/golden/make_ratio.py from the reference codec compiled where it lies)."""
import json
import pathlib

import numpy as np
import pytest

from psyne_amd.tdt import transformation_ratio_of

FIX = pathlib.Path(__file__).resolve().parent / "golden" / "ratio_cases.json"


@pytest.fixture(scope="module")
def ratios():
    return json.loads(FIX.read_text())["cases"]


def test_ratio_formula_matches_reference(golden, ratios):
    """n / encoded_size() from the blob bytes == the reference's transformation_ratio(), bit for
    bit, on every parity-mode golden encode; UNCP blobs leave the ratio unchanged."""
    by_name = {c.name: c for c in golden if c.op == "encode"}
    assert len(ratios) > 100
    for name, r in ratios.items():
        c = by_name[name]
        got = transformation_ratio_of(c.expected.tobytes(), r["n"])
        if r["overhead_updated"]:
            assert got is not None and got.hex() == r["ratio"], name
        else:  # passthrough: the reference keeps its initial 1.0
            assert got is None and float.fromhex(r["ratio"]) == 1.0, name


@pytest.mark.gpu
def test_protocol_metrics_on_gpu(golden, ratios):
    """The GPU-backed TDTCompressionProtocol reports the reference's transformation_ratio()
    exactly and moves processing_overhead_ms() exactly when the reference does (:332-334:
    mean of the last encode and decode times; only compressing encodes / TDT decodes update)."""
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    from psyne_amd import TDTCompressionProtocol, TDTConfig
    by_name = {c.name: c for c in golden if c.op == "encode"}
    protos = {}
    checked = 0
    for name, r in sorted(ratios.items()):
        c = by_name[name]
        if c.input.size > (1 << 16):
            continue
        ws = r["ws"]
        if ws not in protos:
            protos[ws] = TDTCompressionProtocol(TDTConfig(sample_fraction=1.0, word_size=ws))
        p = protos[ws]
        p.update_network_metrics(c.bandwidth, 1.0)
        # a sentinel encode time: whether encode() set a new one is what the reference decides
        # (two real timings of a ~30 us call can be equal to the clock's resolution)
        p.last_encode_time_ms_ = -1.0
        before_ratio, before_ms = p.transformation_ratio(), p.processing_overhead_ms()
        blob = p.encode(c.input.tobytes())
        assert blob == c.expected.tobytes(), name
        if r["overhead_updated"]:
            assert p.transformation_ratio().hex() == r["ratio"], name
            assert p.last_encode_time_ms_ >= 0.0 and p.processing_overhead_ms() != before_ms, name
        else:
            assert p.transformation_ratio() == before_ratio and p.processing_overhead_ms() == before_ms, name
            assert p.last_encode_time_ms_ == -1.0, name
        enc_ms = p.last_encode_time_ms_
        assert p.decode(blob) == c.input.tobytes()
        assert p.processing_overhead_ms() == (enc_ms + p.last_decode_time_ms_) / 2.0
        checked += 1
    assert checked > 50
