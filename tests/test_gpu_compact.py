"""Compacted batch API (tdt_encode_batch / tdt_decode_batch) on mixed-size batches.

Batches holding a message (or decoded blob) longer than 64 KiB take the two-phase path
(slotted message-class kernels, scan of the lengths, gather into the compacted buffer — or, for
decode, sizes + scan then the slotted kernels writing in place); the rest take the look-back
kernel.  Both must give the same bytes, offsets and statuses (TDT_OPT_NO_TWO_PHASE forces
the look-back path), every blob must equal the oracle's, and the capacity semantics of the
compacted API (`out_cap` smaller than the total) must match too."""

import numpy as np
import pytest

from oracle.oracle import Oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"


def _codec():
    from psyne_amd import TDTConfig, TdtCodec
    c = TdtCodec(TDTConfig(sample_fraction=1.0))
    c.set_metrics(10.0, 1.0, 0.5)
    return c


def _gradient(rng, n):
    x = rng.normal(0, 0.01, n // 4).astype(np.float32)
    x[rng.random(n // 4) < 0.7] = 0
    return x.view(np.uint8)


def _batch(seed):
    rng = np.random.default_rng(seed)
    sizes = [64, 1024, 4096, 65536, 100 * 1024, 300 * 1024, 4, 0, 2048, 1 << 20, 64 * 3, 70000 * 4]
    msgs = [(_gradient(rng, s) if s % 4 == 0 and s >= 64 else rng.integers(0, 256, s, dtype=np.uint8))
            for s in sizes]
    off = np.zeros(len(msgs) + 1, np.int64)
    off[1:] = np.cumsum([m.size for m in msgs])
    return msgs, np.concatenate(msgs), off


def _both(codec, fn):
    """fn() under the two-phase path and under the forced look-back path."""
    from psyne_amd._lib import TDT_OPT_NO_TWO_PHASE
    codec.set_option(TDT_OPT_NO_TWO_PHASE, 0)
    a = fn()
    codec.set_option(TDT_OPT_NO_TWO_PHASE, 1)
    try:
        b = fn()
    finally:
        codec.set_option(TDT_OPT_NO_TWO_PHASE, 0)
    return a, b


@pytest.mark.parametrize("seed", [1, 2])
def test_two_phase_matches_lookback_and_oracle(seed):
    codec = _codec()
    msgs, data, off = _batch(seed)
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off).cuda()

    def enc():
        out, eoff, st = codec.encode_batch(d, o)
        torch.cuda.synchronize()
        return out.cpu().numpy(), eoff.cpu().numpy(), st.cpu().numpy()

    (b1, o1, s1), (b2, o2, s2) = _both(codec, enc)
    assert (s1 == 0).all() and (s2 == 0).all()
    assert np.array_equal(o1, o2)
    assert np.array_equal(b1[:o1[-1]], b2[:o2[-1]])
    orc = Oracle()
    cfg = orc.config(sample_fraction=1.0)
    for i, m in enumerate(msgs):
        want = orc.encode(m, cfg=cfg, bandwidth=10.0)
        assert bytes(b1[o1[i]:o1[i + 1]]) == bytes(want), i

    blobs = torch.from_numpy(b1[:o1[-1]].copy()).cuda()
    bo = torch.from_numpy(o1).cuda()

    def dec():
        out, doff, st = codec.decode_batch(blobs, bo)
        torch.cuda.synchronize()
        return out.cpu().numpy(), doff.cpu().numpy(), st.cpu().numpy()

    (d1, p1, t1), (d2, p2, t2) = _both(codec, dec)
    assert (t1 == 0).all() and (t2 == 0).all()
    assert np.array_equal(p1, off) and np.array_equal(p2, off)
    assert np.array_equal(d1[:off[-1]], data) and np.array_equal(d2[:off[-1]], data)


def test_two_phase_capacity_semantics():
    """out_cap below the total: the same statuses (TDT_E_CAPACITY for blobs past the end),
    offsets (the full prefix sum) and fitting bytes on both paths."""
    codec = _codec()
    msgs, data, off = _batch(3)
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off).cuda()
    full, foff, _ = codec.encode_batch(d, o)
    torch.cuda.synchronize()
    total = int(foff[-1].item())
    cap = total // 2

    def enc():
        out = torch.zeros(total, dtype=torch.uint8, device="cuda")
        _, eoff, st = codec.encode_batch(d, o, out=out, out_capacity=cap)
        torch.cuda.synchronize()
        return out.cpu().numpy(), eoff.cpu().numpy(), st.cpu().numpy()

    (b1, o1, s1), (b2, o2, s2) = _both(codec, enc)
    assert np.array_equal(o1, o2) and np.array_equal(s1, s2)
    assert (s1 == 5).any() and (s1 == 0).any()
    for i in range(len(msgs)):
        if s1[i] == 0:
            assert np.array_equal(b1[o1[i]:o1[i + 1]], b2[o2[i]:o2[i + 1]])


def test_compacted_under_graph_capture():
    """Under hipGraph stream capture the compacted API takes the one-pass look-back kernels
    (the two-phase path reads back on the host); the replayed graph gives the eager bytes."""
    codec = _codec()
    msgs, data, off = _batch(4)
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off).cuda()
    ref, roff, rst = codec.encode_batch(d, o)          # eager (two-phase), also sizes the scratch
    torch.cuda.synchronize()
    out = torch.zeros_like(ref)
    eoff = torch.empty_like(roff)
    st = torch.empty_like(rst)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):                        # warm the look-back path's scratch
        from psyne_amd._lib import TDT_OPT_NO_TWO_PHASE
        codec.set_option(TDT_OPT_NO_TWO_PHASE, 1)
        try:
            codec.encode_batch(d, o, out=out, out_offsets=eoff, status=st)
        finally:
            codec.set_option(TDT_OPT_NO_TWO_PHASE, 0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    out.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        codec.encode_batch(d, o, out=out, out_offsets=eoff, status=st)
    g.replay()
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert np.array_equal(eoff.cpu().numpy(), roff.cpu().numpy())
    n = int(roff[-1].item())
    assert np.array_equal(out[:n].cpu().numpy(), ref[:n].cpu().numpy())


@pytest.mark.parametrize("variant", ["resident", "odd_size", "unaligned"])
def test_lookback_resident_only_kernel(variant):
    """Batches of 16-64 KiB messages take the one-pass look-back kernel; when every message is
    aligned, whole 16-byte groups and at most 64 KiB (checked on the device before the launch)
    it is the resident-only instance, otherwise the one with both bodies.  Either way every blob
    equals the oracle's, the offsets are the blob sizes' prefix sums, and the batch decodes
    back."""
    rng = np.random.default_rng({"resident": 11, "odd_size": 12, "unaligned": 13}[variant])
    sizes = list(rng.integers(1024, 4097, 240) * 16)
    if variant == "odd_size":
        sizes[100] += 4  # a partial 16-byte group
    msgs = [_gradient(rng, int(s)) for s in sizes]
    lead = 4 if variant == "unaligned" else 0
    off = np.zeros(len(msgs) + 1, np.int64)
    off[0] = lead
    off[1:] = lead + np.cumsum([m.size for m in msgs])
    data = np.zeros(int(off[-1]), np.uint8)
    for i, m in enumerate(msgs):
        data[off[i]:off[i + 1]] = m
    codec = _codec()
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off).cuda()
    out, eoff, st = codec.encode_batch(d, o)
    torch.cuda.synchronize()
    b, eo, s = out.cpu().numpy(), eoff.cpu().numpy(), st.cpu().numpy()
    assert (s == 0).all()
    assert codec.error_flags() == 0
    orc = Oracle()
    cfg = orc.config(sample_fraction=1.0)
    for i, m in enumerate(msgs):
        assert bytes(b[eo[i]:eo[i + 1]]) == bytes(orc.encode(m, cfg=cfg, bandwidth=10.0)), i
    back, doff, dst = codec.decode_batch(torch.from_numpy(b[:eo[-1]].copy()).cuda(), torch.from_numpy(eo).cuda())
    torch.cuda.synchronize()
    assert int(dst.abs().sum()) == 0
    assert np.array_equal(back.cpu().numpy()[: off[-1] - off[0]], data[lead:])
