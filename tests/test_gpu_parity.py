"""GPU parity: the HIP codec (through the C ABI) against the golden vectors made by the
reference codec, and against the CPU oracle on seeded inputs.  Bit-exact everywhere: this
is byte/integer work (the only floating point, the entropy decision, is restated
bit-exactly; tests/test_log2_restatement.py)."""
import pathlib
import struct

import numpy as np
import pytest

from oracle.oracle import Oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

E_CAPACITY, E_UNSUPPORTED = 5, 6


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from psyne_amd import _lib
    _lib.load()  # the HIP library must be the thing under test


def make_codec(ws=4, min_tensor=1024, bw=10.0, cpu=0.5, hint=None):
    from psyne_amd import TDTConfig, TdtCodec
    c = TdtCodec(TDTConfig(sample_fraction=1.0, word_size=ws, min_tensor_size=min_tensor))
    c.set_metrics(bw, 1.0, cpu)
    if hint is not None:
        c.set_size_hint(hint)
    return c


def pack(msgs, lead=0, align=1):
    """Concatenate messages (optionally misaligned by `lead` bytes) → device tensors."""
    sizes = [len(m) for m in msgs]
    off = np.zeros(len(msgs) + 1, np.int64)
    pos = lead
    for i, s in enumerate(sizes):
        off[i] = pos
        pos += s
        if align > 1:
            pos = (pos + align - 1) // align * align
    off[-1] = pos
    buf = np.zeros(max(pos, 1), np.uint8)
    for i, m in enumerate(msgs):
        buf[off[i]:off[i] + len(m)] = np.frombuffer(bytes(m), np.uint8) if not isinstance(m, np.ndarray) else m
    # with align>1 the gaps belong to the preceding message; rebuild exact offsets
    if align > 1:
        exact = []
        for i, m in enumerate(msgs):
            exact.append((off[i], off[i] + len(m)))
        return buf, exact
    return buf, off


def encode_list(codec, msgs, lead=0):
    buf, off = pack(msgs, lead)
    # offsets are absolute into buf; the message list starts at `lead`
    d = torch.from_numpy(buf).cuda()
    o = torch.from_numpy(off).cuda()
    enc, eoff, st = codec.encode_batch(d, o)
    torch.cuda.synchronize()
    e, eo, s = enc.cpu().numpy(), eoff.cpu().numpy(), st.cpu().numpy()[: len(msgs)]
    return [e[eo[i]:eo[i + 1]].tobytes() for i in range(len(msgs))], s, eo


def decode_list(codec, blobs, cap=None):
    buf, off = pack(blobs)
    d = torch.from_numpy(buf).cuda()
    o = torch.from_numpy(off).cuda()
    if cap is None:
        out, doff, st = codec.decode_batch(d, o)
    else:
        out = torch.empty(max(cap, 1), dtype=torch.uint8, device="cuda")
        out, doff, st = codec.decode_batch(d, o, out=out)
    torch.cuda.synchronize()
    x, xo, s = out.cpu().numpy(), doff.cpu().numpy(), st.cpu().numpy()[: len(blobs)]
    return [x[xo[i]:xo[i + 1]].tobytes() for i in range(len(blobs))], s


def grad(rng, nfloat):
    x = rng.normal(0, 0.01, nfloat).astype(np.float32)
    x[rng.random(nfloat) < 0.7] = 0
    return x.view(np.uint8)


# ----------------------------------------------------------------------------- golden
def _encode_groups(golden, op):
    groups = {}
    for c in golden:
        if c.op == op:
            groups.setdefault((c.ws, c.bandwidth, c.cpu, c.min_tensor), []).append(c)
    return groups


@pytest.mark.parametrize("hint", [1024, 65536])
def test_golden_encode(golden, hint):
    n = 0
    for (ws, bw, cpu, mt), cases in _encode_groups(golden, "encode").items():
        codec = make_codec(ws, mt, bw, cpu, hint)
        got, st, _ = encode_list(codec, [c.input for c in cases])
        for c, g, s in zip(cases, got, st):
            assert s == 0, (c.name, s)
            assert g == c.expected.tobytes(), c.name
            n += 1
    assert n > 100


def test_golden_encode_with_mapping(golden):
    cases = [c for c in golden if c.op == "encode_with_mapping"]
    codec = make_codec(4)
    buf, off = pack([c.input for c in cases])
    mp = torch.tensor(np.array([c.mapping for c in cases], np.int32).reshape(-1)).cuda()
    enc, eoff, st = codec.encode_batch(torch.from_numpy(buf).cuda(), torch.from_numpy(off).cuda(), mapping=mp)
    torch.cuda.synchronize()
    e, eo = enc.cpu().numpy(), eoff.cpu().numpy()
    for i, c in enumerate(cases):
        assert int(st[i]) == 0
        assert e[eo[i]:eo[i + 1]].tobytes() == c.expected.tobytes(), c.name


@pytest.mark.parametrize("hint", [1024, 65536])
def test_golden_decode(golden, hint):
    codec = make_codec(4, hint=hint)
    blobs, want = [], []
    for c in golden:
        if c.op in ("encode", "encode_with_mapping"):
            blobs.append(c.expected.tobytes())
            want.append((0, c.input.tobytes(), c.name))
        elif c.op == "decode":
            blobs.append(c.input.tobytes())
            want.append((c.status, c.expected.tobytes() if c.status == 0 else b"", c.name))
    got, st = decode_list(codec, blobs)
    for (ws_, exp, name), g, s in zip(want, got, st):
        assert s == ws_, (name, s, ws_)
        if s == 0:
            assert g == exp, name


def test_golden_policy(golden):
    for c in golden:
        if c.op != "policy":
            continue
        codec = make_codec(c.ws, c.min_tensor, c.bandwidth, c.cpu)
        assert codec.should_transform(c.n) == c.expect, c.name


# ------------------------------------------------------------------------- vs oracle
def check_vs_oracle(orc, codec, msgs, ws=4, lead=0, bw=10.0, cpu=0.5, mt=1024):
    got, st, eo = encode_list(codec, msgs, lead)
    cfg = orc.config(word_size=ws, min_tensor_size=mt)
    blobs = []
    for i, m in enumerate(msgs):
        want = orc.encode(m, cfg=cfg, bandwidth=bw, cpu=cpu)
        assert st[i] == 0
        assert got[i] == want, f"message {i} (n={len(m)})"
        blobs.append(want)
    dec, dst = decode_list(codec, blobs)
    for i, m in enumerate(msgs):
        assert dst[i] == 0 and dec[i] == bytes(m), f"decode {i}"
    return got


@pytest.mark.parametrize("hint", [1024, 65536])
def test_uniform_1k(orc, hint):
    rng = np.random.default_rng(11)
    msgs = [rng.integers(0, 256, 1024, dtype=np.uint8) for _ in range(512)]
    check_vs_oracle(orc, make_codec(hint=hint), msgs)


def test_gradient_64k(orc):
    rng = np.random.default_rng(12)
    msgs = [grad(rng, 16384) for _ in range(24)]
    check_vs_oracle(orc, make_codec(), msgs)


@pytest.mark.parametrize("hint", [1024, 65536])
def test_large_streaming_path(orc, hint):
    # > 64 KiB (resident limit) → the non-resident streaming rounds
    rng = np.random.default_rng(13)
    msgs = [grad(rng, 262144), rng.integers(0, 256, 200000, dtype=np.uint8), grad(rng, 70000)]
    check_vs_oracle(orc, make_codec(hint=hint), msgs)


def test_zipf_mix(orc):
    rng = np.random.default_rng(14)
    r = np.minimum(rng.zipf(1.5, 300), 1024)
    msgs = []
    for i, k in enumerate(r):
        n = int(64 * k)
        msgs.append(grad(rng, n // 4) if i % 2 else rng.integers(0, 256, n, dtype=np.uint8))
    msgs += [rng.integers(0, 256, n, dtype=np.uint8) for n in (0, 1, 3, 63, 64, 1022, 1026, 1027, 1028)]
    check_vs_oracle(orc, make_codec(), msgs)


@pytest.mark.parametrize("lead", [1, 2, 3, 4, 8, 12])
def test_misaligned_inputs(orc, lead):
    rng = np.random.default_rng(15 + lead)
    msgs = [rng.integers(0, 4, int(n), dtype=np.uint8) for n in rng.integers(256, 3000, 40) * 4]
    msgs += [grad(rng, 4099), rng.integers(0, 256, 1030, dtype=np.uint8)]
    check_vs_oracle(orc, make_codec(), msgs, lead=lead)


def test_rle_cap_boundaries(orc):
    """Runs around the 255 cap at every phase relative to the 16-byte groups."""
    rng = np.random.default_rng(16)
    msgs = [np.zeros(65536, np.uint8), np.full(65536, 7, np.uint8)]
    for L in (254, 255, 256, 509, 510, 511, 765, 766, 1020, 4000):
        for phase in (0, 1, 5, 15):
            v = rng.integers(0, 256, 2048, dtype=np.uint8)
            v[100 + phase:100 + phase + L] = 0x55
            msgs.append(v)
    # stream-position runs that cross many groups in one stream only
    w = np.zeros((8192, 4), np.uint8)
    w[:, 0] = rng.integers(0, 256, 8192)
    msgs.append(w.reshape(-1))
    w2 = np.zeros((8192, 4), np.uint8)
    w2[:, 3] = rng.integers(0, 2, 8192)
    msgs.append(w2.reshape(-1))
    check_vs_oracle(orc, make_codec(), msgs)
    check_vs_oracle(orc, make_codec(hint=1024), msgs)


def test_cap_exclusion_near_threshold(orc):
    """64 KiB messages (8-wave resident kernel) with word-level runs of 110-140 words (~256
    stream bytes per 2-byte stream, 30-34 groups): the pass-A1 block test must send every
    message that can hit the 255-cap through pass A2 (tests/test_cap_exclusion.py)."""
    rng = np.random.default_rng(18)
    msgs = []
    for t in range(24):
        x = grad(rng, 16384).view(np.uint32).copy()
        for _ in range(1 + t % 3):
            L = int(rng.integers(110, 141))
            at = int(rng.integers(0, 16384 - L))
            x[at:at + L] = 0 if t % 2 else x[at]
        msgs.append(x.view(np.uint8))
    check_vs_oracle(orc, make_codec(), msgs)
    check_vs_oracle(orc, make_codec(hint=1024), msgs[:6])


@pytest.mark.parametrize("ws", [1, 2, 8, 16])
def test_word_sizes(orc, ws):
    rng = np.random.default_rng(17 + ws)
    msgs = [grad(rng, 1024 * (i + 1)) if i % 2 else rng.integers(0, 256, 2048 * (i + 1), dtype=np.uint8)
            for i in range(6)]
    msgs += [rng.integers(0, 3, 4096, dtype=np.uint8), np.zeros(4096, np.uint8)]
    msgs += [rng.integers(0, 256, 1028, dtype=np.uint8)]  # 1028 % 8 != 0 → UNCP for ws 8/16
    check_vs_oracle(orc, make_codec(ws=ws), msgs, ws=ws)


def test_policy_passthrough(orc):
    rng = np.random.default_rng(18)
    msgs = [rng.integers(0, 256, 4096, dtype=np.uint8) for _ in range(8)]
    for bw, cpu in ((100.0, 0.5), (1000.0, 0.3), (25.0, 0.9)):
        got, st, _ = encode_list(make_codec(bw=bw, cpu=cpu), msgs)
        for g, m in zip(got, msgs):
            assert g == b"PCNU" + m.tobytes()


def test_empty_and_tiny(orc):
    codec = make_codec(min_tensor=0)
    msgs = [np.zeros(0, np.uint8), np.arange(4, dtype=np.uint8), np.arange(64, dtype=np.uint8),
            np.zeros(64, np.uint8), np.arange(68, dtype=np.uint8)]
    check_vs_oracle(orc, codec, msgs, mt=0)


def test_capacity_error():
    rng = np.random.default_rng(19)
    msgs = [rng.integers(0, 256, 4096, dtype=np.uint8) for _ in range(16)]
    codec = make_codec()
    buf, off = pack(msgs)
    out = torch.empty(20000, dtype=torch.uint8, device="cuda")
    _, eoff, st = codec.encode_batch(torch.from_numpy(buf).cuda(), torch.from_numpy(off).cuda(), out=out)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    eo = eoff.cpu().numpy()
    assert st[0] == 0 and st[-1] == E_CAPACITY
    # offsets still describe the full (unwritten) layout
    assert np.all(np.diff(eo) > 0)


def test_analyze(orc):
    rng = np.random.default_rng(20)
    msgs = [grad(rng, 16384), rng.integers(0, 256, 1024, dtype=np.uint8), np.zeros(2048, np.uint8)]
    codec = make_codec()
    buf, off = pack(msgs)
    hist, ent, mp, st = codec.analyze_batch(torch.from_numpy(buf).cuda(), torch.from_numpy(off).cuda())
    for i, m in enumerate(msgs):
        h, e, p = orc.analyze(m)
        assert np.array_equal(hist[i].cpu().numpy().astype(np.uint32), h)
        assert ent[i].cpu().numpy().tobytes() == e.tobytes()  # bit-exact doubles
        assert np.array_equal(mp[i].cpu().numpy(), p)


def test_roundtrip_many_64k():
    """Size-independent properties at scale: round trip, offsets = prefix of blob sizes."""
    rng = np.random.default_rng(21)
    n = 2048
    x = torch.empty(n * 16384, dtype=torch.float32, device="cuda").normal_(0, 0.01)
    x[torch.rand(n * 16384, device="cuda") < 0.7] = 0
    d = x.view(torch.uint8)
    o = torch.arange(n + 1, dtype=torch.int64, device="cuda") * 65536
    codec = make_codec()
    enc, eoff, st = codec.encode_batch(d, o)
    dec, doff, dst = codec.decode_batch(enc, eoff)
    torch.cuda.synchronize()
    assert int(st[:n].abs().sum()) == 0 and int(dst[:n].abs().sum()) == 0
    assert torch.equal(dec[: n * 65536], d)
    assert torch.equal(doff, o)
    eo = eoff.cpu().numpy()
    e = enc.cpu().numpy()
    orc = Oracle()
    for i in rng.integers(0, n, 16):
        want = orc.encode(d[i * 65536:(i + 1) * 65536].cpu().numpy(), cfg=orc.config(), bandwidth=10.0)
        assert e[eo[i]:eo[i + 1]].tobytes() == want


@pytest.mark.parametrize("path", ["lookback", "two_phase"])
def test_many_tiny_lookback(path):
    # 200k UNCP messages: the look-back chain at depth (forced: small-message batches take the
    # two-phase compaction by default) and the two-phase path's scan + gather
    from psyne_amd._lib import TDT_OPT_NO_TWO_PHASE
    rng = np.random.default_rng(22)
    sizes = rng.integers(0, 40, 200000)
    data = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8)
    off = np.zeros(sizes.size + 1, np.int64)
    off[1:] = np.cumsum(sizes)
    codec = make_codec(hint=64)
    codec.set_option(TDT_OPT_NO_TWO_PHASE, 1 if path == "lookback" else 0)
    enc, eoff, st = codec.encode_batch(torch.from_numpy(data).cuda(), torch.from_numpy(off).cuda())
    torch.cuda.synchronize()
    eo = eoff.cpu().numpy()
    assert np.array_equal(np.diff(eo), sizes + 4)
    e = enc.cpu().numpy()
    i = 12345
    assert e[eo[i]:eo[i + 1]].tobytes() == b"PCNU" + data[off[i]:off[i + 1]].tobytes()


def test_protocol_mirror():
    from psyne_amd import TDTCompressionProtocol, TDTConfig
    p = TDTCompressionProtocol(TDTConfig(sample_fraction=1.0))
    rng = np.random.default_rng(23)
    m = grad(rng, 4096).tobytes()
    assert p.protocol_name() == "TDT-Compression" and p.is_lossless()
    blob = p.encode(m)
    assert blob[:4] == b"PCNU"  # default bandwidth 100 Mbps → passthrough (:200, :352)
    p.update_network_metrics(10.0, 1.0)
    assert p.should_transform(m, len(m))
    blob = p.encode(m)
    assert blob[:4] == b"DTDT" and p.decode(blob) == m
    assert p.transformation_ratio() > 1.0
    orc = Oracle()
    assert blob == orc.encode(np.frombuffer(m, np.uint8), cfg=orc.config(), bandwidth=10.0)
    with pytest.raises(RuntimeError, match="TDT: Invalid encoded data size"):
        p.decode(b"ab")
    with pytest.raises(RuntimeError, match="Invalid TDT magic number"):
        p.decode(b"XXXXYYYYZZZZ")
    p.analyze_data(m, len(m))
    _, e, _ = orc.analyze(np.frombuffer(m, np.uint8))
    assert p.get_average_entropy() == sum(float(v) for v in e) / 4


def test_cpp_protocol_dropin():
    """The header-only C++ HipTDTCompressionProtocol, used through psyne's Protocol concept."""
    import pathlib
    import subprocess
    exe = pathlib.Path(__file__).resolve().parent / "cpp" / "test_protocol"
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cpp protocol OK" in r.stdout


# ------------------------------------------------------------------ slotted batches
def test_slotted_golden_and_roundtrip(golden):
    """tdt_encode_batch_into / tdt_decode_batch_into: every golden encode case in its own
    slot, byte-identical blobs, lengths, decode back through the slots."""
    for hint in (1024, 65536):
        for (ws, bw, cpu, mt), cases in _encode_groups(golden, "encode").items():
            codec = make_codec(ws, mt, bw, cpu, hint)
            buf, off = pack([c.input for c in cases])
            d, o = torch.from_numpy(buf).cuda(), torch.from_numpy(off).cuda()
            out, slots, lens, st = codec.encode_into(d, o)
            torch.cuda.synchronize()
            sl, ln, e = slots.cpu().numpy(), lens.cpu().numpy(), out.cpu().numpy()
            sizes = np.diff(off)
            bounds = np.array([codec.encode_bound(int(s)) for s in sizes])
            assert np.array_equal(np.diff(sl), bounds)
            for i, c in enumerate(cases):
                assert int(st[i]) == 0, c.name
                assert ln[i] == c.expected.size, c.name
                assert e[sl[i]:sl[i] + ln[i]].tobytes() == c.expected.tobytes(), c.name
            back, dsl, dln, dst = codec.decode_into(out, slots, in_lengths=lens)
            torch.cuda.synchronize()
            assert np.array_equal(dsl.cpu().numpy(), off - off[0])
            assert int(dst[: len(cases)].abs().sum()) == 0
            assert np.array_equal(dln.cpu().numpy()[: len(cases)], sizes)
            assert np.array_equal(back.cpu().numpy()[: int(sizes.sum())], buf[off[0]:off[-1]])


def test_slotted_capacity_and_errors():
    rng = np.random.default_rng(31)
    msgs = [rng.integers(0, 256, 4096, dtype=np.uint8) for _ in range(8)]
    codec = make_codec()
    buf, off = pack(msgs)
    d, o = torch.from_numpy(buf).cuda(), torch.from_numpy(off).cuda()
    slots = codec.encode_slots(o)
    s = slots.cpu().numpy().copy()
    s[4] = s[3] + 100  # slot 3 too small
    sl = torch.from_numpy(s).cuda()
    out = torch.empty(int(s[-1]), dtype=torch.uint8, device="cuda")
    out, _, lens, st = codec.encode_into(d, o, slots=sl, out=out)
    torch.cuda.synchronize()
    st, ln = st.cpu().numpy(), lens.cpu().numpy()
    assert st[3] == E_CAPACITY and ln[3] == 0
    assert all(st[i] == 0 for i in range(8) if i != 3)
    # decode side: a blob with a bad magic reports status 2 and length 0; slots skip it
    blobs = [b"PCNU" + bytes(range(10)), b"XXXXabc", b"PCNU"]
    bb, bo = pack(blobs)
    dd, do = torch.from_numpy(bb).cuda(), torch.from_numpy(bo).cuda()
    back, dsl, dln, dst = codec.decode_into(dd, do)
    torch.cuda.synchronize()
    assert list(dst.cpu().numpy()[:3]) == [0, 2, 0]
    assert list(dln.cpu().numpy()[:3]) == [10, 0, 0]
    assert back.cpu().numpy()[:10].tobytes() == bytes(range(10))


def _craft_blob(rng, orig, ws, mapping, stream_fill):
    """A valid TDT blob (tdt_compression.hpp:81-117 layout) with arbitrary RLE streams:
    stream_fill(c, need) returns the pair bytes of stream c (may be short, long, contain count 0
    pairs or an odd trailing byte)."""
    ns = max(mapping) + 1
    wc = orig // ws
    hdr = struct.pack("<5I", 0x54445444, orig, ns, ws, ws) + struct.pack("<%di" % ws, *mapping)
    body = b""
    for c in range(ns):
        need = wc * mapping.count(c)
        s = stream_fill(c, need)
        body += struct.pack("<I", len(s)) + s
    return hdr + body


def _pairs(rng, total, zero_frac=0.0, maxrun=255, odd=False):
    out = bytearray()
    left = total
    while left > 0:
        if zero_frac and rng.random() < zero_frac:
            out += bytes([0, int(rng.integers(0, 256))])
            continue
        c = int(min(left, rng.integers(1, maxrun + 1)))
        out += bytes([c, int(rng.integers(0, 256))])
        left -= c
    if odd:
        out += bytes([int(rng.integers(1, 256))])
    return bytes(out)


def test_decode_crafted_fast_path(orc):
    """Decoder windows/blocks: streams shorter or longer than needed, count-0 pairs, odd
    trailing bytes, 1 and 2 referenced streams, messages spanning many windows (head-array
    generations), run lengths from 1 to 255; compared with the oracle's decode."""
    rng = np.random.default_rng(31)
    blobs = []
    maps = [[0, 0, 0, 0], [1, 1, 0, 0], [0, 1, 1, 1], [1, 0, 0, 0], [0, 1, 0, 1], [1, 1, 1, 0]]
    for i in range(60):
        orig = int(rng.choice([64, 1024, 4096, 20000, 65536, 65540, 140000]))
        mp = maps[i % len(maps)]
        mode = i % 5
        maxrun = int(rng.choice([1, 2, 3, 8, 255]))

        def fill(c, need, mode=mode, maxrun=maxrun):
            if mode == 0:
                return _pairs(rng, need, maxrun=maxrun)
            if mode == 1:  # short stream: leaves zeros
                return _pairs(rng, int(need * rng.random()), maxrun=maxrun)
            if mode == 2:  # long stream: extra ignored
                return _pairs(rng, need + int(rng.integers(1, 3000)), maxrun=maxrun)
            if mode == 3:
                return _pairs(rng, need, zero_frac=0.2, maxrun=maxrun, odd=True)
            return _pairs(rng, need // 2, maxrun=maxrun, odd=True)
        blobs.append(_craft_blob(rng, orig, 4, mp, fill))
    codec = make_codec()
    got, st = decode_list(codec, blobs)
    for i, b in enumerate(blobs):
        s, want = orc.decode(b)
        assert st[i] == s == 0, (i, st[i], s)
        assert got[i] == want, f"crafted blob {i}"


def test_decode_blob_cache_edges(orc):
    """The small-blob decode list (blobs decoding to <= 8 KiB) reads each blob's first 1,504
    bytes into LDS and takes a stream's pair blocks from there when the whole stream lies inside
    (tdt_decode.h DecLayoutT::BLOBC, decode_fast `cached`).  Blobs whose streams end just before,
    at and just past that edge — stream 0 stored first or second, one or two streams, even and
    odd stream lengths, every 4-byte phase of the blob start — against the oracle's decode."""
    rng = np.random.default_rng(1504)
    maps = [[1, 1, 0, 0], [0, 1, 1, 1], [0, 1, 0, 1], [0, 0, 0, 0], [1, 0, 0, 0]]
    blobs = []
    for i in range(120):
        mp = maps[i % len(maps)]
        orig = int(rng.choice([1024, 1100, 2048, 4096, 8192]))
        ns = max(mp) + 1
        hdr = struct.pack("<5I", 0x54445444, orig, ns, 4, 4) + struct.pack("<4i", *mp)
        body = b""
        for c in range(ns):
            if c == 0:
                # the first stored stream ends at blob offset 1504 + d
                end = 1504 + int(rng.integers(-8, 9))
                nbytes = end - (len(hdr) + 4)
            else:
                nbytes = int(rng.integers(0, 700))
            k, odd = nbytes // 2, nbytes % 2
            s = bytearray()
            for _ in range(k):
                s += bytes([int(rng.integers(1, 4)), int(rng.integers(0, 256))])
            if odd:
                s += bytes([int(rng.integers(1, 256))])
            body += struct.pack("<I", len(s)) + bytes(s)
        blobs.append(hdr + body)
    # (concatenated: the blob starts fall on every phase; a 1-3 byte spacer shifts them further)
    for lead in (0, 1, 3):
        got, st = decode_list(make_codec(), ([b"PCNU" + bytes(lead)] if lead else []) + blobs)
        got, st = (got[1:], st[1:]) if lead else (got, st)
        for i, b in enumerate(blobs):
            s, want = orc.decode(b)
            assert st[i] == s, (lead, i, st[i], s)
            assert got[i] == want, f"blob {i} (lead {lead}, len {len(b)})"


def test_every_ws4_mapping_device_decode(orc):
    """Every one of the 16 word-size-4 byte-plane mappings through the device encoder
    (tdt_encode_with_mapping_batch) and the device decoder's recombine forms (12+4, 4+12, 8+8
    bits, one stream; `[1,1,1,1]` leaves stream 0 empty): blobs byte for byte against the
    oracle's encode with that mapping, then the device's blobs decoded on the device against
    the oracle's decode (status and bytes) and the input (recombine_byte_streams :614-637).
    Sizes 1 KiB (one-wave decode), 64 KiB, 100,000 B and 100,004 B (a partial last 16-byte
    group), 1 MiB (tiled decode); gradient-like and uniform bytes."""
    rng = np.random.default_rng(606)
    maps = [[(mb >> b) & 1 for b in range(4)] for mb in range(16)]
    msgs, mapping = [], []
    for mp in maps:
        for n in (1024, 65536, 100000, 100004, 1 << 20):
            for kind in ("grad", "uniform"):
                if kind == "uniform" and n > 65536:
                    continue  # (incompressible large blobs add bytes, not decode forms)
                m = grad(rng, n // 4) if kind == "grad" else rng.integers(0, 256, n, dtype=np.uint8)
                msgs.append(np.ascontiguousarray(m))
                mapping.append(mp)
    codec = make_codec()
    buf, off = pack(msgs)
    mp_t = torch.tensor(np.array(mapping, np.int32).reshape(-1)).cuda()
    enc, eoff, st = codec.encode_batch(torch.from_numpy(buf).cuda(), torch.from_numpy(off).cuda(), mapping=mp_t)
    torch.cuda.synchronize()
    e, eo, st = enc.cpu().numpy(), eoff.cpu().numpy(), st.cpu().numpy()
    cfg = orc.config(word_size=4)
    blobs = []
    for i, (m, mp) in enumerate(zip(msgs, mapping)):
        want = orc.encode(m, cfg=cfg, mapping=mp)
        got = e[eo[i]:eo[i + 1]].tobytes()
        assert int(st[i]) == 0, (i, mp, len(m))
        assert got == want, f"encode, mapping {mp}, n={len(m)}"
        blobs.append(got)
    dec, dst = decode_list(codec, blobs)
    for i, (m, mp) in enumerate(zip(msgs, mapping)):
        s, want = orc.decode(blobs[i])
        assert dst[i] == s == 0, (i, mp, len(m), dst[i], s)
        assert dec[i] == want == bytes(m), f"decode, mapping {mp}, n={len(m)}"
    # every blob up to 256 KiB once more through tdt_decode_host with one message per call: the
    # one-message kernels (one wave up to 4 KiB, the 16-wave tiled kernel above)
    for i, b in enumerate(blobs):
        if len(msgs[i]) > 256 * 1024:
            continue
        arr = np.frombuffer(b, np.uint8)
        d1, _, s1 = codec.decode_host(arr, np.array([0, arr.size], np.uint64), len(msgs[i]))
        assert s1[0] == 0 and d1.tobytes() == bytes(msgs[i]), f"one-message decode, mapping {mapping[i]}, n={len(msgs[i])}"


def test_copy_device():
    """tdt_copy_device (the hand-written HBM copy bench.py reports as roofline.copy_ceiling):
    every size class (byte head / 64 KiB pieces / partial last piece / byte tail) at equal and
    unequal 16-byte phases, nothing written outside [dst, dst + n)."""
    from psyne_amd._lib import check, load
    lib = load()
    rng = np.random.default_rng(77)
    src = torch.from_numpy(rng.integers(0, 256, (3 << 20) + 64, dtype=np.uint8)).cuda()
    for n in (0, 1, 15, 16, 17, 4095, 65536, 65536 * 3 + 17, (3 << 20) - 5):
        for so, do in ((0, 0), (3, 3), (5, 9), (16, 0)):
            dst = torch.full(((3 << 20) + 128,), 0xA5, dtype=torch.uint8, device="cuda")
            check(lib.tdt_copy_device(dst.data_ptr() + do, src.data_ptr() + so, n, None))
            torch.cuda.synchronize()
            assert torch.equal(dst[do:do + n], src[so:so + n]), (n, so, do)
            assert int((dst[:do] != 0xA5).sum()) == 0 and int((dst[do + n:] != 0xA5).sum()) == 0, (n, so, do)


@pytest.mark.parametrize("n", [0, 1, 8191, 8192, 8193, 20000, 50001])
def test_slot_offsets_multi_chunk(n):
    """tdt_encode_slots (closed form) and tdt_decode_slots (two-pass chunked scan, 8192
    sizes per workgroup) against numpy cumsums, across chunk boundaries, with a non-zero
    first input offset and with a slot array that is only 8-byte aligned (scalar path)."""
    from psyne_amd._lib import check
    rng = np.random.default_rng(n + 7)
    codec = make_codec()
    lib, h = codec._lib, codec._h
    sizes = rng.integers(0, 40, n)
    lead = 12
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64) + lead
    o = torch.from_numpy(off).cuda()
    for shift in (0, 1):  # slot array 16-byte aligned / 8-byte aligned
        raw = torch.full((n + 3,), -1, dtype=torch.int64, device="cuda")
        sl = raw[shift:shift + n + 1]
        check(lib.tdt_encode_slots(h, o.data_ptr(), n, sl.data_ptr(), 0))
        torch.cuda.synchronize()
        want = np.concatenate([[0], np.cumsum(2 * sizes + 28 + 16)]).astype(np.int64)
        assert np.array_equal(sl.cpu().numpy(), want)
    # decode side: UNCP blobs of the drawn payload sizes; decoded size = blob length - 4
    blobs = [b"PCNU" + bytes(rng.integers(0, 256, int(s), dtype=np.uint8)) for s in sizes]
    bb, bo = pack(blobs) if n else (np.zeros(1, np.uint8), np.zeros(1, np.int64))
    dd, do = torch.from_numpy(bb).cuda(), torch.from_numpy(bo).cuda()
    st = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")
    for shift in (0, 1):
        raw = torch.full((n + 3,), -1, dtype=torch.int64, device="cuda")
        sl = raw[shift:shift + n + 1]
        check(lib.tdt_decode_slots(h, dd.data_ptr(), do.data_ptr(), 0, n, sl.data_ptr(), st.data_ptr(), 0))
        torch.cuda.synchronize()
        want = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        assert np.array_equal(sl.cpu().numpy(), want)
        assert int(st[:n].abs().sum()) == 0
        assert int(raw[shift + n + 1]) == -1  # nothing written past off[n]


def test_mapping_ties_exact_fallback(orc):
    """Messages whose byte-position entropies tie (or nearly tie) with their mean: the
    kernel's hardware-log2 entropy sums cannot decide them (|a_b - mean| <= kFastMargin), so it
    must fall back to the reference's sequential fma chains (tdt_compression.hpp:470-480) —
    compared here with the oracle byte for byte, for the 512-lane (64 KiB) and the one-wave
    (1-4 KiB) teams.  The near ties (a copied position with k samples changed) straddle the
    margin: some messages take the fast decision, some the exact one."""
    rng = np.random.default_rng(41)
    msgs = []
    for n in (1024, 4096, 65536):
        w = n // 4
        x = rng.integers(0, 256, w, dtype=np.uint8)
        msgs.append(np.repeat(x, 4))                                  # 4 equal positions: exact tie
        msgs.append(np.full(n, 0x3C, np.uint8))                       # constant: all entropies 0
        y = rng.integers(0, 256, (w, 4), dtype=np.uint8)
        y[:, 1] = y[:, 0]                                             # two equal positions
        y[:, 3] = np.roll(y[:, 2], 1)                                 # same distribution, shifted
        msgs.append(y.reshape(-1))
        z = np.tile(np.arange(256, dtype=np.uint8), n // 256)         # every position uniform
        msgs.append(z)
        g = grad(rng, w)
        msgs.append(g)
        for k in (1, 2, 3, 5, 9, 17):                                  # near ties around the margin
            y = rng.integers(0, 256, (w, 4), dtype=np.uint8)
            y[:, 1] = y[:, 0]
            idx = rng.choice(w, k, replace=False)
            y[idx, 1] = rng.integers(0, 256, k, dtype=np.uint8)
            y[:, 3] = np.roll(y[:, 2], 3)
            msgs.append(y.reshape(-1))
    check_vs_oracle(orc, make_codec(), msgs)
    check_vs_oracle(orc, make_codec(hint=1024), msgs)


@pytest.mark.parametrize("ws", [4, 8])
def test_one_message_host_path(orc, ws):
    """tdt_encode_host / tdt_decode_host with ONE message (the drop-in Protocol::encode / decode
    call, protocol_demo.cpp:135-189) take the zero-copy one-message path up to 256 KiB: every
    size class (UNCP, one-wave, 256-lane, 512-lane resident and streaming), odd and unaligned
    sizes, the 256 KiB bound and just past it (the pipeline), each blob equal to the oracle's and
    decoded back; corrupted blobs report the reference's errors through the status."""
    from psyne_amd._lib import TDT_OK
    rng = np.random.default_rng(90 + ws)
    codec = make_codec(ws=ws)
    cfg = orc.config(word_size=ws, sample_fraction=1.0)
    sizes = [0, 3, 64, 1020, 1024, 1032, 4096, 4104, 8192, 32768, 32776, 65536, 65544, 100000, 131072,
             262144, 262144 + 8, 1 << 20]
    for n in sizes:
        m = grad(rng, n // 4).view(np.uint8) if n % 4 == 0 else rng.integers(0, 256, n, dtype=np.uint8)
        m = np.ascontiguousarray(m[:n])
        enc, eoff, st = codec.encode_host(m, np.array([0, n], np.uint64))
        assert int(st[0]) == TDT_OK, n
        want = orc.encode(m, cfg=cfg, bandwidth=10.0)
        assert enc.tobytes() == want, "encode n=%d ws=%d" % (n, ws)
        dec, doff, dst = codec.decode_host(enc, eoff, max(n, 1))
        assert int(dst[0]) == TDT_OK and int(doff[1]) == n and np.array_equal(dec, m), "decode n=%d" % n
    # errors: short blob, bad magic, truncated TDT header
    for bad, code in ((b"\x01\x02", 1), (b"ABCDEFGH", 2), (bytes.fromhex("44544454") + b"\x00" * 6, 3)):
        b = np.frombuffer(bad, np.uint8)
        dec, doff, dst = codec.decode_host(b, np.array([0, b.size], np.uint64), 64)
        assert int(dst[0]) == code and int(doff[1]) == 0
    assert codec.error_flags() == 0


def _runs(rng, n, mean_run, alphabet=4):
    out = np.empty(n, np.uint8)
    i = 0
    while i < n:
        L = int(rng.geometric(1.0 / mean_run))
        out[i:i + L] = rng.integers(0, alphabet)
        i += L
    return out


@pytest.mark.parametrize("env", [{}, {"PSYNE_TDT_ONE_SPIN": "0"}, {"PSYNE_TDT_ONE_WAVE": "1"}],
                         ids=["tiles", "tiles_sync", "one_wave"])
def test_one_message_decode_tiles(orc, env, monkeypatch):
    """The one-message decode (tdt_decode_one_kernel: block sums, their scan in LDS and 16 waves'
    output tiles in one launch) on blobs whose runs cross every tile boundary, whose streams end
    before the output does (zeros), hold count-0 pairs or one empty stream, and on the shapes it
    hands to wave 0's decode_one (UNCP, a ws-8 generic mapping, truncated blobs): statuses and
    bytes equal the oracle's.  Completion seen by the spin on the stream-written word or by the
    stream sync, and the round-4 one-wave kernel, give the same results."""
    import sys
    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent))
    from test_gpu_large import build_blob, parse_blob
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(131)
    codec = make_codec()
    cfg = orc.config(sample_fraction=1.0)
    blobs = []
    for n, mr in ((65536, 0), (262144, 0), (262144, 300), (200000, 40), (131072, 5000), (4096, 0), (65536 + 16, 900)):
        m = grad(rng, n // 4) if mr == 0 else _runs(rng, n, mr)
        blobs.append(orc.encode(np.ascontiguousarray(m), cfg=cfg, bandwidth=10.0))
    w, mp, streams = parse_blob(blobs[1])
    assert len(streams) == 2
    blobs.append(build_blob(w, mp, [streams[0], streams[1][: (len(streams[1]) // 6) * 2]]))  # stream 1 short
    blobs.append(build_blob(w, mp, [streams[0][:(len(streams[0]) // 3) * 2], streams[1]]))  # stream 0 short
    blobs.append(build_blob(w, mp, [b"", streams[1]]))  # stream 0 empty
    s0 = bytearray(streams[0])
    for k in range(0, len(s0) - 1, 2 * 211):
        s0[k] = 0
    blobs.append(build_blob(w, mp, [bytes(s0), streams[1]]))  # count-0 pairs
    blobs.append(blobs[1][:-7])  # truncated
    x = grad(rng, 32768)
    blobs.append(orc.encode(x, cfg=orc.config(word_size=8, sample_fraction=1.0), bandwidth=10.0,
                            mapping=[1, 1, 1, 0, 0, 0, 0, 0]))  # generic shape (ws 8)
    blobs.append(orc.encode(rng.integers(0, 256, 100001, dtype=np.uint8), cfg=cfg, bandwidth=10.0))  # UNCP
    for i, b in enumerate(blobs):
        arr = np.frombuffer(b, np.uint8).copy()
        ost, want = orc.decode(b)
        dec, doff, dst = codec.decode_host(arr, np.array([0, arr.size], np.uint64), 1 << 18)
        assert int(dst[0]) == ost, "blob %d (%d B) status %d vs oracle %d" % (i, arr.size, dst[0], ost)
        if ost == 0:
            assert dec.tobytes() == want, "blob %d (%d B) bytes" % (i, arr.size)
    assert codec.error_flags() == 0


def test_encode_host_gather(orc):
    """tdt_encode_host_v (the substrate send path: messages in separate caller buffers, gathered by
    the copy pool straight into pinned staging) equals the oracle blob for blob, over a batch
    large enough to be split into several 64 MiB pipeline chunks and gather pieces (small,
    medium, 1 MiB and 3 MiB messages, odd sizes)."""
    import ctypes as C
    from psyne_amd._lib import check
    rng = np.random.default_rng(97)
    sizes = list(rng.integers(1, 2048, 3000) * 4) + [65536] * 600 + [1 << 20] * 60 + [3 << 20] * 4 + [1021, 0, 7]
    rng.shuffle(sizes)
    msgs = [np.ascontiguousarray(grad(rng, int(n) // 4).view(np.uint8)[: int(n)]) if n % 4 == 0 else
            rng.integers(0, 256, int(n), dtype=np.uint8) for n in sizes]
    n = len(msgs)
    codec = make_codec()
    ptrs = (C.c_void_p * n)(*[m.ctypes.data for m in msgs])
    sz = np.array(sizes, np.uint64)
    cap = int(sum(codec.encode_bound(int(s)) for s in sizes))
    out = np.empty(cap, np.uint8)
    ooff = np.zeros(n + 1, np.uint64)
    st = np.zeros(n, np.int32)
    check(codec._lib.tdt_encode_host_v(codec._h, C.addressof(ptrs), sz.ctypes.data, n, out.ctypes.data, cap,
                                       ooff.ctypes.data, st.ctypes.data))
    assert int(np.abs(st).sum()) == 0
    for i, m in enumerate(msgs):
        assert out[ooff[i]:ooff[i + 1]].tobytes() == orc.encode(m, bandwidth=10.0), "message %d (%d B)" % (i, m.size)


def test_encode_host_gather_pinned(orc):
    """tdt_encode_host_v over messages in pinned memory (a channel's pinned message buffers): no
    staging, one DMA per run of adjacent messages (runs broken by gaps and by a reversed order),
    blobs equal to the oracle's; then the same messages pageable give the same bytes."""
    import ctypes as C
    from psyne_amd._lib import check
    rng = np.random.default_rng(98)
    sizes = [1 << 20] * 12 + list(rng.integers(1, 2048, 40) * 4) + [65536] * 6 + [0, 12]
    total = sum(sizes) + 4096 * len(sizes)
    pin = torch.empty(total, dtype=torch.uint8).pin_memory()
    host = pin.numpy()
    starts, pos = [], 0
    for k, n in enumerate(sizes):
        starts.append(pos)
        pos += n + (4096 if k % 5 == 4 else 0)  # every fifth message leaves a gap (a new run)
    order = list(range(len(sizes)))
    order[20:30] = order[20:30][::-1]  # not in memory order: each of these starts a run
    msgs = []
    for k in order:
        n = sizes[k]
        host[starts[k]:starts[k] + n] = grad(rng, n // 4).view(np.uint8)[:n] if n % 4 == 0 else rng.integers(0, 256, n)
        msgs.append((int(starts[k]), int(n)))
    n = len(msgs)
    codec = make_codec()
    base = pin.data_ptr()
    ptrs = (C.c_void_p * n)(*[int(base + a) for a, _ in msgs])
    sz = np.array([b for _, b in msgs], np.uint64)
    cap = int(sum(codec.encode_bound(int(b)) for b in sz))
    out = np.empty(cap, np.uint8)
    ooff = np.zeros(n + 1, np.uint64)
    st = np.zeros(n, np.int32)
    check(codec._lib.tdt_encode_host_v(codec._h, C.addressof(ptrs), sz.ctypes.data, n, out.ctypes.data, cap,
                                       ooff.ctypes.data, st.ctypes.data))
    assert int(np.abs(st).sum()) == 0
    for i, (a, b) in enumerate(msgs):
        assert out[ooff[i]:ooff[i + 1]].tobytes() == orc.encode(host[a:a + b].copy(), bandwidth=10.0), "message %d" % i
    copies = [np.array(host[a:a + b]) for a, b in msgs]
    ptrs2 = (C.c_void_p * n)(*[m.ctypes.data for m in copies])
    out2 = np.empty(cap, np.uint8)
    ooff2 = np.zeros(n + 1, np.uint64)
    check(codec._lib.tdt_encode_host_v(codec._h, C.addressof(ptrs2), sz.ctypes.data, n, out2.ctypes.data, cap,
                                       ooff2.ctypes.data, st.ctypes.data))
    assert np.array_equal(ooff2, ooff) and np.array_equal(out2[: int(ooff[-1])], out[: int(ooff[-1])])
