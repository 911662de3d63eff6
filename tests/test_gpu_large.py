"""Large messages on the tiled path (DESIGN.md §4 "large messages"): span histograms, the
mapping pass, per-tile counts, the scan that stitches the run carried across tile boundaries
(255-cap chunk starts inside the next tile), and the emit pass — every blob compared with the
oracle byte for byte, then decoded back.  Also the fallback to the whole-message kernel when
the tile budget is spent."""

import numpy as np
import pytest

from oracle.oracle import Oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"


def codec_for(ws=4):
    from psyne_amd import TDTConfig, TdtCodec
    c = TdtCodec(TDTConfig(sample_fraction=1.0, word_size=ws))
    c.set_metrics(10.0, 1.0, 0.5)
    return c


def runs_message(rng, n, mean_run, alphabet=4):
    """Bytes in runs of geometric length (mean `mean_run`): many runs cross 255 and the tile
    boundaries, so the cap chunk starts of carried runs land inside later tiles."""
    out = np.empty(n, np.uint8)
    i = 0
    while i < n:
        L = int(rng.geometric(1.0 / mean_run))
        out[i:i + L] = rng.integers(0, alphabet)
        i += L
    return out


def gradient(rng, n):
    x = rng.normal(0, 0.01, n // 4).astype(np.float32)
    x[rng.random(x.size) < 0.7] = 0
    return x.view(np.uint8)


def check_batch(msgs, ws=4, lead=0, codec=None):
    off = np.zeros(len(msgs) + 1, np.int64)
    off[0] = lead
    for i, m in enumerate(msgs):
        off[i + 1] = off[i] + m.size
    buf = np.zeros(int(off[-1]), np.uint8)
    for i, m in enumerate(msgs):
        buf[off[i]:off[i + 1]] = m
    codec = codec or codec_for(ws)
    d, o = torch.from_numpy(buf).cuda(), torch.from_numpy(off).cuda()
    out, slots, lens, st = codec.encode_into(d, o)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0
    orc = Oracle()
    sl, ln, ob = slots.cpu().numpy(), lens.cpu().numpy(), out.cpu().numpy()
    for i, m in enumerate(msgs):
        got = ob[sl[i]:sl[i] + ln[i]].tobytes()
        want = orc.encode(m, cfg=orc.config(word_size=ws), bandwidth=10.0)
        assert got == want, "message %d (%d bytes)" % (i, m.size)
    back, dsl, dln, dst = codec.decode_into(out, slots, in_lengths=lens)
    torch.cuda.synchronize()
    assert int(dst.abs().sum()) == 0
    assert torch.equal(back[: int(off[-1] - off[0])], d[int(off[0]):])
    assert codec.error_flags() == 0


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mean_run", [40, 300, 900])
def test_runs_across_tiles(mean_run):
    rng = np.random.default_rng(mean_run)
    check_batch([runs_message(rng, 3 << 20, mean_run), runs_message(rng, (1 << 20) + 4 * 4099, mean_run)])


@pytest.mark.timeout(300)
def test_constant_and_sparse_large():
    rng = np.random.default_rng(5)
    zeros = np.zeros(5 << 20, np.uint8)
    sparse = np.zeros(2 << 20, np.uint8)
    sparse[rng.integers(0, sparse.size, 200)] = rng.integers(1, 256, 200)
    # one run starting exactly at a tile boundary and one ending 1 byte past a span boundary
    edge = np.zeros(1 << 20, np.uint8)
    edge[65536:65536 + 700] = 7
    edge[524288 - 5:524288 + 1] = 9
    check_batch([zeros, sparse, edge])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("lead", [1, 3, 8])
def test_mixed_unaligned(lead):
    """Large messages at misaligned starts (streaming tiles) among small and medium ones."""
    rng = np.random.default_rng(100 + lead)
    msgs = []
    for k in range(24):
        kind = k % 4
        if kind == 0:
            msgs.append(gradient(rng, int(rng.integers(65, 800)) * 4096))
        elif kind == 1:
            msgs.append(runs_message(rng, int(rng.integers(70, 700)) * 4096 + 4 * int(rng.integers(0, 1000)), 200))
        elif kind == 2:
            msgs.append(rng.integers(0, 256, int(rng.integers(1, 64)) * 64, dtype=np.uint8))
        else:
            msgs.append(gradient(rng, int(rng.integers(2, 16)) * 4096))
    check_batch(msgs, lead=lead)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("ws", [1, 2, 8, 16])
def test_word_sizes_large(ws):
    rng = np.random.default_rng(ws)
    check_batch([gradient(rng, 3 << 20), runs_message(rng, (2 << 20) + 16 * 1000, 350), gradient(rng, 1 << 19)], ws=ws)


@pytest.mark.timeout(300)
def test_large_uncompressible_passthrough():
    """Large messages that the policy leaves uncompressed (size not a multiple of 4) are
    copied span by span."""
    rng = np.random.default_rng(9)
    check_batch([rng.integers(0, 256, (3 << 20) + 1, dtype=np.uint8), gradient(rng, 1 << 20),
                 rng.integers(0, 256, (1 << 20) + 3, dtype=np.uint8)])


@pytest.mark.timeout(300)
def test_tile_budget_fallback():
    """A tile budget of 64 tiles (4 MiB): the first large messages take the tiled path, the
    rest the whole-message kernel — the blobs are the same either way."""
    from psyne_amd._lib import TDT_OPT_TILE_CAP
    codec = codec_for(4)
    codec.set_option(TDT_OPT_TILE_CAP, 64)
    rng = np.random.default_rng(17)
    msgs = [runs_message(rng, int(rng.integers(5, 20)) * 65536 + 4 * k, 280) for k in range(12)]
    check_batch(msgs, codec=codec)


def parse_blob(b):
    """(header words, mapping, [stream bytes]) of a TDT blob."""
    w = np.frombuffer(b[:20], np.uint32)
    msize = int(w[4])
    mapping = np.frombuffer(b[20:20 + 4 * msize], np.int32).copy()
    off, streams = 20 + 4 * msize, []
    for _ in range(int(w[2])):
        ln = int.from_bytes(b[off:off + 4], "little")
        streams.append(b[off + 4:off + 4 + ln])
        off += 4 + ln
    return w.copy(), mapping, streams


def build_blob(w, mapping, streams):
    out = w.astype(np.uint32).tobytes() + mapping.astype(np.int32).tobytes()
    for st in streams:
        out += len(st).to_bytes(4, "little") + st
    return out


def decode_vs_oracle(blobs):
    from psyne_amd import TDTConfig, TdtCodec
    codec = TdtCodec(TDTConfig(sample_fraction=1.0))
    off = np.zeros(len(blobs) + 1, np.int64)
    off[1:] = np.cumsum([len(b) for b in blobs])
    buf = np.frombuffer(b"".join(blobs), np.uint8).copy()
    d, o = torch.from_numpy(buf).cuda(), torch.from_numpy(off).cuda()
    out, slots, lens, st = codec.decode_into(d, o)
    torch.cuda.synchronize()
    orc = Oracle()
    sl, ln, ob, sts = slots.cpu().numpy(), lens.cpu().numpy(), out.cpu().numpy(), st.cpu().numpy()
    for i, b in enumerate(blobs):
        ost, want = orc.decode(b)
        assert int(sts[i]) == ost, "blob %d status %d vs oracle %d" % (i, sts[i], ost)
        if ost == 0:
            assert ob[sl[i]:sl[i] + ln[i]].tobytes() == want, "blob %d bytes" % i
    assert codec.error_flags() == 0


@pytest.mark.timeout(300)
def test_large_decode_crafted():
    rng = np.random.default_rng(23)
    orc = Oracle()
    good = orc.encode(gradient(rng, 3 << 20), bandwidth=10.0)
    w, mp, streams = parse_blob(good)
    assert len(streams) == 2
    # stream 1 cut to a third of its pairs: its positions past that decode as zeros
    s1 = streams[1][: (len(streams[1]) // 6) * 2]
    short = build_blob(w, mp, [streams[0], s1])
    # stream 0 empty, stream 1 whole
    empty0 = build_blob(w, mp, [b"", streams[1]])
    # truncated blob (stream table runs past the end)
    trunc = good[:-7]
    # a stream with count-0 pairs sprinkled in (emit nothing)
    s0 = bytearray(streams[0])
    for k in range(0, len(s0) - 1, 2 * 997):
        s0[k] = 0
    zeros = build_blob(w, mp, [bytes(s0), streams[1]])
    decode_vs_oracle([good, short, empty0, trunc, zeros])


@pytest.mark.timeout(300)
def test_large_decode_generic_shapes():
    """A large blob the fast path does not take (word size 8, three positions in stream 1:
    6-byte segments): decoded whole by one wave in the prep pass, still bit-exact."""
    rng = np.random.default_rng(29)
    orc = Oracle()
    x = gradient(rng, 2 << 20)
    b8 = orc.encode(x, cfg=orc.config(word_size=8), bandwidth=10.0, mapping=[1, 1, 1, 0, 0, 0, 0, 0])
    assert parse_blob(b8)[0][3] == 8
    decode_vs_oracle([b8, orc.encode(x, bandwidth=10.0)])


def test_compacted_offsets_past_4gib():
    """The compacted one-pass encode (decoupled look-back) over 6 GiB of C3-style messages:
    blob offsets pass 2^31 and 2^32, so the 64-bit offsets must survive every wave-uniform
    broadcast (a sign-extended low half faulted here).  Offsets equal the scan of the slotted
    lengths, sampled blobs (first, around 2 / 4 GiB, last) equal the oracle's, and the round
    trip is exact."""
    codec = codec_for(4)
    n, mb = 98304, 65536  # 6 GiB in, ~4.8 GiB of blobs
    g = torch.Generator(device="cuda")
    g.manual_seed(41)
    x = torch.empty(n * mb // 4, dtype=torch.float32, device="cuda").normal_(0, 0.01, generator=g)
    x.masked_fill_(torch.rand(x.numel(), device="cuda", generator=g) < 0.7, 0.0)
    data = x.view(torch.uint8)
    off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * mb
    out, eoff, st = codec.encode_batch(data, off)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0
    eo = eoff.cpu().numpy()
    assert eo[-1] > (1 << 32) and np.all(np.diff(eo) > 0)
    # slotted lengths, scanned, give the same offsets
    slots = codec.encode_slots(off)
    buf = torch.empty(int(slots[-1].item()), dtype=torch.uint8, device="cuda")
    lens = torch.empty(n, dtype=torch.int64, device="cuda")
    sst = torch.empty(n, dtype=torch.int32, device="cuda")
    from psyne_amd._lib import check
    check(codec._lib.tdt_encode_batch_into(codec._h, data.data_ptr(), off.data_ptr(), n, buf.data_ptr(),
                                           slots.data_ptr(), lens.data_ptr(), sst.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert np.array_equal(np.diff(eo), lens.cpu().numpy())
    del buf
    orc = Oracle()
    cfg = orc.config(sample_fraction=1.0)
    picks = {0, n - 1}
    for lim in (1 << 31, 1 << 32):
        k = int(np.searchsorted(eo, lim))
        picks.update({k - 1, k})
    for i in sorted(picks):
        m = data[i * mb:(i + 1) * mb].cpu().numpy()
        assert out[eo[i]:eo[i + 1]].cpu().numpy().tobytes() == orc.encode(m, cfg=cfg, bandwidth=10.0), i
    back, doff, dst = codec.decode_batch(out, eoff, out_capacity=n * mb,
                                         out=torch.empty(n * mb, dtype=torch.uint8, device="cuda"))
    torch.cuda.synchronize()
    assert int(dst.abs().sum()) == 0 and torch.equal(back, data)
    assert torch.equal(doff, off)


@pytest.mark.timeout(300)
def test_count_list_history_on_warm_context():
    """The count pass runs over the tiles the map pass lists (a message whose mapping is not the
    speculated one, or a tile whose fused count could not rule the 255-cap out); its grid comes
    from the previous call's list length.  One warm context alternates batches whose list is
    empty (gradients: the speculation holds), long (runs data: every tile) and mixed — every
    blob equals the oracle's each time."""
    rng = np.random.default_rng(31)
    codec = codec_for(4)
    grads = [gradient(rng, 1 << 20) for _ in range(6)]
    runs = [runs_message(rng, (1 << 20) + 4 * 77, 300) for _ in range(5)]
    for batch in (grads, runs, grads, grads + runs[:2] + [np.zeros(3 << 20, np.uint8)], runs):
        check_batch(batch, codec=codec)


def gradient64(rng, n):
    """float64 gradients (70 % zeros): six high-entropy mantissa bytes and two low-entropy
    sign / exponent bytes per word, so word size 8 takes the speculated mapping 0x3f."""
    x = rng.normal(0, 0.01, n // 8)
    x[rng.random(x.size) < 0.7] = 0
    return x.view(np.uint8)


@pytest.mark.timeout(300)
def test_speculated_mapping_ws8():
    """Word size 8 messages whose mapping IS the speculated [1,1,1,1,1,1,0,0] (the
    ws=8 tests used float32 data, which never produces it): streaming messages (64 KiB up to the
    tile threshold) and tiled ones (above it), every blob against the oracle."""
    rng = np.random.default_rng(88)
    msgs = [gradient64(rng, 96 * 1024), gradient64(rng, 200 * 1024), gradient64(rng, 1 << 20),
            gradient64(rng, (3 << 20) + 8 * 77), gradient64(rng, 16 * 1024)]
    orc = Oracle()
    for m in msgs[:3]:  # (the premise: the speculated mapping is the real one)
        b = orc.encode(m, cfg=orc.config(word_size=8), bandwidth=10.0)
        assert list(np.frombuffer(b[20:52], np.int32)) == [1, 1, 1, 1, 1, 1, 0, 0]
    check_batch(msgs, ws=8)


@pytest.mark.timeout(300)
def test_speculated_tile_recount():
    """A word size 4 gradient above the tile threshold with a long constant stretch: its mapping
    is the speculated one, but the tiles holding the stretch cannot rule the 255-cap out and are
    counted again (kRecount) — the branch ADVICE r04 found untested."""
    rng = np.random.default_rng(44)
    m = gradient(rng, 2 << 20)
    f = m.view(np.float32)
    f[100000:100000 + 60000] = np.float32(0.5)      # 240 KB of one nonzero value: runs >> 255
    f[300000:300003] = np.float32(-0.25)
    m2 = gradient(rng, (1 << 20) + 4096)
    m2.view(np.float32)[5000:9000] = np.float32(1e-3)
    orc = Oracle()
    b = orc.encode(m, cfg=orc.config(), bandwidth=10.0)
    assert list(np.frombuffer(b[20:36], np.int32)) == [1, 1, 1, 0]
    check_batch([m, m2, gradient(rng, 512 * 1024)])
