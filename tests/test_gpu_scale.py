"""GPU parity at BASELINE sizes: the HIP codec through the C ABI against
the C oracle (pinned by tests/golden/) on the full C2, C3 and C4 bench batches, on 100 k mixed
messages, and on
single messages up to SimpleTCP's 100 MB frame cap (tcp_simple.hpp:127-134) at several
alignments.  Bit-exact: byte/integer work with a bit-exact restated entropy decision."""
import numpy as np
import pytest

from oracle.oracle import Oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"


def make_codec():
    from psyne_amd import TDTConfig, TdtCodec
    c = TdtCodec(TDTConfig(sample_fraction=1.0))
    c.set_metrics(10.0, 1.0, 0.5)  # bandwidth < 100 Mbps: compression on
    return c


def valid_mask(slot, lens, total):
    """Bytes [slot[i], slot[i] + lens[i]) of a slotted buffer of `total` bytes."""
    d = np.zeros(total + 1, np.int32)
    np.add.at(d, slot[:-1].astype(np.int64), 1)
    np.add.at(d, (slot[:-1] + lens).astype(np.int64), -1)
    return np.cumsum(d[:-1]) > 0


def check_slotted(codec, data, off, chunk=131072):
    """Encode the batch on the GPU into slots, compare every blob with the oracle (threaded,
    chunked), then decode the GPU blobs back and compare with the input on the device."""
    orc = Oracle()
    n = off.numel() - 1
    out, slots, lens, st = codec.encode_into(data, off)
    torch.cuda.synchronize()
    assert int(st[:n].abs().sum()) == 0
    offh = off.cpu().numpy().astype(np.uint64)
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        a, b = int(offh[c0]), int(offh[c1])
        host = data[a:b].cpu().numpy()
        want, wslot, wlen = orc.encode_slotted(host, offh[c0:c1 + 1] - offh[c0], bandwidth=10.0)
        glen = lens[c0:c1].cpu().numpy().astype(np.uint64)
        assert np.array_equal(glen, wlen), "blob lengths differ in chunk %d" % c0
        s0, s1 = int(slots[c0].item()), int(slots[c1].item())
        got = out[s0:s1].cpu().numpy()
        gslot = slots[c0:c1 + 1].cpu().numpy().astype(np.uint64) - np.uint64(s0)
        assert np.array_equal(gslot, wslot), "slot layout differs"
        m = valid_mask(wslot, wlen, int(wslot[-1]))
        assert np.array_equal(got[m], want[: m.size][m]), "blob bytes differ in chunk %d" % c0
    back, dsl, dln, dst = codec.decode_into(out, slots, in_lengths=lens)
    torch.cuda.synchronize()
    assert int(dst[:n].abs().sum()) == 0
    assert torch.equal(back[: int(offh[-1] - offh[0])], data[int(offh[0]):int(offh[-1])])


@pytest.mark.timeout(600)
def test_c2_full_batch_bitexact():
    """BASELINE configs[1] as bench.py --workload c2 runs it: 1,048,576 x 1 KiB uniform random
    payloads generated on the device (seed 0x5EED0001), every blob compared with the oracle."""
    import bench
    n = 1 << 20
    data = bench.gen_uniform(torch, n * 1024, 0x5EED0001, torch.device("cuda"))
    off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * 1024
    check_slotted(make_codec(), data, off)


@pytest.mark.timeout(900)
def test_c3_full_batch_bitexact():
    """The headline batch (BASELINE configs[2], bench.py's default): 262,144 x 64 KiB
    gradient-like float32 messages generated on the device as bench.py does (seed 0x5EED0002),
    16 GiB; every blob of the slotted encode compared byte for byte with the oracle's (chunks of
    8,192 messages), then the whole batch decoded back on the device."""
    import bench
    n, mb = 262144, 65536
    data = bench.gen_gradient(torch, n, mb, 0x5EED0002, torch.device("cuda"))
    off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * mb
    codec = make_codec()
    out, slots, lens, st = codec.encode_into(data, off)
    torch.cuda.synchronize()
    assert int(st[:n].abs().sum()) == 0
    orc = Oracle()
    sl = slots.cpu().numpy().astype(np.int64)
    ln = lens[:n].cpu().numpy().astype(np.int64)
    chunk = 8192
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        host = data[c0 * mb:c1 * mb].cpu().numpy()
        want, wslot, wlen = orc.encode_slotted(host, np.arange(c1 - c0 + 1, dtype=np.uint64) * mb, bandwidth=10.0)
        assert np.array_equal(ln[c0:c1], wlen.astype(np.int64)), "blob lengths differ in chunk %d" % c0
        got = out[int(sl[c0]):int(sl[c1])].cpu().numpy()
        gs = sl[c0:c1] - sl[c0]
        ws = wslot.astype(np.int64)
        for i in range(c1 - c0):
            L, a, b = int(ln[c0 + i]), int(gs[i]), int(ws[i])
            assert np.array_equal(got[a:a + L], want[b:b + L]), "blob %d differs" % (c0 + i)
    back, dsl, dln, dst = codec.decode_into(out, slots, in_lengths=lens)
    torch.cuda.synchronize()
    assert int(dst[:n].abs().sum()) == 0
    assert torch.equal(back[:n * mb], data)


@pytest.mark.timeout(900)
def test_c4_full_batch_bitexact():
    """The C4 bench batch itself (bench.py --workload c4): 4 Mi messages of Zipf(1.5) sizes
    64 B - 1 MiB (24.6 GiB, every message class), gradient-like data from the bench's generator
    and seed; every blob byte for byte against the oracle (chunks of 262,144 messages, blob by
    blob), then the whole batch decoded back on the device."""
    import bench
    sizes = bench.zipf_sizes(1 << 22, 0x5EED0003)
    off = np.zeros(sizes.size + 1, np.int64)
    off[1:] = np.cumsum(sizes)
    data = bench.gen_gradient(torch, 1, int(off[-1]), 0x5EED0003, torch.device("cuda"))
    n = sizes.size
    codec = make_codec()
    doff = torch.from_numpy(off).cuda()
    out, slots, lens, st = codec.encode_into(data, doff)
    torch.cuda.synchronize()
    assert int(st[:n].abs().sum()) == 0
    orc = Oracle()
    sl = slots.cpu().numpy().astype(np.int64)
    ln = lens[:n].cpu().numpy().astype(np.int64)
    chunk = 262144
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        host = data[int(off[c0]):int(off[c1])].cpu().numpy()
        want, wslot, wlen = orc.encode_slotted(host, (off[c0:c1 + 1] - off[c0]).astype(np.uint64), bandwidth=10.0)
        assert np.array_equal(ln[c0:c1], wlen.astype(np.int64)), "blob lengths differ in chunk %d" % c0
        got = out[int(sl[c0]):int(sl[c1])].cpu().numpy()
        gs = sl[c0:c1] - sl[c0]
        ws = wslot.astype(np.int64)
        for i in range(c1 - c0):
            L, a, b = int(ln[c0 + i]), int(gs[i]), int(ws[i])
            assert np.array_equal(got[a:a + L], want[b:b + L]), "blob %d differs" % (c0 + i)
    back, dsl, dln, dst = codec.decode_into(out, slots, in_lengths=lens)
    torch.cuda.synchronize()
    assert int(dst[:n].abs().sum()) == 0
    assert torch.equal(back[:int(off[-1])], data)


@pytest.mark.timeout(900)
def test_c5_per_rank_batch_bitexact():
    """BASELINE configs[4] (C5) at ONE rank's size, as bench.py --workload c5 generates it: 524,288 x
    64 KiB (32 GiB) gradient-like messages per GPU (seed 0x5EED0005 + rank 0).  Input offsets run to
    32 GiB and slot offsets past 64 GiB, where offset-width bugs live (round 3 found one past 2 GiB).
    The whole batch is encoded slotted and decoded back on the device; the blobs of the first and
    last 8,192 messages and of 8,192 random ones in between are compared byte for byte with the
    oracle's."""
    import bench
    n, mb = 524288, 65536
    data = bench.gen_gradient(torch, n, mb, 0x5EED0005, torch.device("cuda"))
    off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * mb
    codec = make_codec()
    out, slots, lens, st = codec.encode_into(data, off)
    torch.cuda.synchronize()
    assert int(st[:n].abs().sum()) == 0
    sl = slots.cpu().numpy().astype(np.int64)
    ln = lens[:n].cpu().numpy().astype(np.int64)
    assert sl[n - 1] > (64 << 30) and int(sl[n]) <= out.numel()
    orc = Oracle()
    rng = np.random.default_rng(0xC5)
    mid = np.sort(rng.choice(np.arange(8192, n - 8192), 8192, replace=False))
    for idx in (np.arange(8192), np.arange(n - 8192, n), mid):
        ti = torch.from_numpy(idx).cuda()
        host = data.view(n, mb).index_select(0, ti).cpu().numpy().reshape(-1)
        want, wslot, wlen = orc.encode_slotted(host, np.arange(idx.size + 1, dtype=np.uint64) * mb, bandwidth=10.0)
        assert np.array_equal(ln[idx], wlen.astype(np.int64)), "blob lengths differ"
        # the GPU blobs of these messages, gathered on the device into one buffer
        got = torch.cat([out[int(sl[i]):int(sl[i]) + int(ln[i])] for i in idx]).cpu().numpy()
        g = 0
        for k, i in enumerate(idx):
            L, w = int(ln[i]), int(wslot[k])
            assert np.array_equal(got[g:g + L], want[w:w + L]), "blob %d differs" % i
            g += L
    back, dsl, dln, dst = codec.decode_into(out, slots, in_lengths=lens)
    torch.cuda.synchronize()
    assert int(dst[:n].abs().sum()) == 0
    assert torch.equal(back[:n * mb], data)


@pytest.mark.timeout(600)
def test_c4_zipf_full_range_bitexact():
    """C4's size distribution over its FULL range (bench.zipf_sizes: 64 B - 1 MiB, Zipf(1.5),
    the C4 seed) on 500,000 messages (~3 GiB, every message class incl. the tiled > 256 KiB
    path), gradient-like content generated on the device as bench.py --workload c4 does; every
    blob of the slotted batch compared with the oracle, then decoded back."""
    import bench
    sizes = bench.zipf_sizes(500_000, 0x5EED0003)
    assert sizes.max() > (256 << 10) and sizes.min() == 64  # the tiled and the UNCP classes occur
    off = np.zeros(sizes.size + 1, np.int64)
    off[1:] = np.cumsum(sizes)
    data = bench.gen_gradient(torch, 1, int(off[-1]), 0x5EED0003, torch.device("cuda"))
    check_slotted(make_codec(), data, torch.from_numpy(off).cuda(), chunk=65536)


@pytest.mark.timeout(300)
def test_mid_class_slotted():
    """The 256-lane class (4 KiB < n <= 32 KiB) beside its neighbours: 3,000 messages of every
    size around the class bounds and inside it (multiples of 4 and not, so most start
    unaligned: the streaming body), gradient-like and uniform, every slotted blob compared with
    the oracle, then decoded back."""
    rng = np.random.default_rng(61)
    edges = [4092, 4096, 4100, 4104, 8192, 16380, 16384, 16388, 32764, 32768, 32772, 32776, 65536]
    sizes = np.concatenate([np.array(edges * 40, np.int64), rng.integers(4097, 32769, 2480)])
    rng.shuffle(sizes)
    off = np.zeros(sizes.size + 1, np.int64)
    off[1:] = np.cumsum(sizes)
    buf = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    for i in range(0, sizes.size, 2):
        k = int(sizes[i]) // 4
        x = rng.normal(0, 0.01, k).astype(np.float32)
        x[rng.random(k) < 0.7] = 0
        buf[off[i]:off[i] + 4 * k] = x.view(np.uint8)
    check_slotted(make_codec(), torch.from_numpy(buf).cuda(), torch.from_numpy(off).cuda())


@pytest.mark.timeout(300)
def test_100k_mixed_vs_oracle():
    """100,000 messages of 64 B - 8 KiB (UNCP below 1 KiB), half uniform bytes, half
    gradient-like float32, every blob compared with the oracle."""
    rng = np.random.default_rng(51)
    n = 100_000
    sizes = rng.integers(1, 129, n) * 64
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(sizes)
    buf = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    for i in range(0, n, 2):  # gradient-like content in every other message
        k = int(sizes[i]) // 4
        x = rng.normal(0, 0.01, k).astype(np.float32)
        x[rng.random(k) < 0.7] = 0
        buf[off[i]:off[i + 1]] = x.view(np.uint8)
    check_slotted(make_codec(), torch.from_numpy(buf).cuda(), torch.from_numpy(off).cuda())


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n,lead", [(16 << 20, 0), (16 << 20, 1), (16 << 20, 3), (16 << 20, 8),
                                    (100 * 1024 * 1024, 0), (100 * 1024 * 1024, 3)])
def test_large_message(n, lead):
    """One message of 16 MiB or 100 MB (SimpleTCP's frame cap, tcp_simple.hpp:127-134) at a
    misaligned start, between two small neighbours: compacted encode (look-back) and decode."""
    rng = np.random.default_rng(n % 1000 + lead)
    k = n // 4
    x = rng.normal(0, 0.01, k).astype(np.float32)
    x[rng.random(k) < 0.7] = 0
    big = x.view(np.uint8)
    small = [rng.integers(0, 256, 4096, dtype=np.uint8), rng.integers(0, 4, 2048, dtype=np.uint8)]
    msgs = [small[0], big, small[1]]
    off = np.zeros(4, np.int64)
    off[0] = lead
    for i, m in enumerate(msgs):
        off[i + 1] = off[i] + m.size
    buf = np.zeros(int(off[-1]), np.uint8)
    for i, m in enumerate(msgs):
        buf[off[i]:off[i + 1]] = m
    codec = make_codec()
    d, o = torch.from_numpy(buf).cuda(), torch.from_numpy(off).cuda()
    enc, eoff, st = codec.encode_batch(d, o)
    torch.cuda.synchronize()
    assert int(st[:3].abs().sum()) == 0
    e, eo = enc.cpu().numpy(), eoff.cpu().numpy()
    orc = Oracle()
    for i, m in enumerate(msgs):
        assert e[eo[i]:eo[i + 1]].tobytes() == orc.encode(m, bandwidth=10.0), "message %d" % i
    dec, doff, dst = codec.decode_batch(enc, eoff)
    torch.cuda.synchronize()
    assert int(dst[:3].abs().sum()) == 0
    assert torch.equal(dec[: int(off[-1] - off[0])], d[int(off[0]):])


@pytest.mark.timeout(300)
def test_host_pipeline_multichunk():
    """tdt_encode_host / tdt_decode_host (pageable caller buffers: pinned staging) on a batch of
    ~600 MB of messages <= 64 KiB, so the one-pass encode runs over ten 64 MiB chunks rotating
    through the four pipeline slots: every blob equals the oracle's, the decode restores the input,
    and no chunk raised a device flag."""
    rng = np.random.default_rng(77)
    sizes = np.concatenate([rng.integers(1, 65, 2000) * 64, np.full(9000, 65536, np.int64)])
    rng.shuffle(sizes)
    off = np.zeros(sizes.size + 1, np.uint64)
    off[1:] = np.cumsum(sizes)
    x = rng.normal(0, 0.01, int(off[-1]) // 4).astype(np.float32)
    x[rng.random(x.size) < 0.7] = 0
    buf = x.view(np.uint8)
    codec = make_codec()
    enc, eoff, st = codec.encode_host(buf, off)
    assert int(np.abs(st).sum()) == 0
    orc = Oracle()
    idx = np.concatenate([np.arange(50), rng.choice(sizes.size, 400, replace=False), np.arange(sizes.size - 50, sizes.size)])
    for i in idx:
        assert enc[eoff[i]:eoff[i + 1]].tobytes() == orc.encode(buf[off[i]:off[i + 1]], bandwidth=10.0), "blob %d" % i
    dec, doff, dst = codec.decode_host(enc, eoff, int(off[-1]))
    assert int(np.abs(dst).sum()) == 0
    assert np.array_equal(doff, off) and np.array_equal(dec, buf)
    assert codec.error_flags() == 0


@pytest.mark.timeout(300)
def test_host_pipeline_slotted_pinned():
    """A socket-sized batch of 1 MiB messages (the C1 substrate's send_batch) through the host
    pipeline: messages over 64 KiB take the slotted class kernels (tiles) and the gather straight
    into the host buffer.  Pinned caller buffers (direct DMA, output written by the gather kernel
    through the mapped pointer) and pageable ones (staging) give the same blobs, equal to the
    oracle's; both decode back; a too-small output buffer is TDT_E_CAPACITY."""
    import ctypes as C
    from psyne_amd._lib import TDT_E_CAPACITY, check
    rng = np.random.default_rng(123)
    sizes = np.array([1 << 20] * 40 + list(rng.integers(1, 256, 60) * 64) + [3 << 20, 4, 65536 + 64], np.int64)
    rng.shuffle(sizes)
    off = np.zeros(sizes.size + 1, np.uint64)
    off[1:] = np.cumsum(sizes)
    x = rng.normal(0, 0.01, int(off[-1]) // 4).astype(np.float32)
    x[rng.random(x.size) < 0.7] = 0
    buf = x.view(np.uint8)
    codec = make_codec()
    enc, eoff, st = codec.encode_host(buf, off)  # pageable
    assert int(np.abs(st).sum()) == 0
    orc = Oracle()
    for i in list(range(6)) + list(range(sizes.size - 6, sizes.size)) + [int(np.argmax(sizes))]:
        assert enc[eoff[i]:eoff[i + 1]].tobytes() == orc.encode(buf[off[i]:off[i + 1]], bandwidth=10.0), "blob %d" % i
    n = sizes.size
    cap = int(sum(codec.encode_bound(int(s)) for s in sizes))
    pin_in = torch.from_numpy(buf).pin_memory()
    pin_out = torch.empty(cap, dtype=torch.uint8).pin_memory()
    poff = np.zeros(n + 1, np.uint64)
    pst = np.zeros(n, np.int32)
    check(codec._lib.tdt_encode_host(codec._h, pin_in.data_ptr(), off.ctypes.data, n, pin_out.data_ptr(), cap,
                                     poff.ctypes.data, pst.ctypes.data))
    assert int(np.abs(pst).sum()) == 0 and np.array_equal(poff, eoff)
    assert np.array_equal(pin_out[: int(poff[-1])].numpy(), enc[: int(eoff[-1])])
    dec, doff, dst = codec.decode_host(enc, eoff, int(off[-1]))
    assert int(np.abs(dst).sum()) == 0 and np.array_equal(doff, off) and np.array_equal(dec, buf)
    pin_dec = torch.empty(int(off[-1]), dtype=torch.uint8).pin_memory()
    doff2 = np.zeros(n + 1, np.uint64)
    dst2 = np.zeros(n, np.int32)
    check(codec._lib.tdt_decode_host(codec._h, pin_out.data_ptr(), poff.ctypes.data, n, pin_dec.data_ptr(),
                                     int(off[-1]), doff2.ctypes.data, dst2.ctypes.data))
    assert int(np.abs(dst2).sum()) == 0 and np.array_equal(doff2, off)
    assert torch.equal(pin_dec, pin_in)
    small = np.empty(int(eoff[-1]) // 2, np.uint8)
    r = codec._lib.tdt_encode_host(codec._h, buf.ctypes.data, off.ctypes.data, n, small.ctypes.data, small.size,
                                   poff.ctypes.data, pst.ctypes.data)
    assert r == TDT_E_CAPACITY
    assert codec.error_flags() == 0
