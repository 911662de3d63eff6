"""The slotted batch API never waits on the host (SURVEY.md §8(b) Threading: "calls are async
on a caller hipStream_t") and is capturable into a hipGraph.

The plan kernels' class counts stay in device memory; grids come from an earlier call's counts
plus overflow launches (psyne_amd/csrc/tdt_api.hip, launch_slotted / launch_decode_slotted).
These tests check the observable contract: (1) with a long kernel queued ahead of them, the four
slotted calls return at once and an event recorded after them is still pending; (2) a captured
graph of the four calls replays to the same bytes as the eager calls, for a mixed batch with
large (tiled) messages, small and UNCP ones; (3) capturing on a cold context is refused with
TDT_E_CAPTURE instead of allocating inside the capture; (4) a batch of another shape on a warm
context (its counts exceed the earlier grids) is still exact (overflow launches)."""
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _codec():
    from psyne_amd import TDTConfig, TdtCodec
    c = TdtCodec(TDTConfig(sample_fraction=1.0))
    c.set_metrics(10.0, 1.0, 0.5)
    return c


def _gradient(rng, n):
    x = rng.normal(0, 0.01, n // 4).astype(np.float32)
    x[rng.random(x.size) < 0.7] = 0
    return x.view(np.uint8)


def _mixed(seed):
    rng = np.random.default_rng(seed)
    sizes = [1 << 20, 300 * 1024, 64, 1024, 2048, 4096, 65536, 100000, 1 << 19, 3, 0, 8192 + 4]
    sizes += [int(s) for s in 64 * rng.integers(1, 64, 200)]
    msgs = [_gradient(rng, s) if s % 4 == 0 and s >= 64 else rng.integers(0, 256, s, dtype=np.uint8) for s in sizes]
    off = np.zeros(len(msgs) + 1, np.int64)
    off[1:] = np.cumsum([m.size for m in msgs])
    return np.concatenate(msgs), off


class _Slotted:
    """encode_slots → encode_into → decode_slots → decode_into with preallocated buffers."""

    def __init__(self, codec, data, off):
        self.c, self.d, self.o = codec, data, off
        n = off.numel() - 1
        self.n = n
        ob = off.cpu().numpy()
        cap = int(sum(codec.encode_bound(int(s)) for s in np.diff(ob)))
        dev = data.device
        self.enc = torch.zeros(max(cap, 1), dtype=torch.uint8, device=dev)
        self.eslot = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        self.elen = torch.zeros(n, dtype=torch.int64, device=dev)
        self.est = torch.zeros(n, dtype=torch.int32, device=dev)
        self.dec = torch.zeros(max(int(ob[-1]), 1), dtype=torch.uint8, device=dev)
        self.dslot = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        self.dlen = torch.zeros(n, dtype=torch.int64, device=dev)
        self.dst = torch.zeros(n, dtype=torch.int32, device=dev)

    def run(self):
        from psyne_amd._lib import check
        lib, h = self.c._lib, self.c._h
        sp = torch.cuda.current_stream().cuda_stream
        P = lambda t: t.data_ptr()  # noqa: E731
        check(lib.tdt_encode_slots(h, P(self.o), self.n, P(self.eslot), sp))
        check(lib.tdt_encode_batch_into(h, P(self.d), P(self.o), self.n, P(self.enc), P(self.eslot), P(self.elen),
                                        P(self.est), sp))
        check(lib.tdt_decode_slots(h, P(self.enc), P(self.eslot), P(self.elen), self.n, P(self.dslot), P(self.dst),
                                   sp))
        check(lib.tdt_decode_batch_into(h, P(self.enc), P(self.eslot), P(self.elen), self.n, P(self.dec),
                                        P(self.dslot), P(self.dlen), P(self.dst), sp))

    def blobs(self):
        e, so, ln = self.enc.cpu().numpy(), self.eslot.cpu().numpy(), self.elen.cpu().numpy()
        return [e[so[i]:so[i] + ln[i]].tobytes() for i in range(self.n)]

    def zero(self):
        for t in (self.enc, self.eslot, self.elen, self.est, self.dec, self.dslot, self.dlen, self.dst):
            t.zero_()


def test_slotted_calls_never_wait():
    codec = _codec()
    n, mb = 32768, 65536  # 2 GiB of C3-style messages
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    x = torch.empty(n * mb // 4, dtype=torch.float32, device="cuda").normal_(0, 0.01, generator=g)
    x.masked_fill_(torch.rand(x.numel(), device="cuda", generator=g) < 0.7, 0.0)
    data = x.view(torch.uint8)
    off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * mb
    s = _Slotted(codec, data, off)
    s.run()  # warm: workspaces and the count history exist from here on
    torch.cuda.synchronize()
    assert torch.equal(s.dec, data)
    # a long kernel ahead of the calls: a host that waited on the stream would wait for it too
    torch.cuda._sleep(int(2e8))
    t0 = time.perf_counter()
    s.run()
    host_s = time.perf_counter() - t0
    ev = torch.cuda.Event()
    ev.record()
    pending = not ev.query()
    torch.cuda.synchronize()
    assert pending, "the event after the slotted calls had completed: a call waited on the device"
    assert host_s < 0.05, "slotted calls took %.3f s on the host" % host_s
    assert torch.equal(s.dec, data) and int(s.est.abs().sum()) == 0 and int(s.dst.abs().sum()) == 0
    assert codec.error_flags() == 0


def test_slotted_graph_replay_equals_eager():
    from oracle.oracle import Oracle
    data_h, off_h = _mixed(31)
    data = torch.from_numpy(data_h).cuda()
    off = torch.from_numpy(off_h).cuda()
    codec = _codec()
    s = _Slotted(codec, data, off)
    s.run()
    torch.cuda.synchronize()
    eager = s.blobs()
    orc = Oracle()
    for i in range(s.n):
        m = data_h[off_h[i]:off_h[i + 1]]
        assert eager[i] == orc.encode(m, cfg=orc.config(sample_fraction=1.0), bandwidth=10.0), "message %d" % i
    assert torch.equal(s.dec[: data.numel()], data)
    s.zero()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        s.run()
    gr.replay()
    torch.cuda.synchronize()
    assert s.blobs() == eager
    assert torch.equal(s.dec[: data.numel()], data)
    assert int(s.est.abs().sum()) == 0 and int(s.dst.abs().sum()) == 0


def test_capture_on_cold_context_is_refused():
    from psyne_amd._lib import TDT_E_CAPTURE, TdtError
    data_h, off_h = _mixed(32)
    data = torch.from_numpy(data_h).cuda()
    off = torch.from_numpy(off_h).cuda()
    s = _Slotted(_codec(), data, off)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with pytest.raises(TdtError) as ei:
        with torch.cuda.graph(gr):
            s.run()
    assert ei.value.code == TDT_E_CAPTURE


def test_batches_of_other_shapes_on_a_warm_context():
    """Grids come from the previous batch's counts: a following batch with more small, medium
    and large messages runs through the overflow launches and must be exact.  Every blob of
    every shape is compared with the oracle (round 4 sampled 40: its r04_k1 failure showed only
    as a round-trip mismatch)."""
    from oracle.oracle import Oracle
    orc = Oracle()
    codec = _codec()
    rng = np.random.default_rng(33)
    shapes = [[65536] * 8, [1024] * 3000 + [65536] * 40 + [1 << 20] * 6, [2048] * 50, [600 * 1024] * 12 + [512] * 10]
    for k, sizes in enumerate(shapes):
        msgs = [_gradient(rng, sz) for sz in sizes]
        off_h = np.zeros(len(msgs) + 1, np.int64)
        off_h[1:] = np.cumsum(sizes)
        data_h = np.concatenate(msgs)
        data = torch.from_numpy(data_h).cuda()
        s = _Slotted(codec, data, torch.from_numpy(off_h).cuda())
        s.run()
        torch.cuda.synchronize()
        got = s.blobs()
        cfg = orc.config(sample_fraction=1.0)
        bad = [i for i in range(len(msgs)) if got[i] != orc.encode(msgs[i], cfg=cfg, bandwidth=10.0)]
        assert not bad, (k, len(bad), bad[:8])
        assert torch.equal(s.dec[: data.numel()], data), k
        assert int(s.est.abs().sum()) == 0 and int(s.dst.abs().sum()) == 0
    assert codec.error_flags() == 0


def test_graph_replay_after_workspace_growth():
    """A graph captured on a warm context keeps working after a later eager batch has grown the
    context's workspaces (more large messages than the large-message budget held): grown
    workspaces retire the old buffers instead of freeing them (tdt_api.hip
    ensure_elarge / ensure_dlarge / ensure_plan)."""
    data_h, off_h = _mixed(34)
    data = torch.from_numpy(data_h).cuda()
    off = torch.from_numpy(off_h).cuda()
    codec = _codec()
    s = _Slotted(codec, data, off)
    s.run()
    torch.cuda.synchronize()
    eager = s.blobs()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        s.run()
    # a batch with 1,100 messages of 300 KiB (the starting budget holds 1,024 large messages),
    # twice: the second call grows the large-message and plan workspaces from the first's counts
    rng = np.random.default_rng(35)
    big = [_gradient(rng, 300 * 1024) for _ in range(1100)]
    boff = np.zeros(len(big) + 1, np.int64)
    boff[1:] = np.cumsum([m.size for m in big])
    bdata = torch.from_numpy(np.concatenate(big)).cuda()
    b = _Slotted(codec, bdata, torch.from_numpy(boff).cuda())
    for _ in range(2):
        b.run()
        torch.cuda.synchronize()
        assert torch.equal(b.dec, bdata) and int(b.est.abs().sum()) == 0 and int(b.dst.abs().sum()) == 0
    s.zero()
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    assert s.blobs() == eager
    assert torch.equal(s.dec[: data.numel()], data)
    assert int(s.est.abs().sum()) == 0 and int(s.dst.abs().sum()) == 0
    assert codec.error_flags() == 0
