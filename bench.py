#!/usr/bin/env python3
"""TDT encode+decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2] = SURVEY.md §8(d) C3): per GPU, 262,144 messages of
64 KiB float32 "gradient-like" payload (70 % exact 0.0f, else N(0, 0.01) — the
GRADIENTS generator of the reference's tdt_compression_benchmark.cpp:52-66), generated on
the device with a fixed seed.  One STEP = tdt_encode_slots + tdt_encode_batch_into over the
whole batch (each blob in its own slot, lengths returned — one vector per message, as the
reference's encode returns) followed by tdt_decode_slots + tdt_decode_batch_into of those
blobs, inputs already resident in HBM.  Compression is on (bandwidth 10 Mbps < 100 Mbps threshold) and the
mapping is computed from every word (the reference's sample_fraction = 1.0, deterministic).

value = payload bytes round-tripped by all ranks / max-over-ranks wall time, in GiB/s.
Multi-GPU: messages are independent, so each rank owns its own batch (weak scaling, no
collective on the data path; the only collectives are the timing barriers/all-reduce).

Extra fields: roofline (dominant kernel, HIP events on the launch stream), cpu_baseline
(the reference codec compiled where it lies, timed on this host), ratio and per-kernel ms.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--msgs", type=int, default=262144)
    ap.add_argument("--msg-bytes", type=int, default=65536)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline duration (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = all usable host cores")
    ap.add_argument("--host-inclusive", action="store_true", help="also time pinned H2D+kernel+D2H")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--workload", choices=["c2", "c3", "c4"], default="c3",
                    help="c3 (default, the BASELINE metric): 262,144 x 64 KiB gradient; c2: 1 Mi x 1 KiB "
                         "uniform bytes; c4: 4 Mi Zipf(1.5)-sized (64 B - 1 MiB) gradient messages")
    a = ap.parse_args()
    if a.workload == "c2":
        a.msgs = a.msgs if a.msgs != 262144 else 1 << 20
        a.msg_bytes = 1024 if a.msg_bytes == 65536 else a.msg_bytes
    if a.workload == "c4" and a.msgs == 262144:
        a.msgs = 1 << 22
    if a.seed is None:
        a.seed = {"c2": 0x5EED0001, "c3": 0x5EED0002, "c4": 0x5EED0003}[a.workload]
    return a


def gen_gradient(torch, n_msgs, msg_bytes, seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    nf = n_msgs * msg_bytes // 4
    x = torch.empty(nf, dtype=torch.float32, device=device)
    chunk = 1 << 28
    for s in range(0, nf, chunk):
        e = min(nf, s + chunk)
        v = torch.empty(e - s, dtype=torch.float32, device=device).normal_(0.0, 0.01, generator=g)
        m = torch.rand(e - s, device=device, generator=g) < 0.7
        v.masked_fill_(m, 0.0)
        x[s:e] = v
        del v, m
    return x.view(torch.uint8)


def gen_uniform(torch, nbytes, seed, device):
    """C2 payloads: uniform random bytes."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=device, generator=g)


def zipf_sizes(n, seed, world=1, rank=0):
    """C4 message sizes: 64 * r, r ~ Zipf(1.5) on [1, 16384] (64 B - 1 MiB); the whole
    job's list is drawn once and each rank takes its byte-balanced shard."""
    import numpy as np
    from psyne_amd.shard import shard_bounds
    rng = np.random.default_rng(seed)
    # truncated Zipf: P(r) ∝ r^-1.5 on [1, 16384] (inverse CDF; mean ≈ 6.3 KB)
    pmf = np.arange(1, 16385, dtype=np.float64) ** -1.5
    cdf = np.cumsum(pmf / pmf.sum())
    r = np.minimum(np.searchsorted(cdf, rng.random(n), side="right") + 1, 16384).astype(np.int64)
    sizes = 64 * r
    b = shard_bounds(sizes, world)
    return sizes[b[rank]:b[rank + 1]]


def load_traffic(config_key):
    """HBM bytes per launch measured with rocprofv3 PMC passes (profiles/*_traffic.json)."""
    best = None
    for p in sorted((ROOT / "profiles").glob("*_traffic.json")):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get("config") == config_key:
            best = d
    return best


def cpu_baseline(data_u8, msg_bytes, target_s, threads):
    """Time the REFERENCE codec (oracle/_ref, compiled from the reference header) on a
    bounded sample of the same messages; fall back to the C restatement if absent."""
    import numpy as np
    from oracle.oracle import Reference, Oracle
    n_sample = 512
    sample = data_u8[: n_sample * msg_bytes].cpu().numpy()
    off = np.arange(n_sample + 1, dtype=np.uint64) * msg_bytes
    if Reference.available():
        ref = Reference()
        # calibrate on 1 thread, then scale reps to ~target_s on `threads` threads
        t1, _ = ref.bench(sample[: 32 * msg_bytes], off[:33], sample_fraction=0.3, threads=1, reps=1)
        per_msg = t1 / 32
        reps = max(1, int(target_s * threads / (per_msg * n_sample)))
        secs, enc = ref.bench(sample, off, sample_fraction=0.3, threads=threads, reps=reps)
        payload = n_sample * msg_bytes * reps
        return dict(value=payload / secs / 2**30, unit="GiB/s", cores=threads, kind="reference",
                    sample="%d x %d B messages x %d reps, reference TDTCompressionProtocol (default "
                           "TDTConfig, sample_fraction 0.3), encode+decode, one object per thread, %.1f s"
                           % (n_sample, msg_bytes, reps, secs),
                    ratio=float(payload / enc))
    orc = Oracle()
    t0 = time.perf_counter()
    reps = 0
    while time.perf_counter() - t0 < target_s:
        for i in range(n_sample):
            b = orc.encode(sample[off[i]:off[i + 1]], bandwidth=10.0)
            orc.decode(b)
        reps += 1
    secs = time.perf_counter() - t0
    return dict(value=n_sample * msg_bytes * reps / secs / 2**30, unit="GiB/s", cores=1, kind="port",
                sample="%d x %d B messages x %d reps, oracle restatement, 1 thread" % (n_sample, msg_bytes, reps))


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from psyne_amd import TDTConfig, TdtCodec

    from psyne_amd.shard import all_true, reduce_max, reduce_sum
    n, mb = a.msgs, a.msg_bytes
    if a.workload == "c4":
        import numpy as np
        sizes = zipf_sizes(n * world, a.seed, world, rank)  # the job's list, this rank's shard
        n = int(sizes.size)
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(sizes)
        payload = int(offs[-1])
        data = gen_gradient(torch, 1, payload, a.seed + rank, dev)  # sizes are multiples of 64
        off = torch.from_numpy(offs).to(dev)
        cap = int(sum(int(s) for s in (2 * sizes + 28 + 16)))  # Σ tdt_encode_bound (ws 4)
        hint = 65536
    else:
        payload = n * mb
        data = (gen_uniform(torch, payload, a.seed + rank, dev) if a.workload == "c2"
                else gen_gradient(torch, n, mb, a.seed + rank, dev))
        off = torch.arange(n + 1, dtype=torch.int64, device=dev) * mb
        hint = mb
    codec = TdtCodec(TDTConfig(sample_fraction=1.0), device=local)
    codec.set_metrics(10.0, 1.0, 0.5)  # slow network → compression on (tdt_compression.hpp:200)
    codec.set_size_hint(hint)
    # Slotted batches (tdt_encode_batch_into / tdt_decode_batch_into): blob i lands in its own
    # slot of the output buffer, as the reference returns one vector per message; the slot
    # offsets (prefix sums of the encode bounds / of the decoded sizes) are computed on the
    # device inside every step.
    if a.workload != "c4":
        cap = n * codec.encode_bound(mb)
    enc = torch.empty(cap, dtype=torch.uint8, device=dev)
    eslot = torch.empty(n + 1, dtype=torch.int64, device=dev)
    elen = torch.empty(n, dtype=torch.int64, device=dev)
    est = torch.empty(n, dtype=torch.int32, device=dev)
    dec = torch.empty(payload, dtype=torch.uint8, device=dev)
    dslot = torch.empty(n + 1, dtype=torch.int64, device=dev)
    dlen = torch.empty(n, dtype=torch.int64, device=dev)
    dst = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    from psyne_amd._lib import check
    lib, h, sp = codec._lib, codec._h, stream.cuda_stream
    P = lambda t: t.data_ptr()

    def step(ev=None):
        if ev:
            ev[0].record(stream)
        check(lib.tdt_encode_slots(h, P(off), n, P(eslot), sp))
        check(lib.tdt_encode_batch_into(h, P(data), P(off), n, P(enc), P(eslot), P(elen), P(est), sp))
        if ev:
            ev[1].record(stream)
        check(lib.tdt_decode_slots(h, P(enc), P(eslot), P(elen), n, P(dslot), P(dst), sp))
        check(lib.tdt_decode_batch_into(h, P(enc), P(eslot), P(elen), n, P(dec), P(dslot), P(dlen), P(dst), sp))
        if ev:
            ev[2].record(stream)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    # correctness of the measured configuration (size-independent property): round trip
    ok = bool(torch.equal(dec, data)) and int(est.abs().sum()) == 0 and int(dst.abs().sum()) == 0
    ok = ok and bool(torch.equal(dslot, off))
    enc_bytes = int(elen.sum().item())

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.steps)]
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(evs[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t_enc = sum(e[0].elapsed_time(e[1]) for e in evs) / a.steps  # ms, encode launch incl. memset
    t_dec = sum(e[1].elapsed_time(e[2]) for e in evs) / a.steps
    elapsed = reduce_max(elapsed, dev)  # whole-job time = the slowest rank
    ok = all_true(ok, dev)
    job_payload = int(reduce_sum(payload, dev))

    ms_per_step = elapsed / a.steps * 1e3
    value = job_payload * a.steps / elapsed / 2**30

    host = None
    if a.host_inclusive and rank == 0 and a.workload != "c4":
        host = host_inclusive(torch, codec, data, off, n, mb)

    if rank == 0:
        alg = payload + enc_bytes  # algorithmic bytes per launch (read input once, write output once)
        dom, t_dom = ("tdt_encode_kernel", t_enc) if t_enc >= t_dec else ("tdt_decode_kernel", t_dec)
        achieved = alg / (t_dom * 1e-3) / 1e9
        key = "%s_%dx%d" % (a.workload, n, mb)
        tr = load_traffic(key) if a.workload == "c3" else None
        traffic = None
        if tr and dom in tr.get("kernels", {}):
            traffic = tr["kernels"][dom].get("hbm_bytes_per_launch")
        cpu = None
        if a.cpu_seconds > 0 and a.workload == "c3":
            thr = a.cpu_threads or min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "1024")))
            cpu = cpu_baseline(data, mb, a.cpu_seconds, thr)
        if a.workload == "c3":
            metric = "TDT encode+decode GiB/s (device-resident), 64 KiB msgs, 1/2/4/8 MI355X"
            workload = "C3: %d x %d B float32 gradient-like messages per GPU, encode+decode" % (n, mb)
            data_desc = "synthetic (device-generated gradient-like float32: 70% zeros, N(0,0.01); seed 0x5EED0002+rank)"
        elif a.workload == "c2":
            metric = "TDT encode+decode GiB/s (device-resident), 1 KiB uniform msgs"
            workload = "C2: %d x %d B uniform random messages per GPU, encode+decode" % (n, mb)
            data_desc = "synthetic (device-generated uniform bytes; seed 0x5EED0001+rank)"
        else:
            metric = "TDT encode+decode GiB/s (device-resident), Zipf 64 B-1 MiB mix"
            workload = ("C4: %d Zipf(1.5)-sized messages (64 B - 1 MiB, %.2f GiB) on this rank of %d, "
                        "gradient-like content, encode+decode" % (n, payload / 2**30, a.msgs * world))
            data_desc = "synthetic (device-generated gradient-like float32; sizes seed 0x5EED0003)"
        line = {
            "metric": metric,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": data_desc,
            "config": {"workload": workload, "msgs_per_gpu": n, "msg_bytes": mb if a.workload != "c4" else None,
                       "word_size": 4, "sample_fraction": 1.0,
                       "bandwidth_mbps": 10.0, "parallelism": "independent message shards (dp%d)" % world},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "algorithmic_bytes_per_launch": alg},
            "kernels_ms": {"encode": round(t_enc, 4), "decode": round(t_dec, 4)},
            "compression_ratio": round(payload / enc_bytes, 4),
            "roundtrip_ok": ok,
            "cpu_baseline": cpu,
        }
        if host:
            line["host_inclusive"] = host
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def host_inclusive(torch, codec, data, off, n, mb, reps=3):
    """The TCP socket-buffer path: pinned host payloads -> tdt_encode_host (chunked, two
    streams: H2D, kernel and D2H of neighbouring chunks overlap) -> pinned host blobs ->
    tdt_decode_host -> pinned host payloads.  GiB/s of payload per direction, best of reps."""
    import ctypes as C
    from psyne_amd._lib import check
    lib, h = codec._lib, codec._h
    m = min(n, 32768)
    src = torch.empty(m * mb, dtype=torch.uint8, pin_memory=True)
    src.copy_(data[: m * mb])
    hoff = torch.arange(m + 1, dtype=torch.int64) * mb
    cap = m * codec.encode_bound(mb)
    henc = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    heoff = torch.empty(m + 1, dtype=torch.int64)
    hst = torch.empty(m, dtype=torch.int32)
    hdec = torch.empty(m * mb, dtype=torch.uint8, pin_memory=True)
    hdoff = torch.empty(m + 1, dtype=torch.int64)
    hdst = torch.empty(m, dtype=torch.int32)
    torch.cuda.synchronize()
    te, td = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        check(lib.tdt_encode_host(h, src.data_ptr(), hoff.data_ptr(), m, henc.data_ptr(), cap, heoff.data_ptr(),
                                  hst.data_ptr()))
        te.append(time.perf_counter() - t0)
        nb = int(heoff[-1])
        t0 = time.perf_counter()
        check(lib.tdt_decode_host(h, henc.data_ptr(), heoff.data_ptr(), m, hdec.data_ptr(), m * mb, hdoff.data_ptr(),
                                  hdst.data_ptr()))
        td.append(time.perf_counter() - t0)
    ok = bool(torch.equal(hdec, src)) and int(hst.abs().sum()) == 0 and int(hdst.abs().sum()) == 0
    b = m * mb
    return {"msgs": m, "encode_GiBps": round(b / min(te) / 2**30, 3), "decode_GiBps": round(b / min(td) / 2**30, 3),
            "roundtrip_GiBps": round(b / (min(te) + min(td)) / 2**30, 3), "encoded_bytes": nb, "ok": ok,
            "note": "pinned host buffers; C-ABI tdt_encode_host/tdt_decode_host: 256 MiB chunks on two streams "
                    "(H2D, kernel, D2H overlapped); payload bytes / wall"}


if __name__ == "__main__":
    main()
