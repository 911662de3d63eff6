#!/usr/bin/env python3
"""TDT encode+decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2] = SURVEY.md §8(d) C3): per GPU, 262,144 messages of
64 KiB float32 "gradient-like" payload (70 % exact 0.0f, else N(0, 0.01) — the
GRADIENTS generator of the reference's tdt_compression_benchmark.cpp:52-66), generated on
the device with a fixed seed.  One STEP = tdt_encode_slots + tdt_encode_batch_into over the
whole batch (each blob in its own slot, lengths returned — one vector per message, as the
reference's encode returns) followed by tdt_decode_slots + tdt_decode_batch_into of those
blobs, inputs already resident in HBM.  Compression is on (bandwidth 10 Mbps < 100 Mbps
threshold) and the mapping is computed from every word (the reference's sample_fraction =
1.0, deterministic).  --workload c2 / c4 run the other BASELINE configs (parity-test sizes
for the headline; benched for the record, not as the metric).

value = payload bytes round-tripped by all ranks / max-over-ranks wall time, in GiB/s.
Multi-GPU: messages are independent, so each rank owns its own batch (weak scaling, no
collective on the data path; the only collectives are the timing barriers and the gathers of
the per-rank figures).

Measurement:
  * kernels_ms: HIP events on the launch stream around EACH codec kernel alone (the slot
    kernels are timed separately in slots_ms);
  * roofline: the dominant kernel's algorithmic bytes per launch (Σ n + Σ E: input read once,
    output written once) ÷ its own event time, against the 8 TB/s HBM peak; roofline.combined
    is §8(d)'s 2(n+E) / (t_enc + t_dec);
  * roofline.traffic: HBM bytes per launch from rocprofv3 FETCH/WRITE passes, taken only from a
    profiles/*_traffic.json whose lib_sha256 matches the library being run (else null);
  * cpu_baseline: the reference codec itself (oracle/_ref, compiled from the reference header
    where it lies) on this host: 1 thread and all usable cores, sample_fraction 0.3 (the
    reference default) and 1.0 (parity mode); value = the default-config all-cores row.  A
    missing reference build is an error, not a silent fallback (--cpu-kind port times the C
    restatement instead, labelled as such);
  * host_inclusive (--host-inclusive): pinned host buffers through tdt_encode_host /
    tdt_decode_host, every rank, next to the pinned hipMemcpyAsync H2D / D2H ceiling.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import pathlib
import subprocess
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
    ap.add_argument("--cpu-seconds", type=float, default=3.0,
                    help="target duration of EACH of the four CPU-baseline rows (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the all-cores CPU baseline row (0 = one per physical core of the host)")
    ap.add_argument("--cpu-kind", choices=["reference", "port"], default="reference")
    ap.add_argument("--host-inclusive", action="store_true",
                    help="also time host buffers (pinned and pageable) through H2D+kernel+D2H")
    ap.add_argument("--latency", action="store_true",
                    help="also time one message per call (1 KiB / 64 KiB / 1 MiB) against the reference CPU codec")
    ap.add_argument("--latency-sizes", default="1024,65536,1048576",
                    help="message sizes of the --latency rows (comma-separated bytes)")
    ap.add_argument("--compacted-steps", type=int, default=3,
                    help="timed steps of the compacted (look-back) API leg after the headline (0 = skip)")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default="c3",
                    help="c3 (default, the BASELINE metric): 262,144 x 64 KiB gradient; c2: 1 Mi x 1 KiB "
                         "uniform bytes; c4: 4 Mi Zipf(1.5)-sized (64 B - 1 MiB) gradient messages; c5: "
                         "32 GiB of C3-style messages per GPU (256 GiB at 8 GPUs), host-inclusive leg on")
    a = ap.parse_args()
    if a.workload == "c2":
        a.msgs = a.msgs if a.msgs != 262144 else 1 << 20
        a.msg_bytes = 1024 if a.msg_bytes == 65536 else a.msg_bytes
    if a.workload == "c4" and a.msgs == 262144:
        a.msgs = 1 << 22
    if a.workload == "c5":
        if a.msgs == 262144:
            a.msgs = (32 << 30) // a.msg_bytes  # 32 GiB per GPU
        a.host_inclusive = True
        a.compacted_steps = 0  # (its staging buffer would add 2x the payload again)
    if a.seed is None:
        a.seed = {"c2": 0x5EED0001, "c3": 0x5EED0002, "c4": 0x5EED0003, "c5": 0x5EED0005}[a.workload]
    return a


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# sysfs roots of the topology helpers (tests point them at a fake tree)
KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"
SYSFS_DRM = "/sys/class/drm"
SYSFS_NODE = "/sys/devices/system/node"


def visible_gpus() -> list:
    """The GPUs this process may use, found WITHOUT touching HIP (no torch, no HIP runtime: the
    launcher parent must never initialise the GPU): KFD topology nodes with SIMDs
    (/sys/class/kfd/kfd/topology/nodes/*/properties), in node order (the HIP device order),
    narrowed by ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES.  Each entry
    is that node's properties (drm_render_minor, location_id, ...)."""
    root = pathlib.Path(KFD_NODES)
    gpus = []
    try:
        nodes = sorted(root.iterdir(), key=lambda q: int(q.name) if q.name.isdigit() else 1 << 30)
    except OSError:
        return []
    for d in nodes:
        # A node this process may not read is a GPU it cannot open either (the 1-GPU boxes expose
        # one render node and deny the others' properties): skip it, do not give up on the rest
        # (round 4's helper returned [] there, so numa_bind never ran on a real box).
        try:
            text = (d / "properties").read_text()
        except OSError:
            continue
        props = {}
        for line in text.splitlines():
            f = line.split()
            if len(f) == 2 and f[1].lstrip("-").isdigit():
                props[f[0]] = int(f[1])
        if props.get("simd_count", 0) > 0:
            gpus.append(props)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None or v.strip() == "":
            continue
        sel = []
        for tok in (t.strip() for t in v.split(",")):
            if tok.isdigit():
                i = int(tok)
                if 0 <= i < len(gpus):
                    sel.append(gpus[i])
            elif tok.upper().startswith("GPU-"):
                # UUID form: GPU-<unique_id as 16 hex digits> (rocm-smi / ROCr spelling)
                want = tok[4:].lower()
                sel += [g for g in gpus if "unique_id" in g and ("%016x" % g["unique_id"]) == want.rjust(16, "0")]
        gpus = sel
    return gpus


def parse_cpulist(text: str) -> set:
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def numa_bind(local_rank: int):
    """Bind this rank's threads to the NUMA node of its GPU's PCIe root (before its first GPU
    call), so that its pinned staging and host threads are node-local.  Returns what was done
    (None: no topology information)."""
    gpus = visible_gpus()
    if local_rank >= len(gpus) or "drm_render_minor" not in gpus[local_rank]:
        return None
    minor = gpus[local_rank]["drm_render_minor"]
    try:
        node = int(pathlib.Path(SYSFS_DRM, "renderD%d" % minor, "device", "numa_node").read_text())
    except (OSError, ValueError):
        return None
    if node < 0:
        return {"numa_node": node, "bound": False}
    try:
        cpus = parse_cpulist(pathlib.Path(SYSFS_NODE, "node%d" % node, "cpulist").read_text())
        allowed = os.sched_getaffinity(0) & cpus
        if not allowed:
            return {"numa_node": node, "bound": False}
        os.sched_setaffinity(0, allowed)
    except OSError:
        return {"numa_node": node, "bound": False}
    return {"numa_node": node, "bound": True, "cpus": len(allowed)}


def launch_ranks(a) -> int:
    """`bench.py --gpus N` outside a torch.distributed launch: start N ranks (one process per GPU)
    as a child `torch.distributed.run` and relay its exit code.  This parent never touches HIP:
    it counts GPUs from the KFD topology (visible_gpus) and imports neither torch nor the codec.
    (The child ranks see WORLD_SIZE == N and run main().)"""
    shared = os.environ.get("PSYNE_BENCH_SHARED_DEVICE") == "1"
    if not shared:
        have = len(visible_gpus())
        if have < a.gpus:
            # The topology count is advisory up to one node's worth of GPUs (8): sysfs may hide
            # nodes this process can still use, or be unreadable, so up to 8 ranks start anyway and
            # each checks its own device count (main(): a rank whose LOCAL_RANK has no device exits
            # with status 2).  More than a node's worth beyond what the topology shows is refused.
            if a.gpus > max(have, 8):
                print("bench.py: --gpus %d but only %d visible GPU(s)" % (a.gpus, have), file=sys.stderr, flush=True)
                return 2
            print("bench.py: --gpus %d, the KFD topology shows %d visible GPU(s); starting the ranks, each checks "
                  "its device" % (a.gpus, have), file=sys.stderr, flush=True)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "bench.py")] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "16")
    sys.stdout.flush()
    return subprocess.run(cmd, cwd=str(ROOT), env=env).returncode  # rank 0's JSON line goes to our stdout


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


def lib_sha256() -> str:
    from psyne_amd import _lib
    p = pathlib.Path(os.environ.get("PSYNE_TDT_LIB") or _lib.LIB_PATH)
    return hashlib.sha256(p.read_bytes()).hexdigest()


def load_traffic(config_key, sha, src=None):
    """HBM bytes per launch measured with rocprofv3 PMC passes of THIS library build
    (profiles/**/*traffic.json with a matching lib_sha256, or — hipcc builds are not
    byte-reproducible — with a matching src_sha256: the same kernel sources and build recipe),
    or None."""
    for p in sorted((ROOT / "profiles").glob("**/*traffic.json")):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get("config") == config_key and (d.get("lib_sha256") == sha or (src and d.get("src_sha256") == src)):
            d["_file"] = str(p.relative_to(ROOT))
            return d
    return None


def host_cores():
    """(nproc, physical cores from lscpu) of this host."""
    nproc = os.cpu_count() or 1
    phys = None
    try:
        out = subprocess.run(["lscpu", "-p=CORE,SOCKET"], capture_output=True, text=True, timeout=20).stdout
        cores = {tuple(l.split(",")) for l in out.splitlines() if l and not l.startswith("#")}
        phys = len(cores) or None
    except Exception:
        pass
    return nproc, phys


def affinity_desc():
    """(cpu count, compact list) of this process's CPU affinity mask."""
    cpus = sorted(os.sched_getaffinity(0))
    runs, start = [], None
    for i, c in enumerate(cpus):
        if start is None:
            start = c
        if i + 1 == len(cpus) or cpus[i + 1] != c + 1:
            runs.append("%d-%d" % (start, c) if c > start else "%d" % c)
            start = None
    return len(cpus), ",".join(runs)


def physical_core_cpus():
    """One logical CPU per physical core (lscpu's CORE,SOCKET pairs), within this process's
    affinity: the pinning list of the all-cores CPU baseline."""
    allowed = os.sched_getaffinity(0)
    try:
        out = subprocess.run(["lscpu", "-p=CPU,CORE,SOCKET"], capture_output=True, text=True, timeout=20).stdout
    except Exception:
        return sorted(allowed)
    first = {}
    for line in out.splitlines():
        if not line or line.startswith("#"):
            continue
        f = line.split(",")
        cpu, key = int(f[0]), (f[1], f[2])
        if cpu in allowed and key not in first:
            first[key] = cpu
    return sorted(first.values()) or sorted(allowed)


def cpu_baseline(data_u8, msg_bytes, target_s, threads, kind):
    """CPU rows of the REFERENCE codec (oracle/_ref, the reference header compiled where it lies)
    on bounded samples of the same messages, sample_fraction 0.3 (reference default) and 1.0
    (parity mode), one protocol object per thread: 1 thread, and `threads` workers pinned one per
    physical core (default: every physical core of the host); plus 16-, 32- and
    64-thread rows (16 = the one-GPU box's CPU share).  `value` is the best sample-0.3 row and
    `cores` its thread count.  The multi-thread rows run over 4 GiB of DISTINCT messages
    (no cache-resident working set), repeated to last about 2 s; the 1-thread rows over as many
    distinct messages as take about `target_s`."""
    import numpy as np
    from oracle.oracle import Oracle, Reference
    n_all = data_u8.numel() // msg_bytes
    n_big = min(n_all, max(1, (4 << 30) // msg_bytes))
    sample = data_u8[: n_big * msg_bytes].cpu().numpy()
    off = np.arange(n_big + 1, dtype=np.uint64) * msg_bytes
    nproc, phys = host_cores()
    aff_n, aff = affinity_desc()
    rows = []
    if kind == "reference":
        if not Reference.available():
            raise RuntimeError("cpu_baseline: oracle/_ref/libtdt_ref.so (the compiled reference) is missing; "
                               "build it in the container that has /root/reference (make -C oracle) or pass "
                               "--cpu-kind port")
        ref = Reference()
        cores = physical_core_cpus()
        if threads <= 0:
            threads = len(cores)
        pins = [cores[i % len(cores)] for i in range(threads)] if ref.has_pinned else None
        for sf in (0.3, 1.0):
            t1, _ = ref.bench(sample[: 16 * msg_bytes], off[:17], sample_fraction=sf, threads=1, reps=1)
            per_msg = t1 / 16
            # (sample 0.3: 1 thread, 16 (the one-GPU box's CPU share), 32, 64 and every physical
            # core — the reference stops scaling well before all cores, so the best row is reported)
            thr_list = sorted({1, 16, 32, 64, threads} if sf == 0.3 else {1, threads})
            for thr in (t for t in thr_list if t <= max(threads, 1) or t == 1):
                if thr > 1:
                    k, reps = n_big, 1  # (one pass over 4 GiB: 2.5-3 s on the MI355X box's host)
                    cp = pins if thr == threads else ([cores[i % len(cores)] for i in range(thr)] if pins else None)
                else:
                    k = int(min(n_big, max(16, target_s / per_msg)))
                    reps, cp = 1, None
                secs, enc = ref.bench(sample[: k * msg_bytes], off[: k + 1], sample_fraction=sf, threads=thr,
                                      reps=reps, cpus=cp)
                payload = k * msg_bytes * reps
                rows.append(dict(value=payload / secs / 2**30, unit="GiB/s", cores=thr, sample_fraction=sf,
                                 seconds=round(secs, 2), msgs=k, reps=reps, distinct_bytes=k * msg_bytes,
                                 pinned=cp is not None, ratio=float(payload / enc)))
        # the baseline is the BEST reference configuration measured (default sample 0.3), with its
        # thread count (round 4 reported the all-core row, slower than 16 threads)
        main = max((r for r in rows if r["sample_fraction"] == 0.3), key=lambda r: r["value"])
        return dict(value=main["value"], unit="GiB/s", cores=main["cores"], kind="reference",
                    sample="%d x %d B distinct msgs (first %.1f GiB of the payload) x %d passes; reference "
                           "encode+decode, sample_fraction 0.3, one object per thread, %d threads pinned one per "
                           "physical core (the best of the rows: 1 / 16 / 32 / 64 / all %d physical cores), %.1f s"
                           % (main["msgs"], msg_bytes, main["distinct_bytes"] / 2**30, main["reps"], main["cores"],
                              threads, main["seconds"]),
                    rows=rows, nproc=nproc, lscpu_physical_cores=phys, affinity_cpus=aff_n, affinity_mask=aff)
    orc = Oracle()
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < target_s and k < n_big:
        b = orc.encode(sample[off[k]:off[k + 1]], bandwidth=10.0)
        orc.decode(b)
        k += 1
    secs = time.perf_counter() - t0
    return dict(value=k * msg_bytes / secs / 2**30, unit="GiB/s", cores=1, kind="port",
                sample="%d distinct x %d B messages, oracle C restatement (sample_fraction 1.0), 1 thread"
                       % (k, msg_bytes), nproc=nproc, lscpu_physical_cores=phys, affinity_cpus=aff_n,
                affinity_mask=aff)


def copy_ceiling(torch, dev, nbytes=4 << 30, reps=5):
    """Achievable HBM rate of a device-to-device copy on this box (the
    "achievable stream-copy ceiling" beside the 8 TB/s peak), read + write bytes counted, HIP
    events around `reps` copies of 4 GiB (far past the 256 MiB Infinity Cache): the codec's
    hand-written copy (tdt_copy_device: 64 KiB per 512-lane workgroup, every load in flight before
    the non-temporal stores — the best copy shape of tools/ubench_hbm.hip), which is the reported
    ceiling, and torch copy_ beside it (round 5's figure)."""
    from psyne_amd import _lib
    lib = _lib.load()
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(1)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def hand():
        _lib.check(lib.tdt_copy_device(b.data_ptr(), a.data_ptr(), nbytes, sp))

    def torch_copy():
        b.copy_(a)

    out = {}
    for name, fn in (("hand", hand), ("torch", torch_copy)):
        fn()
        fn()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(reps):
            fn()
        ev[1].record(stream)
        torch.cuda.synchronize(dev)
        out[name] = 2 * nbytes / (ev[0].elapsed_time(ev[1]) / reps * 1e-3) / 1e9
    ok = bool(torch.equal(a[:1 << 20], b[:1 << 20]))
    del a, b
    return {"GBps": round(out["hand"], 1), "torch_copy_GBps": round(out["torch"], 1), "bytes_copied": nbytes,
            "copy_ok": ok,
            "note": "tdt_copy_device (hand-written: 64 KiB pieces, nt stores), read + write bytes / HIP-event "
                    "time, %d reps of 4 GiB; torch copy_ beside it" % reps}


def pcie_ceiling(torch, dev, nbytes=256 << 20, reps=5):
    """Pinned hipMemcpyAsync ceilings (GB/s): H2D alone, D2H alone, and both directions at once
    on two streams — the bound of the host-inclusive pipeline."""
    h_src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d_b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def timed(fn):
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            best = min(best, time.perf_counter() - t0)
        return best

    with torch.cuda.stream(s1):
        h2d = timed(lambda: d_a.copy_(h_src, non_blocking=True))
        d2h = timed(lambda: h_dst.copy_(d_b, non_blocking=True))

    def both():
        with torch.cuda.stream(s1):
            d_a.copy_(h_src, non_blocking=True)
        with torch.cuda.stream(s2):
            h_dst.copy_(d_b, non_blocking=True)
    bi = timed(both)
    return {"h2d_GBps": round(nbytes / h2d / 1e9, 2), "d2h_GBps": round(nbytes / d2h / 1e9, 2),
            "bidir_GBps_each_way": round(nbytes / bi / 1e9, 2), "bytes": nbytes,
            "note": "pinned host <-> device hipMemcpyAsync, best of %d" % reps}


def host_inclusive(torch, codec, data, off, n, mb, reps=3):
    """The TCP socket-buffer path: host payloads -> tdt_encode_host (64 MiB chunks on two
    streams: H2D, kernel and D2H of neighbouring chunks overlap) -> host blobs -> tdt_decode_host
    -> host payloads.  Two callers: PINNED buffers (DMA'd directly) and PAGEABLE ones (numpy
    arrays, as a socket buffer or std::vector is: staged through the context's pinned buffers by
    its copy threads).  GiB/s of payload per direction, best of reps."""
    import numpy as np
    from psyne_amd._lib import check
    lib, h = codec._lib, codec._h
    m = min(n, 32768)
    b = m * mb
    hoff = np.arange(m + 1, dtype=np.uint64) * mb
    cap = m * codec.encode_bound(mb)
    heoff = np.zeros(m + 1, np.uint64)
    hst = np.zeros(m, np.int32)
    hdoff = np.zeros(m + 1, np.uint64)
    hdst = np.zeros(m, np.int32)
    out = {"msgs": m}
    for kind in ("pinned", "pageable"):
        if kind == "pinned":
            t_src = torch.empty(b, dtype=torch.uint8, pin_memory=True)
            t_src.copy_(data[:b])
            t_enc = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
            t_dec = torch.empty(b, dtype=torch.uint8, pin_memory=True)
            src, enc, dec = t_src.numpy(), t_enc.numpy(), t_dec.numpy()
        else:
            src = data[:b].cpu().numpy().copy()
            enc = np.empty(cap, np.uint8)
            dec = np.empty(b, np.uint8)
        enc[:] = 0  # touch the pages (a socket buffer's pages are resident)
        dec[:] = 0
        torch.cuda.synchronize()
        te, td = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            check(lib.tdt_encode_host(h, src.ctypes.data, hoff.ctypes.data, m, enc.ctypes.data, cap,
                                      heoff.ctypes.data, hst.ctypes.data))
            te.append(time.perf_counter() - t0)
            nb = int(heoff[-1])
            t0 = time.perf_counter()
            check(lib.tdt_decode_host(h, enc.ctypes.data, heoff.ctypes.data, m, dec.ctypes.data, b, hdoff.ctypes.data,
                                      hdst.ctypes.data))
            td.append(time.perf_counter() - t0)
        ok = bool(np.array_equal(dec, src)) and int(np.abs(hst).sum()) == 0 and int(np.abs(hdst).sum()) == 0
        out[kind] = {"encode_GiBps": round(b / min(te) / 2**30, 3), "decode_GiBps": round(b / min(td) / 2**30, 3),
                     "roundtrip_GiBps": round(b / (min(te) + min(td)) / 2**30, 3), "encoded_bytes": nb, "ok": ok}
    out["pageable_vs_pinned"] = round(out["pageable"]["roundtrip_GiBps"] / out["pinned"]["roundtrip_GiBps"], 3)
    out["note"] = ("C-ABI tdt_encode_host/tdt_decode_host, %d x %d B; payload bytes / wall; pageable buffers staged "
                   "by %s copy threads" % (m, mb, os.environ.get("PSYNE_TDT_COPY_THREADS", "the default")))
    return out


def message_latency(torch, codec, data, sizes=(1024, 65536, 1 << 20), calls=200):
    """One message per call, as the reference's Protocol::encode / decode are called
    (protocol_demo.cpp:135-189): tdt_encode_host + tdt_decode_host on a pageable buffer (the
    HipTDTCompressionProtocol path), median microseconds per call; beside it the reference codec
    on one host thread (oracle/_ref), microseconds per message, default and parity config."""
    import numpy as np
    from oracle.oracle import Reference
    from psyne_amd._lib import check
    lib, h = codec._lib, codec._h
    ref = Reference() if Reference.available() else None
    rows = []
    for n in sizes:
        src = data[:n].cpu().numpy().copy()
        off = np.array([0, n], np.uint64)
        cap = codec.encode_bound(n)
        enc = np.empty(cap, np.uint8)
        eoff = np.zeros(2, np.uint64)
        dec = np.empty(n, np.uint8)
        doff = np.zeros(2, np.uint64)
        st = np.zeros(1, np.int32)
        te, td = [], []
        for i in range(calls + 5):
            t0 = time.perf_counter()
            check(lib.tdt_encode_host(h, src.ctypes.data, off.ctypes.data, 1, enc.ctypes.data, cap, eoff.ctypes.data,
                                      st.ctypes.data))
            t1 = time.perf_counter()
            check(lib.tdt_decode_host(h, enc.ctypes.data, eoff.ctypes.data, 1, dec.ctypes.data, n, doff.ctypes.data,
                                      st.ctypes.data))
            t2 = time.perf_counter()
            if i >= 5:
                te.append(t1 - t0)
                td.append(t2 - t1)
        row = {"bytes": n, "gpu_encode_us": round(float(np.median(te)) * 1e6, 1),
               "gpu_decode_us": round(float(np.median(td)) * 1e6, 1), "ok": bool(np.array_equal(dec, src))}
        if ref is not None:
            k = max(4, min(256, (64 << 20) // n))
            rep = np.tile(src, k)
            roff = np.arange(k + 1, dtype=np.uint64) * n
            for sf in (0.3, 1.0):
                secs, _ = ref.bench(rep, roff, sample_fraction=sf, threads=1, reps=1)
                row["ref_cpu_us_sf%.1f" % sf] = round(secs / k * 1e6, 1)
        row["gpu_roundtrip_us"] = round(row["gpu_encode_us"] + row["gpu_decode_us"], 1)
        rows.append(row)
    return {"rows": rows, "note": "one message per call: GPU = tdt_encode_host + tdt_decode_host (pageable buffers; "
                                  "H2D, kernel, D2H per call), median of %d; reference = the compiled reference "
                                  "codec, encode+decode per message on one host thread (ref_cpu_us_*)" % calls}


def gather_obj(obj, world):
    import torch.distributed as dist
    if world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (a.gpus, world), file=sys.stderr, flush=True)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # before the first GPU call: this rank's threads on its GPU's NUMA node (pinned staging and
    # copy threads node-local)
    orig_affinity = os.sched_getaffinity(0)
    numa = None if os.environ.get("PSYNE_BENCH_SHARED_DEVICE") == "1" else numa_bind(local)
    import torch
    import torch.distributed as dist

    # PSYNE_BENCH_SHARED_DEVICE=1: rehearsal of the N-rank path on a one-GPU box (every rank on
    # device 0, gloo for the barrier and reductions); never used for a reported number
    shared = os.environ.get("PSYNE_BENCH_SHARED_DEVICE") == "1"
    if shared:
        local = 0
    elif local >= torch.cuda.device_count():
        print("bench.py: rank %d has LOCAL_RANK %d but sees %d GPU(s)" % (rank, local, torch.cuda.device_count()),
              file=sys.stderr, flush=True)
        sys.exit(2)
    if world > 1:
        torch.cuda.set_device(local)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    red = None if shared else dev  # where the reduction tensors live (gloo: host)
    observed_world = dist.get_world_size() if world > 1 else 1
    if observed_world != a.gpus:
        raise SystemExit("bench.py: process group has %d ranks, --gpus %d" % (observed_world, a.gpus))
    props = torch.cuda.get_device_properties(dev)
    my_dev = {"local_rank": local, "name": props.name, "arch": getattr(props, "gcnArchName", ""),
              "pci": "%04x:%02x:%02x" % (getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", 0),
                                          getattr(props, "pci_device_id", 0))}

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
        # events (on the launch stream): [0] slots [1] encode kernel [2] slots [3] decode kernel [4]
        if ev:
            ev[0].record(stream)
        check(lib.tdt_encode_slots(h, P(off), n, P(eslot), sp))
        if ev:
            ev[1].record(stream)
        check(lib.tdt_encode_batch_into(h, P(data), P(off), n, P(enc), P(eslot), P(elen), P(est), sp))
        if ev:
            ev[2].record(stream)
        check(lib.tdt_decode_slots(h, P(enc), P(eslot), P(elen), n, P(dslot), P(dst), sp))
        if ev:
            ev[3].record(stream)
        check(lib.tdt_decode_batch_into(h, P(enc), P(eslot), P(elen), n, P(dec), P(dslot), P(dlen), P(dst), sp))
        if ev:
            ev[4].record(stream)

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(a.steps)]
    for _ in range(a.warmup):
        step()
    # the timed steps follow the warm-up steps directly (no host work in between: an idle gap
    # lets the clocks drop, and the first steps after it run up to 25 % slower)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(evs[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # correctness of the measured configuration (size-independent property): the last timed
    # step's round trip
    ok = bool(torch.equal(dec, data)) and int(est.abs().sum()) == 0 and int(dst.abs().sum()) == 0
    ok = ok and bool(torch.equal(dslot, off - off[0]))
    enc_bytes = int(elen.sum().item())
    avg = lambda i, j: sum(e[i].elapsed_time(e[j]) for e in evs) / a.steps  # ms
    t_enc, t_dec = avg(1, 2), avg(3, 4)
    t_eslot, t_dslot = avg(0, 1), avg(2, 3)
    my_rate = payload * a.steps / elapsed / 2**30
    job_elapsed = reduce_max(elapsed, red)  # whole-job time = the slowest rank
    ok = all_true(ok, red)
    job_payload = int(reduce_sum(payload, red))
    ms_per_step = job_elapsed / a.steps * 1e3
    value = job_payload * a.steps / job_elapsed / 2**30

    # Compacted API leg (tdt_encode_batch / tdt_decode_batch: blobs and decoded messages packed
    # in message order, offsets by the kernels' decoupled look-back — the north_star's
    # variable-length output compaction), on the same batch after the timed loop; reported
    # beside the headline, never as `value`.  Reuses the slotted buffers.
    compacted = None
    if a.compacted_steps > 0:
        coff = torch.empty(n + 1, dtype=torch.int64, device=dev)
        cdoff = torch.empty(n + 1, dtype=torch.int64, device=dev)

        def cstep(ev=None):
            if ev:
                ev[0].record(stream)
            check(lib.tdt_encode_batch(h, P(data), P(off), n, P(enc), cap, P(coff), P(est), sp))
            if ev:
                ev[1].record(stream)
            check(lib.tdt_decode_batch(h, P(enc), P(coff), n, P(dec), payload, P(cdoff), P(dst), sp))
            if ev:
                ev[2].record(stream)

        cstep()
        torch.cuda.synchronize(dev)
        cok = bool(torch.equal(dec, data)) and int(est.abs().sum()) == 0 and int(dst.abs().sum()) == 0
        cok = cok and int(coff[-1].item()) == enc_bytes and bool(torch.equal(cdoff, off - off[0]))
        cev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.compacted_steps)]
        for k in range(a.compacted_steps):
            cstep(cev[k])
        torch.cuda.synchronize(dev)
        c_enc = sum(e[0].elapsed_time(e[1]) for e in cev) / a.compacted_steps
        c_dec = sum(e[1].elapsed_time(e[2]) for e in cev) / a.compacted_steps
        compacted = {"api": "tdt_encode_batch / tdt_decode_batch (outputs compacted in message order; encode: one "
                            "pass with decoupled look-back for messages <= 64 KiB averaging >= 16 KiB, else "
                            "slotted kernels + scan of the lengths + gather; decode: sizes + scan, then the "
                            "slotted kernels in place)",
                     "steps": a.compacted_steps, "encode_ms": round(c_enc, 4), "decode_ms": round(c_dec, 4),
                     "GiBps_kernels": round(payload / ((c_enc + c_dec) * 1e-3) / 2**30, 3),
                     "roundtrip_ok": cok, "blob_bytes_equal_slotted": int(coff[-1].item()) == enc_bytes}

    host = None
    if a.host_inclusive and a.workload != "c4":
        host = host_inclusive(torch, codec, data, off, n, mb)
        host["pcie_ceiling"] = pcie_ceiling(torch, dev)
    latency = (message_latency(torch, codec, data, sizes=[int(x) for x in a.latency_sizes.split(",")])
               if a.latency and rank == 0 else None)
    per_rank = gather_obj({"rank": rank, "device": my_dev, "numa": numa, "msgs": n, "payload_bytes": payload,
                           "GiBps": round(my_rate, 3), "kernels_ms": [round(t_enc, 4), round(t_dec, 4)],
                           "host_inclusive": host}, world)

    if rank == 0:
        alg = payload + enc_bytes  # algorithmic bytes per launch (read input once, write output once)
        dom, t_dom = ("tdt_encode_kernel", t_enc) if t_enc >= t_dec else ("tdt_decode_kernel", t_dec)
        achieved = alg / (t_dom * 1e-3) / 1e9
        combined = 2 * alg / ((t_enc + t_dec) * 1e-3) / 1e9
        key = "%s_%dx%d" % (a.workload, n, mb)
        sha = lib_sha256()
        from psyne_amd import _lib
        from psyne_amd.srchash import recorded
        # the source hash the build recorded beside the library (a variant without one: its sha only)
        src = recorded(pathlib.Path(os.environ.get("PSYNE_TDT_LIB") or _lib.LIB_PATH))
        tr = load_traffic(key, sha, src)
        traffic = tr["kernels"][dom].get("hbm_bytes_per_launch") if tr and dom in tr.get("kernels", {}) else None
        ceil = copy_ceiling(torch, dev)  # (after the timed region; rank 0)
        cpu = None
        if a.cpu_seconds > 0 and a.workload == "c3" and world == 1:  # rank 0 at N=1 only
            if orig_affinity:
                os.sched_setaffinity(0, orig_affinity)  # the whole host, not the GPU's NUMA node
            cpu = cpu_baseline(data, mb, a.cpu_seconds, a.cpu_threads, a.cpu_kind)
        if a.workload == "c3":
            metric = "TDT encode+decode GiB/s (device-resident), 64 KiB msgs, 1/2/4/8 MI355X"
            workload = "C3: %d x %d B float32 gradient-like messages per GPU, encode+decode" % (n, mb)
            data_desc = "synthetic (device-generated gradient-like float32: 70% zeros, N(0,0.01); seed 0x5EED0002+rank)"
        elif a.workload == "c5":
            metric = "TDT encode+decode GiB/s (device-resident), 64 KiB msgs, 32 GiB per GPU stream"
            workload = ("C5: %d x %d B (%.1f GiB) C3-style gradient messages per GPU, %.1f GiB job, encode+decode"
                        % (n, mb, payload / 2**30, job_payload / 2**30))
            data_desc = ("synthetic (device-generated gradient-like float32, resident in HBM: %.0f GB per GPU "
                         "incl. slots; seed 0x5EED0005+rank)" % ((payload * 2 + cap) / 1e9))
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
            "world_size_observed": observed_world,
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
                         "traffic_source": tr["_file"] if traffic is not None else
                         "no PMC record for this library build (lib sha256 %s)" % sha[:16],
                         "algorithmic_bytes_per_launch": alg,
                         "copy_ceiling": ceil, "frac_of_copy_ceiling": round(achieved / ceil["GBps"], 4),
                         "combined": {"achieved": round(combined, 2), "frac": round(combined / HBM_PEAK_GBS, 4),
                                      "def": "2(n+E) / (t_enc + t_dec), SURVEY.md 8(d)"}},
            "kernels_ms": {"encode": round(t_enc, 4), "decode": round(t_dec, 4)},
            "slots_ms": {"encode_slots": round(t_eslot, 4), "decode_slots": round(t_dslot, 4)},
            "lib_sha256": sha[:16],
            "src_sha256": src[:16] if src else None,
            "compression_ratio": round(payload / enc_bytes, 4) if enc_bytes else None,
            "roundtrip_ok": ok,
            "per_rank": per_rank,
            "cpu_baseline": cpu,
        }
        if compacted:
            line["compacted"] = compacted
        if host:
            line["host_inclusive"] = host
        if latency:
            line["message_latency"] = latency
        if shared:
            line["rehearsal"] = "all ranks on device 0 over gloo (PSYNE_BENCH_SHARED_DEVICE=1): not a scaling number"
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
