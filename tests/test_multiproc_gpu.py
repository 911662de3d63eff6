"""Multi-rank path through the HIP codec, rehearsed on a one-GPU box.

Two gloo ranks share device 0 (RCCL refuses two ranks on one GPU; the 8-GPU node is the
driver's).  Each rank encodes its byte-balanced shard with the HIP codec (compacted API) and
decodes it back; the gathered blobs must equal the oracle's single-process encoding.  Then
bench.py's N-rank path (barriers, max-over-ranks time, all-gathered per-rank figures) runs
under torch.distributed.run with PSYNE_BENCH_SHARED_DEVICE=1."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from psyne_amd.shard import all_true, reduce_max, shard_bounds, shard_offsets  # noqa: E402

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _batch():
    rng = np.random.default_rng(43)
    sizes = (64 * np.minimum(rng.zipf(1.5, 2000), 1024)).astype(np.int64)
    msgs = []
    for i, n in enumerate(sizes):
        x = rng.normal(0, 0.01, int(n) // 4).astype(np.float32)
        x[rng.random(x.size) < 0.7] = 0
        msgs.append(x.view(np.uint8) if i % 3 else rng.integers(0, 256, int(n), dtype=np.uint8))
    off = np.zeros(len(msgs) + 1, np.int64)
    off[1:] = np.cumsum([m.size for m in msgs])
    return msgs, off


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from psyne_amd import TDTConfig, TdtCodec
        msgs, off = _batch()
        b = shard_bounds(np.diff(off), world)
        lo, hi = int(b[rank]), int(b[rank + 1])
        loff = shard_offsets(off, b, rank)
        buf = np.concatenate(msgs[lo:hi]) if hi > lo else np.zeros(0, np.uint8)
        codec = TdtCodec(TDTConfig(sample_fraction=1.0))
        codec.set_metrics(10.0, 1.0, 0.5)
        d = torch.from_numpy(buf).cuda()
        o = torch.from_numpy(loff).cuda()
        enc, eoff, st = codec.encode_batch(d, o)
        dec, doff, dst = codec.decode_batch(enc, eoff)
        torch.cuda.synchronize()
        ok = (int(st.abs().sum()) == 0 and int(dst.abs().sum()) == 0 and torch.equal(dec[: d.numel()], d)
              and codec.error_flags() == 0)
        e, eo = enc.cpu().numpy(), eoff.cpu().numpy()
        mine = [e[eo[i]:eo[i + 1]].tobytes() for i in range(hi - lo)]
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        t = reduce_max(float(rank + 1))
        ok_all = all_true(ok)
        if rank == 0:
            q.put((gathered, t, ok_all, b.tolist()))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(240)
def test_two_ranks_hip_codec_shards_match_oracle():
    from oracle.oracle import Oracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, t, ok, bounds = q.get(timeout=200)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 2.0 and ok
    msgs, off = _batch()
    orc = Oracle()
    flat = [blob for shard in gathered for blob in shard]
    assert len(flat) == len(msgs)
    for i, m in enumerate(msgs):
        assert flat[i] == orc.encode(m, bandwidth=10.0), "message %d" % i
    assert bounds[0] == 0 and bounds[-1] == len(msgs) and 0 < bounds[1] < len(msgs)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("launcher", ["plain", "torchrun"])
def test_bench_two_ranks_shared_device(launcher):
    """`python bench.py --gpus 2` (what the driver runs) must start two ranks itself; under an
    explicit torch.distributed.run it must join the launched ranks."""
    env = dict(os.environ, PSYNE_BENCH_SHARED_DEVICE="1", OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    args = ["bench.py", "--gpus", "2", "--msgs", "4096", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0"]
    if launcher == "plain":
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=220)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["world_size_observed"] == 2 and r["roundtrip_ok"] is True
    assert [x["rank"] for x in r["per_rank"]] == [0, 1]
    assert all(x["device"]["local_rank"] == 0 for x in r["per_rank"])  # shared-device rehearsal
    assert r["value"] > 0 and r["cpu_baseline"] is None


@pytest.mark.timeout(300)
def test_bench_eight_ranks_shared_device():
    """8-rank rehearsal of the driver's SCALE point: `bench.py --gpus 8`
    starts eight ranks itself; on this one-GPU box they share device 0 (PSYNE_BENCH_SHARED_DEVICE),
    each with its own 4,096-message C3 shard, and rank 0 prints one line with eight per-rank
    entries and a checked round trip.  (The driver's own --gpus 8 run on an 8-GPU node gives each
    rank its own GPU; nothing else differs.)"""
    env = dict(os.environ, PSYNE_BENCH_SHARED_DEVICE="1", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "bench.py", "--gpus", "8", "--msgs", "4096", "--steps", "2", "--warmup", "1",
           "--cpu-seconds", "0", "--compacted-steps", "0"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 8 and r["world_size_observed"] == 8 and r["roundtrip_ok"] is True
    assert [x["rank"] for x in r["per_rank"]] == list(range(8))
    assert r["scaling"] == "weak" and r["value"] > 0


@pytest.mark.timeout(240)
def test_topology_on_the_box():
    """The launcher's topology helpers on a real MI355X box (round 4 reported
    numa: null in every box run): the GPU is found without HIP, numa_bind returns a record, and a
    one-GPU bench.py run reports it in per_rank[0].numa."""
    code = ("import json, bench; g = bench.visible_gpus(); r = bench.numa_bind(0); "
            "print(json.dumps({'n': len(g), 'numa': r}))")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout.strip().splitlines()[-1])
    assert got["n"] >= 1, got
    assert isinstance(got["numa"], dict) and "numa_node" in got["numa"], got
    env = dict(os.environ, OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    env.pop("PSYNE_BENCH_SHARED_DEVICE", None)
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--msgs", "4096", "--steps", "2", "--warmup", "1",
                        "--cpu-seconds", "0", "--compacted-steps", "0"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=220)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert isinstance(r["per_rank"][0]["numa"], dict), r["per_rank"][0]
