"""Multi-rank path on CPU: world_size 2 over gloo.

Each rank takes its byte-balanced shard of one batch (psyne_amd.shard), encodes it with the
CPU oracle (test infrastructure, standing in for the GPU codec), and the gathered shards must
equal the single-process encoding byte for byte; the bench's max-over-ranks time and
all-ranks-ok reductions are exercised on the same group."""
import os
import pathlib
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from psyne_amd.shard import all_true, reduce_max, shard_bounds, shard_offsets  # noqa: E402


def _batch():
    rng = np.random.default_rng(41)
    sizes = (64 * np.minimum(rng.zipf(1.5, 300), 256)).astype(np.int64)
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
        from oracle.oracle import Oracle
        orc = Oracle()
        msgs, off = _batch()
        b = shard_bounds(np.diff(off), world)
        mine = [orc.encode(m, bandwidth=10.0) for m in msgs[b[rank]:b[rank + 1]]]
        local_off = shard_offsets(off, b, rank)
        assert local_off[0] == 0 and local_off[-1] == off[b[rank + 1]] - off[b[rank]]
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        t = reduce_max(float(rank + 1))
        ok = all_true(rank == 0)  # rank 1 says False → AND is False
        if rank == 0:
            q.put((gathered, t, ok, b.tolist()))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_balanced():
    sizes = np.array([100, 1, 1, 1, 1, 1, 100, 1, 1000, 1], np.int64)
    for world in (1, 2, 3, 4, 8):
        b = shard_bounds(sizes, world)
        assert b[0] == 0 and b[-1] == sizes.size and np.all(np.diff(b) >= 0)
        per = [int(sizes[b[r]:b[r + 1]].sum()) for r in range(world)]
        assert sum(per) == sizes.sum()
        assert max(per) - min(per) <= sizes.max() + sizes.sum() // world
    assert shard_bounds(np.zeros(5, np.int64), 2).tolist() == [0, 2, 5]


def test_two_rank_gloo_shards_match_single_process():
    from oracle.oracle import Oracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, t, ok, bounds = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 2.0 and ok is False
    msgs, off = _batch()
    orc = Oracle()
    single = [orc.encode(m, bandwidth=10.0) for m in msgs]
    flat = [blob for shard in gathered for blob in shard]
    assert flat == single
    assert bounds[0] == 0 and bounds[-1] == len(msgs) and 0 < bounds[1] < len(msgs)


def test_bench_refuses_world_size_mismatch():
    """bench.py --gpus N must run exactly N ranks: a launch of another size exits non-zero
    before touching a GPU (the driver's SCALE points would be mislabelled otherwise)."""
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=root, env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 2 and "WORLD_SIZE=3" in p.stderr


def test_bench_launcher_never_initialises_hip():
    """`bench.py --gpus N` (the driver's SCALE launch) starts its ranks from a parent that never
    touches HIP: it counts GPUs from the KFD topology, never imports torch, and refuses more GPUs
    than the host has with exit code 2 and a clear message."""
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k != "PSYNE_BENCH_SHARED_DEVICE"}
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "9999"], capture_output=True, text=True,
                       timeout=120, env=env, cwd=str(root))
    assert p.returncode == 2, p.stdout + p.stderr
    assert "--gpus 9999 but only" in p.stderr and "visible GPU" in p.stderr
    probe = ("import sys; sys.argv = ['bench.py', '--gpus', '9999']; import bench; "
             "rc = bench.launch_ranks(bench.parse()); maps = open('/proc/self/maps').read(); "
             "print(rc, 'libamdhip64' in maps, 'torch' in sys.modules, 'psyne_amd' in sys.modules)")
    p = subprocess.run([sys.executable, "-c", probe], capture_output=True, text=True, timeout=120, env=env,
                       cwd=str(root))
    assert p.stdout.split() == ["2", "False", "False", "False"], p.stdout + p.stderr


def test_visible_gpus_and_cpulist_parsing(tmp_path, monkeypatch):
    import bench
    assert bench.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "-1")
    assert bench.visible_gpus() == []


def _fake_sysfs(tmp_path, monkeypatch):
    """The layout a 1-GPU MI355X box showed (gpurun_out/r05_a/topo.txt): two CPU nodes, seven
    GPU nodes this process may not read, one readable GPU node (render minor 160, NUMA node 1)."""
    import bench
    kfd, drm, node = tmp_path / "kfd", tmp_path / "drm", tmp_path / "node"
    for i in range(10):
        d = kfd / str(i)
        d.mkdir(parents=True)
        if i in (0, 1):
            (d / "properties").write_text("cpu_cores_count 128\nsimd_count 0\ndrm_render_minor 0\n")
        elif i == 6:
            (d / "properties").write_text("simd_count 1024\ndrm_render_minor 160\nlocation_id 62464\n"
                                          "unique_id 12784088038668414734\n")
        # other nodes: no readable properties (the box answered EPERM)
    (drm / "renderD160" / "device").mkdir(parents=True)
    (drm / "renderD160" / "device" / "numa_node").write_text("1\n")
    allowed = sorted(os.sched_getaffinity(0))
    (node / "node1").mkdir(parents=True)
    (node / "node1" / "cpulist").write_text("%d-%d\n" % (allowed[0], allowed[-1]))
    monkeypatch.setattr(bench, "KFD_NODES", str(kfd))
    monkeypatch.setattr(bench, "SYSFS_DRM", str(drm))
    monkeypatch.setattr(bench, "SYSFS_NODE", str(node))
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    return bench


def test_visible_gpus_skips_unreadable_nodes(tmp_path, monkeypatch):
    """Round 4's helper gave up on the first unreadable node, so every box run reported numa: null
    (VERDICT r04 item 3): unreadable nodes are skipped, the readable GPU is found, indices and
    UUIDs in the visibility variables select it, and numa_bind binds to its node."""
    bench = _fake_sysfs(tmp_path, monkeypatch)
    g = bench.visible_gpus()
    assert [x["drm_render_minor"] for x in g] == [160]
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert len(bench.visible_gpus()) == 1
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "GPU-%016x" % 12784088038668414734)
    assert len(bench.visible_gpus()) == 1
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "GPU-0123456789abcdef")
    assert bench.visible_gpus() == []
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1")
    assert bench.visible_gpus() == []
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0")
    before = os.sched_getaffinity(0)
    try:
        r = bench.numa_bind(0)
    finally:
        os.sched_setaffinity(0, before)
    assert r == {"numa_node": 1, "bound": True, "cpus": len(before)}
    assert bench.numa_bind(1) is None
