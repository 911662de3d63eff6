"""TCP substrate path: PosixTcpSubstrate framing and the
TdtSubstrate decorator, through the loopback harness tests/native/tcp_loopback (C1 counterpart
of the reference's benchmarks/tcp_tdt_benchmark.cpp) and the C++ decorator test
tests/cpp/test_substrate (oversized-claim rejection, per-frame batch statuses)."""
import json
import pathlib
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
BIN = ROOT / "tests" / "native" / "tcp_loopback"
SUBSTRATE_BIN = ROOT / "tests" / "cpp" / "test_substrate"
REF_LIB = ROOT / "oracle" / "_ref" / "libtdt_ref.so"


def run(*args, timeout=120):
    if not BIN.exists():
        pytest.skip("tests/native/tcp_loopback not built (python -m psyne_amd.build)")
    p = subprocess.run([str(BIN), *args], capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr + p.stdout
    return json.loads(p.stdout.strip().splitlines()[-1])


def read_frames(path):
    raw = path.read_bytes()
    frames, i = [], 0
    while i < len(raw):
        n = int.from_bytes(raw[i:i + 4], "little")
        frames.append(raw[i + 4:i + 4 + n])
        i += 4 + n
    return frames


def check_frames_vs_oracle(dump, count, floats):
    """Every wire frame is what the oracle encodes for the corresponding tensor."""
    from oracle.oracle import Oracle
    inputs = np.fromfile(dump / "inputs.bin", np.uint8).reshape(count, floats * 4)
    frames = read_frames(dump / "frames.bin")
    assert len(frames) == count
    orc = Oracle()
    for i in range(count):
        assert frames[i] == orc.encode(inputs[i], bandwidth=10.0), "frame %d" % i


def test_framing_passthrough_loopback():
    # no codec: u32-length frames over 127.0.0.1 (tcp_simple.hpp:68-150), byte-exact
    r = run("--codec", "none", "--count", "64", "--floats", "16384", "--batch", "8", "--port", "18181")
    assert r["mismatches"] == 0 and r["tensors"] == 64
    assert abs(r["compression_ratio"] - 1.0) < 1e-9


def test_framing_passthrough_two_processes():
    # --procs 2: the receiving end in a forked child (its own process, as the far host's end would
    # be); the child's end time and mismatch count come back through a pipe
    r = run("--codec", "none", "--count", "64", "--floats", "16384", "--batch", "8", "--port", "18185",
            "--procs", "2")
    assert r["mismatches"] == 0 and r["tensors"] == 64 and r["procs"] == 2
    assert r["seconds"] > 0


def test_reference_codec_loopback(tmp_path):
    # psyne's own CPU path (the compiled reference protocol) over the same frames; its wire
    # blobs are the oracle's (the oracle is pinned against this library)
    if not REF_LIB.exists():
        pytest.skip("oracle/_ref not built (make -C oracle ref; needs /root/reference)")
    r = run("--codec", "cpu", "--count", "12", "--floats", "16384", "--batch", "4", "--port", "18183",
            "--dump", str(tmp_path))
    assert r["mismatches"] == 0 and r["compression_ratio"] > 1.1
    check_frames_vs_oracle(tmp_path, 12, 16384)


@pytest.mark.gpu
def test_tdt_substrate_gpu_loopback(tmp_path):
    # GPU codec on both ends: batches encoded/decoded by the C-ABI host pipeline, every payload
    # verified by the receiver and every wire frame compared with the oracle
    r = run("--codec", "gpu", "--count", "40", "--floats", "65536", "--batch", "8", "--port", "18182",
            "--dump", str(tmp_path))
    assert r["mismatches"] == 0
    assert r["compression_ratio"] > 1.1  # gradient tensors: ~1.25 (BASELINE C3 ratio)
    check_frames_vs_oracle(tmp_path, 40, 65536)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_tdt_substrate_gpu_loopback_c1_workload(tmp_path):
    """BASELINE configs[0] at its own workload (tcp_tdt_benchmark.cpp:542-543): 1,000 tensors of
    256 Ki float32 (1 MiB) GRADIENTS over loopback TCP through TdtSubstrate on both ends; the
    receiver verifies every payload and every one of the 1,000 wire frames equals the oracle's
    encoding of its tensor."""
    r = run("--codec", "gpu", "--count", "1000", "--floats", str(256 * 1024), "--batch", "50", "--port", "18184",
            "--dump", str(tmp_path), timeout=300)
    assert r["mismatches"] == 0 and r["tensors"] == 1000
    assert r["compression_ratio"] > 1.2
    check_frames_vs_oracle(tmp_path, 1000, 256 * 1024)


@pytest.mark.gpu
def test_tdt_substrate_gpu_loopback_two_processes(tmp_path):
    # each end in its own process with its own GPU codec context (forked before either touches
    # the GPU); every payload verified by the child, every wire frame against the oracle
    r = run("--codec", "gpu", "--count", "40", "--floats", "65536", "--batch", "8", "--port", "18186",
            "--procs", "2", "--dump", str(tmp_path))
    assert r["mismatches"] == 0 and r["procs"] == 2
    assert r["compression_ratio"] > 1.1
    check_frames_vs_oracle(tmp_path, 40, 65536)


@pytest.mark.gpu
def test_tdt_substrate_decorator_cpp():
    # crafted frame claiming 0xFFFFFFF0 decoded bytes rejected before decoding; the connection
    # stays usable; one oversized frame in a batch gets TDT_E_CAPACITY, its neighbours decode
    if not SUBSTRATE_BIN.exists():
        pytest.skip("tests/cpp/test_substrate not built (python -m psyne_amd.build)")
    p = subprocess.run([str(SUBSTRATE_BIN)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "cpp substrate OK" in p.stdout, p.stdout + p.stderr
