"""The drop-in boundary against the reference's OWN contracts: compiles
tests/native/ref_concepts.cpp with the reference's include directory (static_asserts on
psyne::concepts::Protocol / ProtocolStack, a TdtSubstrate over a SimpleTCP-shaped
SubstrateBehavior, and an explicit instantiation of psyne's ChannelBridge).  Build container
only: /root/reference does not exist on the GPU box."""
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
REF = pathlib.Path("/root/reference/include")


@pytest.mark.skipif(not REF.is_dir(), reason="reference headers absent (GPU box)")
def test_reference_concepts_compile():
    gxx = shutil.which("g++")
    assert gxx
    r = subprocess.run([gxx, "-std=c++20", "-fsyntax-only", "-I", str(ROOT / "include"), "-I", str(REF),
                        "-I", str(REF / "psyne" / "global"), str(ROOT / "tests" / "native" / "ref_concepts.cpp")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
