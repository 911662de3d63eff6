"""Decode recombine forms (tdt_decode.h make_rec_layout): every word-size-4 mapping's selected
form reproduces the reference's byte order (include/psyne/protocol/tdt_compression.hpp
recombine_byte_streams :615-637) on random stream words.  Host code only:
tests/cpp/test_recombine.cpp built with hipcc, run on the CPU; the GPU parity tests cover the
same forms end to end."""
import pathlib
import re
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
SRC = ROOT / "tests" / "cpp" / "test_recombine.cpp"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not pathlib.Path(HIPCC).exists(), reason="hipcc not available")
def test_recombine_forms_ws4(tmp_path):
    exe = tmp_path / "test_recombine"
    subprocess.check_call([HIPCC, "-std=c++17", "-O1", "-x", "hip", "--offload-arch=gfx950", "-I",
                           str(ROOT / "include"), str(SRC), "-o", str(exe)], timeout=600)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"mismatches (\d+); forms 0-4: (\d+) (\d+) (\d+) (\d+) (\d+)", r.stdout)
    assert m, r.stdout
    forms = [int(x) for x in m.groups()[1:]]
    assert int(m.group(1)) == 0
    assert sum(forms) == 16
    # every specialised form is exercised (12+4, 4+12, 8+8, one stream); none falls back
    assert forms[0] == 0 and all(f > 0 for f in forms[1:]), forms
