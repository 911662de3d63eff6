"""CPU-side checks of the C ABI boundary: the gfx950 library loads on a GPU-less host and
exports every function include/psyne_tdt.h declares (no compute calls here)."""
import pathlib
import re

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def declared_functions():
    src = (ROOT / "include" / "psyne_tdt.h").read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tdt_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_surface():
    names = declared_functions()
    for n in ("tdt_ctx_create", "tdt_encode_batch", "tdt_decode_batch", "tdt_encode_with_mapping_batch",
              "tdt_analyze_batch", "tdt_encode_bound", "tdt_last_error"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from psyne_amd import _lib
    if not _lib.LIB_PATH.exists():
        pytest.skip("libpsyne_tdt.so not built (run __graft_entry__.build())")
    lib = _lib.load()
    for n in declared_functions():
        assert hasattr(lib, n), n
    assert set(declared_functions()) == set(_lib.SIGNATURES)


def test_host_only_entry_points():
    from psyne_amd import _lib
    if not _lib.LIB_PATH.exists():
        pytest.skip("libpsyne_tdt.so not built")
    lib = _lib.load()
    assert lib.tdt_encode_bound(1024, 4) == 28 + 16 + 2048
    assert lib.tdt_encode_bound(0, 4) == 44
    assert lib.tdt_status_string(1) == b"TDT: Invalid encoded data size"
    assert lib.tdt_status_string(2) == b"Invalid TDT magic number"
    cfg = _lib.TdtConfigC()
    lib.tdt_default_config(cfg)
    assert cfg.word_size == 4 and cfg.min_tensor_size == 1024 and abs(cfg.sample_fraction - 0.3) < 1e-7


def test_product_never_imports_oracle():
    # the product package must not reach the CPU checker
    for p in (ROOT / "psyne_amd").rglob("*.py"):
        src = p.read_text()
        assert "import oracle" not in src and "from oracle" not in src, p
