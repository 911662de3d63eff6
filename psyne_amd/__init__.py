"""psyne_amd — MI355X-native (gfx950) implementation of psyne's TDT payload codec.

The product is libpsyne_tdt.so (C ABI: include/psyne_tdt.h) built from psyne_amd/csrc/;
this package is its Python host mirror (psyne_amd.tdt)."""
from .tdt import TDTConfig, TdtCodec, TDTCompressionProtocol, encode_bound  # noqa: F401

__all__ = ["TDTConfig", "TdtCodec", "TDTCompressionProtocol", "encode_bound"]
