"""Host-side mirror of psyne's TDT protocol over the gfx950 codec (libpsyne_tdt.so).

Reference interface (include/psyne/protocol/tdt_compression.hpp):
  TDTConfig                 :31-43
  TDTCompressionProtocol    :176-638 — should_transform, analyze_data, encode, decode,
                            update_network_metrics, update_system_metrics, protocol_name,
                            is_lossless, transformation_ratio, processing_overhead_ms,
                            get_average_entropy, get_bandwidth_mbps, get_cpu_usage
satisfying psyne::concepts::Protocol (include/psyne/concepts/protocol_concepts.hpp:22-47).

Two layers:
  * ``TdtCodec`` — the batch API: device-resident torch.uint8 tensors of concatenated
    messages plus int64 offsets (n+1), asynchronous on the current torch stream.  This is
    the hot path (bench.py measures it).
  * ``TDTCompressionProtocol`` — the reference's one-message-per-call API (host bytes in,
    host bytes out) with the same names, defaults, exceptions and metric semantics, built
    on the C ABI's host path.

torch is used only for device memory and streams; all codec work is in the HIP kernels.
"""
from __future__ import annotations

import ctypes as C
import time
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import TdtConfigC, TdtError, check

MAGIC_TDT = 0x54445444
MAGIC_UNCP = 0x554E4350


@dataclass
class TDTConfig:
    """TDTConfig (tdt_compression.hpp:31-43).  auto_detect_clusters / max_clusters /
    enable_simd are declared by the reference but never read; kept for API parity.
    sample_fraction is accepted, but the GPU always analyses every word (the reference's
    sample_fraction = 1.0 behaviour, which is the only deterministic one)."""
    sample_fraction: float = 0.3
    word_size: int = 4
    auto_detect_clusters: bool = True
    max_clusters: int = 4
    enable_simd: bool = True
    bandwidth_threshold_mbps: float = 100.0
    cpu_usage_threshold: float = 0.8
    min_tensor_size: int = 1024

    def to_c(self) -> TdtConfigC:
        return TdtConfigC(self.sample_fraction, self.word_size, self.bandwidth_threshold_mbps,
                          self.cpu_usage_threshold, self.min_tensor_size)


def transformation_ratio_of(blob: bytes, n: int) -> float | None:
    """The reference's transformation_ratio() after encoding n bytes into `blob`
    (compress_tdt :395-396): n / TDTEncodedData::encoded_size() (:71-78), which counts the RLE
    stream bytes, the mapping ints and sizeof(TDTEncodedData) = 72 (x86-64 libstdc++: two
    vectors, size_t, int, double) — not the serialized length.  None for a UNCP blob (the
    reference leaves the ratio unchanged on the passthrough path, :230-236 and :256-265)."""
    if len(blob) < 20 or int.from_bytes(blob[:4], "little") != MAGIC_TDT:
        return None
    ns = int.from_bytes(blob[8:12], "little")
    msize = int.from_bytes(blob[16:20], "little")
    streams = len(blob) - 20 - 4 * msize - 4 * ns
    return float(n) / float(streams + 4 * msize + 72)


def encode_bound(n: int, word_size: int = 4) -> int:
    return int(_lib.load().tdt_encode_bound(n, word_size))


def _ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


class TdtCodec:
    """Batched TDT codec bound to one HIP device."""

    def __init__(self, config: TDTConfig | None = None, device: int = 0, lib=None):
        self.config = config or TDTConfig()
        self.device = device
        self._lib = lib if lib is not None else _lib.load()  # `lib`: diagnostic builds only
        h = C.c_void_p()
        cfg = self.config.to_c()
        check(self._lib.tdt_ctx_create(device, C.byref(cfg), C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.tdt_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- policy (update_network_metrics / update_system_metrics :309-319)
    def set_metrics(self, bandwidth_mbps: float, latency_ms: float = 1.0, cpu_usage: float = 0.5):
        self._lib.tdt_ctx_set_metrics(self._h, bandwidth_mbps, latency_ms, cpu_usage)

    def get_metrics(self) -> tuple[float, float, float]:
        b, l, c = C.c_double(), C.c_double(), C.c_double()
        self._lib.tdt_ctx_get_metrics(self._h, C.byref(b), C.byref(l), C.byref(c))
        return b.value, l.value, c.value

    def set_size_hint(self, typical_message_bytes: int):
        self._lib.tdt_ctx_set_size_hint(self._h, typical_message_bytes)

    def should_transform(self, n: int) -> bool:
        return bool(self._lib.tdt_should_transform(self._h, n))

    def encode_bound(self, n: int) -> int:
        return int(self._lib.tdt_encode_bound(n, self.config.word_size))

    # ---- batches (device tensors) ------------------------------------------------------
    @staticmethod
    def _stream(stream):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        return C.c_void_p(s.cuda_stream)

    def batch_bound(self, offsets_host: np.ndarray) -> int:
        sizes = np.diff(np.asarray(offsets_host, dtype=np.int64))
        ws = self.config.word_size
        return int(np.maximum(sizes + 4, 28 + 4 * ws + 2 * sizes).sum()) if sizes.size else 0

    def encode_batch(self, data, offsets, out=None, out_offsets=None, status=None, mapping=None,
                     out_capacity: int | None = None, stream=None):
        """Encode messages data[offsets[i]:offsets[i+1]] (torch uint8 / int64 on the GPU).
        Returns (out, out_offsets, status); blobs are compacted in message order."""
        import torch
        n = offsets.numel() - 1
        if out is None:
            cap = out_capacity if out_capacity is not None else self.batch_bound(offsets.cpu().numpy())
            out = torch.empty(max(cap, 1), dtype=torch.uint8, device=data.device)
        if out_offsets is None:
            out_offsets = torch.empty(n + 1, dtype=torch.int64, device=data.device)
        if status is None:
            status = torch.empty(max(n, 1), dtype=torch.int32, device=data.device)
        cap = out.numel() if out_capacity is None else out_capacity
        if mapping is None:
            check(self._lib.tdt_encode_batch(self._h, _ptr(data), _ptr(offsets), n, _ptr(out), cap,
                                             _ptr(out_offsets), _ptr(status), self._stream(stream)))
        else:
            check(self._lib.tdt_encode_with_mapping_batch(self._h, _ptr(data), _ptr(offsets), n, _ptr(mapping),
                                                          _ptr(out), cap, _ptr(out_offsets), _ptr(status),
                                                          self._stream(stream)))
        return out, out_offsets, status

    def decode_batch(self, blobs, offsets, out=None, out_offsets=None, status=None,
                     out_capacity: int | None = None, stream=None):
        """Decode blobs[offsets[i]:offsets[i+1]].  If `out` is None the decoded sizes are
        computed first (tdt_decoded_sizes_batch) to size it."""
        import torch
        n = offsets.numel() - 1
        if out is None:
            sizes, _ = self.decoded_sizes(blobs, offsets, stream=stream)
            cap = int(sizes.sum().item())
            out = torch.empty(max(cap, 1), dtype=torch.uint8, device=blobs.device)
        if out_offsets is None:
            out_offsets = torch.empty(n + 1, dtype=torch.int64, device=blobs.device)
        if status is None:
            status = torch.empty(max(n, 1), dtype=torch.int32, device=blobs.device)
        cap = out.numel() if out_capacity is None else out_capacity
        check(self._lib.tdt_decode_batch(self._h, _ptr(blobs), _ptr(offsets), n, _ptr(out), cap,
                                         _ptr(out_offsets), _ptr(status), self._stream(stream)))
        return out, out_offsets, status

    # ---- slotted batches (no inter-message dependency: the hot path) -------------------
    def encode_slots(self, offsets, stream=None):
        """Slot offsets (n+1, int64, device) = prefix sum of the encode bounds."""
        import torch
        n = offsets.numel() - 1
        slots = torch.empty(n + 1, dtype=torch.int64, device=offsets.device)
        check(self._lib.tdt_encode_slots(self._h, _ptr(offsets), n, _ptr(slots), self._stream(stream)))
        return slots

    def decode_slots(self, blobs, offsets, lengths=None, status=None, stream=None):
        """Slot offsets (n+1) = prefix sum of the decoded sizes (header parse).  With
        `lengths`, blob i is blobs[offsets[i]:offsets[i]+lengths[i]] (offsets may then have n
        or n+1 entries)."""
        import torch
        n = lengths.numel() if lengths is not None else offsets.numel() - 1
        slots = torch.empty(n + 1, dtype=torch.int64, device=offsets.device)
        if status is None:
            status = torch.empty(max(n, 1), dtype=torch.int32, device=offsets.device)
        check(self._lib.tdt_decode_slots(self._h, _ptr(blobs), _ptr(offsets), _ptr(lengths), n, _ptr(slots),
                                         _ptr(status), self._stream(stream)))
        return slots

    def encode_into(self, data, offsets, slots=None, out=None, lengths=None, status=None, stream=None):
        """Encode message i into out[slots[i]:slots[i+1]]; returns (out, slots, lengths, status)."""
        import torch
        n = offsets.numel() - 1
        if slots is None:
            slots = self.encode_slots(offsets, stream=stream)
        if out is None:
            out = torch.empty(max(int(slots[-1].item()), 1), dtype=torch.uint8, device=data.device)
        if lengths is None:
            lengths = torch.empty(max(n, 1), dtype=torch.int64, device=data.device)
        if status is None:
            status = torch.empty(max(n, 1), dtype=torch.int32, device=data.device)
        check(self._lib.tdt_encode_batch_into(self._h, _ptr(data), _ptr(offsets), n, _ptr(out), _ptr(slots),
                                              _ptr(lengths), _ptr(status), self._stream(stream)))
        return out, slots, lengths, status

    def decode_into(self, blobs, offsets, in_lengths=None, slots=None, out=None, lengths=None, status=None,
                    stream=None):
        """Decode blob i (blobs[offsets[i]:offsets[i]+in_lengths[i]], or up to offsets[i+1]) into
        out[slots[i]:slots[i+1]]; returns (out, slots, lengths, status)."""
        import torch
        n = in_lengths.numel() if in_lengths is not None else offsets.numel() - 1
        if slots is None:
            slots = self.decode_slots(blobs, offsets, lengths=in_lengths, stream=stream)
        if out is None:
            out = torch.empty(max(int(slots[-1].item()), 1), dtype=torch.uint8, device=blobs.device)
        if lengths is None:
            lengths = torch.empty(max(n, 1), dtype=torch.int64, device=blobs.device)
        if status is None:
            status = torch.empty(max(n, 1), dtype=torch.int32, device=blobs.device)
        check(self._lib.tdt_decode_batch_into(self._h, _ptr(blobs), _ptr(offsets), _ptr(in_lengths), n, _ptr(out),
                                              _ptr(slots), _ptr(lengths), _ptr(status), self._stream(stream)))
        return out, slots, lengths, status

    def decoded_sizes(self, blobs, offsets, stream=None):
        import torch
        n = offsets.numel() - 1
        sizes = torch.empty(max(n, 1), dtype=torch.int64, device=blobs.device)
        status = torch.empty(max(n, 1), dtype=torch.int32, device=blobs.device)
        check(self._lib.tdt_decoded_sizes_batch(self._h, _ptr(blobs), _ptr(offsets), n, _ptr(sizes),
                                                _ptr(status), self._stream(stream)))
        return sizes[:n], status[:n]

    def analyze_batch(self, data, offsets, stream=None):
        """Full-sample histograms (n, ws, 256), entropies (n, ws), mapping (n, ws), status."""
        import torch
        n = offsets.numel() - 1
        ws = self.config.word_size
        hist = torch.empty((max(n, 1), ws, 256), dtype=torch.int32, device=data.device)
        ent = torch.empty((max(n, 1), ws), dtype=torch.float64, device=data.device)
        mp = torch.empty((max(n, 1), ws), dtype=torch.int32, device=data.device)
        st = torch.empty(max(n, 1), dtype=torch.int32, device=data.device)
        check(self._lib.tdt_analyze_batch(self._h, _ptr(data), _ptr(offsets), n, _ptr(hist), _ptr(ent), _ptr(mp),
                                          _ptr(st), self._stream(stream)))
        return hist[:n], ent[:n], mp[:n], st[:n]

    def error_flags(self, stream=None) -> int:
        """Device invariant flags (tdt_ctx_error_flags; 0 for a correct build).  Synchronises
        the stream the batches were issued on (default: the current torch stream)."""
        fl = C.c_uint32(0)
        check(self._lib.tdt_ctx_error_flags(self._h, self._stream(stream), C.byref(fl)))
        return int(fl.value)

    def set_option(self, option: int, value: int):
        """tdt_ctx_set_option (tuning / diagnostic knobs; results are the same bytes)."""
        check(self._lib.tdt_ctx_set_option(self._h, option, int(value)))

    # ---- host path (socket buffers) -------------------------------------------------------
    def encode_host(self, data: np.ndarray, offsets: np.ndarray):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        cap = self.batch_bound(offsets)
        out = np.empty(max(cap, 1), np.uint8)
        out_off = np.zeros(n + 1, np.uint64)
        st = np.zeros(max(n, 1), np.int32)
        check(self._lib.tdt_encode_host(self._h, data.ctypes.data, offsets.ctypes.data, n, out.ctypes.data, cap,
                                        out_off.ctypes.data, st.ctypes.data))
        return out[: int(out_off[-1])], out_off, st[:n]

    def decode_host(self, blobs: np.ndarray, offsets: np.ndarray, capacity: int):
        blobs = np.ascontiguousarray(blobs, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        out = np.empty(max(capacity, 1), np.uint8)
        out_off = np.zeros(n + 1, np.uint64)
        st = np.zeros(max(n, 1), np.int32)
        check(self._lib.tdt_decode_host(self._h, blobs.ctypes.data, offsets.ctypes.data, n, out.ctypes.data,
                                        capacity, out_off.ctypes.data, st.ctypes.data))
        return out[: int(out_off[-1])], out_off, st[:n]


class TDTCompressionProtocol:
    """psyne::protocol::TDTCompressionProtocol (tdt_compression.hpp:176-638) on the GPU.

    Same method names, defaults and semantics; encode/decode move one message through the
    C ABI's host path (H2D, kernel, D2H).  Errors raise RuntimeError with the reference's
    messages ("TDT: Invalid encoded data size", "Invalid TDT magic number")."""

    def __init__(self, config: TDTConfig | None = None, device: int = 0):
        self.config_ = config or TDTConfig()
        self.codec = TdtCodec(self.config_, device)
        self._bandwidth = 100.0   # :352
        self._latency = 1.0       # :353
        self._cpu = 0.5           # :354
        self.last_compression_ratio_ = 1.0
        self.last_encode_time_ms_ = 0.0
        self.last_decode_time_ms_ = 0.0
        self.avg_entropy_ = 0.0

    # PROTOCOL CONCEPT ---------------------------------------------------------------------
    def should_transform(self, data, size: int) -> bool:
        return self.codec.should_transform(size)

    def _is_tensor_data(self, size: int) -> bool:  # :409-413
        return size % 4 == 0 and size >= 64

    def analyze_data(self, data, size: int) -> None:
        """analyze_data :206-222, full sample, on the GPU (tdt_analyze_batch)."""
        import torch
        if not self._is_tensor_data(size):
            return
        ws = self.config_.word_size
        words = size // ws
        if words == 0:
            self.avg_entropy_ = 0.0
            return
        buf = np.frombuffer(bytes(memoryview(data)[: words * ws]), dtype=np.uint8)
        d = torch.from_numpy(buf.copy()).cuda(self.codec.device)
        off = torch.tensor([0, words * ws], dtype=torch.int64, device=d.device)
        _, ent, _, st = self.codec.analyze_batch(d, off)
        e = ent[0].cpu().numpy()
        total = 0.0
        for b in range(ws):
            total += float(e[b])
        self.avg_entropy_ = total / ws

    def encode(self, data, size: int | None = None) -> bytes:
        t0 = time.perf_counter()
        buf = bytes(memoryview(data)) if size is None else bytes(memoryview(data)[:size])
        n = len(buf)
        arr = np.frombuffer(buf, dtype=np.uint8) if n else np.zeros(1, np.uint8)
        out, _, st = self.codec.encode_host(arr[:n] if n else arr[:0], np.array([0, n], np.uint64))
        if int(st[0]) != 0:
            raise TdtError(int(st[0]), "encode")
        blob = out.tobytes()
        ratio = transformation_ratio_of(blob, n)
        if ratio is not None:  # compressed: metrics as :243-248
            self.last_compression_ratio_ = ratio
            self.last_encode_time_ms_ = (time.perf_counter() - t0) * 1e3
        return blob

    def decode(self, encoded: bytes) -> bytes:
        t0 = time.perf_counter()
        if len(encoded) < 4:
            raise RuntimeError("TDT: Invalid encoded data size")
        arr = np.frombuffer(bytes(encoded), dtype=np.uint8)
        off = np.array([0, arr.size], np.uint64)
        magic = int.from_bytes(encoded[:4], "little")
        if magic == MAGIC_UNCP:
            cap = arr.size - 4
        elif magic == MAGIC_TDT and arr.size >= 8:
            cap = int.from_bytes(encoded[4:8], "little")
        else:
            cap = 0
        out, _, st = self.codec.decode_host(arr, off, cap)
        s = int(st[0])
        if s != 0:
            msg = _lib.load().tdt_status_string(s).decode()
            raise RuntimeError(msg)
        if magic != MAGIC_UNCP:
            self.last_decode_time_ms_ = (time.perf_counter() - t0) * 1e3
        return out.tobytes()

    def update_network_metrics(self, bandwidth_mbps: float, latency_ms: float) -> None:
        self._bandwidth, self._latency = bandwidth_mbps, latency_ms
        self.codec.set_metrics(self._bandwidth, self._latency, self._cpu)

    def update_system_metrics(self, cpu_usage: float) -> None:
        self._cpu = cpu_usage
        self.codec.set_metrics(self._bandwidth, self._latency, self._cpu)

    # IDENTITY ------------------------------------------------------------------------------
    def protocol_name(self) -> str:
        return "TDT-Compression"

    def is_lossless(self) -> bool:
        return True

    def transformation_ratio(self) -> float:
        return self.last_compression_ratio_

    def processing_overhead_ms(self) -> float:
        return (self.last_encode_time_ms_ + self.last_decode_time_ms_) / 2.0

    def get_average_entropy(self) -> float:
        return self.avg_entropy_

    def get_bandwidth_mbps(self) -> float:
        return self._bandwidth

    def get_cpu_usage(self) -> float:
        return self._cpu
