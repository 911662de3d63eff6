"""Diagnostic: one pinned tdt_encode_host + three tdt_decode_host calls of 32,768 x 64 KiB
gradient messages (bench.py --host-inclusive's pinned leg), wall time per call, and the host
time spent before the first chunk is issued (decoded-size scan).  Run under rocprofv3
--kernel-trace --memory-copy-trace to see the chunk pipeline (tools/trace_view.py)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from psyne_amd import TDTConfig, TdtCodec  # noqa: E402
from psyne_amd._lib import check  # noqa: E402

m, mb = 32768, 65536
codec = TdtCodec(TDTConfig(sample_fraction=1.0))
codec.set_metrics(10.0, 1.0, 0.5)
lib, h = codec._lib, codec._h
g = torch.Generator(device="cuda")
g.manual_seed(5)
x = torch.empty(m * mb // 4, dtype=torch.float32, device="cuda").normal_(0, 0.01, generator=g)
x.masked_fill_(torch.rand(x.numel(), device="cuda", generator=g) < 0.7, 0.0)
b = m * mb
t_src = torch.empty(b, dtype=torch.uint8, pin_memory=True)
t_src.copy_(x.view(torch.uint8))
cap = m * codec.encode_bound(mb)
t_enc = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
t_dec = torch.empty(b, dtype=torch.uint8, pin_memory=True)
src, enc, dec = t_src.numpy(), t_enc.numpy(), t_dec.numpy()
enc[:] = 0
dec[:] = 0
hoff = np.arange(m + 1, dtype=np.uint64) * mb
heoff = np.zeros(m + 1, np.uint64)
hst = np.zeros(m, np.int32)
hdoff = np.zeros(m + 1, np.uint64)
hdst = np.zeros(m, np.int32)
torch.cuda.synchronize()
for r in range(3):
    t0 = time.perf_counter()
    check(lib.tdt_encode_host(h, src.ctypes.data, hoff.ctypes.data, m, enc.ctypes.data, cap, heoff.ctypes.data,
                              hst.ctypes.data))
    t1 = time.perf_counter()
    check(lib.tdt_decode_host(h, enc.ctypes.data, heoff.ctypes.data, m, dec.ctypes.data, b, hdoff.ctypes.data,
                              hdst.ctypes.data))
    t2 = time.perf_counter()
    print("call %d: encode %.2f ms (%.1f GiB/s), decode %.2f ms (%.1f GiB/s), blobs %d B" %
          (r, (t1 - t0) * 1e3, b / (t1 - t0) / 2**30, (t2 - t1) * 1e3, b / (t2 - t1) / 2**30, int(heoff[-1])))
print("ok", bool(np.array_equal(dec, src)))
