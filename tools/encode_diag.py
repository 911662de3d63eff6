"""Diagnostic (not shipped): encode a few message shapes with the library named by PSYNE_TDT_LIB,
compare every blob with the oracle and print the mismatch counts and the context's error flags
(diagnostic builds may set extra bits).  Run on the GPU box."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle.oracle import Oracle  # noqa: E402
from psyne_amd import TDTConfig, TdtCodec  # noqa: E402


def grad(rng, n):
    x = rng.normal(0, 0.01, n).astype(np.float32)
    x[rng.random(n) < 0.7] = 0
    return x.view(np.uint8)


def main():
    orc = Oracle()
    rng = np.random.default_rng(5)
    cases = {
        "ws1_2k": (1, [rng.integers(0, 4, 2048, dtype=np.uint8) for _ in range(64)]),
        "ws4_2k": (4, [grad(rng, 512) for _ in range(64)]),
        "ws4_64k": (4, [grad(rng, 16384) for _ in range(64)]),
        "ws4_16k": (4, [grad(rng, 4096) for _ in range(64)]),
        "ws2_8k": (2, [rng.integers(0, 3, 8192, dtype=np.uint8) for _ in range(64)]),
    }
    for name, (ws, msgs) in cases.items():
        codec = TdtCodec(TDTConfig(sample_fraction=1.0, word_size=ws))
        codec.set_metrics(10.0, 1.0, 0.5)
        off = np.zeros(len(msgs) + 1, np.int64)
        off[1:] = np.cumsum([m.size for m in msgs])
        d = torch.from_numpy(np.concatenate(msgs)).cuda()
        enc, eoff, st = codec.encode_batch(d, torch.from_numpy(off).cuda())
        torch.cuda.synchronize()
        e, eo = enc.cpu().numpy(), eoff.cpu().numpy()
        cfg = orc.config(word_size=ws)
        bad = []
        for i, m in enumerate(msgs):
            want = orc.encode(m, cfg=cfg)
            got = e[eo[i]:eo[i + 1]].tobytes()
            if got != want:
                k = next((j for j in range(min(len(got), len(want))) if got[j] != want[j]), min(len(got), len(want)))
                bad.append((i, len(got), len(want), k))
        print(name, "mismatches", len(bad), bad[:4], "errflags", codec.error_flags(), flush=True)


if __name__ == "__main__":
    main()
