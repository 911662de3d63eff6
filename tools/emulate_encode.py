#!/usr/bin/env python3
"""CPU emulation of tdt_encode_kernel's round algorithm (psyne_amd/csrc/tdt_encode.h, v3).

Mirrors, lane for lane, what one TEAM-thread workgroup computes for one compressible message:
the transposed two-stream slot layout T (slot j = 4t + q lives in dword q, byte t), the SWAR
run-start mask, the packed two-stream max-scan of run starts, the 255-cap bit, chunk and end
masks, the packed pair-index sum-scan, the branch-free slot emission (clz counts, bcnt
addresses, overwrite order) with its first-end repair sweep, and the flush.  Used by
tests/test_emulator.py to pin the kernel's index arithmetic against the oracle on the golden
vectors without a GPU, and to assert the invariants the kernel's guards rely on.

Everything is 32-bit unsigned arithmetic as on the device; hardware-specific behaviour that
the kernel relies on is modelled explicitly (v_ffbh_u32(0) = 0xffffffff, DPP wave shifts with
an `old` value for the lane whose source is outside the wave).
"""
from __future__ import annotations

import numpy as np

M32 = 0xFFFFFFFF
LANES = np.arange(64, dtype=np.int64)


def perm(hi, lo, sel):
    """v_perm_b32 over lane arrays; selector bytes in {0..7, 0x0c}."""
    hi = np.asarray(hi, np.int64)
    lo = np.asarray(lo, np.int64)
    out = np.zeros(np.broadcast(hi, lo).shape, np.int64)
    for t in range(4):
        s = (sel >> (8 * t)) & 0xFF
        if s < 4:
            b = (lo >> (8 * s)) & 0xFF
        elif s < 8:
            b = (hi >> (8 * (s - 4))) & 0xFF
        elif s == 0x0C:
            b = 0
        else:
            raise ValueError(s)
        out |= b << (8 * t)
    return out


def ffbh(x):
    """v_ffbh_u32: leading zeros, 0xffffffff for 0."""
    x = np.asarray(x, np.int64) & M32
    out = np.full(x.shape, M32, np.int64)
    nz = x != 0
    out[nz] = 32 - np.vectorize(lambda v: int(v).bit_length())(x[nz]) if nz.any() else out[nz]
    return out


def ffbl(x):
    x = np.asarray(x, np.int64) & M32
    out = np.full(x.shape, M32, np.int64)
    nz = x != 0
    if nz.any():
        v = x[nz]
        out[nz] = np.vectorize(lambda a: (int(a) & -int(a)).bit_length() - 1)(v)
    return out


def popc(x):
    return np.vectorize(lambda v: bin(int(v) & M32).count("1"))(np.asarray(x, np.int64))


def hibit(x):
    return np.vectorize(lambda v: int(v).bit_length() - 1)(np.asarray(x, np.int64))


def wave_shr1(x, old):
    """DPP wave_shr:1 — lane l gets lane l-1, lane 0 keeps `old`."""
    y = np.empty_like(x)
    y[1:] = x[:-1]
    y[0] = old
    return y


def wave_shl1(x, old):
    y = np.empty_like(x)
    y[:-1] = x[1:]
    y[-1] = old
    return y


def pk_max_scan(x):
    lo = np.maximum.accumulate(x & 0xFFFF)
    hi = np.maximum.accumulate(x >> 16)
    return lo | (hi << 16)


class Desc:
    """Uniform per-message description (thread 0 in the kernel)."""

    def __init__(self, mapping, ws):
        self.ws = ws
        self.wpg = 16 // ws
        mapping = [int(m) for m in mapping]
        self.ns = 2 if any(mapping) else 1
        pos = [[b for b in range(ws) if mapping[b] == c] for c in range(2)]
        if self.ns == 1:
            pos = [list(range(ws)), []]
        self.pos = pos
        self.k = [len(pos[0]), len(pos[1])]
        self.L = [self.wpg * self.k[0], self.wpg * self.k[1]]
        self.L0 = self.L[0]
        # slot -> source byte of the group
        sb = []
        for j in range(16):
            if j < self.L0:
                sb.append((j // self.k[0]) * ws + pos[0][j % self.k[0]])
            else:
                jj = j - self.L0
                sb.append((jj // self.k[1]) * ws + pos[1][jj % self.k[1]])
        self.sb = sb
        self.selA, self.selB = [], []
        for q in range(4):
            a = b = 0
            for t in range(4):
                s = sb[4 * t + q]
                a |= (s if s < 8 else 0x0C) << (8 * t)
                b |= (s - 8 if s >= 8 else 0x0C) << (8 * t)
            self.selA.append(a)
            self.selB.append(b)
        # edges: byte0 stream-0 last slot, byte1 slot 15, byte2 stream-1 first slot
        e = [sb[self.L0 - 1] if self.L0 > 0 else None, sb[15], sb[self.L0] if self.ns == 2 else None, None]
        a = b = 0
        for t, s in enumerate(e):
            a |= (s if (s is not None and s < 8) else 0x0C) << (8 * t)
            b |= (s - 8 if (s is not None and s >= 8) else 0x0C) << (8 * t)
        self.edA, self.edB = a, b

    def valid_mask(self, nvw):
        if nvw >= self.wpg:
            return 0xFFFF
        v = (1 << (nvw * self.k[0])) - 1
        if self.ns == 2:
            v |= ((1 << (nvw * self.k[1])) - 1) << self.L0
        return v


class Msg:
    def __init__(self, data: bytes, sd: Desc):
        self.n = len(data)
        self.ngroups = (self.n + 15) // 16
        buf = np.zeros(self.ngroups * 16 + 16 * 64 * 4, np.uint8)
        buf[:self.n] = np.frombuffer(data, np.uint8)
        self.dw = buf.view(np.uint32).astype(np.int64).reshape(-1, 4)
        self.sd = sd

    def load(self, g):
        g = np.asarray(g)
        d = self.dw[np.minimum(g, len(self.dw) - 1)].copy()
        d[g >= self.ngroups] = 0
        return d

    def vmask(self, g):
        vb = np.clip(self.n - 16 * np.asarray(g, np.int64), 0, 16)
        return np.array([self.sd.valid_mask(int(v) // self.sd.ws) for v in vb], np.int64)


def tmat(d, sd):
    return [perm(d[:, 1], d[:, 0], sd.selA[q]) | perm(d[:, 3], d[:, 2], sd.selB[q]) for q in range(4)]


def edges(d, sd):
    return perm(d[:, 1], d[:, 0], sd.edA) | perm(d[:, 3], d[:, 2], sd.edB)


def run_mask(T, ed, ed_carry, g, V, sd):
    pe = wave_shr1(ed, ed_carry)
    P0 = perm(T[3], pe, 0x06050400)
    X = [T[0] ^ P0, T[1] ^ T[0], T[2] ^ T[1], T[3] ^ T[2]]
    Y = [(((x & 0x7F7F7F7F) + 0x7F7F7F7F) & M32) | x for x in X]
    m = ((Y[0] >> 7) & 0x01010101) | ((Y[1] >> 6) & 0x02020202) | ((Y[2] >> 5) & 0x04040404) | \
        ((Y[3] >> 4) & 0x08080808)
    m = (m | (m >> 4)) & 0x00FF00FF
    m = (m | (m >> 8)) & 0xFFFF
    if sd.ns == 2:
        fx = ((ed >> 16) ^ (pe >> 8)) & 0xFF
        m = (m & ~(1 << sd.L0)) | (np.where(fx != 0, 1, 0) << sd.L0)
    first = (g == 0)
    m = np.where(first, m | 1 | ((1 << sd.L0) if sd.ns == 2 else 0), m)
    return m & V


def split(m, sd):
    return [m & ((1 << sd.L0) - 1), (m >> sd.L0) & 0xFFFF if sd.ns == 2 else np.zeros_like(m)]


def run_scan(m, rbase, sd):
    """Packed max-scan of (last run start + 1), round-relative.  Returns per-lane carried
    run start (+1, round-relative, 0 = from an earlier round) and the inclusive scan."""
    lr = np.zeros_like(m)
    ms = split(m, sd)
    for c in range(sd.ns):
        v = np.where(ms[c] != 0, LANES * sd.L[c] + hibit(np.maximum(ms[c], 1)) + 1, 0)
        lr |= v << (16 * c)
    inc = pk_max_scan(lr)
    exc = wave_shr1(inc, 0)
    return exc, inc


def caps(m, exc, rcarry, rbase, g, V, sd):
    """Cap bits (combined layout) and the carried run start (absolute) per stream."""
    out = np.zeros_like(m)
    ms = split(m, sd)
    cs_all = []
    for c in range(sd.ns):
        er = (exc >> (16 * c)) & 0xFFFF
        cs = np.where(er != 0, rbase[c] + er - 1, rcarry[c] - 1)  # -1 = none
        cs_all.append(cs)
        Lv = popc(split(V, sd)[c])
        gpos = g * sd.L[c]
        mc = ms[c]
        has = (cs >= 0) & ((mc & 1) == 0) & (Lv > 0)
        d = gpos - cs
        mcap = (d + 254) // 255
        rel = 255 * mcap - d
        fs = ffbl(mc | (1 << Lv))
        bit = has & (rel < fs)
        off = 0 if c == 0 else sd.L0
        out |= np.where(bit, 1 << np.where(bit, rel + off, 0), 0)
    return out, cs_all


def encode(data: bytes, mapping, ws=4, team=256, G=16, check=True):
    sd = Desc(mapping, ws)
    n = len(data)
    msg = Msg(data, sd)
    ngroups = msg.ngroups
    W = team // 64
    RW = (ngroups + team - 1) // team
    ns = sd.ns

    def groups(w, r):
        return w * RW * 64 + r * 64 + LANES

    def ed_carry0(w):
        gp = w * RW * 64 - 1
        if gp < 0:
            return 0
        return int(edges(msg.load(np.array([gp])), sd)[0])

    # ---------------------------------------------------------------- pass A1
    wmax = np.zeros((W, 2), np.int64)
    for w in range(W):
        edc = ed_carry0(w)
        for r in range(RW):
            g = groups(w, r)
            d = msg.load(g)
            V = msg.vmask(g)
            T, ed = tmat(d, sd), edges(d, sd)
            m = run_mask(T, ed, edc, g, V, sd)
            edc = int(ed[63])
            ms = split(m, sd)
            for c in range(ns):
                v = np.where(ms[c] != 0, g * sd.L[c] + hibit(np.maximum(ms[c], 1)) + 1, 0)
                wmax[w, c] = max(wmax[w, c], int(v.max()))
    rin = np.zeros((W, 2), np.int64)
    for w in range(1, W):
        rin[w] = np.maximum(rin[w - 1], wmax[w - 1])

    # ---------------------------------------------------------------- pass A2
    cstore = {}
    psum = np.zeros((W, 2), np.int64)
    fb = np.zeros(W, np.int64)
    for w in range(W):
        edc = ed_carry0(w)
        rcarry = list(rin[w])
        for r in range(RW):
            g = groups(w, r)
            d = msg.load(g)
            V = msg.vmask(g)
            T, ed = tmat(d, sd), edges(d, sd)
            m = run_mask(T, ed, edc, g, V, sd)
            edc = int(ed[63])
            rbase = [(w * RW * 64 + r * 64) * sd.L[c] for c in range(2)]
            exc, inc = run_scan(m, rbase, sd)
            cp, _ = caps(m, exc, rcarry, rbase, g, V, sd)
            C = m | cp
            cstore[(w, r)] = C
            for c in range(ns):
                i63 = (int(inc[63]) >> (16 * c)) & 0xFFFF
                if i63:
                    rcarry[c] = max(rcarry[c], rbase[c] + i63)
                psum[w, c] += int(popc(split(C, sd)[c]).sum())
            if r == 0:
                fb[w] = int(C[0]) & (1 | ((1 << sd.L0) if ns == 2 else 0))
    P = psum.sum(axis=0)
    pin = np.zeros((W, 2), np.int64)
    for w in range(1, W):
        pin[w] = pin[w - 1] + psum[w - 1]

    hdr = 20 + 4 * ws
    E = hdr + 4 + 2 * int(P[0]) + (4 + 2 * int(P[1]) if ns == 2 else 0)
    out = bytearray(E)
    import struct
    struct.pack_into("<IIIII", out, 0, 0x54445444, n, ns, ws, ws)
    for b in range(ws):
        struct.pack_into("<i", out, 20 + 4 * b, int(mapping[b]))
    sdata = [hdr + 4, hdr + 4 + 2 * int(P[0]) + 4]
    struct.pack_into("<I", out, hdr, 2 * int(P[0]))
    if ns == 2:
        struct.pack_into("<I", out, sdata[1] - 4, 2 * int(P[1]))

    # ---------------------------------------------------------------- pass B
    for w in range(W):
        edc = ed_carry0(w)
        rcarry = list(rin[w])
        pr = list(pin[w])
        nfb = int(fb[w + 1]) if w + 1 < W else 0
        for r in range(RW):
            g = groups(w, r)
            d = msg.load(g)
            V = msg.vmask(g)
            T, ed = tmat(d, sd), edges(d, sd)
            m = run_mask(T, ed, edc, g, V, sd)
            edc = int(ed[63])
            rbase = [(w * RW * 64 + r * 64) * sd.L[c] for c in range(2)]
            exc, inc = run_scan(m, rbase, sd)
            _, cs = caps(m, exc, rcarry, rbase, g, V, sd)
            C = cstore[(w, r)]
            for c in range(ns):
                i63 = (int(inc[63]) >> (16 * c)) & 0xFFFF
                if i63:
                    rcarry[c] = max(rcarry[c], rbase[c] + i63)
            nxt63 = int(cstore[(w, r + 1)][0]) if r + 1 < RW else nfb
            nb = wave_shl1(C, nxt63)
            last = (16 * (g + 1) >= n) & (g < ngroups)
            L0 = sd.L0
            e = (C >> 1) & 0x7FFF
            if L0 > 0:
                e &= ~(1 << (L0 - 1))
                e |= (nb & 1) << (L0 - 1)
            if ns == 2:
                e |= ((nb >> L0) & 1) << 15
            # last group: ends at the last valid slot of each stream
            Vs = split(V, sd)
            lastbits = np.zeros_like(e)
            for c in range(ns):
                off = 0 if c == 0 else L0
                lv = popc(Vs[c])
                lastbits |= np.where(lv > 0, 1 << np.where(lv > 0, off + lv - 1, 0), 0)
            e = np.where(last, ((C >> 1) & V) | lastbits, e)
            e &= V
            # packed pair-index scan
            Cs = split(C, sd)
            pc = popc(Cs[0]) | (popc(Cs[1]) << 16)
            pinc = np.cumsum(pc)
            pexc = pinc - pc
            tot = int(pinc[63])
            es = split(e, sd)
            Tq = T
            # emission
            for c in range(ns):
                off = 0 if c == 0 else L0
                f0 = int(Cs[c][0]) & 1
                v0 = int(Vs[c][0]) != 0
                dang = 1 if (v0 and not f0) else 0
                k0 = pr[c] - dang
                ends = int(popc(es[c]).sum())
                pbase = pr[c] + ((pexc >> (16 * c)) & 0xFFFF)
                fi = pbase - np.where((Cs[c] & 1) != 0, 0, 1)
                gdst = sdata[c] + 2 * k0
                stage = {}
                base = 2 * (fi - k0)
                if c == 1:
                    base = base - 2 * popc(es[0])
                E2 = np.zeros_like(e)
                for j in range(16):
                    E2 |= ((e >> j) & 1) * (3 << (2 * j))
                # sweep 1: every valid slot of stream c, ascending
                for j in range(off, off + sd.L[c]):
                    q, t = j % 4, j // 4
                    clz = ffbh((C << (31 - j)) & M32)
                    cnt = (clz + 1) & 0xFF
                    val = (Tq[q] >> (8 * t)) & 0xFF
                    addr = base + popc(E2 & ((1 << (2 * j)) - 1))
                    # one ds_write per slot: lanes writing the same address in the same
                    # instruction leave an undefined winner (poisoned here)
                    seen = {}
                    for l in range(64):
                        if (int(V[l]) >> j) & 1:
                            a = int(addr[l])
                            seen[a] = None if a in seen else (int(cnt[l]), int(val[l]))
                    stage.update(seen)
                # sweep 2: first end of the stream in each lane
                jf = ffbl(es[c])
                lastchunk = np.where(cs[c] >= 0, cs[c] + 255 * ((g * sd.L[c] - 1 - cs[c]) // 255), 0)
                firstval = (Tq[0] & 0xFF) if c == 0 else ((ed >> 16) & 0xFF)
                for l in range(64):
                    if int(es[c][l]) == 0:
                        continue
                    jr = int(jf[l])  # relative slot within stream
                    if int(Cs[c][l]) & 1:
                        cnt = jr + 1
                    else:
                        cnt = int(g[l]) * sd.L[c] + jr - int(lastchunk[l]) + 1
                    if check:
                        assert 1 <= cnt <= 255, (cnt, w, r, l, c)
                    stage[int(2 * (fi[l] - k0))] = (cnt, int(firstval[l]))
                # flush [0, ends)
                for i in range(ends):
                    if check:
                        assert 2 * i in stage, (w, r, c, i)
                    if check:
                        assert stage[2 * i] is not None, ("poisoned pair survived", w, r, c, i)
                    cnt, val = stage[2 * i]
                    out[gdst + 2 * i] = cnt
                    out[gdst + 2 * i + 1] = val
                pr[c] += (tot >> (16 * c)) & 0xFFFF
    return bytes(out)


if __name__ == "__main__":
    import sys
    sys.path.insert(0, ".")
    from oracle.oracle import Oracle
    o = Oracle()
    rng = np.random.default_rng(1)
    for trial in range(20):
        nw = int(rng.integers(16, 3000))
        x = rng.normal(0, 0.01, nw).astype(np.float32)
        x[rng.random(nw) < 0.7] = 0
        v = x.view(np.uint8)
        want = o.encode(v, cfg=o.config(), bandwidth=10.0)
        if want[:4] != b"DTDT":
            continue
        mp = list(np.frombuffer(want[20:36], np.int32))
        got = encode(v.tobytes(), mp, team=64, G=4)
        print(trial, nw, got == want)
