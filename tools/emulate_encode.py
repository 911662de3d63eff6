#!/usr/bin/env python3
"""CPU emulation of tdt_encode_kernel's round algorithm (psyne_amd/csrc/tdt_encode.h).

Mirrors, lane for lane, what one TEAM-thread workgroup computes for one message: v_perm
gathers, the SWAR run-start masks, the max-scan of run starts, the 255-cap bit, chunk and
end masks, the sum-scans, the staging-window indices (k0, idx) and the flush.  Used by
tests/test_emulator.py to check the kernel's index arithmetic against the oracle on the
golden vectors without a GPU, and to assert the invariants the kernel's guards rely on
(0 <= idx - k0 < ends_in_round).
"""
from __future__ import annotations

import numpy as np


def perm(hi, lo, sel):
    """v_perm_b32 for selector bytes in {0..7, 0x0c}."""
    src = (int(lo) | (int(hi) << 32))
    out = 0
    for t in range(4):
        s = (sel >> (8 * t)) & 0xFF
        if s < 8:
            b = (src >> (8 * s)) & 0xFF
        elif s == 0x0C:
            b = 0
        else:
            raise ValueError(s)
        out |= b << (8 * t)
    return out


def neq_prev_mask4(x, below):
    t = ((x << 8) | (below >> 24)) & 0xFFFFFFFF  # alignbyte(x, below, 3)
    d = x ^ t
    nz = (((d & 0x7F7F7F7F) + 0x7F7F7F7F) | d) & 0x80808080
    return ((((nz >> 7) * 0x00204081) & 0xFFFFFFFF) >> 21) & 0xF


def excl_scan(vals, op):
    out, acc = [], 0
    for v in vals:
        out.append(acc)
        acc = op(acc, v)
    return out, acc


def popc(x):
    return bin(x).count("1")


def hibit(x):
    return x.bit_length() - 1


def lobit(x):
    return (x & -x).bit_length() - 1


def encode(data: bytes, mapping, ws=4, team=64):
    """Encode one compressible message with the kernel's algorithm; returns the blob."""
    data = bytes(data)
    n = len(data)
    wpg = 16 // ws
    ns = 2 if any(mapping) else 1
    k, last, first, selA, selB = [0, 0], [0, 0], [0, 0], [[0] * 4, [0] * 4], [[0] * 4, [0] * 4]
    for c in range(2):
        pos = [b for b in range(ws) if mapping[b] == c]
        k[c] = len(pos)
        last[c] = pos[-1] if pos else 0
        first[c] = pos[0] if pos else 0
        for q in range(4):
            A = B = 0x0C0C0C0C
            for t in range(4):
                j = 4 * q + t
                if k[c] and j < wpg * k[c]:
                    src = (j // k[c]) * ws + pos[j % k[c]]
                    if src < 8:
                        A = (A & ~(0xFF << (8 * t))) | (src << (8 * t))
                    else:
                        B = (B & ~(0xFF << (8 * t))) | ((src - 8) << (8 * t))
            selA[c][q], selB[c][q] = A, B
    ngroups = (n + 15) // 16
    nrounds = (ngroups + team - 1) // team
    padded = data + bytes(16 * nrounds * team - n)

    def group(g):
        d = padded[16 * g:16 * g + 16]
        return [int.from_bytes(d[4 * i:4 * i + 4], "little") for i in range(4)]

    def analyze(g, c, prevb):
        dw = group(g)
        vb = max(0, min(16, n - 16 * g))
        L = (vb // ws) * k[c]
        gpos = g * wpg * k[c]
        s = [perm(dw[1], dw[0], selA[c][q]) | perm(dw[3], dw[2], selB[c][q]) for q in range(4)]
        m = (neq_prev_mask4(s[0], prevb << 24) | (neq_prev_mask4(s[1], s[0]) << 4) |
             (neq_prev_mask4(s[2], s[1]) << 8) | (neq_prev_mask4(s[3], s[2]) << 12))
        if g == 0:
            m |= 1
        mask = (m & ((1 << L) - 1)) if L else 0
        return dict(s=s, L=L, gpos=gpos, mask=mask)

    def byte_of(s, j):
        return (s[j >> 2] >> (8 * (j & 3))) & 0xFF

    def run_pass(emit, out=None, ob=0, sdata=(0, 0), check=None):
        carry_max, carry_P = [0, 0], [0, 0]
        for r in range(nrounds):
            xs = []
            for lane in range(team):
                g = r * team + lane
                last_group = 16 * (g + 1) >= n
                row = []
                for c in range(2):
                    prevb = nextb = 0
                    if c < ns and k[c]:
                        if g > 0 and 16 * g < n:
                            prevb = data[16 * g - ws + last[c]]
                        if emit and not last_group:
                            nextb = data[16 * (g + 1) + first[c]]
                    x = analyze(g, c, prevb)
                    if ns < 2 and c == 1:
                        x["L"] = 0
                        x["mask"] = 0
                    x["nextb"], x["last_group"] = nextb, last_group
                    row.append(x)
                xs.append(row)
            for c in range(2):
                mv = [(x[c]["gpos"] + hibit(x[c]["mask"]) + 1) if x[c]["mask"] else 0 for x in xs]
                ex, tot = excl_scan(mv, max)
                for lane, x in enumerate(xs):
                    x[c]["cs_enc"] = max(ex[lane], carry_max[c])
                carry_max[c] = max(carry_max[c], tot)
                for x in xs:
                    xc = x[c]
                    cap = 0
                    if xc["L"] and not (xc["mask"] & 1) and xc["cs_enc"]:
                        cs = xc["cs_enc"] - 1
                        fs = lobit(xc["mask"]) if xc["mask"] else xc["L"]
                        kk = (xc["gpos"] - cs + 254) // 255
                        cpos = cs + 255 * kk
                        if cpos < xc["gpos"] + fs:
                            cap = 1 << (cpos - xc["gpos"])
                    xc["chunk"] = xc["mask"] | cap
                    xc["end"] = 0
                    if emit and xc["L"]:
                        lend = xc["last_group"]
                        if not lend:
                            lb = byte_of(xc["s"], xc["L"] - 1)
                            rs = xc["gpos"] + hibit(xc["mask"]) if xc["mask"] else xc["cs_enc"] - 1
                            lend = (xc["nextb"] != lb) or ((xc["gpos"] + xc["L"] - rs) % 255 == 0)
                        xc["end"] = ((xc["chunk"] >> 1) | (int(lend) << (xc["L"] - 1))) & ((1 << xc["L"]) - 1)
            tots = [0, 0, 0, 0]
            for c in range(2):
                exP, tots[c] = excl_scan([popc(x[c]["chunk"]) for x in xs], lambda a, b: a + b)
                exE, tots[2 + c] = excl_scan([popc(x[c]["end"]) for x in xs], lambda a, b: a + b)
                for lane, x in enumerate(xs):
                    x[c]["sv"] = exP[lane]
            if emit:
                for c in range(2):
                    dang = 1 if (xs[0][c]["L"] and not (xs[0][c]["chunk"] & 1)) else 0
                    k0 = carry_P[c] - dang
                    stage = {}
                    for x in xs:
                        xc = x[c]
                        em = xc["end"]
                        pb = carry_P[c] + xc["sv"]
                        while em:
                            j = lobit(em)
                            em &= em - 1
                            below = xc["chunk"] & ((2 << j) - 1)
                            if below:
                                cnt = j - hibit(below) + 1
                                idx = pb + popc(below) - 1
                            else:
                                cs = xc["cs_enc"] - 1
                                st0 = cs + 255 * ((xc["gpos"] + j - cs) // 255)
                                cnt = xc["gpos"] + j - st0 + 1
                                idx = pb - 1
                            rel = idx - k0
                            if check is not None:
                                check(0 <= rel < tots[2 + c], (r, c, idx, k0, tots[2 + c]))
                                check(1 <= cnt <= 255, (r, c, cnt))
                            stage[rel] = (cnt, byte_of(xc["s"], j))
                    for rel, (cnt, val) in stage.items():
                        p = ob + sdata[c] + 2 * (k0 + rel)
                        out[p] = cnt
                        out[p + 1] = val
            for c in range(2):
                carry_P[c] += tots[c]
        return carry_P

    P = run_pass(False)
    P0, P1 = P[0], P[1] if ns > 1 else 0
    hdr = 20 + 4 * ws
    E = hdr + 4 + 2 * P0 + (4 + 2 * P1 if ns > 1 else 0)
    out = bytearray(E)
    out[0:4] = (0x54445444).to_bytes(4, "little")
    out[4:8] = n.to_bytes(4, "little")
    out[8:12] = ns.to_bytes(4, "little")
    out[12:16] = ws.to_bytes(4, "little")
    out[16:20] = ws.to_bytes(4, "little")
    for b in range(ws):
        out[20 + 4 * b:24 + 4 * b] = int(mapping[b]).to_bytes(4, "little")
    sdata = (hdr + 4, hdr + 4 + 2 * P0 + 4)
    out[hdr:hdr + 4] = (2 * P0).to_bytes(4, "little")
    if ns > 1:
        out[sdata[1] - 4:sdata[1]] = (2 * P1).to_bytes(4, "little")
    problems = []

    def check(cond, info):
        if not cond:
            problems.append(info)

    run_pass(True, out, 0, sdata, check)
    if problems:
        raise AssertionError("index invariant violated: %r" % problems[:5])
    return bytes(out)
