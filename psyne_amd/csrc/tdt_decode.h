// tdt_decode.h — batched TDT decode for CDNA4 (gfx950).
//
// Restates include/psyne/protocol/tdt_compression.hpp (reference):
//   decode                  :271-304  size < 4 → error; UNCP → payload; else TDT
//   TDTEncodedData::deserialize :119-170 (+ the bounds checks the reference lacks)
//   simple_rle_decompress   :596-612  pairs while i+1 < len; count 0 emits nothing
//   recombine_byte_streams  :614-637  zero-initialised output; short streams leave zeros
//
// Work decomposition: one TEAM-thread workgroup per blob.  Output is
// produced in WINDOWS of TEAM 16-byte groups (thread t owns group t of the window, so
// stores are one coalesced 16 B/lane sweep).  For every stream the window covers a range
// [P0, P1) of stream positions.  Rounds of pairs (8 per lane) are prefix-summed across the
// team; each non-empty pair writes its value at its start position into an LDS "heads"
// array (u16, 0xFFFF = no head).  Each thread then fills its own 4·k positions forward
// from the last head (carry-in from a team max-scan), zeroes positions past the decoded
// stream length, and scatters the bytes into output words with v_perm_b32 selectors.
#pragma once
#include "tdt_device.h"
#include "tdt_encode.h"

namespace psy {

struct DecodeArgs {
    const uint8_t *in;
    const uint64_t *in_off;
    uint32_t n_msgs;
    uint8_t *out;
    uint64_t out_cap;
    uint64_t *out_off;
    int32_t *status;
    uint64_t *sizes_out;  // sizes-only mode
    uint64_t *lookback;
    uint32_t *ticket;
    uint32_t *errflags;
    const uint64_t *slot_off;  // slotted outputs (LB = 0)
    const uint64_t *in_len;    // optional blob lengths (blob i = in[in_off[i] .. +in_len[i]))
    uint64_t *out_len;
};

constexpr int kMaxRef = 16;  // referenced streams <= word_size <= 16

template <int TEAM>
struct DecLayout {
    static constexpr int W = TEAM / 64;
    static constexpr int HEADS = TEAM * 16 * 2;  // u16 per stream position of a window
    static constexpr int SLOTS = 2 * W * 4 * 4;
    // misc (uint32): [0] msg [1] status [2] is_uncp [3] orig [4] ws [5] nref [6..7] base(u64)
    //   [8..8+16) ref stream k, [24..) soff, [40..) npairs,
    //   [56..56+128) selectors A/B per ref (8 each), [184..200) pidx, [200..216) pos, [216..232) carry
    static constexpr int MISC = 256 * 4;
    static constexpr int OFF_HEADS = 0;
    static constexpr int OFF_SLOTS = OFF_HEADS + HEADS;
    static constexpr int OFF_MISC = OFF_SLOTS + SLOTS;
    static constexpr int BYTES = OFF_MISC + MISC;
};

enum { D_MSG = 0, D_STATUS = 1, D_UNCP = 2, D_ORIG = 3, D_WS = 4, D_NREF = 5, D_BASE = 6,
       D_K = 8, D_SOFF = 24, D_NP = 40, D_SEL = 56, D_PIDX = 184, D_POS = 200, D_CARRY = 216 };

template <int TEAM, int SIZES_ONLY, int LB>
__global__ __launch_bounds__(TEAM) void tdt_decode_kernel(DecodeArgs a) {
    using Lay = DecLayout<TEAM>;
    constexpr int W = Lay::W;
    __shared__ __attribute__((aligned(16))) uint8_t smem[Lay::BYTES];
    uint16_t *heads = reinterpret_cast<uint16_t *>(smem + Lay::OFF_HEADS);
    uint32_t *slots = reinterpret_cast<uint32_t *>(smem + Lay::OFF_SLOTS);
    uint32_t *misc = reinterpret_cast<uint32_t *>(smem + Lay::OFF_MISC);
    const int tid = threadIdx.x;
    PSY_PROF_BEGIN();

    if (tid == 0) misc[D_MSG] = atomicAdd(a.ticket, 1u);
    team_sync<W>();
    const uint32_t msg = __builtin_amdgcn_readfirstlane(misc[D_MSG]);
    if (msg >= a.n_msgs) return;
    const uint64_t boff = a.in_off[msg];
    const uint64_t len = a.in_len ? a.in_len[msg] : a.in_off[msg + 1] - boff;
    const uint8_t *blob = a.in + boff;

    // ------------------------------------------------ header parse (thread 0)
    if (tid == 0) {
        uint32_t st = ST_OK, uncp = 0, orig = 0, ws = 0, nref = 0;
        uint64_t osize = 0;
        if (len < 4) {
            st = ST_SHORT;
        } else {
            const uint32_t magic = ld_u32_bytes(blob);
            if (magic == kMagicUNCP) {
                uncp = 1;
                osize = len - 4;
            } else if (magic != kMagicTDT) {
                st = ST_MAGIC;
            } else if (len < 20) {
                st = ST_TRUNCATED;
            } else {
                orig = ld_u32_bytes(blob + 4);
                const uint32_t ns = ld_u32_bytes(blob + 8);
                ws = ld_u32_bytes(blob + 12);
                const uint32_t msize = ld_u32_bytes(blob + 16);
                const int32_t wsi = (int32_t)ws;
                // deserialize :131-165 — header, mapping and stream table must fit
                const uint64_t toff = 20 + 4ull * msize;
                uint64_t off = toff;
                if (off > len) st = ST_TRUNCATED;
                for (uint32_t s = 0; s < ns && st == ST_OK; ++s) {
                    if (off + 4 > len) {
                        st = ST_TRUNCATED;
                        break;
                    }
                    const uint32_t sl = ld_u32_bytes(blob + off);
                    off += 4;
                    if (off + sl > len) st = ST_TRUNCATED;
                    off += sl;
                }
                // recombine :618-631 — word_size 0 divides by zero; mapping must cover ws
                // entries with values < num_streams whenever at least one word exists
                const uint64_t wc = wsi > 0 ? orig / (uint64_t)wsi : 0;
                if (st == ST_OK && wsi == 0) st = ST_BAD_HEADER;
                if (st == ST_OK && wc > 0) {
                    if (msize < ws) st = ST_BAD_MAPPING;
                    for (uint32_t b = 0; b < ws && st == ST_OK; ++b) {
                        const int32_t m = (int32_t)ld_u32_bytes(blob + 20 + 4 * b);
                        if (m < 0 || (uint32_t)m >= ns) st = ST_BAD_MAPPING;
                    }
                    if (st == ST_OK && (ws > 16 || (16 % ws) != 0)) st = ST_UNSUPPORTED;
                }
                uint32_t refc[kMaxRef];
                if (st == ST_OK && wc > 0) {
                    // distinct referenced streams, in order of first use
                    for (uint32_t b = 0; b < ws; ++b) {
                        const uint32_t m = ld_u32_bytes(blob + 20 + 4 * b);
                        uint32_t r = 0;
                        while (r < nref && refc[r] != m) ++r;
                        if (r == nref) refc[nref++] = m;
                    }
                    off = toff;
                    for (uint32_t s = 0; s < ns; ++s) {
                        const uint32_t sl = ld_u32_bytes(blob + off);
                        off += 4;
                        for (uint32_t r = 0; r < nref; ++r)
                            if (refc[r] == s) {
                                misc[D_SOFF + r] = (uint32_t)off;
                                misc[D_NP + r] = sl / 2;
                            }
                        off += sl;
                    }
                }
                if (st == ST_OK) {
                    osize = orig;
                    // per referenced stream: k and the scatter selectors (recombine :622-633)
                    const uint32_t WPG = (wc > 0) ? 16 / ws : 0;
                    for (uint32_t r = 0; r < nref; ++r) {
                        uint32_t k = 0;
                        for (uint32_t b = 0; b < ws; ++b) k += ld_u32_bytes(blob + 20 + 4 * b) == refc[r];
                        misc[D_K + r] = k;
                        for (int q = 0; q < 4; ++q) {
                            uint32_t A = 0x0c0c0c0cu, B = 0x0c0c0c0cu;
                            for (int t = 0; t < 4; ++t) {
                                const uint32_t i = 4 * q + t;  // output byte in group
                                const uint32_t w = i / ws, b = i % ws;
                                if (w >= WPG) continue;
                                if (ld_u32_bytes(blob + 20 + 4 * b) != refc[r]) continue;
                                uint32_t rank = 0;
                                for (uint32_t bb = 0; bb < b; ++bb) rank += ld_u32_bytes(blob + 20 + 4 * bb) == refc[r];
                                const uint32_t j = w * k + rank;
                                if (j < 8) A = (A & ~(0xffu << (8 * t))) | (j << (8 * t));
                                else B = (B & ~(0xffu << (8 * t))) | ((j - 8) << (8 * t));
                            }
                            misc[D_SEL + 8 * r + q] = A;
                            misc[D_SEL + 8 * r + 4 + q] = B;
                        }
                        misc[D_PIDX + r] = 0;
                        misc[D_POS + r] = 0;
                        misc[D_CARRY + r] = 0x100;  // none
                    }
                }
            }
        }
        if (st != ST_OK) osize = 0;
        misc[D_STATUS] = st;
        misc[D_UNCP] = uncp;
        misc[D_ORIG] = orig;
        misc[D_WS] = ws;
        misc[D_NREF] = nref;
        if constexpr (SIZES_ONLY) {
            a.sizes_out[msg] = osize;
            if (a.status) a.status[msg] = (int32_t)st;
        } else {
            *reinterpret_cast<uint64_t *>(misc + D_BASE) = osize;
        }
    }
    if constexpr (SIZES_ONLY) return;
    team_sync<W>();
    if (tid < 64) {  // wave 0: output placement (look-back on the decoded size, or slot)
        const uint64_t osize = *reinterpret_cast<const uint64_t *>(misc + D_BASE);
        uint64_t b;
        bool fits;
        if constexpr (LB) {
            b = lookback_excl_wave(a.lookback, msg, osize, a.errflags);
            fits = b + osize <= a.out_cap;
        } else {
            b = a.slot_off[msg];
            fits = osize <= a.slot_off[msg + 1] - b;
        }
        if (tid == 0) {
            uint32_t st = misc[D_STATUS];
            *reinterpret_cast<uint64_t *>(misc + D_BASE) = b;
            if constexpr (LB) {
                a.out_off[msg] = b;
                if (msg == a.n_msgs - 1) a.out_off[a.n_msgs] = b + osize;
            }
            if (st == ST_OK && !fits) {
                st = ST_CAPACITY;
                misc[D_STATUS] = st;
            }
            if constexpr (!LB) {
                if (a.out_len) a.out_len[msg] = st == ST_OK ? osize : 0;
            }
            if (a.status) a.status[msg] = (int32_t)st;
        }
    }
    team_sync<W>();
    const uint32_t st = __builtin_amdgcn_readfirstlane(misc[D_STATUS]);
    if (st != ST_OK) return;
    PSY_PROF_MARK(8);
    const uint64_t ob = *reinterpret_cast<const uint64_t *>(misc + D_BASE);
    uint8_t *dst = a.out + ob;
    if (misc[D_UNCP]) {
        team_copy_g2g<TEAM>(dst, blob + 4, len - 4);
        return;
    }
    const uint32_t orig = __builtin_amdgcn_readfirstlane(misc[D_ORIG]);
    const int32_t wsi = (int32_t)__builtin_amdgcn_readfirstlane(misc[D_WS]);
    const uint64_t wc = wsi > 0 ? orig / (uint64_t)wsi : 0;
    const uint64_t wbytes = wc * (uint64_t)(wsi > 0 ? wsi : 0);
    // recombine :617 zero-initialises; bytes past the last whole word stay zero
    if (orig > wbytes) team_zero<TEAM>(dst + wbytes, orig - wbytes);
    if (wc == 0) return;
    const uint32_t ws = (uint32_t)wsi;
    const uint32_t WPG = 16 / ws;
    const uint32_t nref = __builtin_amdgcn_readfirstlane(misc[D_NREF]);
    const uint32_t ngroups = (uint32_t)((wbytes + 15) / 16);
    const uint64_t total_pos_words = wc;

    for (uint32_t gw0 = 0; gw0 < ngroups; gw0 += TEAM) {
        const uint32_t g = gw0 + tid;
        const int64_t vb64 = (int64_t)wbytes - 16 * (int64_t)g;
        const uint32_t vb = vb64 >= 16 ? 16u : (vb64 <= 0 ? 0u : (uint32_t)vb64);
        const uint32_t nvw = vb / ws;
        uint32_t od[4] = {0, 0, 0, 0};
        const uint64_t wend = (uint64_t)(gw0 + TEAM) * WPG < total_pos_words ? (uint64_t)(gw0 + TEAM) * WPG
                                                                              : total_pos_words;
        for (uint32_t r = 0; r < nref; ++r) {
            const uint32_t k = __builtin_amdgcn_readfirstlane(misc[D_K + r]);
            const uint32_t soff = __builtin_amdgcn_readfirstlane(misc[D_SOFF + r]);
            const uint32_t np = __builtin_amdgcn_readfirstlane(misc[D_NP + r]);
            const uint64_t P0 = (uint64_t)gw0 * WPG * k;
            const uint64_t P1 = wend * k;
            const uint32_t span = (uint32_t)(P1 - P0);
            for (uint32_t i = tid; i < span; i += TEAM) heads[i] = 0xffffu;
            uint32_t pidx = __builtin_amdgcn_readfirstlane(misc[D_PIDX + r]);
            uint64_t pos = __builtin_amdgcn_readfirstlane(misc[D_POS + r]);
            const uint32_t wcarry = __builtin_amdgcn_readfirstlane(misc[D_CARRY + r]);
            uint32_t carry = wcarry;
            team_sync<W>();
            // ---- pair rounds: heads for every pair starting in [P0, P1)
            while (pos < P1 && pidx < np) {
                const uint32_t p0 = pidx + 8u * tid;
                const int64_t vbytes = 2 * ((int64_t)np - (int64_t)p0);
                const int valid = vbytes >= 16 ? 16 : (vbytes <= 0 ? 0 : (int)vbytes);
                const uint4 pv = valid > 0 ? ld16_any(blob + soff + 2ull * p0, valid) : make_uint4(0, 0, 0, 0);
                const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
                uint32_t cnt[8], val[8], tot = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const bool ok = 2 * i + 1 < valid;  // pairs need i+1 < len (:600-601)
                    cnt[i] = ok ? (pw[i >> 1] >> (16 * (i & 1))) & 0xffu : 0u;
                    val[i] = (pw[i >> 1] >> (16 * (i & 1) + 8)) & 0xffu;
                    tot += cnt[i];
                }
                uint32_t ex[1] = {tot}, tt[1];
                team_excl_scan<W, 1, OpAdd>(ex, tt, slots);
                uint64_t s = pos + ex[0];
                uint32_t kc = 0, kv = 0, ke = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const bool real = 2 * i + 1 < valid;
                    if (real && s < P1) {
                        const uint32_t li = 8u * tid + i + 1;  // local index + 1
                        kc = li;
                        const uint64_t e = s + cnt[i];
                        ke = e > 0xffffffffull ? 0xffffffffu : (uint32_t)e;
                        if (cnt[i]) {
                            kv = (li << 8) | val[i];
                            if (s >= P0) heads[s - P0] = (uint16_t)val[i];
                        }
                    }
                    s += cnt[i];
                }
                uint32_t mx[3] = {kc, kv, ke}, mt[3];
                team_excl_scan<W, 3, OpMax>(mx, mt, slots + W * 4);
                const uint32_t consumed = mt[0];
                if (mt[1]) carry = mt[1] & 0xffu;
                if (consumed) pos = mt[2];
                pidx += consumed;
                if (consumed == 0) break;  // defensive: nothing starts below P1
            }
            PSY_PROF_MARK(9);
            const uint64_t cover = pos < P1 ? pos : P1;
            if (tid == 0) {
                misc[D_PIDX + r] = pidx;
                misc[D_POS + r] = (uint32_t)pos;
                misc[D_CARRY + r] = carry;
            }
            team_sync<W>();
            // ---- fill forward inside this thread's group
            const uint32_t L = nvw * k;
            const uint64_t gpos = (uint64_t)g * WPG * k;
            uint32_t hv[16];
            uint32_t lastkey = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                hv[j] = ((uint32_t)j < L) ? heads[gpos - P0 + j] : 0xffffu;
                if (hv[j] != 0xffffu) lastkey = ((uint32_t)(tid + 1) << 8) | hv[j];
            }
            uint32_t lk[1] = {lastkey}, lt[1];
            team_excl_scan<W, 1, OpMax>(lk, lt, slots);
            uint32_t cur = lk[0] ? (lk[0] & 0xffu) : (wcarry & 0xffu);
            uint32_t sb[4] = {0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (hv[j] != 0xffffu) cur = hv[j];
                const uint32_t b = ((uint32_t)j < L && gpos + j < cover) ? cur : 0u;
                sb[j >> 2] |= b << (8 * (j & 3));
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                od[q] |= __builtin_amdgcn_perm(sb[1], sb[0], misc[D_SEL + 8 * r + q]) |
                         __builtin_amdgcn_perm(sb[3], sb[2], misc[D_SEL + 8 * r + 4 + q]);
            team_sync<W>();  // heads are rewritten by the next stream
            PSY_PROF_MARK(10);
        }
        if (vb) st16_any(dst + 16ull * g, make_uint4(od[0], od[1], od[2], od[3]), (int)vb);
        PSY_PROF_MARK(11);
    }
}

}  // namespace psy
