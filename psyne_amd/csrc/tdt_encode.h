// tdt_encode.h — batched TDT encode for CDNA4 (gfx950).
//
// Restates include/psyne/protocol/tdt_compression.hpp (reference):
//   encode                 :227-266  UNCP passthrough / TDT blob
//   should_transform       :186-201  (+ is_tensor_data :409-413) — evaluated per message
//   compress_tdt           :363-399  size % word_size guard → UNCP fallback (:256-265)
//   extract_features       :434-468  full-sample histograms (sample_fraction = 1.0)
//   calculate_entropy      :470-480  fma chain in bin order with glibc log2 (tdt_log2.h)
//   perform_clustering     :507-525  mapping[b] = entropy[b] > mean
//   separate_byte_streams  :527-549  byte-plane gather (v_perm_b32 selectors)
//   simple_rle_compress    :557-582  (count <= 255, value) pairs
//   TDTEncodedData::serialize :81-117
//
// Work decomposition: one TEAM-thread workgroup per message, message ids
// claimed through an atomic ticket.  A message is a sequence of 16-byte GROUPS.  Wave w of
// the team owns the contiguous group range [w·RW·64, (w+1)·RW·64): round r of the wave is
// one coalesced 1 KiB sweep (lane l ↔ group (w·RW + r)·64 + l).  Because every wave owns a
// contiguous stretch of the byte streams, all per-round scans are wave-level DPP scans with
// a uniform running carry; the team synchronises only to exchange wave carries (twice).
// Messages of up to G rounds per wave stay in VGPRs across all passes (the round arrays are
// rotated, never dynamically indexed), so HBM sees each payload byte once.
//
// RLE in parallel, per group and stream c (L = words·k_c consecutive stream bytes):
//   * run starts: SWAR byte compare against the byte before (neq_prev_mask4);
//   * the 255 cap only splits the run carried INTO a group (a run starting inside a 16-byte
//     group cannot reach 255 there), so a max-scan of the last run start gives every group
//     its carried run start and at most one cap boundary → chunk-start mask (kept in VGPRs);
//   * pairs are indexed by a sum-scan of chunk starts and emitted at chunk ENDS (the count
//     is known locally), slot by slot with predicated LDS stores into a per-wave window that
//     is congruent mod 16 with its destination, then flushed with 16-byte stores — the emit
//     pass has no workgroup barrier at all.
// Output offsets across messages come from a single-pass decoupled look-back.
#pragma once
#include "tdt_device.h"
#include "tdt_log2.h"

#include <type_traits>

namespace psy {

__constant__ double c_log2_tab[128] = PSY_LOG2_TAB_INIT;
__constant__ double c_log2_tab2[128] = PSY_LOG2_TAB2_INIT;

enum { MODE_ENCODE = 0, MODE_MAPPED = 1, MODE_ANALYZE = 2 };

// status codes (include/psyne_tdt.h)
enum { ST_OK = 0, ST_SHORT = 1, ST_MAGIC = 2, ST_TRUNCATED = 3, ST_BAD_MAPPING = 4, ST_CAPACITY = 5,
       ST_UNSUPPORTED = 6, ST_BAD_HEADER = 7, ST_CONFIG = 8, ST_ARG = 11 };

constexpr uint32_t kMagicTDT = 0x54445444u;
constexpr uint32_t kMagicUNCP = 0x554E4350u;

struct EncodeArgs {
    const uint8_t *in;
    const uint64_t *in_off;
    uint32_t n_msgs;
    uint8_t *out;
    uint64_t out_cap;
    uint64_t *out_off;
    int32_t *status;
    const int32_t *mapping_in;  // MODE_MAPPED
    uint32_t *hist_out;         // MODE_ANALYZE
    double *ent_out;
    int32_t *map_out;
    uint64_t *lookback;
    uint32_t *ticket;
    uint32_t *errflags;  // bit0 look-back timeout, bit1 staging index, bit2 flush bound
    uint64_t min_tensor;
    int32_t policy_on;  // bandwidth < threshold && cpu <= threshold (host-evaluated atomics)
};

template <int WS, int TEAM>
struct EncLayout {
    static constexpr int W = TEAM / 64;
    static constexpr int WPG = 16 / WS;  // words per 16-byte group
    static constexpr int TB = (TEAM >= 256) ? (WS < 4 ? WS : 4) : (WS < 2 ? WS : 2);
    static constexpr int HIST = WS * 256 * 4;
    static constexpr int WREGION = 2 * 64 * 16 + 16;  // one stream's pairs of one wave-round
    static constexpr int WSTAGE = 2 * WREGION;        // both streams, per wave
    static constexpr int STAGE = W * WSTAGE;
    static constexpr int TERMS = TB * 256 * 16;
    static constexpr int UNION = STAGE > TERMS ? STAGE : TERMS;
    static constexpr int SLOTS = W * 8 * 4;
    static constexpr int MISC = 512;
    static constexpr int OFF_HIST = 0;
    static constexpr int OFF_UNION = OFF_HIST + HIST;
    static constexpr int OFF_SLOTS = OFF_UNION + UNION;
    static constexpr int OFF_MISC = OFF_SLOTS + SLOTS;
    static constexpr int BYTES = OFF_MISC + MISC;
};

// misc area (uint32 index)
enum {
    M_MSG = 0, M_NS = 1, M_K = 2 /*2*/, M_LAST = 4 /*2*/, M_FIRST = 6 /*2*/, M_SELA = 8 /*8*/,
    M_SELB = 16 /*8*/, M_STATUS = 26, M_MAP = 32 /*16*/, M_ENT = 64 /*16 doubles*/, M_BASE = 96 /*u64*/
};
// per-wave slots (uint32, 8 per wave): 0,1 max(last run start+1); 2,3 chunk-start count;
// 4 chunk bit 0 of the wave's first group (stream 1 in bit 16); 5,6 max(last chunk start+1)

__device__ __forceinline__ uint32_t popc(uint32_t x) { return (uint32_t)__builtin_popcount(x); }
__device__ __forceinline__ uint32_t hibit(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }
__device__ __forceinline__ uint32_t lobit(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t dword_of(const uint4 &d, uint32_t q) {
    return q == 0 ? d.x : q == 1 ? d.y : q == 2 ? d.z : d.w;
}
__device__ __forceinline__ uint32_t shfl_up1(uint32_t x) { return (uint32_t)__shfl_up((int)x, 1); }
__device__ __forceinline__ uint32_t shfl_down1(uint32_t x) { return (uint32_t)__shfl_down((int)x, 1); }
__device__ __forceinline__ uint32_t rdlane(uint32_t x, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, l);
}

// Uniform per-message stream description.
struct StreamDesc {
    uint32_t ns;
    uint32_t k[2];
    uint32_t last[2], first[2];
    uint32_t selA[2][4], selB[2][4];
};

template <int WS, int TEAM, int G, int MODE>
__global__ __launch_bounds__(TEAM) void tdt_encode_kernel(EncodeArgs a) {
    using Lay = EncLayout<WS, TEAM>;
    constexpr int W = Lay::W;
    constexpr int WPG = Lay::WPG;
    __shared__ __attribute__((aligned(16))) uint8_t smem[Lay::BYTES];
    uint32_t *hist = reinterpret_cast<uint32_t *>(smem + Lay::OFF_HIST);
    uint32_t *slots = reinterpret_cast<uint32_t *>(smem + Lay::OFF_SLOTS);
    uint32_t *misc = reinterpret_cast<uint32_t *>(smem + Lay::OFF_MISC);
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int wv = tid >> 6;

    if (tid == 0) misc[M_MSG] = atomicAdd(a.ticket, 1u);
    team_sync<W>();
    const uint32_t msg = __builtin_amdgcn_readfirstlane(misc[M_MSG]);
    if (msg >= a.n_msgs) return;

    const uint64_t off0 = a.in_off[msg];
    const uint64_t n = a.in_off[msg + 1] - off0;
    const uint8_t *base = a.in + off0;

    bool compress;
    if constexpr (MODE == MODE_ANALYZE) {
        compress = (n > 0) && (n % WS == 0) && (n < (1ull << 32));
        if (!compress) {
            if (tid == 0 && a.status) a.status[msg] = ST_ARG;
            return;
        }
    } else {
        // should_transform :186-201, then compress_tdt's size guard :364-367.
        compress = a.policy_on && n >= a.min_tensor && (n % 4 == 0) && n >= 64 && (n % WS == 0) &&
                   n > 0 && n < (1ull << 32);
    }

    // ---------------------------------------------------------------- UNCP passthrough
    if (!compress) {
        if constexpr (MODE != MODE_ANALYZE) {
            const uint64_t E = n + 4;
            if (tid == 0) {
                uint64_t b = lookback_excl(a.lookback, msg, E, a.errflags);
                *reinterpret_cast<uint64_t *>(misc + M_BASE) = b;
            }
            team_sync<W>();
            const uint64_t ob = *reinterpret_cast<uint64_t *>(misc + M_BASE);
            const bool fits = ob + E <= a.out_cap;
            if (tid == 0) {
                a.out_off[msg] = ob;
                if (msg == a.n_msgs - 1) a.out_off[a.n_msgs] = ob + E;
                if (a.status) a.status[msg] = fits ? ST_OK : ST_CAPACITY;
            }
            if (fits) {
                uint8_t *dst = a.out + ob;
                if (tid < 4) dst[tid] = (uint8_t)(kMagicUNCP >> (8 * tid));
                team_copy_g2g<TEAM>(dst + 4, base, n);
            }
        }
        return;
    }

    const uint32_t n32 = (uint32_t)n;
    const uint32_t wc = n32 / WS;
    const uint32_t ngroups = (n32 + 15) / 16;
    const uint32_t RW = (ngroups + TEAM - 1) / TEAM;  // rounds per wave
    const bool resident = RW <= (uint32_t)G;
    const bool al16 = ((uintptr_t)base & 15) == 0;
    const uint32_t gw0 = (uint32_t)wv * RW * 64;  // first group of this wave

    auto vbytes = [&](uint32_t g) __attribute__((always_inline)) -> uint32_t {
        const int64_t vb64 = (int64_t)n32 - 16 * (int64_t)g;
        return vb64 >= 16 ? 16u : (vb64 <= 0 ? 0u : (uint32_t)vb64);
    };
    auto load_group = [&](uint32_t r) __attribute__((always_inline)) -> uint4 {
        const uint32_t g = gw0 + r * 64 + lane;
        const uint32_t vb = vbytes(g);
        if (vb == 16 && al16) return *reinterpret_cast<const uint4 *>(base + 16ull * g);
        if (vb == 0) return make_uint4(0, 0, 0, 0);
        return ld16_any(base + 16ull * g, (int)vb);
    };

    // Resident messages keep their RW <= G rounds in VGPRs.  The round loop ROTATES the
    // arrays (compile-time indices only) instead of indexing them with the round number,
    // which would push them to scratch.
    uint4 dres[G];
    uint32_t cres[G];  // chunk-start masks of both streams (stream 1 in the high half)
#pragma unroll
    for (int r = 0; r < G; ++r) {
        dres[r] = (resident && (uint32_t)r < RW) ? load_group(r) : make_uint4(0, 0, 0, 0);
        cres[r] = 0;
    }
    auto rotate = [&]() __attribute__((always_inline)) {
        const uint4 t = dres[0];
        const uint32_t c = cres[0];
#pragma unroll
        for (int q = 0; q < G - 1; ++q) {
            dres[q] = dres[q + 1];
            cres[q] = cres[q + 1];
        }
        dres[G - 1] = t;
        cres[G - 1] = c;
    };
    // body(r, data, chunk_slot&) for every round r < RW of this wave, in order
    auto for_rounds = [&](auto &&body) __attribute__((always_inline)) {
        const uint32_t iters = resident ? (uint32_t)G : RW;
        for (uint32_t r = 0; r < iters; ++r) {
            if (r < RW) body(r, resident ? dres[0] : load_group(r), cres[0]);
            if (resident) rotate();
        }
    };

    // ------------------------------------------------------------ mapping (analysis)
    if constexpr (MODE == MODE_MAPPED) {
        if (tid == 0) {
            uint32_t bad = 0;
            for (int b = 0; b < WS; ++b) {
                int32_t m = a.mapping_in[(uint64_t)msg * WS + b];
                bad |= (m < 0 || m > 1);
                misc[M_MAP + b] = (uint32_t)(m & 1);
            }
            misc[M_STATUS] = bad;
        }
        team_sync<W>();
        if (misc[M_STATUS]) {
            // invalid caller mapping: publish an empty output for this message
            if (tid == 0) {
                uint64_t b = lookback_excl(a.lookback, msg, 0, a.errflags);
                a.out_off[msg] = b;
                if (msg == a.n_msgs - 1) a.out_off[a.n_msgs] = b;
                if (a.status) a.status[msg] = ST_BAD_MAPPING;
            }
            return;
        }
    } else {
        // histograms: extract_features :441-446 over every word (full sample).  Zero bytes
        // (dominant in float tensors) are counted in registers and added once per wave.
        for (int i = tid; i < WS * 256; i += TEAM) hist[i] = 0;
        team_sync<W>();
        uint32_t zc[WS];
#pragma unroll
        for (int b = 0; b < WS; ++b) zc[b] = 0;
        for_rounds([&](uint32_t r, const uint4 d, uint32_t &) __attribute__((always_inline)) {
            const uint32_t vb = vbytes(gw0 + r * 64 + lane);
            const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint32_t v = (dw[i >> 2] >> (8 * (i & 3))) & 0xffu;
                if ((uint32_t)i < vb) {
                    if (v == 0) zc[i % WS]++;
                    else atomicAdd(hist + (i % WS) * 256 + v, 1u);
                }
            }
        });
#pragma unroll
        for (int b = 0; b < WS; ++b) {
            const uint32_t t = wave_reduce<OpAdd>(zc[b]);
            if (lane == 0 && t) atomicAdd(hist + b * 256, t);
        }
        team_sync<W>();

        // entropies: calculate_entropy :470-480, TB byte positions per batch
        double *terms = reinterpret_cast<double *>(smem + Lay::OFF_UNION);
        const double total = (double)wc;
        for (int q0 = 0; q0 < WS; q0 += Lay::TB) {
            for (int i = tid; i < Lay::TB * 256; i += TEAM) {
                const int b = q0 + i / 256;
                if (b < WS) {
                    const uint32_t c = hist[b * 256 + (i & 255)];
                    if (c) {
                        double prob, L;
                        {
#pragma clang fp contract(off)
                            prob = (double)c / total;
                            L = psy_log2_glibc(prob, c_log2_tab, c_log2_tab2);
                        }
                        terms[2 * i] = prob;
                        terms[2 * i + 1] = L;
                    }
                }
            }
            team_sync<W>();
            if (tid < Lay::TB && q0 + tid < WS) {
                const int b = q0 + tid;
                double e = 0.0;
#pragma unroll 8
                for (int v = 0; v < 256; ++v) {
                    const uint32_t c = hist[b * 256 + v];
                    const double p = terms[2 * (tid * 256 + v)];
                    const double L = terms[2 * (tid * 256 + v) + 1];
                    e = c ? __builtin_fma(-p, L, e) : e;
                }
                reinterpret_cast<double *>(misc + M_ENT)[b] = e;
            }
            team_sync<W>();
        }
        // perform_clustering :507-525
        if (tid == 0) {
            const double *ent = reinterpret_cast<const double *>(misc + M_ENT);
            double sum = 0.0;
            for (int b = 0; b < WS; ++b) sum += ent[b];
            double thr;
            {
#pragma clang fp contract(off)
                thr = sum / (double)WS;
            }
            for (int b = 0; b < WS; ++b) misc[M_MAP + b] = ent[b] > thr ? 1u : 0u;
        }
        team_sync<W>();
        if constexpr (MODE == MODE_ANALYZE) {
            const uint64_t mb = (uint64_t)msg * WS;
            if (a.hist_out)
                for (int i = tid; i < WS * 256; i += TEAM) a.hist_out[mb * 256 + i] = hist[i];
            if (tid < WS) {
                if (a.ent_out) a.ent_out[mb + tid] = reinterpret_cast<const double *>(misc + M_ENT)[tid];
                if (a.map_out) a.map_out[mb + tid] = (int32_t)misc[M_MAP + tid];
            }
            if (tid == 0 && a.status) a.status[msg] = ST_OK;
            return;
        }
    }

    if constexpr (MODE != MODE_ANALYZE) {
        // ------------------------------------------------ stream descriptors (thread 0)
        if (tid == 0) {
            uint32_t ns = 1;
            for (int b = 0; b < WS; ++b)
                if (misc[M_MAP + b]) ns = 2;
            misc[M_NS] = ns;
            for (int c = 0; c < 2; ++c) {
                uint32_t pos[WS];
                uint32_t k = 0;
                for (int b = 0; b < WS; ++b)
                    if (misc[M_MAP + b] == (uint32_t)c) pos[k++] = b;
                misc[M_K + c] = k;
                misc[M_LAST + c] = k ? pos[k - 1] : 0;
                misc[M_FIRST + c] = k ? pos[0] : 0;
                for (int q = 0; q < 4; ++q) {
                    uint32_t A = 0x0c0c0c0cu, B = 0x0c0c0c0cu;
                    for (int t = 0; t < 4; ++t) {
                        const uint32_t j = 4 * q + t;
                        if (k && j < WPG * k) {
                            const uint32_t src = (j / k) * WS + pos[j % k];
                            if (src < 8) A = (A & ~(0xffu << (8 * t))) | (src << (8 * t));
                            else B = (B & ~(0xffu << (8 * t))) | ((src - 8) << (8 * t));
                        }
                    }
                    misc[M_SELA + 4 * c + q] = A;
                    misc[M_SELB + 4 * c + q] = B;
                }
            }
        }
        team_sync<W>();
        StreamDesc sd;
        sd.ns = __builtin_amdgcn_readfirstlane(misc[M_NS]);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            sd.k[c] = __builtin_amdgcn_readfirstlane(misc[M_K + c]);
            sd.last[c] = __builtin_amdgcn_readfirstlane(misc[M_LAST + c]);
            sd.first[c] = __builtin_amdgcn_readfirstlane(misc[M_FIRST + c]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                sd.selA[c][q] = __builtin_amdgcn_readfirstlane(misc[M_SELA + 4 * c + q]);
                sd.selB[c][q] = __builtin_amdgcn_readfirstlane(misc[M_SELB + 4 * c + q]);
            }
        }
        if (sd.ns < 2) sd.k[1] = 0;  // stream 1 absent: every group has L = 0 for it
        // the byte of the previous group that precedes stream c's first byte of a group
        uint32_t pq[2], pb[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint32_t i = 16 - WS + sd.last[c];
            pq[c] = i >> 2;
            pb[c] = 8 * (i & 3);
        }

        auto gather = [&](const uint4 &d, int c, uint32_t (&s)[4]) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                s[q] = __builtin_amdgcn_perm(d.y, d.x, sd.selA[c][q]) | __builtin_amdgcn_perm(d.w, d.z, sd.selB[c][q]);
        };
        // run-start masks of both streams for round r (stream 1 in bits 16..31)
        auto run_masks = [&](uint32_t r, const uint4 &d) __attribute__((always_inline)) -> uint32_t {
            const uint32_t g = gw0 + r * 64 + lane;
            const uint32_t nvw = vbytes(g) / WS;
            uint32_t out = 0;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (sd.k[c] == 0) continue;  // uniform
                const uint32_t L = nvw * sd.k[c];
                // previous group's last word from lane-1; lane 0 reads it from memory
                const uint32_t pw = shfl_up1(dword_of(d, pq[c]));
                uint32_t prevb = (pw >> pb[c]) & 0xffu;
                if (lane == 0 && g > 0 && L) prevb = base[16ull * g - WS + sd.last[c]];
                uint32_t s[4];
                gather(d, c, s);
                uint32_t m = neq_prev_mask4(s[0], prevb << 24) | (neq_prev_mask4(s[1], s[0]) << 4) |
                             (neq_prev_mask4(s[2], s[1]) << 8) | (neq_prev_mask4(s[3], s[2]) << 12);
                if (g == 0) m |= 1u;
                m = L ? (m & ((1u << L) - 1u)) : 0u;
                out |= m << (16 * c);
            }
            return out;
        };
        // chunk-start masks for round r given run-start masks m and the carried maximum of
        // (last run start + 1) before the round; advances the carry (rm).
        auto chunk_masks = [&](uint32_t r, uint32_t m, uint32_t (&rm)[2]) __attribute__((always_inline)) -> uint32_t {
            const uint32_t g = gw0 + r * 64 + lane;
            const uint32_t nvw = vbytes(g) / WS;
            uint32_t chunkp = 0;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (sd.k[c] == 0) continue;
                const uint32_t mc = (m >> (16 * c)) & 0xffffu;
                const uint32_t L = nvw * sd.k[c];
                const uint32_t gpos = g * WPG * sd.k[c];
                const uint32_t mv = mc ? gpos + hibit(mc) + 1u : 0u;
                const uint32_t inc = wave_incl_scan<OpMax>(mv);
                uint32_t cs_enc = wave_shift_up1(inc);
                cs_enc = umax(cs_enc, rm[c]);
                rm[c] = umax(rm[c], rdlane(inc, 63));
                // 255-cap inside the carried run (simple_rle_compress :568)
                uint32_t cap = 0;
                if (L && !(mc & 1u) && cs_enc) {
                    const uint32_t cs = cs_enc - 1;
                    const uint32_t fs = mc ? lobit(mc) : L;
                    const uint32_t cpos = cs + 255u * ((gpos - cs + 254u) / 255u);
                    if (cpos < gpos + fs) cap = 1u << (cpos - gpos);
                }
                chunkp |= (mc | cap) << (16 * c);
            }
            return chunkp;
        };

        // ---------------------------------------------------------- pass A1: run starts
        uint32_t wmax[2] = {0, 0};
        for_rounds([&](uint32_t r, const uint4 d, uint32_t &cm) __attribute__((always_inline)) {
            const uint32_t g = gw0 + r * 64 + lane;
            const uint32_t m = run_masks(r, d);
            cm = m;  // kept for A2 (resident messages)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (sd.k[c] == 0) continue;
                const uint32_t mc = (m >> (16 * c)) & 0xffffu;
                const uint32_t gpos = g * WPG * sd.k[c];
                const uint32_t mv = mc ? gpos + hibit(mc) + 1u : 0u;
                wmax[c] = umax(wmax[c], wave_reduce<OpMax>(mv));
            }
        });
        if (lane == 0) {
            slots[wv * 8 + 0] = wmax[0];
            slots[wv * 8 + 1] = wmax[1];
        }
        team_sync<W>();
        uint32_t rin[2] = {0, 0};  // max (run start + 1) before this wave
#pragma unroll
        for (int ww = 0; ww < W; ++ww)
            if (ww < wv) {
                rin[0] = umax(rin[0], slots[ww * 8 + 0]);
                rin[1] = umax(rin[1], slots[ww * 8 + 1]);
            }
        rin[0] = __builtin_amdgcn_readfirstlane(rin[0]);
        rin[1] = __builtin_amdgcn_readfirstlane(rin[1]);

        // ---------------------------------------------------------- pass A2: chunk starts
        uint32_t rm[2] = {rin[0], rin[1]};
        uint32_t psum[2] = {0, 0}, cmaxw[2] = {0, 0};
        uint32_t fb0 = 0;  // chunk bit 0 of this wave's first group (stream 1 in bit 16)
        for_rounds([&](uint32_t r, const uint4 d, uint32_t &cm) __attribute__((always_inline)) {
            const uint32_t g = gw0 + r * 64 + lane;
            const uint32_t m = resident ? cm : run_masks(r, d);
            const uint32_t chunkp = chunk_masks(r, m, rm);
            if (resident) cm = chunkp;  // kept for pass B
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (sd.k[c] == 0) continue;
                const uint32_t ch = (chunkp >> (16 * c)) & 0xffffu;
                const uint32_t gpos = g * WPG * sd.k[c];
                psum[c] += wave_reduce<OpAdd>(popc(ch));
                cmaxw[c] = umax(cmaxw[c], wave_reduce<OpMax>(ch ? gpos + hibit(ch) + 1u : 0u));
            }
            if (r == 0) fb0 = rdlane(chunkp, 0) & 0x10001u;
        });
        if (lane == 0) {
            slots[wv * 8 + 2] = psum[0];
            slots[wv * 8 + 3] = psum[1];
            slots[wv * 8 + 4] = fb0;
            slots[wv * 8 + 5] = cmaxw[0];
            slots[wv * 8 + 6] = cmaxw[1];
        }
        team_sync<W>();
        uint32_t pin[2] = {0, 0}, ptot[2] = {0, 0}, cin[2] = {0, 0};
#pragma unroll
        for (int ww = 0; ww < W; ++ww) {
            const uint32_t s0 = slots[ww * 8 + 2], s1 = slots[ww * 8 + 3];
            if (ww < wv) {
                pin[0] += s0;
                pin[1] += s1;
                cin[0] = umax(cin[0], slots[ww * 8 + 5]);
                cin[1] = umax(cin[1], slots[ww * 8 + 6]);
            }
            ptot[0] += s0;
            ptot[1] += s1;
        }
        const uint32_t nfb = __builtin_amdgcn_readfirstlane((wv + 1 < W) ? slots[(wv + 1) * 8 + 4] : 0u);
        const uint32_t P0 = __builtin_amdgcn_readfirstlane(ptot[0]);
        const uint32_t P1 = sd.ns > 1 ? __builtin_amdgcn_readfirstlane(ptot[1]) : 0u;
        const uint32_t hdr = 20 + 4 * WS;
        const uint64_t E = hdr + (4 + 2ull * P0) + (sd.ns > 1 ? 4 + 2ull * P1 : 0);
        if (tid == 0) {
            uint64_t b = lookback_excl(a.lookback, msg, E, a.errflags);
            *reinterpret_cast<uint64_t *>(misc + M_BASE) = b;
        }
        team_sync<W>();
        const uint64_t ob = *reinterpret_cast<uint64_t *>(misc + M_BASE);
        const bool fits = ob + E <= a.out_cap;
        if (tid == 0) {
            a.out_off[msg] = ob;
            if (msg == a.n_msgs - 1) a.out_off[a.n_msgs] = ob + E;
            if (a.status) a.status[msg] = fits ? ST_OK : ST_CAPACITY;
        }
        if (!fits) return;
        // header :84-106 and stream length words :110-112
        uint8_t *dst = a.out + ob;
        const uint32_t sdata[2] = {hdr + 4, hdr + 4 + 2 * P0 + 4};
        for (uint32_t t = tid; t < hdr; t += TEAM) {
            const int f = t >> 2, sh = 8 * (t & 3);
            uint32_t v;
            if (f == 0) v = kMagicTDT;
            else if (f == 1) v = n32;
            else if (f == 2) v = sd.ns;
            else if (f == 3 || f == 4) v = WS;
            else v = misc[M_MAP + (f - 5)];
            dst[t] = (uint8_t)(v >> sh);
        }
        if (tid < 8) {
            const int c = tid >> 2, sh = 8 * (tid & 3);
            if ((uint32_t)c < sd.ns) {
                const uint32_t len = 2 * (c ? P1 : P0);
                dst[sdata[c] - 4 + (tid & 3)] = (uint8_t)(len >> sh);
            }
        }

        // ---------------------------------------------------------- pass B: emit pairs
        // Everything below is wave-local: per-wave LDS staging, no workgroup barrier.
        const uint32_t wst = Lay::OFF_UNION + wv * Lay::WSTAGE;
        uint32_t pr[2] = {(uint32_t)__builtin_amdgcn_readfirstlane(pin[0]), (uint32_t)__builtin_amdgcn_readfirstlane(pin[1])};
        uint32_t cmc[2] = {(uint32_t)__builtin_amdgcn_readfirstlane(cin[0]), (uint32_t)__builtin_amdgcn_readfirstlane(cin[1])};
        uint32_t rmB[2] = {rin[0], rin[1]};
        for_rounds([&](uint32_t r, const uint4 d, uint32_t &cm) __attribute__((always_inline)) {
            const uint32_t g = gw0 + r * 64 + lane;
            const uint32_t nvw = vbytes(g) / WS;
            const bool last_group = 16ull * (g + 1) >= n;
            const uint32_t chunkp = resident ? cm : chunk_masks(r, run_masks(r, d), rmB);
            const uint32_t nxt = shfl_down1(chunkp);  // next group's chunk starts (lanes < 63)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (sd.k[c] == 0) continue;  // uniform
                const uint32_t L = nvw * sd.k[c];
                const uint32_t gpos = g * WPG * sd.k[c];
                const uint32_t ch = (chunkp >> (16 * c)) & 0xffffu;
                // last chunk start (+1) before this group: wave max-scan + carry
                const uint32_t lc = ch ? gpos + hibit(ch) + 1u : 0u;
                const uint32_t cinc = wave_incl_scan<OpMax>(lc);
                uint32_t ccs = wave_shift_up1(cinc);
                ccs = umax(ccs, cmc[c]);
                const uint32_t ctot = rdlane(cinc, 63);
                // chunk starts before this group → pair indices
                const uint32_t pc = popc(ch);
                const uint32_t pinc = wave_incl_scan<OpAdd>(pc);
                const uint32_t pbase = pr[c] + pinc - pc;
                const uint32_t rtot = rdlane(pinc, 63);
                uint32_t s[4];
                gather(d, c, s);
                // chunk END at slot L-1 iff the next stream byte starts a chunk
                uint32_t e = 0;
                if (L) {
                    bool lend;
                    if (last_group) {
                        lend = true;
                    } else if (lane < 63) {
                        lend = (nxt >> (16 * c)) & 1u;
                    } else if (r + 1 < RW) {
                        // next group = lane 0 of this wave's next round: new run, or exactly
                        // 255 bytes after the start of the chunk holding the last byte
                        const uint32_t nb = base[16ull * (g + 1) + sd.first[c]];
                        const uint32_t lb = (s[(L - 1) >> 2] >> (8 * ((L - 1) & 3))) & 0xffu;
                        const uint32_t lcs = ch ? gpos + hibit(ch) : ccs - 1u;
                        lend = (nb != lb) || (gpos + L - lcs == 255u);
                    } else {
                        lend = (nfb >> (16 * c)) & 1u;  // next wave's first group
                    }
                    e = ((ch >> 1) | ((uint32_t)lend << (L - 1))) & ((1u << L) - 1u);
                }
                // staging window of this wave-round: the pairs ending here, [k0, k0 + ends)
                const uint32_t f0 = rdlane(ch, 0);
                const uint32_t dang = (rdlane(L, 0) && !(f0 & 1u)) ? 1u : 0u;
                const uint32_t k0 = pr[c] - dang;
                const uint32_t ends = wave_reduce<OpAdd>(popc(e));
                const uint64_t gdst = (uint64_t)(uintptr_t)dst + sdata[c] + 2ull * k0;
                const uint32_t ra = (uint32_t)(gdst & 15);
                const uint32_t rb = wst + c * Lay::WREGION + ra;
                // start of the chunk holding slot 0, relative to gpos (<= 0)
                int cst = (!(ch & 1u) && ccs) ? (int)(ccs - 1u) - (int)gpos : 0;
                uint32_t nst = 0;  // chunk starts at slots <= j
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint32_t isst = (ch >> j) & 1u;
                    nst += isst;
                    cst = isst ? j : cst;
                    if ((e >> j) & 1u) {
                        const uint32_t rel = pbase + nst - 1u - k0;
                        const uint32_t cnt = (uint32_t)(j - cst + 1);
                        const uint32_t val = (s[j >> 2] >> (8 * (j & 3))) & 0xffu;
                        if (rel < ends) {
                            smem[rb + 2 * rel] = (uint8_t)cnt;
                            smem[rb + 2 * rel + 1] = (uint8_t)val;
                        } else {
                            atomicOr(a.errflags, 2u);
                        }
                    }
                }
                team_sync<1>();  // this wave's staging writes are visible to its other lanes
                uint32_t len = 2u * ends;
                if (len && sdata[c] + 2ull * k0 + len > E) {  // never for a consistent round
                    if (lane == 0) atomicOr(a.errflags, 4u);
                    len = 0;
                }
                if (len) {
                    uint8_t *gd = dst + sdata[c] + 2ull * k0;
                    const uint32_t head0 = (16u - ra) & 15u;
                    const uint32_t head = head0 < len ? head0 : len;
                    const uint32_t body = (len - head) & ~15u;
                    if ((uint32_t)lane < head) gd[lane] = smem[rb + lane];
                    for (uint32_t k = lane; k < body / 16; k += 64)
                        *reinterpret_cast<uint4 *>(gd + head + 16 * k) =
                            *reinterpret_cast<const uint4 *>(smem + rb + head + 16 * k);
                    const uint32_t tail = len - head - body;
                    if ((uint32_t)lane < tail) gd[head + body + lane] = smem[rb + head + body + lane];
                }
                team_sync<1>();
                pr[c] += rtot;
                cmc[c] = umax(cmc[c], ctot);
            }
        });
    }
}

}  // namespace psy
