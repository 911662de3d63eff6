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
// claimed through an atomic ticket.  A message is a sequence of 16-byte GROUPS; group g
// lives in thread (g mod TEAM) of round (g / TEAM) — every round is one fully coalesced
// 16 B/lane sweep.  Messages of up to G rounds stay in VGPRs across all three passes
// (histogram, count, emit), so HBM sees each payload byte once.
//
// RLE in parallel: for stream c a group holds L = words*k_c consecutive stream bytes,
// packed into 4 dwords.  Run starts come from a SWAR byte compare against the byte before
// (neq_prev_mask4).  The 255-count cap only splits the run that is carried INTO a group
// (runs starting inside a 16-byte group cannot reach 255 there), so one max-scan of "last
// run start" gives every group its carried run start and at most one cap boundary.  A
// sum-scan of chunk starts gives every pair its index; pairs are emitted at chunk ENDS
// (count known locally) into an LDS staging window whose start is congruent to its
// destination mod 16, then flushed with 16-byte stores.  Output offsets across messages
// come from a single-pass decoupled look-back (tdt_device.h), so the batch output is
// compacted with no extra pass.
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
    static constexpr int REGION = 2 * TEAM * 16 + 16;
    static constexpr int STAGE = 2 * REGION;
    static constexpr int TERMS = TB * 256 * 16;
    static constexpr int UNION = STAGE > TERMS ? STAGE : TERMS;
    static constexpr int SLOTS = 2 * W * 4 * 4;
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
    M_SELB = 16 /*8*/, M_DANG = 24 /*2*/, M_STATUS = 26, M_MAP = 32 /*16*/, M_ENT = 64 /*16 doubles*/,
    M_BASE = 96 /*u64*/, M_P = 100 /*2*/
};

__device__ __forceinline__ uint32_t popc(uint32_t x) { return (uint32_t)__builtin_popcount(x); }
__device__ __forceinline__ uint32_t hibit(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }
__device__ __forceinline__ uint32_t lobit(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
__device__ __forceinline__ uint32_t byte_of(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint32_t j) {
    const uint32_t w = j < 4 ? s0 : j < 8 ? s1 : j < 12 ? s2 : s3;
    return (w >> (8 * (j & 3))) & 0xffu;
}

// Uniform per-message stream description, read into SGPRs.
struct StreamDesc {
    uint32_t ns;
    uint32_t k[2];
    uint32_t last[2], first[2];
    uint32_t selA[2][4], selB[2][4];
};

// Per-group, per-stream RLE analysis shared by the count pass and the emit pass.
struct GS {
    uint32_t s[4];
    uint32_t L, gpos, mask, chunk, cs_enc;
};

template <int WS, int TEAM, int G, int MODE>
__global__ __launch_bounds__(TEAM) void tdt_encode_kernel(EncodeArgs a) {
    using Lay = EncLayout<WS, TEAM>;
    constexpr int W = Lay::W;
    constexpr int WPG = Lay::WPG;
    __shared__ __attribute__((aligned(16))) uint8_t smem[Lay::BYTES];
    uint32_t *hist = reinterpret_cast<uint32_t *>(smem + Lay::OFF_HIST);
    uint8_t *uni = smem + Lay::OFF_UNION;
    uint32_t *slots = reinterpret_cast<uint32_t *>(smem + Lay::OFF_SLOTS);
    uint32_t *misc = reinterpret_cast<uint32_t *>(smem + Lay::OFF_MISC);
    const int tid = threadIdx.x;

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
    const uint32_t nrounds = (ngroups + TEAM - 1) / TEAM;
    const bool resident = nrounds <= (uint32_t)G;
    const bool al16 = ((uintptr_t)base & 15) == 0;

    auto load_group = [&](uint32_t r) __attribute__((always_inline)) -> uint4 {
        const uint32_t g = r * TEAM + tid;
        const int64_t vb64 = (int64_t)n32 - 16 * (int64_t)g;
        const int vb = vb64 >= 16 ? 16 : (vb64 <= 0 ? 0 : (int)vb64);
        if (vb == 16 && al16) return *reinterpret_cast<const uint4 *>(base + 16ull * g);
        if (vb <= 0) return make_uint4(0, 0, 0, 0);
        return ld16_any(base + 16ull * g, vb);
    };

    // Resident messages keep their G rounds in VGPRs; the round loop ROTATES the array (all
    // indices compile-time constant) instead of indexing it with the runtime round number,
    // which would push it to scratch.
    uint4 dres[G];
#pragma unroll
    for (int r = 0; r < G; ++r)
        dres[r] = (resident && (uint32_t)r < nrounds) ? load_group(r) : make_uint4(0, 0, 0, 0);
    auto rotate = [&]() __attribute__((always_inline)) {
        const uint4 t = dres[0];
#pragma unroll
        for (int q = 0; q < G - 1; ++q) dres[q] = dres[q + 1];
        dres[G - 1] = t;
    };
    // body(r, data) for every round r < nrounds, in order
    auto for_rounds = [&](auto &&body) __attribute__((always_inline)) {
        const uint32_t iters = resident ? (uint32_t)G : nrounds;
        for (uint32_t r = 0; r < iters; ++r) {
            if (r < nrounds) body(r, resident ? dres[0] : load_group(r));
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
        // histograms: extract_features :441-446 over every word (full sample)
        for (int i = tid; i < WS * 256; i += TEAM) hist[i] = 0;
        team_sync<W>();
        const int lane = lane_id();
        for_rounds([&](uint32_t r, const uint4 d) __attribute__((always_inline)) {
            const uint32_t g = r * TEAM + tid;
            const int64_t vb64 = (int64_t)n32 - 16 * (int64_t)g;
            const int vb = vb64 >= 16 ? 16 : (vb64 <= 0 ? 0 : (int)vb64);
            const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const bool valid = i < vb;
                const uint32_t v = (dw[i >> 2] >> (8 * (i & 3))) & 0xffu;
                const uint64_t act = __ballot(valid);
                if (act == 0) continue;
                const int leader = __builtin_ctzll(act);
                const uint32_t lv = (uint32_t)__builtin_amdgcn_readlane((int)v, leader);
                const uint64_t same = __ballot(valid && v == lv);
                uint32_t *hb = hist + (i % WS) * 256;
                if (lane == leader) atomicAdd(hb + lv, (uint32_t)__builtin_popcountll(same));
                if (valid && v != lv) atomicAdd(hb + v, 1u);
            }
        });
        team_sync<W>();

        // entropies: calculate_entropy :470-480, TB byte positions per batch
        double *terms = reinterpret_cast<double *>(uni);
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
                for (int v = 0; v < 256; ++v) {
                    const uint32_t c = hist[b * 256 + v];
                    if (c) e = __builtin_fma(-terms[2 * (tid * 256 + v)], terms[2 * (tid * 256 + v) + 1], e);
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

        // Per-group analysis of stream c for round r (shared by both passes).
        auto analyze = [&](const uint4 &d, uint32_t g, int c, uint32_t prevb) __attribute__((always_inline)) -> GS {
            GS x;
            const int64_t vb64 = (int64_t)n32 - 16 * (int64_t)g;
            const uint32_t vb = vb64 >= 16 ? 16u : (vb64 <= 0 ? 0u : (uint32_t)vb64);
            x.L = (vb / WS) * sd.k[c];
            x.gpos = g * WPG * sd.k[c];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                x.s[q] = __builtin_amdgcn_perm(d.y, d.x, sd.selA[c][q]) |
                         __builtin_amdgcn_perm(d.w, d.z, sd.selB[c][q]);
            uint32_t m = neq_prev_mask4(x.s[0], prevb << 24) | (neq_prev_mask4(x.s[1], x.s[0]) << 4) |
                         (neq_prev_mask4(x.s[2], x.s[1]) << 8) | (neq_prev_mask4(x.s[3], x.s[2]) << 12);
            if (g == 0) m |= 1u;
            x.mask = x.L ? (m & ((1u << x.L) - 1u)) : 0u;
            x.chunk = 0;
            x.cs_enc = 0;
            return x;
        };

        // carried run start + 255-cap boundary → chunk-start mask (simple_rle_compress :567-575)
        auto chunks = [&](GS &x) __attribute__((always_inline)) {
            uint32_t cap = 0;
            if (x.L && !(x.mask & 1u) && x.cs_enc) {
                const uint32_t cs = x.cs_enc - 1;
                const uint32_t fs = x.mask ? lobit(x.mask) : x.L;
                const uint32_t kk = (x.gpos - cs + 254u) / 255u;
                const uint32_t cpos = cs + 255u * kk;
                if (cpos < x.gpos + fs) cap = 1u << (cpos - x.gpos);
            }
            x.chunk = x.mask | cap;
        };

        uint32_t carry_max[2] = {0, 0};
        uint32_t carry_P[2] = {0, 0};
        uint32_t scan_par = 0;

        // one round of the count pass (EMIT=false) or the emit pass (EMIT=true)
        auto round = [&](uint32_t r, const uint4 d, auto emit_tag, uint64_t out_base, const uint32_t *sdata,
                         uint64_t E) __attribute__((always_inline)) {
            constexpr bool EMIT = decltype(emit_tag)::value;
            const uint32_t g = r * TEAM + tid;
            const bool last_group = 16ull * (g + 1) >= n;
            uint32_t prevb[2] = {0, 0}, nextb[2] = {0, 0};
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if ((uint32_t)c < sd.ns && sd.k[c]) {
                    if (g > 0 && 16ull * g < n) prevb[c] = base[16ull * g - WS + sd.last[c]];
                    if (EMIT && !last_group) nextb[c] = base[16ull * (g + 1) + sd.first[c]];
                }
            }
            GS x[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) x[c] = analyze(d, g, c, prevb[c]);
            if (sd.ns < 2) {
                x[1].L = 0;
                x[1].mask = 0;
            }
            // max-scan of (last run start + 1)
            uint32_t mv[2], mt[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) mv[c] = x[c].mask ? x[c].gpos + hibit(x[c].mask) + 1u : 0u;
            team_excl_scan<W, 2, OpMax>(mv, mt, slots + (scan_par & 1) * W * 4);
            ++scan_par;
            uint32_t sv[4], st[4];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                x[c].cs_enc = mv[c] > carry_max[c] ? mv[c] : carry_max[c];
                carry_max[c] = mt[c] > carry_max[c] ? mt[c] : carry_max[c];
                chunks(x[c]);
                sv[c] = popc(x[c].chunk);
            }
            uint32_t endm[2] = {0, 0};
            if (EMIT) {
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    if (x[c].L) {
                        bool lend = last_group;
                        if (!lend) {
                            const uint32_t lb = byte_of(x[c].s[0], x[c].s[1], x[c].s[2], x[c].s[3], x[c].L - 1);
                            const uint32_t rs = x[c].mask ? x[c].gpos + hibit(x[c].mask) : x[c].cs_enc - 1;
                            lend = (nextb[c] != lb) || ((x[c].gpos + x[c].L - rs) % 255u == 0);
                        }
                        endm[c] = ((x[c].chunk >> 1) | ((uint32_t)lend << (x[c].L - 1))) & ((1u << x[c].L) - 1u);
                    }
                }
                if (tid == 0) {
                    misc[M_DANG + 0] = (x[0].L && !(x[0].chunk & 1u)) ? 1u : 0u;
                    misc[M_DANG + 1] = (x[1].L && !(x[1].chunk & 1u)) ? 1u : 0u;
                }
            }
            sv[2] = popc(endm[0]);
            sv[3] = popc(endm[1]);
            team_excl_scan<W, 4, OpAdd>(sv, st, slots + (scan_par & 1) * W * 4);
            ++scan_par;
            if (EMIT) {
                uint32_t k0[2], ra[2];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    k0[c] = carry_P[c] - misc[M_DANG + c];
                    const uintptr_t dst = (uintptr_t)a.out + out_base + sdata[c] + 2ull * k0[c];
                    ra[c] = (uint32_t)(dst & 15);
                }
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    uint32_t em = endm[c];
                    const uint32_t pb = carry_P[c] + sv[c];
                    const uint32_t rbase = Lay::OFF_UNION + c * Lay::REGION + ra[c];
                    while (em) {
                        const uint32_t j = lobit(em);
                        em &= em - 1u;
                        const uint32_t below = x[c].chunk & ((2u << j) - 1u);
                        uint32_t cnt, idx;
                        if (below) {
                            cnt = j - hibit(below) + 1u;
                            idx = pb + popc(below) - 1u;
                        } else {
                            const uint32_t cs = x[c].cs_enc - 1u;
                            const uint32_t st0 = cs + 255u * ((x[c].gpos + j - cs) / 255u);
                            cnt = x[c].gpos + j - st0 + 1u;
                            idx = pb - 1u;
                        }
                        const uint32_t val = byte_of(x[c].s[0], x[c].s[1], x[c].s[2], x[c].s[3], j);
                        const uint32_t rel = idx - k0[c];
                        if (rel < st[2 + c]) {  // always true for a consistent round
                            smem[rbase + 2u * rel] = (uint8_t)cnt;
                            smem[rbase + 2u * rel + 1u] = (uint8_t)val;
                        } else {
                            atomicOr(a.errflags, 2u);
                        }
                    }
                }
                team_sync<W>();
                // flush both regions: LDS (congruent mod 16 with the destination) → global
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    uint32_t len = 2u * st[2 + c];
                    if (len && sdata[c] + 2ull * k0[c] + len > E) {  // never for a consistent round
                        if (tid == 0) atomicOr(a.errflags, 4u);
                        len = 0;
                    }
                    if (len) {
                        uint8_t *dst = a.out + out_base + sdata[c] + 2ull * k0[c];
                        const uint32_t sb = Lay::OFF_UNION + c * Lay::REGION + ra[c];
                        const uint32_t head0 = (16u - ra[c]) & 15u;
                        const uint32_t head = head0 < len ? head0 : len;
                        const uint32_t body = (len - head) & ~15u;
                        if ((uint32_t)tid < head) dst[tid] = smem[sb + tid];
                        for (uint32_t k = tid; k < body / 16; k += TEAM)
                            *reinterpret_cast<uint4 *>(dst + head + 16 * k) =
                                *reinterpret_cast<const uint4 *>(smem + sb + head + 16 * k);
                        const uint32_t tail = len - head - body;
                        if ((uint32_t)tid < tail) dst[head + body + tid] = smem[sb + head + body + tid];
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < 2; ++c) carry_P[c] += st[c];
        };

        // ---------------------------------------------------------- pass A: count pairs
        const uint32_t nosd[2] = {0, 0};
        for_rounds([&](uint32_t r, const uint4 d) __attribute__((always_inline)) { round(r, d, std::false_type{}, 0, nosd, 0); });
        const uint32_t P0 = carry_P[0], P1 = sd.ns > 1 ? carry_P[1] : 0;
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
        carry_max[0] = carry_max[1] = 0;
        carry_P[0] = carry_P[1] = 0;
        for_rounds([&](uint32_t r, const uint4 d) __attribute__((always_inline)) { round(r, d, std::true_type{}, ob, sdata, E); });
    }
}

}  // namespace psy
