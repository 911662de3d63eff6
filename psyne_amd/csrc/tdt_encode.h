// tdt_encode.h — batched TDT encode for CDNA4 (gfx950), v3.
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
// Work decomposition: one TEAM-thread workgroup per message (message id =
// blockIdx for slotted outputs, an atomic ticket for the compacted look-back API).  A message
// is a sequence of 16-byte GROUPS.  Wave w owns the contiguous group range [w·RW·64,
// (w+1)·RW·64); round r of the wave is one coalesced 1 KiB sweep (lane l ↔ group
// (w·RW + r)·64 + l).  Aligned whole-group messages of up to G rounds per wave stay in VGPRs
// across all passes (a separate instantiation of the kernel body: fully unrolled round loops,
// compile-time array indices); pass A1 replaces each round's bytes by its slot word T.
//
// Both streams of a group live in ONE 16-slot word — stream 0 in slots [0, L0), stream 1 in
// [L0, 16) — transposed so that slot j = 4t + q is byte t of dword q: the byte before slot j
// is then the same byte of the previous dword, and the run-start mask of all 16 slots costs
// one v_perm plus a SWAR zero-byte test per dword.  Both streams' scans run as ONE packed
// scan (two u16 halves: v_pk_max_u16 / carry-free adds).  Passes per message:
//   H   histograms into replicated LDS bins (+ per-lane zero bins: no same-address atomics)
//   E   entropies (exact fma chain) → mapping → slot selectors
//   A1  run-start masks → each wave's last run start; a per-round block test that rules the
//       255-cap out for the message                                   (team exchange 1)
//   A2  only if the cap may occur: chunk-start masks (255-cap of the carried run)
//       → pair counts                                                  (team exchange 2)
//       → output slot (or decoupled look-back on the blob size) → header
//   B   per wave and round, every chunk start writes an entry (value, position) at its rank
//       (a running per-lane address: one mul24 select between the entry and a lane-private
//       junk dword); the flush forms pair k from entries k and k+1 (count = position
//       difference) with 2-byte stores coalesced across the wave; the round's last chunk stays
//       pending into the next round.  No workgroup barrier in pass B.
// tools/emulate_encode.py restates this algorithm lane for lane (tests/test_emulator.py).
#pragma once
#include "tdt_device.h"
#include "tdt_log2.h"

#include <type_traits>

namespace psy {

static __constant__ __attribute__((aligned(16))) double c_log2_tab[128] = PSY_LOG2_TAB_INIT;
static __constant__ __attribute__((aligned(16))) double c_log2_tab2[128] = PSY_LOG2_TAB2_INIT;

enum { MODE_ENCODE = 0, MODE_MAPPED = 1, MODE_ANALYZE = 2 };

// status codes (include/psyne_tdt.h)
enum { ST_OK = 0, ST_SHORT = 1, ST_MAGIC = 2, ST_TRUNCATED = 3, ST_BAD_MAPPING = 4, ST_CAPACITY = 5,
       ST_UNSUPPORTED = 6, ST_BAD_HEADER = 7, ST_CONFIG = 8, ST_ARG = 11 };

constexpr uint32_t kMagicTDT = 0x54445444u;
constexpr uint32_t kMagicUNCP = 0x554E4350u;

constexpr uint32_t kNone = 0xffffffffu;
constexpr uint32_t kTileGroups = 4096;  // one tile of a large message: 64 KiB = 512 lanes x 8 rounds
constexpr uint32_t kSpanTiles = 8;      // the histogram pass takes 8 tiles (512 KiB) per workgroup

// A large message on the tiled path (DESIGN.md §4 "large messages"): written by the plan
// kernel, completed by the histogram pass (mapping) and the scan (pair count, fit).
struct LMeta {
    uint32_t msg;      // message id (kNone: this entry fell back to the whole-message kernel)
    uint32_t ntiles;   // 64 KiB tiles
    uint32_t tile0;    // its first tile record
    uint32_t span0;    // its first span histogram (kSpanTiles tiles per span)
    uint32_t mapbits;  // bit b = mapping[b] (map pass)
    uint32_t P0;       // stream 0's pair count (scan)
    uint32_t fits;     // the blob fits its slot (scan)
    uint32_t pad;
};
// One tile: the count pass writes its local figures, the scan rewrites them in place for the
// emit pass.  Positions are stream positions (bytes of that stream before them in the message).
struct TileRec {
    uint32_t lrs[2];  // count: last run start + 1 in the tile (0: none) | scan: the same before the tile
    uint32_t frs[2];  // count: first run start in the tile (kNone: none)
    uint32_t cnt[2];  // count: chunk starts from the first run start on | scan: chunk starts before the tile
    uint32_t clean;   // count: the tile rules the 255-cap out | scan: and the run carried in has no cap
    uint32_t pad;
};

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
    uint32_t *errflags;  // bit0 look-back timeout, bit2 flush bound, bit3 a resident-only kernel got a streaming message
    const uint64_t *slot_off;  // slotted outputs (LB = 0): blob i at out + slot_off[i]
    uint64_t *out_len;         // slotted outputs: blob lengths
    uint64_t min_tensor;
    int32_t policy_on;  // bandwidth < threshold && cpu <= threshold (host-evaluated atomics)
    // slotted kernels: message ids from a class list (null: message id = blockIdx)
    const uint32_t *list;
    const uint32_t *list_count;  // the list's length (device memory: the plan's counter)
    uint32_t list_base;  // first list / tile entry of this launch (grids of < 2^32 threads)
    // (medium list only) the streaming-size messages, dispatched before `list`: a 256 KiB team
    // started late would run alone in the kernel's tail
    const uint32_t *list2;
    const uint32_t *list2_count;
    // tiled large messages: tile / span entries (L index | tile << 32); the plan's counters
    // (u32 view: [4] large messages, [6] tiles, [8] spans claimed) and the budgets it ran with
    const uint64_t *tiles;
    const uint32_t *pcnt;
    uint32_t lcap, tcap;  // large-message entries, tiles (spans: tcap / kSpanTiles)
    const uint64_t *spans;
    LMeta *lmeta;
    TileRec *trec;
    uint32_t *shist;  // per span: WS x 256 bin counts
    // the count pass's work list, appended by the map pass: every tile of a message whose mapping
    // is not the speculated one, and the tiles whose fused count could not rule the 255-cap out
    // (entries as `tiles`; its length is plan counter 11, u32 view pcnt[22])
    uint64_t *rtiles;
    unsigned long long *rcount;
};

template <int WS, int TEAM, int LB = 0>
struct EncLayout {
    static constexpr int W = TEAM / 64;
    static constexpr int WPG = 16 / WS;  // words per 16-byte group
    // histogram, per byte position (uint32): bins 1..255 x HC copies (bin v copy k at
    // (v - 1)·HC + k), one unused row, then 64 (unused) dwords.  Zero bytes are not counted in
    // LDS: their atomic is aimed past the allocation (dropped) and the zero count is the words
    // minus the nonzero total (round 5).
    // 16 KiB of copies whatever the word size for message-sized teams; one copy for the
    // one-wave small-message kernel (its LDS footprint sets how many messages a CU holds)
    static constexpr int HC = TEAM >= 256 ? 16 / WS : 1;
    static constexpr int LOG_HC = HC == 1 ? 0 : HC == 2 ? 1 : HC == 4 ? 2 : HC == 8 ? 3 : 4;
    static constexpr int ZB = 256 * HC;
    static constexpr int PS = 64 + 256 * HC;
    static constexpr int bin(int v, int k) { return (v - 1) * HC + k; }  // v >= 1
    static constexpr int HIST = WS * PS * 4;
    static constexpr int HISTA = HIST;
    // positions per batch of the exact (tie) path: 4 for message-sized teams; one for the
    // 256-lane team, whose LDS footprint (staging of 4 waves) sets its occupancy
    static constexpr int TB = (TEAM >= 512) ? (WS < 4 ? WS : 4) : 1;
    // one stream's pairs of one wave-round: alignment pad + 1024 pairs + one garbage pair
    static constexpr int WREGION = 16 + 2 * 64 * 16 + 16;
    // per wave: v4 emit — both streams' pair windows + a junk pair; v5 emit — 64 junk dwords,
    // then (pending + up to 64·16 entries) for the two streams together
    static constexpr int WSTAGE_V4 = 2 * WREGION + 16;
    static constexpr int WSTAGE_V5 = 256 + 4 * (2 + 64 * 16);
    // v6 (u16 entries): NB rounds per flush — 3 for message-sized teams (fewer flushes, the LDS
    // fits 3 workgroups per CU), 2 for the one-wave team (whose LDS sets messages per CU)
    // (512-lane teams: 2 rounds of staging, so that the team's LDS (38.3 KB) lets four teams share
    // a CU — 8 waves per SIMD, round 6 — where 3 rounds (50.9 KB) allowed three)
#ifndef PSY_ENC_NB6
#define PSY_ENC_NB6 2
#endif
// (the compacted look-back instances run at 6 waves per SIMD, three teams per CU: they keep 3
// rounds of staging — their first flush, where the team waits for its offset, comes a round
// later: C3 compacted encode 9.36-9.41 -> 8.80-8.82 ms, profiles/r06_bc/ab_compact/lb3/)
#ifndef PSY_ENC_NB6_LB
#define PSY_ENC_NB6_LB 3
#endif
    static constexpr int NB6 = TEAM >= 512 ? (LB ? PSY_ENC_NB6_LB : PSY_ENC_NB6) : TEAM >= 256 ? 3 : 2;
    static constexpr int WSTAGE_V6 = 16 + 2 * (3 + NB6 * 64 * 16);
    static constexpr int WSTAGE_45 = WSTAGE_V4 > WSTAGE_V5 ? WSTAGE_V4 : WSTAGE_V5;
    static constexpr int WSTAGE = ((WSTAGE_45 > WSTAGE_V6 ? WSTAGE_45 : WSTAGE_V6) + 15) / 16 * 16;
    static constexpr int STAGE = W * WSTAGE;
    static constexpr int TERMS = TEAM >= 256 ? TB * 256 * 16 : 0;  // one-wave teams: in registers
    // Two phases share one region: histogram + entropy terms + log2 tables (dead once the
    // mapping is known) and pass B's per-wave staging windows.
    // + log2 tables (2 KiB) + the per-message term table for counts 1..64 (1 KiB); one-wave
    // teams read the tables from constant memory and keep the term table in registers (their
    // LDS footprint sets how many messages a CU holds)
    static constexpr int ANALYSIS = HISTA + TERMS + (TEAM >= 256 ? 2048 + 1024 : 0);
    static constexpr int REGION = STAGE > ANALYSIS ? STAGE : ANALYSIS;
    static constexpr int SLOTS = W * 8 * 4;
    static constexpr int MISC = 512;
    static constexpr int WM = 176;  // mapping state (uint32)
    static constexpr int OFF_HIST = 0;
    static constexpr int OFF_TERMS = HISTA;
    static constexpr int OFF_LOG2 = HISTA + TERMS;
    static constexpr int OFF_CTAB = HISTA + TERMS + 2048;
    static constexpr int OFF_STAGE = 0;
    static constexpr int OFF_SLOTS = REGION;
    static constexpr int OFF_MISC = OFF_SLOTS + SLOTS;
    static constexpr int OFF_WMISC = OFF_MISC + MISC;
    static constexpr int BYTES = OFF_WMISC + WM * 4;
    static_assert((1 << LOG_HC) == HC, "histogram copies");
};

// misc area (uint32 index)
enum {
    M_MSG = 0, M_NS = 1, M_L0 = 2, M_K0 = 3, M_K1 = 4, M_SELA = 8 /*4*/, M_SELB = 12 /*4*/, M_EDA = 16,
    M_EDB = 17, M_EXACT = 18, M_STATUS = 26, M_MAP = 32 /*16*/, M_ENT = 64 /*16 doubles*/, M_BASE = 96 /*u64*/,
    M_SB = 100 /*16*/, M_PART = 128 /*16 doubles: per-wave entropy partials*/, M_Z = 48 /*16: zero-bin totals*/,
    M_MAPBITS = 5 /*bit b = mapping[b]*/, M_READY = 6 /*deferred look-back: offset published*/,
    M_CPART = 160 /*16: per-wave (or per-position) nonzero byte counts*/
};
// decision margin of the mapping fast path, in bits of entropy: > 2x its worst-case error
// delta <= 2^-18 (hardware log2 per count) + 5·2^-24·log2 N (float sums of <= 4 bins, plus the
// float count above 2^24) < 1.34e-5 for every N < 2^32.  (Was 1e-4 with 16-bin float groups: 0.7 % of C2's 1 KiB
// uniform messages fell inside it and ran the exact fma chains, ~20k VALU each.)
constexpr double kFastMargin = 3e-5;
// bins summed per float group before the double accumulation
constexpr int kFloatGroup = 4;

// The slot layout of a byte-plane mapping (separate_byte_streams :527-549): slot j < L0 of a
// 16-byte group is stream-0 byte j (word j / k0, position = the (j % k0)-th position mapped to
// 0), slot j >= L0 stream-1 byte j - L0; selA / selB are the v_perm selectors that gather T
// (slot 4t + q in byte t of T[q]) from the group's dwords (x,y) / (z,w); edA / edB the edges
// word (byte 0: stream 0's last slot, 1: slot 15, 2: stream 1's first slot).  A pure function of
// the mapping bits: compiled into constant tables for word sizes <= 8 (2^WS entries), so a
// message reads its layout with scalar loads instead of deriving it.
struct SlotLayout {
    uint32_t ns, L0, k0, k1, selA[4], selB[4], edA, edB, pad[2];
};
template <int WS>
struct SlotTable {
    SlotLayout e[1 << WS];
};
template <int WS>
constexpr SlotLayout make_slot_layout(uint32_t mb) {
    SlotLayout L{};
    uint32_t k[2] = {0, 0};
    for (int b = 0; b < WS; ++b) k[(mb >> b) & 1u]++;
    constexpr uint32_t WPG = 16 / WS;
    const uint32_t L0 = WPG * k[0];
    uint32_t sb[16] = {};
    for (uint32_t j = 0; j < 16; ++j) {
        const uint32_t c = j < L0 ? 0u : 1u;
        const uint32_t jj = c ? j - L0 : j;
        const uint32_t rank = jj % k[c];
        uint32_t b = 0, seen = 0;
        for (uint32_t bb = 0; bb < (uint32_t)WS; ++bb)
            if (((mb >> bb) & 1u) == c) {
                if (seen == rank) b = bb;
                ++seen;
            }
        sb[j] = (jj / k[c]) * WS + b;
    }
    L.ns = k[1] ? 2u : 1u;
    L.L0 = L0;
    L.k0 = k[0];
    L.k1 = k[1];
    for (uint32_t q = 0; q < 5; ++q) {
        uint32_t A = 0x0c0c0c0cu, B = 0x0c0c0c0cu;
        for (uint32_t t = 0; t < 4; ++t) {
            uint32_t sv = 0xffu;
            if (q < 4) sv = sb[4 * t + q];
            else if (t == 0 && L0 > 0) sv = sb[L0 - 1];
            else if (t == 1) sv = sb[15];
            else if (t == 2 && k[1]) sv = sb[L0];
            if (sv == 0xffu) continue;
            if (sv < 8) A = (A & ~(0xffu << (8 * t))) | (sv << (8 * t));
            else B = (B & ~(0xffu << (8 * t))) | ((sv - 8) << (8 * t));
        }
        if (q < 4) {
            L.selA[q] = A;
            L.selB[q] = B;
        } else {
            L.edA = A;
            L.edB = B;
        }
    }
    return L;
}
template <int WS>
constexpr SlotTable<WS> make_slot_table() {
    SlotTable<WS> t{};
    for (uint32_t mb = 0; mb < (1u << WS); ++mb) t.e[mb] = make_slot_layout<WS>(mb);
    return t;
}
static __constant__ SlotTable<1> c_slots1 = make_slot_table<1>();
static __constant__ SlotTable<2> c_slots2 = make_slot_table<2>();
static __constant__ SlotTable<4> c_slots4 = make_slot_table<4>();
static __constant__ SlotTable<8> c_slots8 = make_slot_table<8>();
template <int WS>
__device__ __forceinline__ const SlotLayout &slot_layout(uint32_t mb) {
    if constexpr (WS == 1) return c_slots1.e[mb];
    else if constexpr (WS == 2) return c_slots2.e[mb];
    else if constexpr (WS == 4) return c_slots4.e[mb];
    else return c_slots8.e[mb];
}
// Speculated mapping of the fused count (DESIGN.md §4 "speculated count"): the byte-plane
// mapping float gradients take (word size 4: the three low bytes high-entropy, the
// sign/exponent byte low: mapping [1,1,1,0]; word size 8: [1,1,1,1,1,1,0,0]).  The histogram pass
// of a streaming or tiled message also counts run starts under it; when the message's real
// mapping turns out to be this one the count pass over the message is skipped (one read less).
template <int WS>
constexpr uint32_t spec_mapbits() {
    return WS == 4 ? 0x7u : WS == 8 ? 0x3fu : 0xffffffffu;
}
// TileRec.clean written by the fused count when the tile may hold a 255-cap chunk start: the
// count pass runs for that tile whatever the mapping
constexpr uint32_t kRecount = 0xffffffffu;

// per-wave slots (uint32, 8 per wave): 0,1 max(last run start+1); 2,3 chunk-start count;
// 4 chunk bits of the wave's first group (combined slot layout)

typedef uint32_t u32_a2 __attribute__((aligned(2)));  // a dword stored at a 2-byte aligned address
__device__ __forceinline__ void st32a2_nt(uint8_t *p, uint32_t v) {  // (non-temporal: tdt_device.h st16_nt)
    __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32_a2 *)(p));
}
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t popc(uint32_t x) { return (uint32_t)__builtin_popcount(x); }
__device__ __forceinline__ uint32_t hibit(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }
__device__ __forceinline__ uint32_t lobit(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t rdlane(uint32_t x, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, l);
}
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
// Byte-lane layout of a group's 16 slot bits (resident bodies, word size <= 4): slot j = 4t + q
// at bit 8t + q, the position the SWAR zero-byte test of T[q] leaves it in, so that pass A1
// skips the compaction into 16 bits (round 5).  Monotonic in j, so hibit / lobit / "a bit above
// a low mask" keep their meaning; sb_slot maps a bit position back to the slot.
__host__ __device__ constexpr uint32_t sb_pos(uint32_t j) { return 8u * (j >> 2) + (j & 3u); }
__host__ __device__ constexpr uint32_t sb_slot(uint32_t b) { return ((b >> 3) << 2) | (b & 3u); }
__device__ __forceinline__ uint32_t sb_spread(uint32_t x) {  // 16-bit compact -> byte-lane
    return (x & 0xfu) | ((x & 0xf0u) << 4) | ((x & 0xf00u) << 8) | ((x & 0xf000u) << 12);
}
__device__ __forceinline__ uint32_t sb_compact(uint32_t x) {  // byte-lane -> 16-bit compact
    x = (x | (x >> 4)) & 0x00ff00ffu;
    return (x | (x >> 8)) & 0xffffu;
}
// bit j of e duplicated into bits 2j and 2j+1 (16 → 32 bits)
__device__ __forceinline__ uint32_t spread2(uint32_t e) {
    uint32_t x = e & 0xffffu;
    x = (x | (x << 8)) & 0x00ff00ffu;
    x = (x | (x << 4)) & 0x0f0f0f0fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x | (x << 1);
}

// LB = 1: compacted output, offsets by decoupled look-back (out_off written);
// LB = 0: slotted output at caller offsets (slot_off), lengths to out_len — no dependency
//         between messages.
// Occupancy target (min waves per SIMD) of the 512-lane teams: 4 workgroups per CU = 8 waves per
// SIMD (64 VGPRs; round 6: the C3 encode 7.44 -> 7.29 ms against 6 waves at 73 VGPRs, same box,
// alternating runs; its 8-VGPR spill is stored in pass A1 and reloaded in pass B, 3 dwords per
// lane).  The 256-lane teams stay at 6: their LDS (26 KB) allows no more.
#ifndef PSY_ENC_WPE
#define PSY_ENC_WPE 8
#endif
// cache policy of the resident message loads (raw buffer loads; gfx950: 2 = nt)
#ifndef PSY_ENC_LDAUX
#define PSY_ENC_LDAUX 0
#endif
#ifndef PSY_ENC_WPE_LB
#define PSY_ENC_WPE_LB 6
#endif
#define PSY_ENC_WAVES(TEAM, LB) ((TEAM) >= 512 ? ((LB) ? PSY_ENC_WPE_LB : PSY_ENC_WPE) : (TEAM) >= 256 ? 6 : 7)

// One message — or, TL > 0, part of a large message: TL 1 the histogram of one span of
// kSpanTiles tiles (UNCP messages: the span's copy), 4 the mapping from the message's span
// histograms (one team per message), 2 count and 3 emit one 64 KiB tile.
// PATH: which bodies the instance holds — 0 both (resident and streaming), 1 resident only
// (every message of its list is aligned and at most TEAM·G groups: the plan's medium list),
// 2 streaming only (any message: the plan's big list).  Separate instances keep the streaming
// body's live state out of the resident body's register allocation.
enum { PATH_BOTH = 0, PATH_RES = 1, PATH_STREAM = 2 };

template <int WS, int TEAM, int G, int MODE, int LB, int TL, int PATH = PATH_BOTH>
__device__ __forceinline__ void encode_one(const EncodeArgs &a, uint8_t *smem, uint32_t msg, uint32_t lj,
                                           uint32_t tile) {
    static_assert(TL == 0 || (TEAM * G == (int)kTileGroups && MODE == MODE_ENCODE && !LB), "tile shape");
    constexpr uint32_t kTG = TL == 1 ? kTileGroups * kSpanTiles : kTileGroups;  // groups per team
    using Lay = EncLayout<WS, TEAM, LB>;
    constexpr int W = Lay::W;
    constexpr int WPG = Lay::WPG;
    uint32_t *slots = reinterpret_cast<uint32_t *>(smem + Lay::OFF_SLOTS);
    uint32_t *misc = reinterpret_cast<uint32_t *>(smem + Lay::OFF_MISC);
    const int tid = threadIdx.x;
    const int lane = lane_id();
    // wave index, made provably uniform: everything derived from it (group ranges, round
    // bounds, full-round tests) is then scalar code instead of per-lane VALU work
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    PSY_PROF_BEGIN();

    if (msg >= a.n_msgs) return;
    PSY_PROF_MARK(0);

    const uint64_t off0 = a.in_off[msg];
    const uint64_t n = a.in_off[msg + 1] - off0;
    const uint8_t *base = a.in + off0;
    // slotted outputs: the slot is known now; loading it here keeps its latency off the
    // critical path between the count pass and the emit pass (round 6: loaded at its first use
    // instead, the C3 encode took 8.2-8.7 ms against 7.26)
    uint64_t slot_b = 0, slot_e = 0;
    if constexpr (!LB) {
        slot_b = a.slot_off[msg];
        slot_e = a.slot_off[msg + 1];
    }

    // Output placement of an E-byte result (all threads call it): returns the offset in
    // a.out and whether the result fits.
    auto place = [&](uint64_t E, bool &fits) __attribute__((always_inline)) -> uint64_t {
        uint64_t ob;
        if constexpr (LB) {
            if (wv == 0) {
#ifndef PSY_X_NOLB
                const uint64_t b = lookback_excl_wave(a.lookback, msg, E, a.errflags);
#else
                const uint64_t b = (uint64_t)msg * (28 + 4 * WS + 2ull * n);  // diagnostic: no look-back
#endif
                if (lane == 0) *reinterpret_cast<uint64_t *>(misc + M_BASE) = b;
            }
            team_sync<W>();
            ob = *reinterpret_cast<uint64_t *>(misc + M_BASE);
            fits = ob + E <= a.out_cap;
            if (tid == 0) {
                a.out_off[msg] = ob;
                if (msg == a.n_msgs - 1) a.out_off[a.n_msgs] = ob + E;
            }
        } else {
            ob = slot_b;
            fits = E <= slot_e - ob;
            if (tid == 0 && a.out_len) a.out_len[msg] = fits ? E : 0;
        }
        return ob;
    };

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
        if constexpr (TL == 1) {
            const uint64_t E = n + 4;
            const bool fits = E <= slot_e - slot_b;
            if (tile == 0 && tid == 0) {
                if (a.status) a.status[msg] = fits ? ST_OK : ST_CAPACITY;
                if (a.out_len) a.out_len[msg] = fits ? E : 0;
            }
            if (fits) {
                uint8_t *dst = a.out + slot_b;
                if (tile == 0 && tid < 4) dst[tid] = (uint8_t)(kMagicUNCP >> (8 * tid));
                const uint64_t t0 = 16ull * kTG * tile;  // this span's bytes
                team_copy_g2g<TEAM>(dst + 4 + t0, base + t0, n - t0 < 16ull * kTG ? n - t0 : 16ull * kTG);
            }
        } else if constexpr (MODE != MODE_ANALYZE && TL == 0) {
            const uint64_t E = n + 4;
            bool fits;
            const uint64_t ob = place(E, fits);
            if (tid == 0 && a.status) a.status[msg] = fits ? ST_OK : ST_CAPACITY;
            if (fits) {
                uint8_t *dst = a.out + ob;
                if (tid < 4) dst[tid] = (uint8_t)(kMagicUNCP >> (8 * tid));
                team_copy_g2g<TEAM>(dst + 4, base, n);
            }
        }
        return;
    }

    constexpr uint32_t kSpec = spec_mapbits<WS>();
    // the histogram pass counts run starts under the speculated mapping: tiled messages (TL 1,
    // one wave per tile) and streaming whole messages (TL 0)
    constexpr bool SPECA1 = kSpec != 0xffffffffu && MODE == MODE_ENCODE && (TL == 0 || TL == 1);
    // streaming rounds in flight per wave: the streaming-only kernel and the span pass have the
    // registers (37 / 30 VGPRs with one); kernels holding the resident body too keep one
    constexpr int PF = PATH == PATH_STREAM || TL == 1 ? 4 : 1;
    if constexpr (TL == 2 && kSpec != 0xffffffffu) {
        // the span pass counted this tile under the speculated mapping and it is the real one
        const LMeta &lm = a.lmeta[lj];
        if (lm.mapbits == kSpec && a.trec[lm.tile0 + tile].clean != kRecount) return;
    }

    const uint32_t n32 = (uint32_t)n;
    const uint32_t wc = n32 / WS;
    const uint32_t ngroups = (n32 + 15) / 16;
    // the team's groups: the whole message, or one tile of it
    const uint32_t tg0 = TL ? tile * kTG : 0u;
    const uint32_t tgn = TL == 4 ? 0u : TL ? umin(ngroups - tg0, kTG) : ngroups;
    // rounds per wave; a span pass that counts gives every wave exactly one tile
    const uint32_t RW = TL == 1 && SPECA1 ? kTileGroups / 64u : (tgn + TEAM - 1) / TEAM;
    const bool al16 = ((uintptr_t)base & 15) == 0;
    // Resident: the rounds fit in VGPRs and every group is a whole aligned 16 bytes, so the
    // loads are straight-line dwordx4s (below); anything else streams.
    const bool resident = TL != 4 && RW <= (uint32_t)G && al16 && (n32 & 15u) == 0;
    const uint32_t gw0 = tg0 + (uint32_t)wv * RW * 64;  // first group of this wave

    auto vbytes = [&](uint32_t g) __attribute__((always_inline)) -> uint32_t {
        const int64_t vb64 = (int64_t)n32 - 16 * (int64_t)g;
        return vb64 >= 16 ? 16u : (vb64 <= 0 ? 0u : (uint32_t)vb64);
    };
    auto load_group = [&](uint32_t g) __attribute__((always_inline)) -> uint4 {
        const uint32_t vb = vbytes(g);
        if (vb == 16 && al16) return *reinterpret_cast<const uint4 *>(base + 16ull * g);
        if (vb == 0) return make_uint4(0, 0, 0, 0);
        return ld16_any(base + 16ull * g, (int)vb);
    };
    // FULL round: its 64 groups all hold 16 message bytes (uniform; 32-bit so that it stays
    // on the scalar unit: gfx9 has no 64-bit scalar ordered compare, and the u64 form cost a
    // VGPR copy, two v_cmp_*_u64 and a select per round)
    const uint32_t nfull = n32 >> 4;  // whole groups of the message
    auto full_round = [&](uint32_t r) __attribute__((always_inline)) -> bool {
        return gw0 + r * 64u + 64u <= nfull;
    };

    // The rest of the kernel is instantiated twice: RES (the message's RW <= G rounds stay in
    // VGPRs) and streaming (every pass re-reads its rounds from HBM).  Two separate code paths,
    // so the register allocator never has to keep the resident arrays alive across the
    // streaming loops (which spilled them to scratch when both shared one path).
    auto run = [&](auto res_tag) __attribute__((always_inline)) {
    constexpr bool RES = decltype(res_tag)::value;
    constexpr int GR = RES ? G : 1;
    // Resident rounds live in fully unrolled loops (compile-time indices only): indexing the
    // arrays with a run-time round number would push them to scratch.
    uint4 dres[GR];     // the round's 16 bytes per lane; after pass A1 its slot word T
    uint32_t cres[GR];  // run-start masks (A1 → A2), then chunk-start masks (A2 → B)
    // glibc log2 tables for the entropy pass, fetched BEFORE the message's rounds so that the
    // LDS copy below waits for these loads only (issued after the rounds, its wait would
    // cover every round's load and stall the team until the whole message had arrived)
    constexpr int NL2 = W == 1 ? 1 : (128 + TEAM - 1) / TEAM;
    uint4 l2v[NL2];
    if constexpr (MODE != MODE_MAPPED && W > 1) {
#pragma unroll
        for (int k = 0; k < NL2; ++k) {
            const int i = (tid + k * TEAM) & 127;
            l2v[k] = reinterpret_cast<const uint4 *>(i < 64 ? c_log2_tab : c_log2_tab2)[i & 63];
        }
    }
    if constexpr (RES) {
        // One unconditional dwordx4 per lane and round, all in flight before the first use (a
        // branchy load per round made the compiler wait for each before issuing the next).
        // Raw buffer loads over the message (num_records = n): the round offsets are scalar
        // and lanes past the end read zeros from the hardware range check, so no per-round
        // address arithmetic (round 4: a compare, a select and a 64-bit address per round);
        // every pass masks those lanes by vbytes / vmask.  (A resident message is whole 16-byte
        // groups, n % 16 == 0, so num_records = n = ngroups·16: the range check never splits a
        // dword — ADVICE r05 asked.)
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), (short)0, (int)n32, 0x00020000);
        const int vo = (int)((gw0 + (uint32_t)lane) * 16u);
#pragma unroll
        for (int r = 0; r < G; ++r) {
            typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
            const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo, r * 1024, PSY_ENC_LDAUX);
            dres[r] = make_uint4(v.x, v.y, v.z, v.w);
            cres[r] = 0;
        }
    }
    // body(r, data&, cres&, res) for every round r < RW of this wave, in order.
    auto for_rounds = [&](auto &&body) __attribute__((always_inline)) {
        if constexpr (RES) {
#pragma unroll
            for (int r = 0; r < G; ++r)
                if ((uint32_t)r < RW) body((uint32_t)r, dres[r], cres[r], std::true_type{});
        } else {
            // rounds r < RW of the wave that hold a group of the message (uniform)
            auto live = [&](uint32_t r) __attribute__((always_inline)) {
                return r < RW && gw0 + r * 64u < ngroups;
            };
            if constexpr (PF == 1) {
                for (uint32_t r = 0; live(r); ++r) {
                    uint4 d = load_group(gw0 + r * 64 + lane);
                    uint32_t c = 0;
                    body(r, d, c, std::false_type{});
                }
            } else {
                // PF rounds in flight: round r + PF is loaded before round r is processed (one
                // load per round and its full HBM latency in front of every round left the
                // streaming kernels at half the resident kernels' rate: C4's 64 KiB - 1 MiB list)
                uint4 q[PF];
#pragma unroll
                for (int k = 0; k < PF; ++k) q[k] = live((uint32_t)k) ? load_group(gw0 + k * 64 + lane) : uint4{};
                bool go = true;
                for (uint32_t r0 = 0; go; r0 += PF) {
#pragma unroll
                    for (int k = 0; k < PF; ++k) {
                        const uint32_t r = r0 + (uint32_t)k;
                        if (!live(r)) {
                            go = false;
                            break;
                        }
                        uint4 d = q[k];
                        if (live(r + PF)) q[k] = load_group(gw0 + (r + PF) * 64 + lane);
                        uint32_t c = 0;
                        body(r, d, c, std::false_type{});
                    }
                }
            }
        }
    };

    // The message's mapping state: after the entropy terms wave 0 alone derives entropies,
    // mapping, slot layout and selectors (wave-local syncs), then ONE workgroup barrier.
    uint32_t *wm = reinterpret_cast<uint32_t *>(smem + Lay::OFF_WMISC);

    // ---- speculated count (streaming / tiled messages): pass A1 below, restated on the
    // speculated mapping's slot layout (a compile-time constant), run inside the histogram's
    // rounds; the accumulators stand in for pass A1's when the real mapping is kSpec
    constexpr bool SPEC_ON = SPECA1 && !RES;
    constexpr SlotLayout SS = make_slot_layout<WS>(SPEC_ON ? kSpec : 0u);
    constexpr bool s_ns2 = SS.ns == 2;
    constexpr uint32_t s_L0 = SS.L0, s_Ls0 = SS.L0, s_Ls1 = s_ns2 ? 16u - SS.L0 : 0u;
    constexpr uint32_t s_low = s_L0 >= 16 ? 0xffffu : ((1u << s_L0) - 1u);
    constexpr bool s_fold = WS <= 4;
    constexpr uint32_t s_p0sel =
        s_fold && s_ns2 ? (0x06050400u & ~(0xffu << (2u * s_L0))) | (0x01u << (2u * s_L0)) : 0x06050400u;
    constexpr uint64_t s_zk1[2] = {s_Ls0 < 16u ? 0x0101010101010101ull : 0x1111111111111111ull,
                                   s_Ls1 < 16u ? 0x0101010101010101ull : 0x1111111111111111ull};
    constexpr uint64_t s_zk8[2] = {s_Ls0 == 0u ? 0ull : s_Ls0 < 16u ? 0x8080808080808080ull : 0x8888888888888888ull,
                                   s_Ls1 == 0u ? 0ull : s_Ls1 < 16u ? 0x8080808080808080ull : 0x8888888888888888ull};
    uint32_t s_wmax[2] = {0, 0}, s_fmx[2] = {0, 0}, s_pc0 = 0, s_pc1 = 0, s_edc = 0;
    uint64_t s_zacc = 0;
    auto s_edges = [&](const uint4 &d) __attribute__((always_inline)) -> uint32_t {
        return perm(d.y, d.x, SS.edA) | perm(d.w, d.z, SS.edB);
    };
    if constexpr (SPEC_ON) {
        if (gw0 > 0 && gw0 - 1 < ngroups) s_edc = __builtin_amdgcn_readfirstlane(s_edges(load_group(gw0 - 1)));
    }
    auto spec_round = [&](uint32_t r, const uint4 &d) __attribute__((always_inline)) {
        const uint32_t g = gw0 + r * 64 + lane;
        uint32_t T[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) T[q] = perm(d.y, d.x, SS.selA[q]) | perm(d.w, d.z, SS.selB[q]);
        const uint32_t ed = s_edges(d);
        uint32_t V = 0xffffu;
        if (!full_round(r)) {
            const uint32_t nvw = vbytes(g) / WS;
            if (nvw < (uint32_t)(16 / WS)) {
                V = (1u << (nvw * SS.k0)) - 1u;
                if (s_ns2) V |= ((1u << (nvw * SS.k1)) - 1u) << s_L0;
            }
        }
        // run-start mask (the run_mask lambda of pass A1, on the constant layout)
        const uint32_t pe = wave_shr1(ed, s_edc);
        const uint32_t P0 = perm(T[3], pe, s_p0sel);
        const uint32_t X[4] = {T[0] ^ P0, T[1] ^ T[0], T[2] ^ T[1], T[3] ^ T[2]};
        uint32_t m = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t y = ((X[q] & 0x7f7f7f7fu) + 0x7f7f7f7fu) | X[q];
            m |= (y >> (7 - q)) & (0x01010101u << q);
        }
        m = (m | (m >> 4)) & 0x00ff00ffu;
        m = (m | (m >> 8)) & 0xffffu;
        if constexpr (!s_fold && s_ns2) {
            const uint32_t fx = ((ed >> 16) ^ (pe >> 8)) & 0xffu;
            m = (m & ~(1u << s_L0)) | ((fx ? 1u : 0u) << s_L0);
        }
        if (r == 0u && gw0 == 0u && lane == 0) m |= 1u | (s_ns2 ? (1u << s_L0) : 0u);
        m &= V;
        s_edc = rdlane(ed, 63);
        const uint64_t pastm = full_round(r) ? 0ull : (uint64_t)__ballot(g >= ngroups);
        const uint32_t m0 = m & s_low;
        if (m0) {
            s_wmax[0] = umax(s_wmax[0], g * s_Ls0 + hibit(m0) + 1u);
            if constexpr (TL == 1) s_fmx[0] = umax(s_fmx[0], ~(g * s_Ls0 + lobit(m0)));
        }
        s_pc0 += popc(m0);
        const uint64_t b0 = (uint64_t)__ballot(m0 != 0u) | pastm;
        s_zacc |= (b0 - s_zk1[0]) & ~b0 & s_zk8[0];
        if constexpr (s_ns2) {
            const uint32_t m1 = m >> s_L0;
            if (m1) {
                s_wmax[1] = umax(s_wmax[1], g * s_Ls1 + hibit(m1) + 1u);
                if constexpr (TL == 1) s_fmx[1] = umax(s_fmx[1], ~(g * s_Ls1 + lobit(m1)));
            }
            s_pc1 += popc(m1);
            const uint64_t b1 = (uint64_t)__ballot(m > s_low) | pastm;
            s_zacc |= (b1 - s_zk1[1]) & ~b1 & s_zk8[1];
        }
    };

    // ------------------------------------------------------------ mapping (analysis)
    if constexpr (MODE == MODE_MAPPED || TL == 2 || TL == 3) {
        uint32_t bad = 0, mbit = 0;
        if (lane < WS) {
            int32_t m;
            if constexpr (TL == 2 || TL == 3) m = (int32_t)((a.lmeta[lj].mapbits >> lane) & 1u);
            else m = a.mapping_in[(uint64_t)msg * WS + lane];
            bad = (m < 0 || m > 1) ? 1u : 0u;
            wm[M_MAP + lane] = (uint32_t)(m & 1);
            mbit = (uint32_t)(m & 1);
        }
        const bool anybad = __any(bad);
        const uint32_t mbits = (uint32_t)__ballot(mbit != 0u);  // (every wave: the same value)
        if (lane == 0) wm[M_MAPBITS] = mbits;
        team_sync<1>();
        if (anybad) {
            // invalid caller mapping: publish an empty output for this message
            bool fits;
            (void)place(0, fits);
            if (tid == 0 && a.status) a.status[msg] = ST_BAD_MAPPING;
            return;
        }
    } else {
        // histograms: extract_features :441-446 over every word (full sample).  Byte value
        // v at position p adds 1 to copy (lane mod HC) of bin v — or, for v = 0 (dominant in
        // float tensors), to this lane's private zero bin — so one ds_add only sends two
        // lanes to the same address when they hold the same nonzero value.
        uint32_t *hist = reinterpret_cast<uint32_t *>(smem + Lay::OFF_HIST);
        for (int i = tid; i < WS * Lay::PS / 4; i += TEAM) reinterpret_cast<uint4 *>(hist)[i] = make_uint4(0, 0, 0, 0);
        if (tid == 0) wm[M_READY] = 0u;  // (published by the barrier below)
        if constexpr (TL == 4) {
            // the message's histogram: the sum of its span histograms, into copy 0 of the bins
            team_sync<W>();
            const LMeta *lm = a.lmeta + lj;
            const uint32_t nsp = (lm->ntiles + kSpanTiles - 1) / kSpanTiles;
            const uint32_t *sh = a.shist + (uint64_t)lm->span0 * WS * 256;
            for (int i = tid; i < WS * 256; i += TEAM) {
                const int v = i & 255;
                if (v == 0) continue;  // (the zero count is derived from the nonzero total below)
                uint32_t c = 0;
                for (uint32_t k = 0; k < nsp; ++k) c += sh[(uint64_t)k * WS * 256 + i];
                hist[(i >> 8) * Lay::PS + Lay::bin(v, 0)] = c;
            }
        }
        // glibc log2 tables → LDS (the bins' log2 evaluations read them with per-lane indices)
        if constexpr (W > 1) {
#pragma unroll
            for (int k = 0; k < NL2; ++k)
                if (tid + k * TEAM < 128) reinterpret_cast<uint4 *>(smem + Lay::OFF_LOG2)[tid + k * TEAM] = l2v[k];
        }
        team_sync<W>();
        // Compare-free bin address: v·4HC + 4(copy - HC) is bin v's copy for v >= 1 and wraps
        // to >= 2^16 - 4HC for v = 0: an address past every encode workgroup's LDS allocation,
        // so the zero byte's atomic is dropped (tools/ubench_lds.hip: out-of-range ds_add lands
        // nowhere) and the zero count is derived from the nonzero total.  Two bytes per
        // instruction in u16 halves (v_pk_mad_u16, then v_and / v_lshrrev split the two
        // addresses): round 4's per-lane zero bins took a v_pk_min_u16 per byte pair more.
        static_assert(Lay::BYTES <= 65536 - 4 * Lay::HC, "zero-byte atomics must fall past the allocation");
        const uint32_t coff = (((uint32_t)lane & (Lay::HC - 1)) - (uint32_t)Lay::HC) * 4u;
        const uint32_t coff2 = (coff & 0xffffu) * 0x10001u;
        constexpr uint32_t kMul2 = (uint32_t)(4 * Lay::HC) * 0x10001u;
        auto hist_group = [&](const uint4 &d, uint32_t vb, bool full) __attribute__((always_inline)) {
            const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                // bytes (0, 2) of a dword with one v_and, bytes (1, 3) with v_lshrrev + v_and
                // (2-cycle ops, where a v_perm costs 4)
                const int w = i >> 2, o = (i >> 1) & 1;
                const uint32_t P = (o ? dw[w] >> 8 : dw[w]) & 0x00ff00ffu;
                uint32_t A;
                asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(A) : "v"(P), "s"(kMul2), "v"(coff2));
                const uint32_t ad2[2] = {A & 0xffffu, A >> 16};
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int b = 4 * w + o + 2 * h;
#ifndef PSY_X_NOHIST
                    if (full || (uint32_t)b < vb)
#else
                    if (vb == 12345u)
#endif
                        atomicAdd(reinterpret_cast<uint32_t *>(smem + Lay::OFF_HIST + (b % WS) * Lay::PS * 4 + ad2[h]), 1u);
                }
            }
        };
        const double *ltab = W == 1 ? c_log2_tab : reinterpret_cast<const double *>(smem + Lay::OFF_LOG2);
        const double *ltab2 = W == 1 ? c_log2_tab2 : ltab + 128;
        const double total = (double)wc;
        if constexpr (TL != 4)
        for_rounds([&](uint32_t r, uint4 &d, uint32_t &, auto) __attribute__((always_inline)) {
            PSY_ASM_ROUND(H);
            if (full_round(r)) hist_group(d, 16, true);
            else hist_group(d, vbytes(gw0 + r * 64 + lane), false);
            if constexpr (SPEC_ON) spec_round(r, d);
        });
        team_sync<W>();
        PSY_PROF_MARK(1);
        if constexpr (TL == 1 && SPEC_ON) {
            // this wave's tile, counted under the speculated mapping (the count pass's record:
            // last run start + 1, first run start, run starts, cap ruled out — or kRecount)
            const LMeta &lm = a.lmeta[lj];
            const uint32_t tl = tile * kSpanTiles + (uint32_t)wv;
            const uint32_t w0 = wave_reduce<OpMax>(s_wmax[0]), w1 = wave_reduce<OpMax>(s_wmax[1]);
            const uint32_t f0 = wave_reduce<OpMax>(s_fmx[0]), f1 = wave_reduce<OpMax>(s_fmx[1]);
            const uint32_t p0 = wave_reduce<OpAdd>(s_pc0), p1 = wave_reduce<OpAdd>(s_pc1);
            if (lane == 0 && tl < lm.ntiles) {
                TileRec *t = a.trec + lm.tile0 + tl;
                t->lrs[0] = w0;
                t->lrs[1] = w1;
                t->frs[0] = ~f0;
                t->frs[1] = ~f1;
                t->cnt[0] = p0;
                t->cnt[1] = p1;
                t->clean = s_zacc != 0ull ? kRecount : 1u;
            }
        }
        if constexpr (TL == 1) {
            // the span's histogram (its LDS copies summed; the zero count = the span's words
            // minus its nonzero total), for the map pass
            uint32_t *sh = a.shist + ((uint64_t)a.lmeta[lj].span0 + tile) * WS * 256;
            uint32_t *tot = wm + M_CPART;
            if (tid < WS) tot[tid] = 0u;
            team_sync<W>();
            for (int i = tid; i < WS * 256; i += TEAM) {
                const int b = i >> 8, v = i & 255;
                if (v == 0) continue;
                uint32_t c = 0;
#pragma unroll
                for (int k = 0; k < Lay::HC; ++k) c += hist[b * Lay::PS + Lay::bin(v, k)];
                sh[i] = c;
                if (c) atomicAdd(&tot[b], c);
            }
            team_sync<W>();
            if (tid < WS) {
                const uint64_t t0 = 16ull * kTG * tile, sb = n - t0 < 16ull * kTG ? n - t0 : 16ull * kTG;
                sh[tid * 256] = (uint32_t)(sb / WS) - tot[tid];
            }
            return;
        }

        auto count = [&](int b, int v) __attribute__((always_inline)) -> uint32_t {
            uint32_t c = 0;
#pragma unroll
            for (int k = 0; k < Lay::HC; ++k) c += v ? hist[b * Lay::PS + Lay::bin(v, k)] : 0u;
            return c;
        };
        double *part = reinterpret_cast<double *>(wm + M_PART);

        // ---- Mapping decision, fast path (DESIGN.md §4 "E").  Per position b, S_b = Σ_v c_v·log2 c_v
        // in double with the hardware log2 (v_log_f32 of (float)c: |error| <= 2^-18 for every count,
        // checked by tests/test_gpu_0_selftest.py).  The entropy calculate_entropy :470-480 computes
        // is e_b = log2 N - S_b/N up to the fma chain's rounding (< 5e-13), so a_b = log2 N - S_b/N
        // differs from it by delta < 2^-18 + 2^-23 + 1e-12, and mean(a) from the reference's mean by as
        // much.  Whenever every |a_b - mean(a)| = |S_b - mean(S)| / N exceeds kFastMargin = 3e-5 (> 2·delta)
        // the mapping a_b > mean(a), i.e. S_b < mean(S), IS the reference's e_b > mean(e) (perform_clustering
        // :507-525).  Otherwise — ties: constant or repeated-distribution data — the exact fma chains in
        // bin order decide (below).  The sweep costs one log per bin and one reduction per position.
        uint32_t exact_needed = 1;
        {
            constexpr int TP = TEAM / WS;  // threads per position (4 .. 512)
            constexpr int BPT = TP >= 256 ? 1 : 256 / TP;
            const int pb = tid / TP, pj = tid % TP;
            // c·log2 c per bin in float (an empty bin: 0·log2 1 = 0), summed in float over groups of
            // at most kFloatGroup bins and in double across groups: <= 5 roundings of 2^-24
            // relative each on positive terms and partial sums (the float count above 2^24, the 4
            // fmas of a group) add at most 5·2^-24·log2 N < 9.6e-6 bits to the hardware log's
            // 2^-18
            double acc = 0.0;
            uint32_t ci = 0;  // nonzero bytes of the position counted by this thread's bins
#pragma unroll
            for (int k0 = 0; k0 < BPT; k0 += kFloatGroup) {
                float accf = 0.0f;
#pragma unroll
                for (int k = k0; k < (k0 + kFloatGroup < BPT ? k0 + kFloatGroup : BPT); ++k) {
                    const int v = pj + k * TP;
                    if (TP > 256 && v >= 256) break;  // (TEAM 512, word size 1: half the team idle)
                    const uint32_t c = count(pb, v);  // (0 for v = 0: its count is derived below)
                    ci += c;
                    if constexpr (MODE != MODE_ANALYZE) {
                        const float cf = (float)c;
                        accf = __builtin_fmaf(cf, __builtin_amdgcn_logf(__builtin_fmaxf(cf, 1.0f)), accf);
                    }
                }
                acc += (double)accf;
            }
            uint32_t *cpart = wm + M_CPART;
            if constexpr (TP >= 64) {
                if constexpr (MODE != MODE_ANALYZE) acc = seg_sum_f64<64>(acc);
                ci = seg_sum_u32<64>(ci);
                if (lane == 63) {  // wave wv: TP / 64 waves per position
                    part[wv] = acc;
                    cpart[wv] = ci;
                }
            } else {
                if constexpr (MODE != MODE_ANALYZE) acc = seg_sum_f64<TP>(acc);
                ci = seg_sum_u32<TP>(ci);
                if (pj == TP - 1) {
                    part[pb] = acc;
                    cpart[pb] = ci;
                }
            }
            team_sync<W>();
            if (wv == 0) {
                // zero count of position lane: its words minus its nonzero bytes
                uint32_t nz = 0;
                double sb = 0.0;
                if (lane < WS) {
                    if constexpr (TP >= 64) {
#pragma unroll
                        for (int w = 0; w < W; ++w)
                            if (w * 64 / TP == lane) {
                                sb += part[w];
                                nz += cpart[w];
                            }
                    } else {
                        sb = part[lane];
                        nz = cpart[lane];
                    }
                    const uint32_t z = wc - nz;
                    wm[M_Z + lane] = z;
                    if (z) sb += (double)z * (double)__builtin_amdgcn_logf((float)z);
                }
              if constexpr (MODE != MODE_ANALYZE) {
                double ss = 0.0;
#pragma unroll
                for (int b = 0; b < WS; ++b) ss += readlane_f64(sb, b);
                const double ms = ss / (double)WS;
                const bool unsafe = lane < WS && !(__builtin_fabs(sb - ms) > kFastMargin * total);
                const bool fast = !__any(unsafe);
                if (fast && lane < WS) wm[M_MAP + lane] = sb < ms ? 1u : 0u;
                const uint32_t mbits = (uint32_t)__ballot(lane < WS && sb < ms);
                if (lane == 0) {
                    wm[M_EXACT] = fast ? 0u : 1u;
                    if (fast) wm[M_MAPBITS] = mbits;
                }
              }
            }
            team_sync<W>();
            if constexpr (MODE != MODE_ANALYZE) exact_needed = __builtin_amdgcn_readfirstlane(wm[M_EXACT]);
        }
#ifdef PSY_X_FIXMAP
        exact_needed = 0;  // diagnostic: no entropy terms / chains
        if (tid == 0) {
            for (int b = 0; b < WS; ++b) wm[M_MAP + b] = b < 3 ? 1u : 0u;
            wm[M_MAPBITS] = 7u & ((1u << WS) - 1u);
        }
        team_sync<W>();
#endif

        // ---- Exact path (ties, and MODE_ANALYZE's entropies): calculate_entropy :470-480 in bin
        // order, step fma(-prob, log2 prob, e) with glibc's log2 (tdt_log2.h).  Each bin's
        // (-prob, log2 prob) is computed in parallel (0, 0 for an empty bin, so the chain needs no
        // select: fma(0, 0, e) == e for the non-negative running sum); then in every wave one lane
        // per position runs the chain.
        if (exact_needed) {
            // Counts repeat: the terms of counts 1..64 are computed once per message (exactly the
            // operations below, so the same bits) and looked up; larger counts are computed.  Lane i
            // holds count i + 1's terms (one-wave teams: in registers, looked up by ds_bpermute).
            double *ctab = reinterpret_cast<double *>(smem + Lay::OFF_CTAB);
            double c_np = 0.0, c_L = 0.0;
            if (tid < 64) {
                double prob;
                {
#pragma clang fp contract(off)
                    prob = (double)(uint32_t)(tid + 1) / total;
                    c_L = psy_log2_glibc(prob, ltab, ltab2);
                }
                c_np = -prob;
                if constexpr (W > 1) {
                    ctab[2 * tid] = c_np;
                    ctab[2 * tid + 1] = c_L;
                }
            }
            team_sync<W>();
            double *terms = reinterpret_cast<double *>(smem + Lay::OFF_TERMS);
            auto shfl_f64 = [&](double x, uint32_t src) __attribute__((always_inline)) -> double {
                const uint64_t u = __builtin_bit_cast(uint64_t, x);
                const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)(uint32_t)u);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)(uint32_t)(u >> 32));
                return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
            };
            // (-prob, log2 prob) of a bin with count c
            auto bin_terms = [&](uint32_t c, double &np, double &L) __attribute__((always_inline)) {
                np = 0.0;
                L = 0.0;
                if constexpr (W == 1) {
                    // every lane takes part in the permutes (counts 0 and > 64 read lane 0 and
                    // are then overwritten / ignored)
                    const uint32_t src = c - 1u <= 63u ? c - 1u : 0u;
                    const double tnp = shfl_f64(c_np, src), tL = shfl_f64(c_L, src);
                    if (c - 1u <= 63u) {
                        np = tnp;
                        L = tL;
                    }
                }
                if (c > 64u) {
                    double prob;
                    {
#pragma clang fp contract(off)
                        prob = (double)c / total;
                        L = psy_log2_glibc(prob, ltab, ltab2);
                    }
                    np = -prob;
                } else if (W > 1 && c) {
                    const double2 t = reinterpret_cast<const double2 *>(ctab)[c - 1];
                    np = t.x;
                    L = t.y;
                }
            };
            constexpr int NKB = (Lay::TB * 256 + TEAM - 1) / TEAM;  // bin batches per thread
            for (int q0 = 0; q0 < WS; q0 += Lay::TB) {
                if (q0 > 0) team_sync<W>();  // every wave's chain has read the previous batch
                // one-wave teams keep their bins' terms in registers (no LDS terms array): bin v
                // = 64·k + lane, read back in bin order by the chain through readlane
                double rnp[W == 1 ? NKB : 1], rL[W == 1 ? NKB : 1];
                {
#pragma unroll
                for (int k = 0; k < NKB; ++k) {
                    const int i = tid + k * TEAM;
                    if (i >= Lay::TB * 256) break;  // wave-uniform
                    const int b = q0 + i / 256;     // wave-uniform
                    double np = 0.0, L = 0.0;
                    if (b < WS) {
                        uint32_t c = count(b, i & 255);
                        if ((i & 255) == 0) c = wm[M_Z + b];  // bin 0: the derived zero count
                        if constexpr (MODE == MODE_ANALYZE) {
                            if (a.hist_out) a.hist_out[((uint64_t)msg * WS + b) * 256 + (i & 255)] = c;
                        }
                        bin_terms(c, np, L);
                    }
                    if constexpr (W == 1) {
                        rnp[k] = np;
                        rL[k] = L;
                    } else {
                        terms[2 * i] = np;
                        terms[2 * i + 1] = L;
                    }
                }
                }
                team_sync<W>();
                if (wv == 0) {
                    if constexpr (W == 1) {
                        static_assert(Lay::TB == 1, "one-wave teams run one position per batch");
                        // uniform: every lane runs the chain on readlane operands
                        double e = 0.0;
#pragma unroll
                        for (int k = 0; k < NKB; ++k)
#pragma unroll 8
                            for (int l = 0; l < 64; ++l)
                                e = __builtin_fma(readlane_f64(rnp[k], l), readlane_f64(rL[k], l), e);
                        if (lane == 0) reinterpret_cast<double *>(wm + M_ENT)[q0] = e;
                    } else if (lane < Lay::TB && q0 + lane < WS) {
                        const int b = q0 + lane;
                        const double2 *tp = reinterpret_cast<const double2 *>(terms) + lane * 256;
                        double e = 0.0;
#pragma unroll 2
                        for (int v = 0; v < 256; ++v) {  // (rare path: few registers, the message's are live)
                            const double2 t = tp[v];
                            e = __builtin_fma(t.x, t.y, e);
                        }
                        reinterpret_cast<double *>(wm + M_ENT)[b] = e;
                    }
                }
            }
            team_sync<1>();
            // perform_clustering :507-525 from the exact entropies
            if (tid == 0) {
                const double *ent = reinterpret_cast<const double *>(wm + M_ENT);
                double sum = 0.0;
                for (int b = 0; b < WS; ++b) sum += ent[b];
                double thr;
                {
#pragma clang fp contract(off)
                    thr = sum / (double)WS;
                }
                uint32_t mbits = 0;
                for (int b = 0; b < WS; ++b) {
                    wm[M_MAP + b] = ent[b] > thr ? 1u : 0u;
                    mbits |= (ent[b] > thr ? 1u : 0u) << b;
                }
                wm[M_MAPBITS] = mbits;
            }
            team_sync<W>();  // every wave reads the mapping next
        }
        if constexpr (MODE == MODE_ANALYZE) {
            const uint64_t mb = (uint64_t)msg * WS;
            if (tid < WS) {
                if (a.ent_out) a.ent_out[mb + tid] = reinterpret_cast<const double *>(wm + M_ENT)[tid];
                if (a.map_out) a.map_out[mb + tid] = (int32_t)wm[M_MAP + tid];
            }
            if (tid == 0 && a.status) a.status[msg] = ST_OK;
            return;
        }
        if constexpr (TL == 4) {
            uint32_t bits = 0;
            for (int b = 0; b < WS; ++b) bits |= wm[M_MAP + b] << b;
            if (tid == 0) a.lmeta[lj].mapbits = bits;
            {
                // the count pass's list (one workgroup per listed tile, instead of one per tile
                // that mostly exits at once: C4's count launch was 2 ms of such workgroups);
                // word sizes without a speculated mapping list every tile
                const uint32_t nt = a.lmeta[lj].ntiles, t0 = a.lmeta[lj].tile0;
                const bool miss = kSpec == 0xffffffffu || bits != kSpec;
                for (uint32_t t = (uint32_t)tid; t < nt; t += TEAM) {
                    const bool need = miss || a.trec[t0 + t].clean == kRecount;
                    const uint64_t bal = __ballot(need);
                    if (bal == 0) continue;
                    const int first = __ffsll((unsigned long long)bal) - 1;
                    uint32_t base = 0;
                    if (lane == first) base = (uint32_t)atomicAdd(a.rcount, (unsigned long long)__popcll(bal));
                    base = (uint32_t)__shfl((int)base, first);
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                    if (need) a.rtiles[base + rank] = ((uint64_t)t << 32) | lj;
                }
            }
            return;
        }
    }

    if constexpr (MODE != MODE_ANALYZE) {
        // ------------------------------------------------ slot layout
        // separate_byte_streams :527-549: slot j < L0 is stream-0 byte j of the group
        // (word j / k0, position pos0[j % k0]); slot j >= L0 is stream-1 byte j - L0.
        uint32_t ns, L0, k0, k1, selA[4], selB[4], edA, edB;
        const uint32_t mapbits = __builtin_amdgcn_readfirstlane(wm[M_MAPBITS]);
        if constexpr (WS <= 8) {
            // a constant table indexed by the mapping bits: scalar loads, no barrier
            const SlotLayout &SL = slot_layout<WS>(mapbits);
            ns = SL.ns;
            L0 = SL.L0;
            k0 = SL.k0;
            k1 = SL.k1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                selA[q] = SL.selA[q];
                selB[q] = SL.selB[q];
            }
            edA = SL.edA;
            edB = SL.edB;
        } else {
            // word size 16 (2^16 mappings): wave 0 derives it (make_slot_layout's steps), 16 lanes
            // for slot j's source byte in the group (no per-thread arrays: scratch-free)
            if (tid < 16) {
                uint32_t k[2] = {0, 0};
                for (int b = 0; b < WS; ++b) k[wm[M_MAP + b]]++;
                const uint32_t L0w = WPG * k[0];
                const uint32_t j = (uint32_t)lane;
                const uint32_t c = j < L0w ? 0u : 1u;
                const uint32_t jj = c ? j - L0w : j;
                const uint32_t rank = jj % k[c];
                uint32_t b = 0, seen = 0;
                for (int bb = 0; bb < WS; ++bb) {
                    if (wm[M_MAP + bb] == c) {
                        if (seen == rank) b = bb;
                        ++seen;
                    }
                }
                wm[M_SB + j] = (jj / k[c]) * WS + b;
                if (j == 0) {
                    wm[M_NS] = k[1] ? 2u : 1u;
                    wm[M_L0] = L0w;
                    wm[M_K0] = k[0];
                    wm[M_K1] = k[1];
                }
            }
            team_sync<1>();
            if (tid < 5) {
                const uint32_t L0w = wm[M_L0];
                const bool two = wm[M_NS] == 2;
                uint32_t A = 0x0c0c0c0cu, B = 0x0c0c0c0cu;
                for (int t = 0; t < 4; ++t) {
                    // T[q] byte t = slot 4t + q; edges byte 0 stream-0 last slot, byte 1 slot 15,
                    // byte 2 stream-1 first slot
                    uint32_t sv = 0xffu;
                    if (lane < 4) sv = wm[M_SB + 4 * t + lane];
                    else if (t == 0 && L0w > 0) sv = wm[M_SB + L0w - 1];
                    else if (t == 1) sv = wm[M_SB + 15];
                    else if (t == 2 && two) sv = wm[M_SB + L0w];
                    if (sv == 0xffu) continue;
                    if (sv < 8) A = (A & ~(0xffu << (8 * t))) | (sv << (8 * t));
                    else B = (B & ~(0xffu << (8 * t))) | ((sv - 8) << (8 * t));
                }
                wm[lane < 4 ? M_SELA + lane : M_EDA] = A;
                wm[lane < 4 ? M_SELB + lane : M_EDB] = B;
            }
            team_sync<W>();
            ns = __builtin_amdgcn_readfirstlane(wm[M_NS]);
            L0 = __builtin_amdgcn_readfirstlane(wm[M_L0]);
            k0 = __builtin_amdgcn_readfirstlane(wm[M_K0]);
            k1 = __builtin_amdgcn_readfirstlane(wm[M_K1]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                selA[q] = __builtin_amdgcn_readfirstlane(wm[M_SELA + q]);
                selB[q] = __builtin_amdgcn_readfirstlane(wm[M_SELB + q]);
            }
            edA = __builtin_amdgcn_readfirstlane(wm[M_EDA]);
            edB = __builtin_amdgcn_readfirstlane(wm[M_EDB]);
        }
        const bool ns2 = ns == 2;
        const uint32_t Ls[2] = {L0, ns2 ? 16u - L0 : 0u};
        const uint32_t lowL0 = L0 >= 16 ? 0xffffu : ((1u << L0) - 1u);
        // start masks of the resident word-size <= 4 bodies are kept in the byte-lane layout
        // (sb_pos); everything else (streaming bodies, tiles' count pass, A2's scans) in the
        // compact 16-bit one
        constexpr bool BL = RES && WS <= 4 && TL != 2;
        const uint32_t lowX = BL ? sb_spread(lowL0) : lowL0;   // stream-0 slots
        const uint32_t highX = BL ? sb_spread(~lowL0 & 0xffffu) : (~lowL0 & 0xffffu);  // stream-1 slots
        const uint32_t fullX = BL ? 0x0f0f0f0fu : 0xffffu;
        // selectors extracting slot L0 (stream 1's first byte) from T: slot j is byte j/4 of
        // T[j%4], i.e. byte (j%4 & 1)*4 + j/4 of perm(T[1],T[0]) or perm(T[3],T[2])
        uint32_t fsA = 0x0c0c0c0cu, fsB = 0x0c0c0c0cu;
        if (ns2) {
            const uint32_t q = L0 & 3u, t = L0 >> 2, sel = 0x0c0c0c00u | ((q & 1u) * 4u + t);
            if (q < 2) fsA = sel;
            else fsB = sel;
        }
        PSY_PROF_MARK(2);

        auto tmat = [&](const uint4 &d, uint32_t (&T)[4]) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < 4; ++q) T[q] = perm(d.y, d.x, selA[q]) | perm(d.w, d.z, selB[q]);
        };
        auto edges = [&](const uint4 &d) __attribute__((always_inline)) -> uint32_t {
            return perm(d.y, d.x, edA) | perm(d.w, d.z, edB);
        };
        // valid slots of a group holding vb message bytes
        auto vmask = [&](uint32_t vb) __attribute__((always_inline)) -> uint32_t {
            const uint32_t nvw = vb / WS;
            if (nvw >= (uint32_t)WPG) return 0xffffu;
            uint32_t v = (1u << (nvw * k0)) - 1u;
            if (ns2) v |= ((1u << (nvw * k1)) - 1u) << L0;
            return v;
        };
        // run-start mask of the 16 slots (bit j: slot j differs from the stream byte before)
        // P0 = the byte before each slot of T[0]: byte t = slot 4t - 1 of the group, byte 0 the
        // previous group's last stream-0 byte.  When stream 1 begins at a dword boundary
        // (L0 % 4 == 0: word size <= 4), its first slot L0 = 4·t0 takes the previous group's last
        // stream-1 byte (edges byte 1) instead, folded into the selector once per message.
        constexpr bool kFold = WS <= 4;  // L0 = (16 / WS)·k0 is then a multiple of 4
        const uint32_t p0sel = kFold && ns2 ? (0x06050400u & ~(0xffu << (2u * L0))) | (0x01u << (2u * L0)) : 0x06050400u;
        // first: this round holds the message's group 0 (uniform)
        // (BLM: the byte-lane layout, V given in it too)
        auto run_mask = [&](const uint32_t (&T)[4], uint32_t ed, uint32_t edc, bool first, uint32_t V,
                            auto blm) __attribute__((always_inline)) -> uint32_t {
            constexpr bool BLM = decltype(blm)::value;
            const uint32_t pe = wave_shr1(ed, edc);  // previous group's edges
            const uint32_t P0 = perm(T[3], pe, p0sel);
            const uint32_t X[4] = {T[0] ^ P0, T[1] ^ T[0], T[2] ^ T[1], T[3] ^ T[2]};
            uint32_t m = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t y = ((X[q] & 0x7f7f7f7fu) + 0x7f7f7f7fu) | X[q];
                m |= (y >> (7 - q)) & (0x01010101u << q);
            }
            if constexpr (BLM) {
                if (first && lane == 0) m |= 1u | (ns2 ? (1u << sb_pos(L0)) : 0u);
                return m & V;
            }
            m = (m | (m >> 4)) & 0x00ff00ffu;
            m = (m | (m >> 8)) & 0xffffu;
            if constexpr (!kFold) {
                if (ns2) {
                    const uint32_t fx = ((ed >> 16) ^ (pe >> 8)) & 0xffu;
                    m = (m & ~(1u << L0)) | ((fx ? 1u : 0u) << L0);
                }
            }
            if (first && lane == 0) m |= 1u | (ns2 ? (1u << L0) : 0u);
            return m & V;
        };
        // packed (stream 1 in the high half) round-relative last start + 1 of a start mask
        auto last_starts = [&](uint32_t m) __attribute__((always_inline)) -> uint32_t {
            const uint32_t m0 = m & lowL0;
            uint32_t lr = m0 ? (uint32_t)lane * Ls[0] + hibit(m0) + 1u : 0u;
            if (ns2) {
                const uint32_t m1 = m >> L0;
                lr |= (m1 ? (uint32_t)lane * Ls[1] + hibit(m1) + 1u : 0u) << 16;
            }
            return lr;
        };
        // the 255-cap bit of the run carried into each group (simple_rle_compress :568).
        // exc: packed exclusive scan of last run start + 1 (round-relative); rcarry:
        // absolute last run start + 1 before the round (0 = none); rb: round base positions.
        auto cap_bits = [&](uint32_t m, uint32_t exc, const uint32_t (&rcarry)[2], const uint32_t (&rb)[2],
                            uint32_t g, uint32_t V) __attribute__((always_inline)) -> uint32_t {
            uint32_t need = 0;
            uint32_t csp[2] = {0, 0}, Lv[2] = {0, 0};
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (c == 1 && !ns2) break;
                const uint32_t er = (exc >> (16 * c)) & 0xffffu;
                csp[c] = er ? rb[c] + er : rcarry[c];
                Lv[c] = c == 0 ? popc(V & lowL0) : popc(V >> L0);
                need |= (csp[c] && g * Ls[c] + Lv[c] >= csp[c] + 255u) ? 1u : 0u;
            }
            if (!__any(need)) return 0u;  // no run of >= 255 bytes reaches this round
            uint32_t out = 0;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (c == 1 && !ns2) break;
                const uint32_t mc = c == 0 ? (m & lowL0) : (m >> L0);
                if (csp[c] && !(mc & 1u) && Lv[c]) {
                    const uint32_t d = g * Ls[c] + 1u - csp[c];  // >= 1
                    const uint32_t rel = 255u * ((d + 254u) / 255u) - d;
                    const uint32_t fs = lobit(mc | (1u << Lv[c]));
                    if (rel < fs) out |= 1u << (rel + (c ? L0 : 0u));
                }
            }
            return out;
        };
        // chunk-start mask of round r given its run-start mask; advances the run carry
        auto chunk_round = [&](uint32_t r, uint32_t m, uint32_t (&rcarry)[2], uint32_t g,
                               uint32_t V) __attribute__((always_inline)) -> uint32_t {
            const uint32_t rb[2] = {(gw0 + r * 64) * Ls[0], (gw0 + r * 64) * Ls[1]};
            const uint32_t inc = wave_incl_scan<OpPkMax>(last_starts(m));
            const uint32_t exc = wave_shr1(inc, 0u);
            const uint32_t C = m | cap_bits(m, exc, rcarry, rb, g, V);
            const uint32_t i63 = rdlane(inc, 63);
            if (i63 & 0xffffu) rcarry[0] = umax(rcarry[0], rb[0] + (i63 & 0xffffu));
            if (i63 >> 16) rcarry[1] = umax(rcarry[1], rb[1] + (i63 >> 16));
            return C;
        };

        // edges of the group before this wave's first group (carry into round 0)
        uint32_t edc0 = 0;
        if (gw0 > 0 && gw0 - 1 < ngroups) edc0 = __builtin_amdgcn_readfirstlane(edges(load_group(gw0 - 1)));

        // ---------------------------------------------------------- pass A1: run starts
        // A1 also proves, for nearly every message, that the 255-cap cannot occur, so that
        // A2's scan is skipped.  A cap needs a run of >= 256 bytes, i.e. at least
        // Zr = floor(255 / Ls) - 1 consecutive groups without a run start in that stream, and
        // any 2B - 1 consecutive groups contain a B-aligned block of B groups (B divides 64, so
        // rounds and waves start on block boundaries).  With B = 8 for Ls < 16 (Zr >= 16) and
        // B = 4 for Ls = 16 (Zr = 14), "every aligned B-group block holds a start (or reaches
        // past the end)" rules the cap out.  Per round and stream: one ballot and a
        // has-zero-byte (B = 8) or has-zero-nibble (B = 4) test on it, on the scalar unit
        // (tests/test_cap_exclusion.py checks the rule against adversarial run lengths).
        uint32_t wmax[2] = {0, 0};
        uint32_t lr[2] = {0, 0};        // resident: last round with a run start, per stream
        uint64_t lb[2] = {0ull, 0ull};  // and that round's ballot of lanes with one
        uint64_t zk1[2], zk8[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const bool b8 = Ls[c] < 16u;
            zk1[c] = b8 ? 0x0101010101010101ull : 0x1111111111111111ull;
            zk8[c] = Ls[c] == 0u ? 0ull : b8 ? 0x8080808080808080ull : 0x8888888888888888ull;
        }
        uint64_t zacc = 0;
        // per-lane chunk-start counts.  Streaming teams count run starts in A1 — the chunk
        // starts when the 255-cap is ruled out, so that A2 (another pass over HBM) is skipped;
        // resident teams count in A2 (registers only; fewer live values across A1)
        uint32_t pc0 = 0, pc1 = 0;
        uint32_t fmx[2] = {0, 0};  // tile count pass: ~(first run start), max-reduced
        // stream position of this lane's group in round 0 (round r adds r·64·Ls)
        const uint32_t gL[2] = {(gw0 + (uint32_t)lane) * Ls[0], (gw0 + (uint32_t)lane) * Ls[1]};
        bool spec_hit = false;
        if constexpr (SPEC_ON && TL == 0) {
            spec_hit = mapbits == kSpec;  // (uniform) the histogram pass counted under this mapping
            if (spec_hit) {
                wmax[0] = s_wmax[0];
                wmax[1] = s_wmax[1];
                pc0 = s_pc0;
                pc1 = s_pc1;
                zacc = s_zacc;
            }
        }
        if (!spec_hit) {
            uint32_t edc = edc0;
            for_rounds([&](uint32_t r, uint4 &d, uint32_t &cm, auto res) __attribute__((always_inline)) {
                PSY_ASM_ROUND(A1);
                const uint32_t g = gw0 + r * 64 + lane;
                const uint32_t ed = edges(d);
                uint32_t T[4];
                tmat(d, T);
                const uint32_t V = full_round(r) ? fullX : (BL ? sb_spread(vmask(vbytes(g))) : vmask(vbytes(g)));
                const uint32_t m = run_mask(T, ed, edc, r == 0u && gw0 == 0u, V, std::integral_constant<bool, BL>{});
                edc = rdlane(ed, 63);
                cm = m;
                if constexpr (decltype(res)::value) d = make_uint4(T[0], T[1], T[2], T[3]);
                constexpr bool SW = decltype(res)::value && TL != 2;  // scalar last-start tracking
                const uint32_t m0 = m & lowX;
                const uint64_t r0 = (uint64_t)__ballot(m0 != 0u);
                if constexpr (SW) {
                    if (r0) {
                        lr[0] = r;
                        lb[0] = r0;
                    }
                } else {
                    if (m0) wmax[0] = umax(wmax[0], gL[0] + r * 64u * Ls[0] + hibit(m0) + 1u);
                }
                pc0 += popc(m0);
                if constexpr (TL == 2) {
                    if (m0) fmx[0] = umax(fmx[0], ~(g * Ls[0] + lobit(m0)));
                }
                const uint64_t pastm = full_round(r) ? 0ull : (uint64_t)__ballot(g >= ngroups);
                const uint64_t b0 = r0 | pastm;
                zacc |= (b0 - zk1[0]) & ~b0 & zk8[0];
                if (ns2) {
                    const uint32_t m1 = BL ? m & highX : m >> L0;
                    const uint64_t r1 = (uint64_t)__ballot(m > lowX);  // m1 != 0 (layouts monotonic in the slot)
                    if constexpr (SW) {
                        if (r1) {
                            lr[1] = r;
                            lb[1] = r1;
                        }
                    } else {
                        if (m1) wmax[1] = umax(wmax[1], gL[1] + r * 64u * Ls[1] + hibit(m1) + 1u);
                    }
                    pc1 += popc(m1);
                    if constexpr (TL == 2) {
                        if (m1) fmx[1] = umax(fmx[1], ~(g * Ls[1] + lobit(m1)));
                    }
                    const uint64_t b1 = r1 | pastm;
                    zacc |= (b1 - zk1[1]) & ~b1 & zk8[1];
                }
            });
        }
        if constexpr (RES && TL != 2) {
            // the wave's last run start per stream: in the last round with a start, its highest
            // lane with one (all scalar but one readlane per stream)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (lb[c] == 0ull) continue;
                const uint32_t l = 63u - (uint32_t)__builtin_clzll(lb[c]);
                uint32_t mv = 0;
#pragma unroll
                for (int r = 0; r < GR; ++r)
                    if ((uint32_t)r == lr[c]) mv = rdlane(cres[r], (int)l);
                uint32_t hb;
                if constexpr (BL) hb = sb_slot(hibit(c ? mv & highX : mv & lowX)) - (c ? L0 : 0u);
                else hb = hibit(c ? mv >> L0 : mv & lowL0);
                wmax[c] = (gw0 + lr[c] * 64u + l) * Ls[c] + hb + 1u;
            }
        } else {
            wmax[0] = wave_reduce<OpMax>(wmax[0]);
            wmax[1] = wave_reduce<OpMax>(wmax[1]);
        }
        if constexpr (TL == 2) {
            fmx[0] = wave_reduce<OpMax>(fmx[0]);
            fmx[1] = wave_reduce<OpMax>(fmx[1]);
        }
        // run-start counts: the chunk-start counts whenever the 255-cap is ruled out (A2 then
        // never runs and its barrier is saved)
        pc0 = wave_reduce<OpAdd>(pc0);
        pc1 = ns2 ? wave_reduce<OpAdd>(pc1) : 0u;
        if (lane == 0) {
            slots[wv * 8 + 0] = wmax[0];
            slots[wv * 8 + 1] = wmax[1];
            slots[wv * 8 + 2] = pc0;
            slots[wv * 8 + 3] = pc1;
            slots[wv * 8 + 5] = zacc != 0ull ? 1u : 0u;
            if constexpr (TL == 2) {
                slots[wv * 8 + 6] = fmx[0];
                slots[wv * 8 + 7] = fmx[1];
            }
        }
        team_sync<W>();
        uint32_t rin[2] = {0, 0};  // max (run start + 1) before this wave
        uint32_t capped = 0;       // some wave cannot rule the 255-cap out
        const TileRec *tr = nullptr;
        if constexpr (TL == 3) {
            // the run carried into the tile (scan): as if a wave before wave 0
            tr = a.trec + a.lmeta[lj].tile0 + tile;
            rin[0] = tr->lrs[0];
            rin[1] = tr->lrs[1];
            capped = tr->clean ? 0u : 1u;
        }
#pragma unroll
        for (int ww = 0; ww < W; ++ww) {
            if (ww < wv) {
                rin[0] = umax(rin[0], slots[ww * 8 + 0]);
                rin[1] = umax(rin[1], slots[ww * 8 + 1]);
            }
            capped |= slots[ww * 8 + 5];
        }
        rin[0] = __builtin_amdgcn_readfirstlane(rin[0]);
        rin[1] = __builtin_amdgcn_readfirstlane(rin[1]);
        const bool clean = __builtin_amdgcn_readfirstlane(capped) == 0u;
        PSY_PROF_MARK(3);

        // ---------------------------------------------------------- pass A2: chunk starts
        if (!clean) {
            pc0 = pc1 = 0;
            uint32_t rcarry[2] = {rin[0], rin[1]};
            uint32_t edc = edc0;
            for_rounds([&](uint32_t r, uint4 &d, uint32_t &cm, auto res) __attribute__((always_inline)) {
                PSY_ASM_ROUND(A2);
                const uint32_t g = gw0 + r * 64 + lane;
                const uint32_t V = full_round(r) ? 0xffffu : vmask(vbytes(g));
                uint32_t m;
                if constexpr (decltype(res)::value) {
                    m = BL ? sb_compact(cm) : cm;
                } else {
                    uint32_t T[4];
                    tmat(d, T);
                    const uint32_t ed = edges(d);
                    m = run_mask(T, ed, edc, r == 0u && gw0 == 0u, V, std::false_type{});
                    edc = rdlane(ed, 63);
                }
                const uint32_t C = chunk_round(r, m, rcarry, g, V);
                cm = BL ? sb_spread(C) : C;
                pc0 += popc(C & lowL0);
                pc1 += popc(C >> L0);
            });
            pc0 = wave_reduce<OpAdd>(pc0);
            pc1 = ns2 ? wave_reduce<OpAdd>(pc1) : 0u;
            if (lane == 0) {  // (slots 2, 3 are first read after the barrier below)
                slots[wv * 8 + 2] = pc0;
                slots[wv * 8 + 3] = pc1;
            }
            team_sync<W>();
        }
        PSY_PROF_MARK(4);
        uint32_t pin[2] = {0, 0}, ptot[2] = {0, 0};
#pragma unroll
        for (int ww = 0; ww < W; ++ww) {
            const uint32_t s0 = slots[ww * 8 + 2], s1 = slots[ww * 8 + 3];
            if (ww < wv) {
                pin[0] += s0;
                pin[1] += s1;
            }
            ptot[0] += s0;
            ptot[1] += s1;
        }
        if constexpr (TL == 2) {
            // the tile's local figures for the scan
            if (tid == 0) {
                uint32_t l[2] = {0, 0}, f[2] = {0, 0};
                for (int ww = 0; ww < W; ++ww) {
                    l[0] = umax(l[0], slots[ww * 8 + 0]);
                    l[1] = umax(l[1], slots[ww * 8 + 1]);
                    f[0] = umax(f[0], slots[ww * 8 + 6]);
                    f[1] = umax(f[1], slots[ww * 8 + 7]);
                }
                TileRec *t = a.trec + a.lmeta[lj].tile0 + tile;
                t->lrs[0] = l[0];
                t->lrs[1] = l[1];
                t->frs[0] = ~f[0];
                t->frs[1] = ~f[1];
                t->cnt[0] = ptot[0];
                t->cnt[1] = ptot[1];
                t->clean = clean ? 1u : 0u;
            }
            return;
        }
        const uint32_t P0 = __builtin_amdgcn_readfirstlane(ptot[0]);
        const uint32_t P1 = ns2 ? __builtin_amdgcn_readfirstlane(ptot[1]) : 0u;
        const uint32_t hdr = 20 + 4 * WS;
        uint64_t ob;
        uint32_t P0m = P0;  // stream 0's pair count in the whole message
        uint64_t Eblob = 0;
        // deferred look-back: compacted output of a resident message (the E6 emit below)
        constexpr bool DEFER = LB && RES && WS <= 4 && TL == 0 && MODE == MODE_ENCODE;
        if constexpr (TL == 3) {
            const LMeta *lm = a.lmeta + lj;
            if (!lm->fits) return;  // the scan gave the message CAPACITY
            ob = slot_b;
            P0m = lm->P0;
            pin[0] += tr->cnt[0];  // chunk starts before the tile
            pin[1] += tr->cnt[1];
        } else {
            const uint64_t E = hdr + (4 + 2ull * P0) + (ns2 ? 4 + 2ull * P1 : 0);
            Eblob = E;
            bool fits = true;
            if constexpr (DEFER) {
                // compacted, resident: publish the blob size now and take the offset only at the
                // first flush (pass B's sweeps fill the LDS staging meanwhile), so the wait for
                // the predecessors' prefixes overlaps this team's own work
                if (wv == 0) lookback_publish(a.lookback, msg, E);
                ob = 0;
            } else {
                ob = place(E, fits);
                if (tid == 0 && a.status) a.status[msg] = fits ? ST_OK : ST_CAPACITY;
                if (!fits) return;
            }
        }
        // header :84-106 and stream length words :110-112
        uint8_t *dst = a.out + ob;
        const uint32_t sdata[2] = {hdr + 4, hdr + 4 + 2 * P0m + 4};
        if constexpr (TL == 0 && !DEFER) {
        for (uint32_t t = tid; t < hdr; t += TEAM) {
            const int f = t >> 2, sh = 8 * (t & 3);
            uint32_t v;
            if (f == 0) v = kMagicTDT;
            else if (f == 1) v = n32;
            else if (f == 2) v = ns;
            else if (f == 3 || f == 4) v = WS;
            else v = (mapbits >> (f - 5)) & 1u;
            dst[t] = (uint8_t)(v >> sh);
        }
        if (tid < 8) {
            const int c = tid >> 2, sh = 8 * (tid & 3);
            if ((uint32_t)c < ns) {
                const uint32_t len = 2 * (c ? P1 : P0);
                dst[sdata[c] - 4 + (tid & 3)] = (uint8_t)(len >> sh);
            }
        }
        }
        PSY_PROF_MARK(5);

        // ---------------------------------------------------------- pass B: emit pairs
        // Wave-local from here on: per-wave LDS staging, no workgroup barrier.
        const uint32_t wst = Lay::OFF_STAGE + wv * Lay::WSTAGE;
        // last chunk start + 1 before this wave: inside the run carried in (start rin - 1),
        // chunks start every 255 bytes (simple_rle_compress :568)
        uint32_t ccarry[2] = {0, 0};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint32_t W0 = gw0 * Ls[c];
            if (rin[c] && W0 > 0) {
                const uint32_t rs = rin[c] - 1;
                ccarry[c] = rs + 255u * ((W0 - 1 - rs) / 255u) + 1u;
            }
        }


        // ---------------------------------------------------------------- emit v5
        // Chunk-START entries: every chunk start writes entry = value << 24 | (position within
        // the round + 256) at its rank among the round's starts (slot 0 of each stream holds
        // the chunk still open from the previous round / wave); the flush then forms pair k
        // from entries k and k+1 — count = their position difference (<= 255 by the cap),
        // value = entry k's — one pair per lane, 2-byte stores coalesced across the wave.  The
        // last chunk of a round stays pending; the stream's final chunk ends at its length.
        uint32_t pi5[2] = {0, 0}, pend[2] = {0, 0};
        bool hp[2] = {false, false};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (c == 1 && !ns2) break;
            const uint32_t p_in = __builtin_amdgcn_readfirstlane(pin[c]);
            if (p_in > 0 && ccarry[c] > 0) {
                hp[c] = true;
                pi5[c] = p_in - 1;
                const uint32_t val = (edc0 >> (8 * c)) & 0xffu;  // the chunk's value: the byte before the wave
                pend[c] = (val << 24) | (ccarry[c] - 1u + 256u - gw0 * Ls[c]);
            }
        }
        const uint32_t slen[2] = {wc * k0, wc * k1};
        // per wave: 64 junk dwords (one per lane), then stream 0's pending entry + entries,
        // then stream 1's (EncLayout::WSTAGE)
        const uint32_t ebase = wst + 256u;
        const uint32_t jl = wst;  // one junk dword for the wave: same-address writes do not conflict
        const uint32_t eoff1 = 4u * (1u + 64u * L0);  // stream 1's entry region (bytes)
        const uint32_t pb0 = (uint32_t)lane * Ls[0] + 256u, pb1 = (uint32_t)lane * Ls[1] + 256u - L0;
        auto emit5 = [&](uint32_t r, const uint4 &Tw, uint32_t C) __attribute__((always_inline)) {
#ifdef PSY_X_NOEMIT
            if (r < 100) return;
#endif
            PSY_ASM_ROUND(B);
            const uint32_t T[4] = {Tw.x, Tw.y, Tw.z, Tw.w};
            const uint32_t gr = gw0 + r * 64;
            const uint32_t c0 = popc(C & lowL0);
            const uint32_t pc = c0 | (popc(C >> L0) << 16);
            const uint32_t pinc = wave_incl_scan<OpAdd>(pc);
            const uint32_t pexc = pinc - pc;
            const uint32_t Stot = rdlane(pinc, 63);
            const uint32_t S[2] = {Stot & 0xffffu, Stot >> 16};
            if (lane == 0) {
                if (hp[0]) *reinterpret_cast<uint32_t *>(smem + ebase) = pend[0];
                if (ns2 && hp[1]) *reinterpret_cast<uint32_t *>(smem + ebase + eoff1) = pend[1];
            }
            // D = (address of this lane's next entry in the current stream) - its junk dword.
            // Slot j writes at jl + bit_j·D (a start: its entry; otherwise the junk dword),
            // then D advances by one entry on a start: 4 VALU per slot, no compares.
            const uint32_t D0 = ebase + 4u * (1u + (pexc & 0xffffu)) - jl;
            const uint32_t D1 = ebase + eoff1 + 4u * (1u + (pexc >> 16)) - jl;
            uint32_t D = L0 == 0 ? D1 : D0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int q = j & 3, t = j >> 2;
                if (j > 0 && j % WPG == 0 && (uint32_t)j == L0) D = D1;  // stream 1 begins (uniform)
                const bool s0 = (uint32_t)j < L0;
                const uint32_t bit = (C >> j) & 1u;
                const uint32_t pos = (s0 ? pb0 : pb1) + (uint32_t)j;
                // (inline asm keeps the running address: the compiler would rebuild it from a
                // running count, one more VALU per slot)
                uint32_t ad;
                asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(ad) : "v"(bit), "v"(D), "v"(jl));
                *reinterpret_cast<uint32_t *>(smem + ad) =
                    perm(T[q], pos, ((uint32_t)(4 + t) << 24) | 0x000c0100u);
                asm("v_lshl_add_u32 %0, %1, 2, %2" : "=v"(D) : "v"(bit), "v"(D));
            }
            team_sync<1>();
            const bool last = gr <= ngroups - 1 && ngroups - 1 < gr + 64;  // the stream's end is here
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (c == 1 && !ns2) break;
#ifdef PSY_X_NOFLUSH
                if (r < 1000u) continue;  // diagnostic: sweep only
#endif
                const uint32_t f0 = hp[c] ? 0u : 1u;
                const uint32_t nent = S[c] + (hp[c] ? 1u : 0u);
                const uint32_t K = nent ? nent - 1u : 0u;
                const uint32_t eb = ebase + (c ? eoff1 : 0u);
                uint8_t *const D = dst + sdata[c] + 2ull * pi5[c];
                const bool even = ((uintptr_t)D & 1) == 0;
                // pair k = (count, value) from entries k and k+1; full 64-pair trips run without
                // exec masking, the tail trip masked; the alignment test is hoisted out of the loop
                auto pair_at = [&](uint32_t k) __attribute__((always_inline)) -> uint32_t {
                    const uint32_t e0 = *reinterpret_cast<const uint32_t *>(smem + eb + 4u * (f0 + k));
                    const uint32_t e1 = *reinterpret_cast<const uint32_t *>(smem + eb + 4u * (f0 + k + 1u));
                    return perm(e0, e1 - e0, 0x0c0c0700u);  // count, value
                };
                if (even) {
                    uint32_t k0 = 0;
                    for (; k0 + 128u <= K; k0 += 128u) {  // two independent trips per iteration
                        const uint32_t k = k0 + (uint32_t)lane;
                        const uint32_t pa = pair_at(k), pb = pair_at(k + 64u);
                        *reinterpret_cast<uint16_t *>(D + 2u * k) = (uint16_t)pa;
                        *reinterpret_cast<uint16_t *>(D + 2u * k + 128u) = (uint16_t)pb;
                    }
                    for (; k0 + 64u <= K; k0 += 64u) {
                        const uint32_t k = k0 + (uint32_t)lane;
                        *reinterpret_cast<uint16_t *>(D + 2u * k) = (uint16_t)pair_at(k);
                    }
                    const uint32_t k = k0 + (uint32_t)lane;
                    if (k < K) *reinterpret_cast<uint16_t *>(D + 2u * k) = (uint16_t)pair_at(k);
                } else {
                    for (uint32_t k0 = 0; k0 < K; k0 += 64) {
                        const uint32_t k = k0 + (uint32_t)lane;
                        if (k < K) {
                            const uint32_t pair = pair_at(k);
                            D[2u * k] = (uint8_t)pair;
                            D[2u * k + 1u] = (uint8_t)(pair >> 8);
                        }
                    }
                }
                pi5[c] += K;
                if (nent) {
                    const uint32_t el = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const uint32_t *>(smem + eb + 4u * S[c]));
                    if (last) {  // the final chunk runs to the end of the stream
                        if (lane == 0) {
                            const uint32_t cnt = slen[c] - (gr * Ls[c] + (el & 0xffffu) - 256u);
                            D[2u * K] = (uint8_t)cnt;
                            D[2u * K + 1u] = (uint8_t)(el >> 24);
                        }
                        pi5[c] += 1;
                    }
                    pend[c] = el - 64u * Ls[c];  // rebased to the next round
                    hp[c] = true;
                }
            }
            team_sync<1>();  // the entries are rewritten by the next round
        };

        // ---------------------------------------------------------------- emit v6
        // Resident messages with word size <= 4: as v5, but entries are u16 (value << 8 |
        // stream position mod 256 — with Ls a multiple of 4 every round starts at a multiple of
        // 256 positions, and consecutive chunk starts are 1..255 apart, so count = (e1 - e0) mod
        // 256) and NB rounds (3 for message-sized teams) share one flush: the per-round flush bookkeeping (pointers, the
        // last-entry read, the pending entry, loop set-up) is paid once per pair of rounds.
        constexpr bool E6 = RES && WS <= 4;
        constexpr bool E6S = WS <= 4;  // (the streaming body batches its rounds the same way)
        const uint32_t eb6 = wst + 16u;
        // stream 1's u16 region (bytes; a multiple of 4 like eb6, so that every region's even
        // entries are dword-aligned for the flush)
        constexpr uint32_t NB = Lay::NB6;  // rounds per flush
        const uint32_t eoff6 = 2u * (2u + NB * 64u * L0);
        // entries staged per stream: the pending chunk (entry 0, when there is one) plus the
        // batch's own (round 6: one integer, so that the flush tests stay on the scalar unit —
        // the pending flag as a bool came out as v_cndmask / v_cmp per round)
        uint32_t u6[2] = {hp[0] ? 1u : 0u, hp[1] ? 1u : 0u};
        uint32_t pend6[2] = {0, 0};
#pragma unroll
        for (int c = 0; c < 2; ++c) pend6[c] = ((pend[c] >> 24) << 8) | ((pend[c] - 256u + gw0 * Ls[c]) & 0xffu);
        // slot 4t + q's stream position mod 256 in byte t of pos6[q] (rounds start at multiples
        // of 256 positions, so these are round-invariant)
        // byte t of pos6[q] = ((j < L0 ? pb0 : pb1) + j) mod 256, j = 4t + q: the lane's two stream
        // bases replicated into 4 bytes, merged by a uniform byte mask, plus the constant bytes
        // j — a byte-wise add with no carries between bytes (low 7 bits added, bit 7 xor-ed back)
        uint32_t pos6[4] = {0, 0, 0, 0};
        if constexpr (E6S) {
            const uint32_t A4 = perm(0u, pb0, 0x00000000u), B4 = perm(0u, pb1, 0x00000000u);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t mq = 0;  // (uniform) bytes t with 4t + q < L0
#pragma unroll
                for (int t = 0; t < 4; ++t) mq |= (4u * t + q < L0 ? 0xffu : 0u) << (8 * t);
                const uint32_t x = (A4 & mq) | (B4 & ~mq);
                const uint32_t jq = 0x0c080400u + (uint32_t)q * 0x01010101u;
                pos6[q] = ((x & 0x7f7f7f7fu) + jq) ^ (x & 0x80808080u);
            }
        }
        // a round's chunk starts: this lane's exclusive rank and the round's total per stream
        // (packed: stream 1 in the high half).  Taken before the round's sweep, so that a batch is
        // flushed only when THIS round's entries would not fit (round 6: the worst-case test,
        // 64·Ls entries per round, flushed C3's 8 rounds three times with 2-round staging)
        auto scan6 = [&](uint32_t C, uint32_t &pexc, uint32_t &Stot) __attribute__((always_inline)) {
            const uint32_t pc = popc(C & lowX) | (popc(C & highX) << 16);
            const uint32_t pinc = wave_incl_scan<OpAdd>(pc);
            pexc = pinc - pc;
            Stot = __builtin_amdgcn_readfirstlane(rdlane(pinc, 63));
        };
        // C in the byte-lane layout for the resident body (BL), compact for the streaming one
        auto sweep6 = [&](const uint4 &Tw, uint32_t C, uint32_t pexc, uint32_t Stot) __attribute__((always_inline)) {
            PSY_ASM_ROUND(B);
            const uint32_t T[4] = {Tw.x, Tw.y, Tw.z, Tw.w};
            // entry 0 of a region holds the pending chunk (when there is one); the batch's own
            // entries follow it
            const uint32_t D0 = eb6 + 2u * (u6[0] + (pexc & 0xffffu)) - jl;
            const uint32_t D1 = eb6 + eoff6 + 2u * (u6[1] + (pexc >> 16)) - jl;
            uint32_t D = L0 == 0 ? D1 : D0;
            // entries of slots q + 4t, two per dword: E[q][0] = slots q, q+4; E[q][1] = q+8, q+12
            uint32_t E[4][2];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                E[q][0] = perm(T[q], pos6[q], 0x05010400u);
                E[q][1] = perm(T[q], pos6[q], 0x07030602u);
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int q = j & 3, t = j >> 2;
                if (j > 0 && j % WPG == 0 && (uint32_t)j == L0) D = D1;  // stream 1 begins (uniform)
                const uint32_t bit = (C >> (BL ? sb_pos(j) : j)) & 1u;
                uint32_t ad;
                asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(ad) : "v"(bit), "v"(D), "s"(jl));
                const uint32_t e = E[q][t >> 1];
                if (t & 1) *reinterpret_cast<uint16_t *>(smem + ad) = (uint16_t)(e >> 16);
                else *reinterpret_cast<uint16_t *>(smem + ad) = (uint16_t)e;
                asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(D) : "v"(bit), "v"(D));
            }
            u6[0] += Stot & 0xffffu;
            u6[1] += Stot >> 16;
        };
        // flush the batch; last: the stream ends in it
        auto flush6 = [&](bool last) __attribute__((always_inline)) {
#if defined(PSY_X_NOEMIT) || defined(PSY_X_NOFLUSH)
            if (ngroups != 0xffffffffu) { u6[0] = u6[1] = 0; return; }  // diagnostic: no flush
#endif
            team_sync<1>();
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (c == 1 && !ns2) break;
                const uint32_t nent = u6[c];
                const uint32_t K = nent ? nent - 1u : 0u;  // pair k = entries k, k + 1
                const uint32_t eb = eb6 + (c ? eoff6 : 0u);
                uint8_t *const Dp = dst + sdata[c] + 2ull * pi5[c];
                auto pair_at = [&](uint32_t k) __attribute__((always_inline)) -> uint32_t {
                    const uint32_t e0 = *reinterpret_cast<const uint16_t *>(smem + eb + 2u * k);
                    const uint32_t e1 = *reinterpret_cast<const uint16_t *>(smem + eb + 2u * k + 2u);
                    return perm(e0, e1 - e0, 0x0c0c0500u);  // count = (e1 - e0) mod 256, value
                };
                // pairs k, k + 1 (k even) from entries k..k+2: one aligned dword and one u16 read,
                // both counts by one packed u16 subtract, one v_perm into (c0, v0, c1, v1)
                auto pairs2_at = [&](uint32_t k) __attribute__((always_inline)) -> uint32_t {
                    const uint32_t E01 = *reinterpret_cast<const uint32_t *>(smem + eb + 2u * k);
                    const uint32_t e2 = *reinterpret_cast<const uint16_t *>(smem + eb + 2u * k + 4u);
                    const uint32_t E12 = __builtin_amdgcn_alignbyte(e2, E01, 2);
                    uint32_t d;
                    asm("v_pk_sub_u16 %0, %1, %2" : "=v"(d) : "v"(E12), "v"(E01));
                    return perm(E01, d, 0x07020500u);
                };
                if (((uintptr_t)Dp & 1) == 0) {
                    // lane l stores pairs k0 + 2l, k0 + 2l + 1 with one (2-byte aligned) dword store.
                    // Non-temporal stores only where a store instruction's 256 bytes cannot hold
                    // the flush's first or last (partial) 128-byte line: plain stores leave those
                    // in L2, where the neighbouring flush's half of the line merges with them
                    // (round 4 wrote every pair non-temporally: 15.86 GB per C3 launch for 13.74 GB
                    // of blobs).  The choice is uniform per store instruction.
                    auto st_pair2 = [&](uint32_t k, uint32_t v, bool edge) __attribute__((always_inline)) {
                        if (edge) *reinterpret_cast<u32_a2 *>(Dp + 2u * k) = v;
                        else st32a2_nt(Dp + 2u * k, v);
                    };
                    uint32_t k0 = 0;
                    for (; k0 + 256u <= K; k0 += 256u) {
                        const uint32_t k = k0 + 2u * (uint32_t)lane;
                        const uint32_t pa = pairs2_at(k), pb = pairs2_at(k + 128u);
                        st_pair2(k, pa, k0 == 0u);
                        st_pair2(k + 128u, pb, K - k0 < 256u + 64u);
                    }
                    for (; k0 + 128u <= K; k0 += 128u) {
                        const uint32_t k = k0 + 2u * (uint32_t)lane;
                        st_pair2(k, pairs2_at(k), k0 == 0u || K - k0 < 128u + 64u);
                    }
                    const uint32_t k = k0 + 2u * (uint32_t)lane;
                    if (k + 1u < K) *reinterpret_cast<u32_a2 *>(Dp + 2u * k) = pairs2_at(k);
                    else if (k < K) *reinterpret_cast<uint16_t *>(Dp + 2u * k) = (uint16_t)pair_at(k);
                } else {
                    for (uint32_t k0 = 0; k0 < K; k0 += 64) {
                        const uint32_t k = k0 + (uint32_t)lane;
                        if (k < K) {
                            const uint32_t pair = pair_at(k);
                            Dp[2u * k] = (uint8_t)pair;
                            Dp[2u * k + 1u] = (uint8_t)(pair >> 8);
                        }
                    }
                }
                pi5[c] += K;
                if (nent) {
                    const uint32_t el = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const uint16_t *>(smem + eb + 2u * K));
                    if (last) {  // the final chunk runs to the end of the stream
                        if (lane == 0) {
                            Dp[2u * K] = (uint8_t)(slen[c] - el);
                            Dp[2u * K + 1u] = (uint8_t)(el >> 8);
                        }
                        pi5[c] += 1;
                    }
                    pend6[c] = el;
                }
                u6[c] = nent ? 1u : 0u;
            }
            team_sync<1>();  // the entries are rewritten by the next batch
        };

        if constexpr (RES) {
          if constexpr (E6) {
            // A batch of rounds is flushed before a round whose entries would overflow a stream's
            // staging region (capacity: the pending entry + NB rounds of 64·Ls entries; the
            // round's own count, scan6), and at the wave's last round — 2 flushes for a C3
            // message's 8 rounds.
            const uint32_t cap6[2] = {1u + NB * 64u * Ls[0], 1u + NB * 64u * Ls[1]};
            bool fresh = true;
            bool resolved = false;
            // (DEFER) wave 0 completes the look-back at its first flush and publishes the offset
            // in LDS; the other waves wait there for it.  Returns whether the blob fits.
            auto resolve_lb = [&]() __attribute__((always_inline)) -> bool {
                uint64_t b;
                uint32_t ok;
                if (wv == 0) {
#ifndef PSY_X_NOLBWAIT
                    b = lookback_resolve(a.lookback, msg, Eblob, a.errflags);
#else
                    b = (uint64_t)msg * (28 + 4 * WS + 2ull * n);  // diagnostic: offsets without the look-back
#endif
                    ok = b + Eblob <= a.out_cap ? 1u : 0u;
                    uint8_t *hd = a.out + b;
                    if (lane == 0) {
                        a.out_off[msg] = b;
                        if (msg == a.n_msgs - 1) a.out_off[a.n_msgs] = b + Eblob;
                        if (a.status) a.status[msg] = ok ? ST_OK : ST_CAPACITY;
                    }
                    if (ok) {
                        const uint32_t t = (uint32_t)lane;
                        if (t < hdr) {
                            const int f = t >> 2, sh = 8 * (t & 3);
                            uint32_t v;
                            if (f == 0) v = kMagicTDT;
                            else if (f == 1) v = n32;
                            else if (f == 2) v = ns;
                            else if (f == 3 || f == 4) v = WS;
                            else v = (mapbits >> (f - 5)) & 1u;
                            hd[t] = (uint8_t)(v >> sh);
                        } else if (t >= 48 && t < 56) {
                            const int c = (t - 48) >> 2, sh = 8 * (t & 3);
                            if ((uint32_t)c < ns) {
                                const uint32_t len = 2 * (c ? P1 : P0);
                                hd[sdata[c] - 4 + (t & 3)] = (uint8_t)(len >> sh);
                            }
                        }
                    }
                    if (lane == 0) {
                        *reinterpret_cast<uint64_t *>(misc + M_BASE) = b;
                        misc[M_BASE + 2] = ok;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        __hip_atomic_store(&wm[M_READY], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                } else {
                    while (__hip_atomic_load(&wm[M_READY], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
                        __builtin_amdgcn_s_sleep(2);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    b = *reinterpret_cast<const uint64_t *>(misc + M_BASE);
                    ok = misc[M_BASE + 2];
                }
                b = rfl_u64(b);
                dst = a.out + b;
                return __builtin_amdgcn_readfirstlane(ok) != 0u;
            };
            uint32_t rb = 0;  // the batch's first round
            // flush the batch of rounds [rb, re)
            auto flush_batch = [&](uint32_t re) __attribute__((always_inline)) -> bool {
                if constexpr (DEFER) {
                    if (!resolved) {
                        resolved = true;
                        if (!resolve_lb()) return false;  // TDT_E_CAPACITY: nothing is written
                    }
                }
                const uint32_t gb = gw0 + rb * 64u, ge = gw0 + re * 64u;
                flush6(gb <= ngroups - 1 && ngroups - 1 < ge);
                fresh = true;
                rb = re;
                return true;
            };
#pragma unroll
            for (int r = 0; r < G; ++r) {
                if ((uint32_t)r < RW) {
                    uint32_t pexc, Stot;
                    scan6(cres[r], pexc, Stot);
                    const uint32_t over = (u6[0] + (Stot & 0xffffu) > cap6[0] ? 1u : 0u) |
                                          (u6[1] + (Stot >> 16) > cap6[1] ? 1u : 0u);
                    if (over != 0u && !fresh) {
                        if (!flush_batch((uint32_t)r)) return;
                    }
                    if (fresh && lane == 0) {  // batch start: the pending entries
                        if (u6[0]) *reinterpret_cast<uint16_t *>(smem + eb6) = (uint16_t)pend6[0];
                        if (ns2 && u6[1]) *reinterpret_cast<uint16_t *>(smem + eb6 + eoff6) = (uint16_t)pend6[1];
                    }
                    fresh = false;
#ifndef PSY_X_NOEMIT
                    sweep6(dres[r], cres[r], pexc, Stot);
#endif
                    if ((uint32_t)(r + 1) == RW) {
                        if (!flush_batch((uint32_t)r + 1u)) return;
                    }
                }
            }
          } else
          {
#pragma unroll
            for (int r = 0; r < G; ++r) {
                if ((uint32_t)r < RW) {
                    emit5((uint32_t)r, dres[r], cres[r]);
                }
            }
          }
        } else {
            // chunk masks are computed one round ahead (lane 63 needs the next round's)
            uint32_t rcarry[2] = {rin[0], rin[1]};
            uint32_t edc = edc0;
            auto chunk_of = [&](uint32_t r, const uint4 &d, uint4 &Tw) __attribute__((always_inline)) -> uint32_t {
                const uint32_t g = gw0 + r * 64 + lane;
                const uint32_t V = full_round(r) ? 0xffffu : vmask(vbytes(g));
                uint32_t T[4];
                tmat(d, T);
                Tw = make_uint4(T[0], T[1], T[2], T[3]);
                const uint32_t ed = edges(d);
                const uint32_t m = run_mask(T, ed, edc, r == 0u && gw0 == 0u, V, std::false_type{});
                edc = rdlane(ed, 63);
                return clean ? m : chunk_round(r, m, rcarry, g, V);
            };
            uint4 Tc;
            uint32_t Cc = chunk_of(0, load_group(gw0 + lane), Tc);
            if constexpr (E6S) {
                // batches of rounds as in the resident body: a flush when the next round could
                // overflow a stream's staging region, or at the wave's last round (a flush per
                // round cost a 256 KiB message's waves 32 flushes instead of ~10)
                const uint32_t cap6[2] = {1u + NB * 64u * Ls[0], 1u + NB * 64u * Ls[1]};
                bool fresh = true;
                uint32_t rb = 0;  // the batch's first round
                for (uint32_t r = 0; r < RW; ++r) {
                    uint4 Tn = make_uint4(0, 0, 0, 0);
                    uint32_t Cn = 0;
                    if (r + 1 < RW) Cn = chunk_of(r + 1, load_group(gw0 + (r + 1) * 64 + lane), Tn);
                    uint32_t pexc, Stot;
                    scan6(Cc, pexc, Stot);
                    const uint32_t over = (u6[0] + (Stot & 0xffffu) > cap6[0] ? 1u : 0u) |
                                          (u6[1] + (Stot >> 16) > cap6[1] ? 1u : 0u);
                    if (over != 0u && !fresh) {  // this round's entries would not fit: flush [rb, r) first
                        const uint32_t gb = gw0 + rb * 64u, ge = gw0 + r * 64u;
                        flush6(gb <= ngroups - 1 && ngroups - 1 < ge);
                        fresh = true;
                        rb = r;
                    }
                    if (fresh && lane == 0) {  // batch start: the pending entries
                        if (u6[0]) *reinterpret_cast<uint16_t *>(smem + eb6) = (uint16_t)pend6[0];
                        if (ns2 && u6[1]) *reinterpret_cast<uint16_t *>(smem + eb6 + eoff6) = (uint16_t)pend6[1];
                    }
                    fresh = false;
                    sweep6(Tc, Cc, pexc, Stot);
                    if (r + 1 == RW) {
                        const uint32_t gb = gw0 + rb * 64u, ge = gw0 + r * 64u + 64u;
                        flush6(gb <= ngroups - 1 && ngroups - 1 < ge);
                        fresh = true;
                        rb = r + 1u;
                    }
                    Tc = Tn;
                    Cc = Cn;
                }
            } else {
                for (uint32_t r = 0; r < RW; ++r) {
                    uint4 Tn = make_uint4(0, 0, 0, 0);
                    uint32_t Cn = 0;
                    if (r + 1 < RW) Cn = chunk_of(r + 1, load_group(gw0 + (r + 1) * 64 + lane), Tn);
                    emit5(r, Tc, Cc);
                    Tc = Tn;
                    Cc = Cn;
                }
            }
        }
        PSY_PROF_MARK(6);
    }
    };  // run
    if constexpr (PATH == PATH_RES) {
        if (resident) {
            run(std::true_type{});
        } else if (tid == 0) {
            // (the plan never lists such a message here) flag it instead of a wild result
            atomicOr(a.errflags, 8u);
            if (a.status) a.status[msg] = ST_ARG;
            if (a.out_len) a.out_len[msg] = 0;
        }
    } else if constexpr (PATH == PATH_STREAM) {
        run(std::false_type{});
    } else {
        if (resident) run(std::true_type{});
        else run(std::false_type{});
    }
}

// Message ids: the compacted API's look-back needs them in dispatch order (atomic ticket);
// slotted batches take them from a class list (or, without one, the workgroup id); TL > 0:
// one large-message / span / tile entry per workgroup.  List and tile entries are bounded by
// the plan's device-side counts, so a launch never needs them on the host: the main launch
// (PS = 0) covers entries [list_base, list_base + grid) with one workgroup each, its grid sized
// from an earlier plan; the overflow launch (PS = 1) walks the entries past it grid-stride.
// (Only the overflow instances loop: around this body a loop makes the compiler keep
// loop-invariant values live across the whole message and spill at the 80-VGPR budget of 6
// waves per SIMD — correct, but slower.)
template <int TL>
__device__ __forceinline__ uint32_t entry_count(const EncodeArgs &a) {
    uint32_t c;
    if constexpr (TL == 0) c = *a.list_count + (a.list2 ? *a.list2_count : 0u);
    else if constexpr (TL == 4) c = umin(a.pcnt[4], a.lcap);
    else if constexpr (TL == 1) c = umin(a.pcnt[8], a.tcap / kSpanTiles);
    else if constexpr (TL == 2) c = umin(a.pcnt[22], a.tcap);
    else c = umin(a.pcnt[6], a.tcap);
    return __builtin_amdgcn_readfirstlane(c);
}

template <int WS, int TEAM, int G, int MODE, int LB, int TL = 0, int PS = 0, int PATH = PATH_BOTH>
__global__ __launch_bounds__(TEAM, PSY_ENC_WAVES(TEAM, LB)) void tdt_encode_kernel(EncodeArgs a) {
    using Lay = EncLayout<WS, TEAM, LB>;
    constexpr int W = Lay::W;
    __shared__ __attribute__((aligned(16))) uint8_t smem[Lay::BYTES];
    if constexpr (LB) {
        uint32_t *misc = reinterpret_cast<uint32_t *>(smem + Lay::OFF_MISC);
        if (threadIdx.x == 0) misc[M_MSG] = atomicAdd(a.ticket, 1u);
        team_sync<W>();
        encode_one<WS, TEAM, G, MODE, LB, 0>(a, smem, __builtin_amdgcn_readfirstlane(misc[M_MSG]), 0, 0);
        return;
    } else {
        // (slotted launches always pass a class list)
        const uint32_t n2 = TL == 0 && a.list2 ? __builtin_amdgcn_readfirstlane(*a.list2_count) : 0u;
        auto one = [&](uint32_t i) __attribute__((always_inline)) {
            if constexpr (TL == 0) {
                encode_one<WS, TEAM, G, MODE, LB, 0, PATH>(a, smem, i < n2 ? a.list2[i] : a.list[i - n2], 0, 0);
            } else if constexpr (TL == 4) {
                const uint32_t msg = a.lmeta[i].msg;  // one large message per workgroup
                if (msg != kNone) encode_one<WS, TEAM, G, MODE, LB, TL>(a, smem, msg, i, 0);
            } else {
                const uint64_t e = TL == 1 ? a.spans[i] : TL == 2 ? a.rtiles[i] : a.tiles[i];  // a span or tile
                const uint32_t lj = (uint32_t)e;
                if (lj == kNone) return;  // a message that did not fit the budgets
                encode_one<WS, TEAM, G, MODE, LB, TL>(a, smem, a.lmeta[lj].msg, lj, (uint32_t)(e >> 32));
            }
        };
        const uint32_t cnt = entry_count<TL>(a);
        const uint32_t i0 = a.list_base + blockIdx.x;
        if constexpr (PS) {
            for (uint32_t i = i0; i < cnt; i += gridDim.x) {
                if (i != i0) team_sync<W>();  // the previous entry is done with the LDS
                one(i);
            }
        } else if constexpr (TL == 0) {
            // the list entry is read beside the counts, not after them (i0 < n_msgs = every
            // class list's capacity; a stale entry past the count is never used)
            const uint32_t ic = i0 < a.n_msgs ? i0 : a.n_msgs - 1u;
            const uint32_t e2 = a.list2 ? a.list2[ic] : 0u, e1 = a.list[ic];
            if (i0 >= cnt) return;
            encode_one<WS, TEAM, G, MODE, LB, 0, PATH>(a, smem, i0 < n2 ? e2 : (n2 == 0u ? e1 : a.list[i0 - n2]), 0,
                                                       0);
        } else {
            if (i0 >= cnt) return;
            one(i0);
        }
    }
}

// ------------------------------------------------------------------ slotted-batch plan
// Message classes: small (<= small_max bytes: one-wave teams), medium (512-lane
// teams), large (> large_min: 64 KiB tiles, so that one message spreads over the whole chip).
// One thread per message; small / medium ids are appended with one atomic per wave (list order
// is irrelevant: every blob goes to its own slot).  A large message claims an LMeta entry and a
// contiguous range of tile entries (tiles of one message in order); when the budgets (lmax
// entries, tile_cap tiles) are spent it stays medium.
struct PlanArgs {
    const uint8_t *in;  // (alignment of each message: the medium list is resident-only)
    const uint64_t *in_off;
    uint32_t n_msgs;
    // [0] small (listed), [1] medium, [2] large entries, [3] tiles, [4] spans claimed, [5] small
    // messages (listed or not: the host's count history switches the small class back on), [6]
    // mid-sized (listed), [7] mid-sized messages (listed or not), [8] medium messages over big_min
    // (their own list, dispatched first), [9] passthrough (UNCP) messages up to large_min (listed or
    // not), [10] UNCP messages listed
    unsigned long long *cnt;
    uint32_t *slist, *mlist, *qlist, *blist, *clist;
    uint64_t *tiles, *spans;
    LMeta *lmeta;
    uint32_t lmax, tile_cap;  // span_cap = tile_cap / kSpanTiles (0, 0: no tiled path)
    uint64_t small_max, mid_max, big_min, large_min;
    uint32_t small_on;  // 0: small messages join the medium list
    uint32_t mid_on;    // 0: mid-sized messages join the medium list
    // should_transform :186-201 + compress_tdt's size guard :364-367, as encode_one evaluates
    // them: messages that stay UNCP go to the copy list (clist null: no copy list)
    uint64_t min_tensor;
    uint32_t policy_on, ws;
    uint32_t copy_on;  // 0: UNCP messages join their size classes (the count history switches it on)
};

constexpr uint32_t kPlanThreads = 1024, kPlanPer = 2;  // messages per plan workgroup: 2048

#ifndef PSY_ENC_INST_TU  // (defined once, in tdt_api.hip)
__global__ __launch_bounds__(kPlanThreads) void tdt_encode_plan_kernel(PlanArgs p) {
    __shared__ uint64_t lds[8 * (kPlanPer * 16 + 1)];
    const uint32_t scap = p.tile_cap / kSpanTiles;
    // A message takes the tiled path above max(large_min, 1/4096 of the batch's bytes), as the
    // decode plan: below that the batch has enough other messages to keep the chip busy while
    // one 512-lane team streams it (long messages are dispatched first), and the streaming body
    // reads it twice like the tiles but without their span / map / scan passes — C4 (1 MiB
    // messages in 24.6 GiB) encode 19.7 -> 18.8 ms with none of its messages tiled.
    uint64_t thr = p.large_min;
    if (p.n_msgs) {
        const uint64_t share = (p.in_off[p.n_msgs] - p.in_off[0]) / 4096;
        thr = share > thr ? share : thr;
    }
    // the claims' values (A: large messages, tiles, spans; B: the lists) and their starts
    uint64_t A[3][kPlanPer], SA[3][kPlanPer], B[8][kPlanPer], SB[8][kPlanPer];
    uint64_t n[kPlanPer];
    auto &isl = A[0], &T = A[1], &S = A[2];
    auto &j = SA[0], &t0 = SA[1], &s0 = SA[2];
#pragma unroll
    for (int k = 0; k < (int)kPlanPer; ++k) {
        const uint32_t i = (blockIdx.x * kPlanPer + k) * kPlanThreads + threadIdx.x;
        n[k] = i < p.n_msgs ? p.in_off[i + 1] - p.in_off[i] : 0;
        isl[k] = i < p.n_msgs && n[k] > thr ? 1u : 0u;
        T[k] = isl[k] ? (n[k] + 16ull * kTileGroups - 1) / (16ull * kTileGroups) : 0;
        S[k] = (T[k] + kSpanTiles - 1) / kSpanTiles;
    }
    {
        constexpr int ia[3] = {2, 3, 4};
        wg_claim_n<3, kPlanPer>(A, SA, p.cnt, ia, lds);
    }
    auto &sm = B[0], &md = B[1], &sc = B[2], &qm = B[3], &qc = B[4], &bm = B[5], &cc = B[6], &cp = B[7];
    auto &ps = SB[0], &pm = SB[1], &pq = SB[3], &pb = SB[5], &pcp = SB[7];
#pragma unroll
    for (int k = 0; k < (int)kPlanPer; ++k) {
        const uint32_t i = (blockIdx.x * kPlanPer + k) * kPlanThreads + threadIdx.x;
        bool large = false;
        if (isl[k]) {
            large = j[k] < p.lmax && t0[k] + T[k] <= p.tile_cap && s0[k] + S[k] <= scap;
            if (large) {
                LMeta m{};
                m.msg = i;
                m.ntiles = (uint32_t)T[k];
                m.tile0 = (uint32_t)t0[k];
                m.span0 = (uint32_t)s0[k];
                p.lmeta[j[k]] = m;
            } else if (j[k] < p.lmax) {
                p.lmeta[j[k]].msg = kNone;
            }
            // tile / span entries (kNone: the message is over a budget and stays medium)
            for (uint64_t t = 0; t < T[k] && t0[k] + t < p.tile_cap; ++t)
                p.tiles[t0[k] + t] = large ? (t << 32 | j[k]) : (uint64_t)kNone;
            for (uint64_t t = 0; t < S[k] && s0[k] + t < scap; ++t)
                p.spans[s0[k] + t] = large ? (t << 32 | j[k]) : (uint64_t)kNone;
        }
        const bool valid = i < p.n_msgs;
        const bool transform = p.policy_on && n[k] >= p.min_tensor && (n[k] % 4 == 0) && n[k] >= 64 &&
                               (n[k] % p.ws == 0) && n[k] < (1ull << 32);
        const bool uncp = valid && !isl[k] && !transform;
        const bool copy = uncp && p.copy_on;
        cc[k] = uncp ? 1u : 0u;
        cp[k] = copy ? 1u : 0u;
        const bool small = valid && !isl[k] && !copy && n[k] <= p.small_max;
        const bool mid = valid && !isl[k] && !copy && !small && n[k] <= p.mid_max;
        sc[k] = small ? 1u : 0u;
        sm[k] = small && p.small_on ? 1u : 0u;
        qc[k] = mid ? 1u : 0u;
        qm[k] = mid && p.mid_on ? 1u : 0u;
        const bool medium = valid && !large && !copy && !sm[k] && !qm[k];
        // the medium list's kernel holds only the resident body: longer or unaligned messages
        // (and those of size not a multiple of 16) take the big list's streaming kernel
        const bool res_ok = n[k] <= p.big_min && (n[k] & 15u) == 0 &&
                            (((uintptr_t)p.in + (valid ? p.in_off[i] : 0ull)) & 15u) == 0;
        bm[k] = medium && p.blist && !res_ok ? 1u : 0u;
        md[k] = medium && !bm[k] ? 1u : 0u;
    }
    {
        constexpr int ib[8] = {0, 1, 5, 6, 7, 8, 9, 10};
        wg_claim_n<8, kPlanPer>(B, SB, p.cnt, ib, lds);
    }
#pragma unroll
    for (int k = 0; k < (int)kPlanPer; ++k) {
        const uint32_t i = (blockIdx.x * kPlanPer + k) * kPlanThreads + threadIdx.x;
        if (sm[k]) p.slist[ps[k]] = i;
        if (md[k]) p.mlist[pm[k]] = i;
        if (qm[k]) p.qlist[pq[k]] = i;
        if (bm[k]) p.blist[pb[k]] = i;
        if (cp[k]) p.clist[pcp[k]] = i;
    }
}

#endif  // PSY_ENC_INST_TU

// Large messages, between the count and emit passes: one wave per message walks its tile
// records in order — prefix max of the last run start (the run carried into each tile),
// the 255-cap chunk starts that carried run makes inside the tile before its first own run
// start, prefix sums of the chunk starts — rewrites the records for the emit pass, and writes
// the blob's size, status and header.
template <int WS>
__global__ __launch_bounds__(64) void tdt_encode_lscan_kernel(EncodeArgs a, const uint32_t *lcnt, uint32_t lmax) {
    const uint32_t nl = umin(*lcnt, lmax);
    const int lane = lane_id();
    for (uint32_t j = blockIdx.x; j < nl; j += gridDim.x) {
        LMeta *lm = a.lmeta + j;
        const uint32_t msg = lm->msg;
        if (msg == kNone) continue;  // fell back to the whole-message kernel
        const uint64_t n = a.in_off[msg + 1] - a.in_off[msg];
        const bool compress = a.policy_on && n >= a.min_tensor && (n % 4 == 0) && n >= 64 && (n % WS == 0) &&
                              n < (1ull << 32);
        if (!compress) continue;  // UNCP: the histogram pass copied it
        const uint32_t wc = (uint32_t)n / WS;
        const uint32_t mapbits = lm->mapbits;
        const uint32_t k1 = (uint32_t)__builtin_popcount(mapbits & ((1u << WS) - 1u)), k0 = WS - k1;
        const bool ns2 = k1 != 0;
        const uint32_t Ls[2] = {(16u / WS) * k0, (16u / WS) * k1};
        const uint32_t slen[2] = {wc * k0, wc * k1};
        const uint32_t T = lm->ntiles;
        TileRec *rec = a.trec + lm->tile0;
        uint32_t Pt[2] = {0, 0};
        for (int c = 0; c < (ns2 ? 2 : 1); ++c) {
            uint32_t carry = 0, P = 0;
            for (uint32_t t0 = 0; t0 < T; t0 += 64) {
                const uint32_t t = t0 + (uint32_t)lane;
                const bool valid = t < T;
                const uint32_t lrs = valid ? rec[t].lrs[c] : 0u;
                const uint32_t frs = valid ? rec[t].frs[c] : kNone;
                const uint32_t cnt = valid ? rec[t].cnt[c] : 0u;
                const uint32_t incl = wave_incl_scan<OpMax>(lrs);
                const uint32_t excl = umax(carry, wave_shr1(incl, 0u));
                const uint64_t ts = (uint64_t)t * kTileGroups * Ls[c];
                const uint64_t te = umin64((uint64_t)(t + 1) * kTileGroups * Ls[c], slen[c]);
                const uint64_t e = frs != kNone ? (uint64_t)frs : te;
                uint32_t h = 0;
                if (valid && excl > 0 && e > ts) {
                    const uint64_t rs = excl - 1u;  // < ts: the run carried into the tile
                    const uint64_t klo = (ts - rs + 254u) / 255u, khi = (e - 1u - rs) / 255u;
                    h = khi >= klo ? (uint32_t)(khi - klo + 1u) : 0u;
                }
                const uint32_t tot = cnt + h;
                const uint32_t pincl = wave_incl_scan<OpAdd>(tot);
                if (valid) {
                    rec[t].lrs[c] = excl;
                    rec[t].cnt[c] = P + pincl - tot;
                    if (h) rec[t].clean = 0u;
                }
                carry = umax(carry, (uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
                P += (uint32_t)__builtin_amdgcn_readlane((int)pincl, 63);
            }
            Pt[c] = P;
        }
        const uint32_t hdr = 20 + 4 * WS;
        const uint64_t E = hdr + (4 + 2ull * Pt[0]) + (ns2 ? 4 + 2ull * Pt[1] : 0);
        const uint64_t ob = a.slot_off[msg];
        const bool fits = E <= a.slot_off[msg + 1] - ob;
        if (lane == 0) {
            if (a.status) a.status[msg] = fits ? ST_OK : ST_CAPACITY;
            if (a.out_len) a.out_len[msg] = fits ? E : 0;
            lm->P0 = Pt[0];
            lm->fits = fits ? 1u : 0u;
        }
        if (!fits) continue;
        uint8_t *dst = a.out + ob;
        for (uint32_t t = (uint32_t)lane; t < hdr; t += 64) {
            const int f = t >> 2, sh = 8 * (t & 3);
            uint32_t v;
            if (f == 0) v = kMagicTDT;
            else if (f == 1) v = (uint32_t)n;
            else if (f == 2) v = ns2 ? 2u : 1u;
            else if (f == 3 || f == 4) v = WS;
            else v = (mapbits >> (f - 5)) & 1u;
            dst[t] = (uint8_t)(v >> sh);
        }
        if (lane < 8) {
            const int c = lane >> 2, sh = 8 * (lane & 3);
            const uint32_t sd0 = hdr + 4, sd1 = hdr + 4 + 2 * Pt[0] + 4;
            if (c == 0 || ns2) dst[(c ? sd1 : sd0) - 4 + (lane & 3)] = (uint8_t)((2 * Pt[c]) >> sh);
        }
    }
}

// The kernel instances of one word size.  The product library instantiates them in
// tdt_enc_ws.hip, one translation unit per word size (compiled in parallel), and tdt_api.hip
// declares them extern; diagnostic single-TU builds instantiate them implicitly.
#define PSY_ENC_INSTANCES(X, WS)                                                                                  \
    X(WS, 512, 8, MODE_ENCODE, 0, 0, 0, 1) X(WS, 512, 8, MODE_ENCODE, 0, 0, 1, 1) X(WS, 512, 8, MODE_ENCODE, 0, 0, 0, 2) \
    X(WS, 512, 8, MODE_ENCODE, 0, 0, 1, 2) X(WS, 512, 8, MODE_ENCODE, 0, 1, 0, 0) X(WS, 512, 8, MODE_ENCODE, 0, 2, 0, 0) \
    X(WS, 512, 8, MODE_ENCODE, 0, 3, 0, 0) X(WS, 512, 8, MODE_ENCODE, 0, 4, 0, 0) X(WS, 64, 4, MODE_ENCODE, 0, 0, 0, 0)  \
    X(WS, 512, 8, MODE_ENCODE, 0, 1, 1, 0) X(WS, 512, 8, MODE_ENCODE, 0, 2, 1, 0) X(WS, 512, 8, MODE_ENCODE, 0, 3, 1, 0) \
    X(WS, 512, 8, MODE_ENCODE, 0, 4, 1, 0) X(WS, 64, 4, MODE_ENCODE, 0, 0, 1, 0) X(WS, 256, 8, MODE_ENCODE, 0, 0, 0, 0)  \
    X(WS, 256, 8, MODE_ENCODE, 0, 0, 1, 0) X(WS, 64, 4, MODE_ENCODE, 1, 0, 0, 0) X(WS, 512, 8, MODE_ENCODE, 1, 0, 0, 0)  \
    X(WS, 64, 4, MODE_MAPPED, 1, 0, 0, 0) X(WS, 512, 8, MODE_MAPPED, 1, 0, 0, 0) X(WS, 64, 4, MODE_ANALYZE, 1, 0, 0, 0)  \
    X(WS, 512, 8, MODE_ANALYZE, 1, 0, 0, 0) X(WS, 512, 8, MODE_ENCODE, 1, 0, 0, 1)

}  // namespace psy
