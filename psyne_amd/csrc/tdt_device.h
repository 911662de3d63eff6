// tdt_device.h — CDNA4 device building blocks shared by the TDT encode/decode kernels.
//
//   * wave64 inclusive scans on DPP (row_shr 1/2/4/8 + row_bcast 15/31: 12 VALU, no LDS)
//   * team (workgroup) exclusive scans: one DPP wave scan + one LDS exchange + one barrier
//   * decoupled look-back over message ids (single-pass compaction of variable-length
//     outputs; the status word carries the value, so no separate flag/fence is needed:
//     MI355X_MICROARCH.md "R2: the data IS the flag", 8-byte relaxed agent-scope atomics)
//   * byte-exact global loads/stores that never touch bytes outside the buffer
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psy {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

// Phase-cycle instrumentation for diagnostic builds only (-DPSY_PROF=1, tools/phase_prof.py):
// wave-lane 0 accumulates s_memtime deltas per phase.  Compiled out of the product library.
#if defined(PSY_PROF) && PSY_PROF
__device__ unsigned long long psy_prof[32];
#define PSY_PROF_BEGIN() uint64_t psy_pt_ = __builtin_amdgcn_s_memtime()
#define PSY_PROF_MARK(i)                                                    \
    do {                                                                    \
        const uint64_t psy_t_ = __builtin_amdgcn_s_memtime();               \
        if (lane_id() == 0) atomicAdd(&psy_prof[(i)], psy_t_ - psy_pt_);    \
        psy_pt_ = psy_t_;                                                   \
    } while (0)
#elif defined(PSY_X_STOP)
// diagnostic attribution builds: the encode kernel returns at phase mark PSY_X_STOP
#define PSY_PROF_BEGIN() ((void)0)
#define PSY_PROF_MARK(i)                        \
    do {                                        \
        if ((i) == PSY_X_STOP) return;          \
    } while (0)
#elif defined(PSY_ASM_MARKS)
#define PSY_PROF_BEGIN() ((void)0)
#define PSY_PROF_MARK(i) asm volatile(";@@MARK " #i ::)
#else
#define PSY_PROF_BEGIN() ((void)0)
#define PSY_PROF_MARK(i) ((void)0)
#endif
#ifdef PSY_ASM_MARKS
#define PSY_ASM_ROUND(p) asm volatile(";@@ROUND " #p ::)
#else
#define PSY_ASM_ROUND(p) ((void)0)
#endif

template <int CTRL, int ROWMASK = 0xf, int BANKMASK = 0xf>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t x) {
    // Lanes whose source is outside the row / disabled by ROWMASK receive 0 (the identity
    // of both scan operators used here).
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, BANKMASK, false);
}

// v_med3_i32 (clamp x to [lo, hi] in one VALU; clang folds smax(smin()) into it only for
// constant bounds)
__device__ __forceinline__ int32_t med3_i32(int32_t x, int32_t lo, int32_t hi) {
    int32_t r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "v"(hi));
    return r;
}

// 2x as v_add_u32 x, x (a fast-issue add; clang turns x + x into v_lshlrev_b32, a slow one)
__device__ __forceinline__ uint32_t add_self(uint32_t x) {
    uint32_t r;
    asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(x));
    return r;
}

struct OpAdd {
    __device__ __forceinline__ static uint32_t f(uint32_t a, uint32_t b) { return a + b; }
};
struct OpMax {
    __device__ __forceinline__ static uint32_t f(uint32_t a, uint32_t b) { return a > b ? a : b; }
};

// DPP move whose disabled / out-of-row lanes return x itself: the identity for idempotent
// operators (max), so no zero-initialised register is needed.
template <int CTRL, int ROWMASK = 0xf, int BANKMASK = 0xf>
__device__ __forceinline__ uint32_t dpp_mov_self(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, CTRL, ROWMASK, BANKMASK, false);
}

template <class Op>
struct ScanIdem {
    static constexpr bool value = false;
};

// Inclusive wave64 scan with identity 0.
template <class Op>
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    if constexpr (ScanIdem<Op>::value) {
        // row shifts with bound_ctrl (out-of-row lanes read 0, the identity): one v_mov_dpp each
        x = Op::f(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true));
        x = Op::f(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true));
        x = Op::f(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true));
        x = Op::f(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true));
        x = Op::f(x, dpp_mov_self<0x142, 0xa>(x));
        x = Op::f(x, dpp_mov_self<0x143, 0xc>(x));
        return x;
    }
    x = Op::f(x, dpp_mov<0x111>(x));       // row_shr:1
    x = Op::f(x, dpp_mov<0x112>(x));       // row_shr:2
    x = Op::f(x, dpp_mov<0x114>(x));       // row_shr:4
    x = Op::f(x, dpp_mov<0x118>(x));       // row_shr:8
    x = Op::f(x, dpp_mov<0x142, 0xa>(x));  // row_bcast:15 into rows 1,3
    x = Op::f(x, dpp_mov<0x143, 0xc>(x));  // row_bcast:31 into rows 2,3
    return x;
}

__device__ __forceinline__ uint32_t wave_shift_up1(uint32_t x) {
    // lane l receives lane l-1's value, lane 0 receives 0
    return (uint32_t)__shfl_up((int)x, 1) * (lane_id() != 0);
}

// DPP wavefront shifts (GFX9 wave_shr:1 / wave_shl:1): lane l receives lane l-1 (resp.
// l+1); the lane whose source lies outside the wave receives `old`.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_shl1(uint32_t x, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x130, 0xf, 0xf, false);
}

// Two independent u16 lanes per dword (v_pk_max_u16).
typedef unsigned short psy_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(psy_u16x2, a),
                                                                  __builtin_bit_cast(psy_u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(psy_u16x2, a),
                                                                  __builtin_bit_cast(psy_u16x2, b)));
}
// (lo, max(hi, lo)) and (max(a.lo, b.hi), max(a.hi, b.hi)): one v_pk_max_u16 each, the half
// broadcast folded into the instruction's op_sel (no shift / v_perm in front of it).
__device__ __forceinline__ uint32_t pk_max_self_lo(uint32_t a) {
    uint32_t r;
    asm("v_pk_max_u16 %0, %1, %1 op_sel:[0,0] op_sel_hi:[1,0]" : "=v"(r) : "v"(a));
    return r;
}
__device__ __forceinline__ uint32_t pk_max_bcast_hi(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_pk_max_u16 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// Two independent u16 adds per dword (v_pk_add_u16, no carry between the halves).
__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(psy_u16x2, a) + __builtin_bit_cast(psy_u16x2, b));
}
__device__ __forceinline__ uint32_t pk_sub_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(psy_u16x2, a) - __builtin_bit_cast(psy_u16x2, b));
}
struct OpPkMax {
    __device__ __forceinline__ static uint32_t f(uint32_t a, uint32_t b) { return pk_max_u16(a, b); }
};
// (OpMax takes the identity-0 path: the compiler folds each DPP move into v_max_u32_dpp, one
// VALU per step; v_pk_max_u16 has no DPP form, so OpPkMax keeps the self-identity moves.)
template <>
struct ScanIdem<OpPkMax> {
    static constexpr bool value = true;
};

// v_ffbh_u32 with its hardware semantics (count of leading zeros, 0xffffffff for 0), so the
// compiler can neither add a zero fix-up nor treat 0 as poison.
__device__ __forceinline__ uint32_t ffbh_u32(uint32_t x) {
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// f64 helpers: DPP moves of both halves (lanes whose source is outside the row get 0)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const uint32_t lo = dpp_mov<CTRL>((uint32_t)u), hi = dpp_mov<CTRL>((uint32_t)(u >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// lane 16r + 15 receives the sum of row r's 16 values (other lanes: partial sums)
__device__ __forceinline__ double row_sum_f64(double x) {
    x += dpp_f64<0x111>(x);  // row_shr:1
    x += dpp_f64<0x112>(x);  // row_shr:2
    x += dpp_f64<0x114>(x);  // row_shr:4
    x += dpp_f64<0x118>(x);  // row_shr:8
    return x;
}
// Segmented sums over SEG consecutive lanes (SEG a power of two, 1..64): the segment's last
// lane receives its sum (other lanes: partial sums).  row_shr steps stay inside 16-lane rows;
// row_bcast:15 / :31 carry row sums across rows.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64_rm(double x) {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const uint32_t lo = dpp_mov<CTRL, ROWMASK>((uint32_t)u), hi = dpp_mov<CTRL, ROWMASK>((uint32_t)(u >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <int SEG>
__device__ __forceinline__ double seg_sum_f64(double x) {
    if constexpr (SEG >= 2) x += dpp_f64_rm<0x111, 0xf>(x);  // row_shr:1
    if constexpr (SEG >= 4) x += dpp_f64_rm<0x112, 0xf>(x);  // row_shr:2
    if constexpr (SEG >= 8) x += dpp_f64_rm<0x114, 0xf>(x);  // row_shr:4
    if constexpr (SEG >= 16) x += dpp_f64_rm<0x118, 0xf>(x);  // row_shr:8
    if constexpr (SEG >= 32) x += dpp_f64_rm<0x142, 0xa>(x);  // row_bcast:15 into rows 1, 3
    if constexpr (SEG >= 64) x += dpp_f64_rm<0x143, 0xc>(x);  // row_bcast:31 into rows 2, 3
    return x;
}
template <int SEG>
__device__ __forceinline__ uint32_t seg_sum_u32(uint32_t x) {
    if constexpr (SEG >= 2) x += dpp_mov<0x111, 0xf>(x);
    if constexpr (SEG >= 4) x += dpp_mov<0x112, 0xf>(x);
    if constexpr (SEG >= 8) x += dpp_mov<0x114, 0xf>(x);
    if constexpr (SEG >= 16) x += dpp_mov<0x118, 0xf>(x);
    if constexpr (SEG >= 32) x += dpp_mov<0x142, 0xa>(x);
    if constexpr (SEG >= 64) x += dpp_mov<0x143, 0xc>(x);
    return x;
}
__device__ __forceinline__ double readlane_f64(double x, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

template <class Op>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan<Op>(x), 63);
}

// Team-wide exclusive scan of NV values per thread in threadIdx order.
// slots: LDS scratch of W*NV uint32 (callers alternate two slot buffers between
// consecutive scans so that only ONE barrier per scan is needed).
// On return v[k] holds the exclusive prefix and tot[k] the team total (uniform).
template <int W, int NV, class Op>
__device__ __forceinline__ void team_excl_scan(uint32_t (&v)[NV], uint32_t (&tot)[NV], uint32_t *slots) {
    const int lane = lane_id();
    uint32_t inc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) inc[k] = wave_incl_scan<Op>(v[k]);
    if constexpr (W == 1) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            tot[k] = (uint32_t)__builtin_amdgcn_readlane((int)inc[k], 63);
            v[k] = wave_shift_up1(inc[k]);
        }
    } else {
        const int w = threadIdx.x >> 6;
        if (lane == 63) {
#pragma unroll
            for (int k = 0; k < NV; ++k) slots[w * NV + k] = inc[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            uint32_t pre = 0, t = 0;
#pragma unroll
            for (int ww = 0; ww < W; ++ww) {
                uint32_t s = slots[ww * NV + k];
                if (ww < w) pre = Op::f(pre, s);
                t = Op::f(t, s);
            }
            tot[k] = t;
            v[k] = Op::f(pre, wave_shift_up1(inc[k]));
        }
    }
}

// Plan kernels (1024 threads, NK values per thread at slots (k, wave, lane) in message order):
// the exclusive prefix of v over the workgroup's slots plus ONE atomic add of its total to
// *ctr — a per-message or per-wave atomic on one counter serialises badly at millions of
// messages.  lds: NK·16 + 1 words.  All threads must call it.
template <int NK>
__device__ __forceinline__ void wg_claim(const uint64_t (&v)[NK], uint64_t (&start)[NK], unsigned long long *ctr,
                                         uint64_t *lds) {
    const int lane = (int)__lane_id(), wv = threadIdx.x >> 6;
    uint64_t incl[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        uint64_t x = v[k];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        incl[k] = x;
        if (lane == 63) lds[k * 16 + wv] = x;
    }
    __syncthreads();
    // the NK·16 wave totals scanned by wave 0, one per lane (a serial loop over them by one
    // thread was ~3 µs of LDS round trips per call: most of a one-workgroup plan's time)
    static_assert(NK * 16 <= 64, "one wave scans the wave totals");
    if (wv == 0) {
        const uint64_t x = lane < NK * 16 ? lds[lane] : 0ull;
        uint64_t s = x;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(s, d);
            if (lane >= d) s += y;
        }
        if (lane < NK * 16) lds[lane] = s - x;
        if (lane == 63) lds[NK * 16] = s ? atomicAdd(ctr, (unsigned long long)s) : 0ull;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NK; ++k) start[k] = lds[NK * 16] + lds[k * 16 + wv] + incl[k] - v[k];
    __syncthreads();  // lds is reused by the next call
}

// wg_claim of NC counters at once (counter c = cnt[idx[c]]): one pair of barriers and NC
// independent atomics in flight together.  A one-workgroup plan (a host-pipeline chunk) is a
// chain of these claims: nine single claims cost ~30 µs of barriers and atomic round trips.
// lds: NC·(NK·16 + 1) words.
template <int NC, int NK>
__device__ __forceinline__ void wg_claim_n(const uint64_t (&v)[NC][NK], uint64_t (&start)[NC][NK],
                                           unsigned long long *cnt, const int (&idx)[NC], uint64_t *lds) {
    constexpr int E = NK * 16;
    static_assert(E <= 64, "one wave scans the wave totals");
    const int lane = (int)__lane_id(), wv = threadIdx.x >> 6;
    uint64_t incl[NC][NK];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            uint64_t x = v[c][k];
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t y = __shfl_up(x, d);
                if (lane >= d) x += y;
            }
            incl[c][k] = x;
            if (lane == 63) lds[c * E + k * 16 + wv] = x;
        }
    __syncthreads();
    if (wv == 0) {
        uint64_t tot[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const uint64_t x = lane < E ? lds[c * E + lane] : 0ull;
            uint64_t s = x;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t y = __shfl_up(s, d);
                if (lane >= d) s += y;
            }
            if (lane < E) lds[c * E + lane] = s - x;
            tot[c] = s;
        }
        if (lane == 63) {
            uint64_t r[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) r[c] = tot[c] ? atomicAdd(cnt + idx[c], (unsigned long long)tot[c]) : 0ull;
#pragma unroll
            for (int c = 0; c < NC; ++c) lds[NC * E + c] = r[c];
        }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int k = 0; k < NK; ++k) start[c][k] = lds[NC * E + c] + lds[c * E + k * 16 + wv] + incl[c][k] - v[c][k];
    __syncthreads();  // lds is reused by the next call
}

template <int W>
__device__ __forceinline__ void team_sync() {
    if constexpr (W == 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------
// Decoupled look-back over message ids.  st[i] = flag(2 bits) | value(62 bits);
// flag 1 = aggregate (this message's size) published, 2 = inclusive prefix published.
// Message ids are claimed through an atomic ticket in launch order, so every predecessor
// is already resident and publishes its aggregate without waiting: no deadlock, whatever
// the dispatch order.  The spin is bounded; on timeout *timeout is set and 0 is assumed.
constexpr uint64_t kLbAgg = 1ull << 62;
constexpr uint64_t kLbInc = 2ull << 62;
constexpr uint64_t kLbVal = (1ull << 62) - 1;

__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_load(uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by ONE thread.  Returns the exclusive prefix of message i.
__device__ __forceinline__ uint64_t lookback_excl(uint64_t *st, uint32_t i, uint64_t agg,
                                                  uint32_t *timeout) {
    if (i == 0) {
        lb_store(&st[0], kLbInc | agg);
        return 0;
    }
    lb_store(&st[i], kLbAgg | agg);
    uint64_t excl = 0;
    int64_t j = (int64_t)i - 1;
    uint32_t spins = 0;
    while (j >= 0) {
        uint64_t s = lb_load(&st[j]);
        uint64_t f = s >> 62;
        if (f == 0) {
            if (++spins > (1u << 26)) {
                atomicOr(timeout, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += s & kLbVal;
        if (f == 2) break;
        --j;
    }
    lb_store(&st[i], kLbInc | (excl + agg));
    return excl;
}

// A u64 made wave-uniform (lane 0's).  readfirstlane returns int: each half goes through
// uint32_t, or a low half >= 2^31 would sign-extend over the high one.
__device__ __forceinline__ uint64_t rfl_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Sum of a u64 over the wave (butterfly on both 32-bit halves).
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

// Wave-parallel look-back: called by ALL lanes of one wave (uniform control flow); returns
// the exclusive prefix of message i in every lane.  Each round trip reads the 64 status
// words below the window's top at once; the nearest inclusive prefix (a ballot) ends the
// walk, windows of aggregates are summed and skipped, a window with an unpublished word is
// re-read.  Message indices below 0 read as "inclusive 0".  Bounded spin as above.
// Split form of lookback_excl_wave for a team that publishes its aggregate early and needs
// its exclusive prefix only later: lookback_publish (wave 0 of the team), then
// lookback_resolve (the same wave) returns the prefix and publishes the inclusive value.
__device__ __forceinline__ void lookback_publish(uint64_t *st, uint32_t i, uint64_t agg);
__device__ __forceinline__ uint64_t lookback_resolve(uint64_t *st, uint32_t i, uint64_t agg, uint32_t *timeout);

__device__ __forceinline__ uint64_t lookback_excl_wave(uint64_t *st, uint32_t i, uint64_t agg,
                                                       uint32_t *timeout) {
    const int lane = lane_id();
    if (i == 0) {
        if (lane == 0) lb_store(&st[0], kLbInc | agg);
        return 0;
    }
    if (lane == 0) lb_store(&st[i], kLbAgg | agg);
    uint64_t excl = 0;
    int64_t top = (int64_t)i;  // window [top - 64, top)
    uint32_t spins = 0;
    while (true) {
        const int64_t j = top - 64 + lane;
        const uint64_t s = j >= 0 ? lb_load(&st[j]) : kLbInc;
        const uint32_t f = (uint32_t)(s >> 62);
        const uint64_t bz = __ballot(f == 0);
        const uint64_t bp = __ballot(f == 2);
        uint64_t need;  // lanes whose value is part of the prefix
        if (bp) {
            const int hp = 63 - __builtin_clzll(bp);
            need = ~0ull << hp;
        } else {
            need = ~0ull;
        }
        if (bz & need) {
#if defined(PSY_PROF) && PSY_PROF
            if (lane == 0) atomicAdd(&psy_prof[16], 1ull);
#endif
            if (++spins > (1u << 24)) {
                if (lane == 0) atomicOr(timeout, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += wave_sum_u64(((need >> lane) & 1ull) ? (s & kLbVal) : 0ull);
#if defined(PSY_PROF) && PSY_PROF
        if (lane == 0) atomicAdd(&psy_prof[17], 1ull);
#endif
        if (bp) break;
        top -= 64;
    }
    if (lane == 0) lb_store(&st[i], kLbInc | (excl + agg));
#if defined(PSY_PROF) && PSY_PROF
    if (lane == 0) {
        atomicAdd(&psy_prof[18], 1ull);
        if (spins) atomicAdd(&psy_prof[19], 1ull);
    }
#endif
    return excl;
}

__device__ __forceinline__ void lookback_publish(uint64_t *st, uint32_t i, uint64_t agg) {
    if (lane_id() == 0) lb_store(&st[i], (i == 0 ? kLbInc : kLbAgg) | agg);
}
__device__ __forceinline__ uint64_t lookback_resolve(uint64_t *st, uint32_t i, uint64_t agg, uint32_t *timeout) {
    const int lane = lane_id();
    if (i == 0) return 0;
    uint64_t excl = 0;
    int64_t top = (int64_t)i;  // window [top - 64, top)
    uint32_t spins = 0;
    while (true) {
        const int64_t j = top - 64 + lane;
        const uint64_t s = j >= 0 ? lb_load(&st[j]) : kLbInc;
        const uint32_t f = (uint32_t)(s >> 62);
        const uint64_t bz = __ballot(f == 0);
        const uint64_t bp = __ballot(f == 2);
        const uint64_t need = bp ? ~0ull << (63 - __builtin_clzll(bp)) : ~0ull;
        if (bz & need) {
            if (++spins > (1u << 24)) {
                if (lane == 0) atomicOr(timeout, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += wave_sum_u64(((need >> lane) & 1ull) ? (s & kLbVal) : 0ull);
        if (bp) break;
        top -= 64;
    }
    if (lane == 0) lb_store(&st[i], kLbInc | (excl + agg));
    return excl;
}

// ---------------------------------------------------------------------------------------
// Loads through the global address space (kernel-argument pointers reach the device code as
// generic pointers; flat loads would also count in lgkmcnt and wait behind LDS traffic).
template <class T>
__device__ __forceinline__ T gload(const void *p) {
    return *(const __attribute__((address_space(1))) T *)(p);
}

// Output stores are non-temporal (nt): the codec writes each output byte once and never reads
// it back, and streaming the lines past the caches measured C2 +1.9 %, C4 +1.5 %, C3 neutral
// (profiles/r04_diag/nt/); non-temporal LOADS lost (C4 -3 %: a streaming message's second read
// then misses the caches).
typedef unsigned int psy_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_nt(void *p, uint4 v) {
    psy_u32x4 t;
    t.x = v.x;
    t.y = v.y;
    t.z = v.z;
    t.w = v.w;
    __builtin_nontemporal_store(t, (__attribute__((address_space(1))) psy_u32x4 *)(p));
}

// Byte-exact accesses.
__device__ __forceinline__ uint32_t ld_u8(const uint8_t *p) { return *p; }

__device__ __forceinline__ uint32_t ld_u32_bytes(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// 16 bytes from p, any alignment; bytes at index >= valid read as 0 and are not touched.
__device__ __forceinline__ uint4 ld16_any(const uint8_t *p, int valid) {
    uint4 r;
    const uintptr_t a = (uintptr_t)p;
    if (valid >= 16 && (a & 15) == 0) {
        r = *reinterpret_cast<const uint4 *>(p);
    } else if (valid >= 16 && (a & 3) == 0) {
        const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
        r.x = q[0];
        r.y = q[1];
        r.z = q[2];
        r.w = q[3];
    } else {
        uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (i < valid) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
        r.x = w[0];
        r.y = w[1];
        r.z = w[2];
        r.w = w[3];
    }
    return r;
}

// Store the first `valid` bytes of v at p (any alignment).
__device__ __forceinline__ void st16_any(uint8_t *p, uint4 v, int valid) {
    const uintptr_t a = (uintptr_t)p;
    if (valid >= 16 && (a & 15) == 0) {
        st16_nt(p, v);
    } else if (valid >= 16 && (a & 3) == 0) {
        uint32_t *q = reinterpret_cast<uint32_t *>(p);
        q[0] = v.x;
        q[1] = v.y;
        q[2] = v.z;
        q[3] = v.w;
    } else {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (i < valid) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
}

// Team copy global -> global, arbitrary alignment and length.
template <int TEAM>
__device__ __forceinline__ void team_copy_g2g(uint8_t *dst, const uint8_t *src, uint64_t len) {
    const int tid = threadIdx.x;
    const uintptr_t d = (uintptr_t)dst, s = (uintptr_t)src;
    if (((d ^ s) & 15) == 0) {
        uint64_t head = ((16 - (d & 15)) & 15);
        if (head > len) head = len;
        if ((uint64_t)tid < head) dst[tid] = src[tid];
        const uint64_t body = (len - head) & ~(uint64_t)15;
        const uint4 *sv = reinterpret_cast<const uint4 *>(src + head);
        uint4 *dv = reinterpret_cast<uint4 *>(dst + head);
        for (uint64_t k = tid; k < body / 16; k += TEAM) dv[k] = sv[k];
        for (uint64_t k = head + body + tid; k < len; k += TEAM) dst[k] = src[k];
    } else if (((d ^ s) & 3) == 0) {
        uint64_t head = ((4 - (d & 3)) & 3);
        if (head > len) head = len;
        if ((uint64_t)tid < head) dst[tid] = src[tid];
        const uint64_t body = (len - head) & ~(uint64_t)3;
        const uint32_t *sv = reinterpret_cast<const uint32_t *>(src + head);
        uint32_t *dv = reinterpret_cast<uint32_t *>(dst + head);
        for (uint64_t k = tid; k < body / 4; k += TEAM) dv[k] = sv[k];
        for (uint64_t k = head + body + tid; k < len; k += TEAM) dst[k] = src[k];
    } else {
        for (uint64_t k = tid; k < len; k += TEAM) dst[k] = src[k];
    }
}

// Team fill of zeros, arbitrary alignment.
template <int TEAM>
__device__ __forceinline__ void team_zero(uint8_t *dst, uint64_t len) {
    const int tid = threadIdx.x;
    const uintptr_t d = (uintptr_t)dst;
    uint64_t head = ((16 - (d & 15)) & 15);
    if (head > len) head = len;
    if ((uint64_t)tid < head) dst[tid] = 0;
    const uint64_t body = (len - head) & ~(uint64_t)15;
    uint4 *dv = reinterpret_cast<uint4 *>(dst + head);
    for (uint64_t k = tid; k < body / 16; k += TEAM) dv[k] = make_uint4(0, 0, 0, 0);
    for (uint64_t k = head + body + tid; k < len; k += TEAM) dst[k] = 0;
}

// Bytes 0..3 of x that differ from the byte before them (prev-byte chain across dwords
// given by `below`, whose top byte precedes byte 0 of x), as a 4-bit mask.
__device__ __forceinline__ uint32_t neq_prev_mask4(uint32_t x, uint32_t below) {
    const uint32_t t = __builtin_amdgcn_alignbyte(x, below, 3);  // byte k = byte k-1 of {x:below}
    const uint32_t d = x ^ t;
    const uint32_t nz = (((d & 0x7f7f7f7fu) + 0x7f7f7f7fu) | d) & 0x80808080u;
    return (((nz >> 7) * 0x00204081u) >> 21) & 0xfu;  // gather bits 0,8,16,24 into bits 0..3
}

}  // namespace psy
