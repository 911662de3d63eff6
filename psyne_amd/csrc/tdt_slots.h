// tdt_slots.h — slot offsets for the slotted (look-back-free) batch entry points.
//
// Encode slots: psyne's encode never exceeds max(n + 4, 28 + 4·ws + 2n), and for n >= 0 the
// second term always wins, so the exclusive prefix of the bounds has a closed form:
// off[i] = (28 + 4·ws)·i + 2·(in_off[i] - in_off[0]).  One thread per offset, no scan.
//
// Decode slots: the decoded sizes (written into off[0..n) by tdt_decode_sizes_kernel) are
// turned into an exclusive prefix (off[n] = total) in place by two launches over
// kSlotChunk-element chunks: (1) one workgroup per chunk writes the chunk's sum to a small
// workspace; (2) one workgroup per chunk adds the sums of the chunks before it (at most a few
// dozen u64s) to a workgroup scan of its own chunk.  Each thread owns 8 consecutive sizes
// (64 bytes, four 16-byte loads when `off` is 16-byte aligned).  The previous single-workgroup
// version walked 256 strided elements per thread and took ~0.45 ms for 262,144 messages.
#pragma once
#include "tdt_device.h"

namespace psy {

constexpr uint32_t kSlotThreads = 1024;
constexpr uint32_t kSlotPer = 8;
constexpr uint32_t kSlotChunk = kSlotThreads * kSlotPer;

// u64 inclusive scan over the wave (shuffle-up on both halves).
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, o);
        const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), o);
        if (lane >= o) v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

// off[0..n] = exclusive prefix of the encode bounds of the messages in in_off.
__global__ __launch_bounds__(256) void tdt_encode_slots_kernel(const uint64_t *in_off, uint64_t *off, uint32_t n,
                                                               uint32_t ws) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i > n) return;
    off[i] = (28ull + 4ull * ws) * i + 2ull * (in_off[i] - in_off[0]);
}

__device__ __forceinline__ bool slot_vec_ok(const uint64_t *off, uint64_t b, uint32_t n) {
    return b + kSlotPer <= n && (reinterpret_cast<uintptr_t>(off) & 15) == 0;
}

// Loads the thread's (up to) 8 sizes of chunk `blk`; elements at or past n read as 0.
__device__ __forceinline__ void slot_load8(const uint64_t *off, uint32_t n, uint32_t blk, uint64_t (&v)[kSlotPer]) {
    const uint64_t b = (uint64_t)blk * kSlotChunk + (uint64_t)threadIdx.x * kSlotPer;
    if (slot_vec_ok(off, b, n)) {
        const uint4 *p = reinterpret_cast<const uint4 *>(off + b);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 q = p[k];
            v[2 * k] = ((uint64_t)q.y << 32) | q.x;
            v[2 * k + 1] = ((uint64_t)q.w << 32) | q.z;
        }
    } else {
#pragma unroll
        for (int k = 0; k < (int)kSlotPer; ++k) v[k] = b + k < n ? off[b + k] : 0;
    }
}

// Pass 1: sums[blk] = Σ off[blk·C .. min(n, (blk+1)·C)).
__global__ __launch_bounds__(kSlotThreads) void tdt_slot_sums_kernel(const uint64_t *off, uint64_t *sums, uint32_t n) {
    __shared__ uint64_t wsum[kSlotThreads / 64];
    uint64_t v[kSlotPer];
    slot_load8(off, n, blockIdx.x, v);
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < (int)kSlotPer; ++k) s += v[k];
    const uint64_t inc = wave_incl_scan_u64(s);
    if (lane_id() == 63) wsum[threadIdx.x >> 6] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t tot = 0;
        for (int k = 0; k < (int)(kSlotThreads / 64); ++k) tot += wsum[k];
        sums[blockIdx.x] = tot;
    }
}

// Pass 2: in-place exclusive prefix of chunk blk, seeded by the sums of chunks 0..blk-1;
// the last chunk also writes off[n] = total.
__global__ __launch_bounds__(kSlotThreads) void tdt_slot_scan_kernel(uint64_t *off, const uint64_t *sums, uint32_t n) {
    __shared__ uint64_t wsum[kSlotThreads / 64];
    __shared__ uint64_t carry_s;
    const uint32_t blk = blockIdx.x;
    if (threadIdx.x < 64) {  // wave 0: carry = Σ sums[0..blk)
        uint64_t c = 0;
        for (uint32_t j = threadIdx.x; j < blk; j += 64) c += sums[j];
        c = wave_incl_scan_u64(c);
        if (threadIdx.x == 63) carry_s = c;
    }
    uint64_t v[kSlotPer];
    slot_load8(off, n, blk, v);
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < (int)kSlotPer; ++k) s += v[k];
    const uint64_t inc = wave_incl_scan_u64(s);
    const int w = (int)(threadIdx.x >> 6);
    if (lane_id() == 63) wsum[w] = inc;
    __syncthreads();
    uint64_t pre = carry_s, tot = carry_s;
    for (int k = 0; k < (int)(kSlotThreads / 64); ++k) {
        if (k < w) pre += wsum[k];
        tot += wsum[k];
    }
    uint64_t run = pre + inc - s;
    const uint64_t b = (uint64_t)blk * kSlotChunk + (uint64_t)threadIdx.x * kSlotPer;
    if (slot_vec_ok(off, b, n)) {
        uint4 *p = reinterpret_cast<uint4 *>(off + b);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t a0 = run;
            const uint64_t a1 = run + v[2 * k];
            run = a1 + v[2 * k + 1];
            p[k] = make_uint4((uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1, (uint32_t)(a1 >> 32));
        }
    } else {
#pragma unroll
        for (int k = 0; k < (int)kSlotPer; ++k) {
            if (b + k < n) off[b + k] = run;
            run += v[k];
        }
    }
    if (blk == gridDim.x - 1 && threadIdx.x == 0) off[n] = tot;
}

}  // namespace psy
