// tdt_slots.h — slot offsets for the slotted (look-back-free) batch entry points.
//
// One 1024-thread workgroup turns per-message sizes into an exclusive prefix sum (n + 1
// offsets, the last one the total): thread t sums a contiguous chunk, the 1024 chunk sums
// are scanned across the workgroup (u64 wave scans + one LDS exchange), and every thread
// rewrites its chunk.  Sizes are either encode bounds (psyne's encode never exceeds
// max(n + 4, 28 + 4·ws + 2n)) or decoded sizes written into the offset array beforehand.
#pragma once
#include "tdt_device.h"

namespace psy {

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

// MODE 0: sizes = tdt_encode_bound(in_off[i+1] - in_off[i], ws), read from in_off;
// MODE 1: sizes already in off[0..n).  Writes off[0..n] = exclusive prefix (off[n] = total).
template <int MODE>
__global__ __launch_bounds__(1024) void tdt_slots_kernel(const uint64_t *in_off, uint64_t *off, uint32_t n,
                                                         uint32_t ws) {
    __shared__ uint64_t wsum[16];
    const uint32_t t = threadIdx.x;
    const uint32_t chunk = (n + 1023) / 1024;
    const uint64_t b0 = (uint64_t)t * chunk;
    const uint64_t b1 = b0 + chunk < n ? b0 + chunk : n;
    auto size = [&](uint64_t i) -> uint64_t {
        if constexpr (MODE == 0) {
            const uint64_t m = in_off[i + 1] - in_off[i];
            const uint64_t tdt = 28 + 4ull * ws + 2 * m;
            return tdt > m + 4 ? tdt : m + 4;
        } else {
            return off[i];
        }
    };
    uint64_t s = 0;
    for (uint64_t i = b0; i < b1; ++i) s += size(i);
    const uint64_t inc = wave_incl_scan_u64(s);
    const int w = (int)(t >> 6), lane = lane_id();
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (int k = 0; k < 16; ++k) {
        if (k < w) pre += wsum[k];
        tot += wsum[k];
    }
    uint64_t run = pre + inc - s;  // exclusive prefix of this chunk
    for (uint64_t i = b0; i < b1; ++i) {
        const uint64_t v = size(i);
        off[i] = run;
        run += v;
    }
    if (t == 0) off[n] = tot;
}

}  // namespace psy
