// Diagnostic (not shipped): does v_mad_u16 on gfx950 zero the upper 16 bits of its VGPR
// destination (op_sel dst = 0), with src0 taken from either half (op_sel:[0/1,...])?  The
// histogram pass could then form each byte's LDS bin address in one instruction.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void k(const uint32_t *in, uint32_t *out) {
    const uint32_t x = in[threadIdx.x];
    uint32_t lo = 0xdead0000u | threadIdx.x, hi = 0xbeef0000u | threadIdx.x;
    const uint32_t m = 64, c = 0xffc0u + (threadIdx.x & 15) * 4;
    asm volatile("v_mad_u16 %0, %1, %2, %3" : "+v"(lo) : "v"(x), "v"(m), "v"(c));
    asm volatile("v_mad_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "+v"(hi) : "v"(x), "v"(m), "v"(c));
    out[2 * threadIdx.x] = lo;
    out[2 * threadIdx.x + 1] = hi;
}

int main() {
    uint32_t h[64], o[128];
    for (int i = 0; i < 64; ++i) h[i] = (uint32_t)(i * 2654435761u) & 0x00ff00ffu;
    uint32_t *d, *r;
    hipMalloc(&d, sizeof h);
    hipMalloc(&r, sizeof o);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    k<<<1, 64>>>(d, r);
    hipMemcpy(o, r, sizeof o, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 64; ++i) {
        const uint32_t c = 0xffc0u + (i & 15) * 4;
        const uint32_t wlo = ((h[i] & 0xffffu) * 64u + c) & 0xffffu, whi = ((h[i] >> 16) * 64u + c) & 0xffffu;
        if (o[2 * i] != wlo || o[2 * i + 1] != whi) {
            if (bad < 4) printf("lane %d: got %08x %08x want %08x %08x\n", i, o[2 * i], o[2 * i + 1], wlo, whi);
            ++bad;
        }
    }
    printf("v_mad_u16 zero-high + op_sel src0-hi: %s (%d bad)\n", bad ? "NO" : "yes", bad);
    return 0;
}
