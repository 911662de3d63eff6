// Diagnostic (not product): raw-buffer range-check semantics on gfx950 — is the SGPR offset
// (soffset) or the instruction offset part of the checked offset? — and buffer_store nt.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__global__ void k(const uint32_t *src, uint32_t *out, uint32_t nrec, int mode) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)src, (short)0, (int)nrec, 0x00020000);
    const int lane = threadIdx.x;
    u32x4_t v;
    if (mode == 0) v = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, 0, 0);         // voffset only
    else if (mode == 1) v = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, 4096, 0); // + soffset 4096
    else if (mode == 2) v = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16 + 4096, 0, 0); // voffset 4096+
    else v = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, 2048, 0);               // soffset 2048
    out[lane] = v.x;
}
__global__ void ks(uint32_t *dst, uint32_t nrec) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)dst, (short)0, (int)nrec, 0x00020000);
    u32x4_t v = {threadIdx.x + 1u, 7u, 8u, 9u};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, threadIdx.x * 16, 1024, 2);
}
int main() {
    uint32_t *src, *out;
    (void)hipMalloc(&src, 1 << 16);
    (void)hipMalloc(&out, 4096);
    uint32_t h[16384];
    for (int i = 0; i < 16384; ++i) h[i] = i + 1;
    (void)hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
    const char *nm[] = {"voffset only (nrec 4096)", "voffset + soffset 4096", "voffset + 4096 in vgpr", "voffset + soffset 2048"};
    for (int m = 0; m < 4; ++m) {
        k<<<1, 64>>>(src, out, 4096, m);
        uint32_t o[64];
        (void)hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
        int nz = 0;
        for (int i = 0; i < 64; ++i) nz += o[i] != 0;
        printf("%-28s lanes with data: %d (lane0 %u lane63 %u)\n", nm[m], nz, o[0], o[63]);
    }
    (void)hipMemset(src, 0, 1 << 16);
    ks<<<1, 64>>>(src, 2048);
    (void)hipMemcpy(h, src, 16384, hipMemcpyDeviceToHost);
    int w = 0;
    for (int i = 0; i < 4096; ++i) w += h[i] != 0;
    printf("store soffset 1024, nrec 2048: dwords written %d (expect 256 if soffset excluded from the check, 64*4=256 either way below 2048?) first %u at %d\n", w, h[256], 256);
    return 0;
}
