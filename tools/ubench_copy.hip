// Diagnostic micro-benchmark (not shipped): the achievable HBM rate of a hand-written
// device-to-device copy on gfx950 — dwordx4 loads and stores, 1..4 per lane per iteration,
// grid-stride over 4 GiB, several grid sizes — beside hipMemcpyDtoD.  Read + write bytes / time.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy4(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n16) v[u] = NT ? __builtin_nontemporal_load(src + i + u * 256) : src[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n16) {
                if (NT) __builtin_nontemporal_store(v[u], dst + i + u * 256);
                else dst[i + u * 256] = v[u];
            }
    }
}

int main() {
    const uint64_t bytes = 4ull << 30, n16 = bytes / 16;
    u32x4 *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto report = [&](const char *name, float ms, int reps) {
        std::printf("{\"copy\": \"%s\", \"TBps_rw\": %.3f}\n", name, 2.0 * bytes * reps / (ms * 1e-3) / 1e12);
    };
    const int reps = 5;
    auto run = [&](auto kern, const char *what, int g) {
        kern<<<g, 256>>>(a, b, n16);
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) kern<<<g, 256>>>(a, b, n16);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        char name[80];
        std::snprintf(name, sizeof name, "%s, grid %d", what, g);
        report(name, ms, reps);
    };
    for (int g : {1024, 2048, 4096, 8192, 16384}) {
        run(copy4<4, true>, "dwordx4 x4 nt", g);
        run(copy4<4, false>, "dwordx4 x4", g);
        run(copy4<1, true>, "dwordx4 x1 nt", g);
        run(copy4<1, false>, "dwordx4 x1", g);
    }
    hipMemcpy(b, a, bytes, hipMemcpyDeviceToDevice);
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    report("hipMemcpyAsync DtoD", ms, reps);
    return 0;
}
