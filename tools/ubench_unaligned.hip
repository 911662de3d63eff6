// Diagnostic micro-benchmark (not shipped): global_store_dwordx4 at 16-byte-aligned vs
// 2-byte-aligned destinations (the encode flush writes pair runs at even, not 16-aligned,
// offsets), checking the bytes and timing each over 1 GiB.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void store16(uint8_t *dst, uint64_t n16) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n16) return;
    const uint32_t v = (uint32_t)i * 2654435761u;
    *reinterpret_cast<uint4 *>(dst + 16 * i) = make_uint4(v, v ^ 1u, v ^ 2u, v ^ 3u);
}

int main() {
    const uint64_t n16 = (1ull << 30) / 16;
    uint8_t *buf;
    if (hipMalloc(&buf, (1ull << 30) + 64) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int offs[3] = {0, 2, 6};
    for (int k = 0; k < 3; ++k) {
        uint8_t *d = buf + offs[k];
        store16<<<n16 / 256, 256>>>(d, n16);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) store16<<<n16 / 256, 256>>>(d, n16);
        hipEventRecord(e1);
        if (hipEventSynchronize(e1) != hipSuccess) return 2;
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<uint8_t> h(64 * 16);
        hipMemcpy(h.data(), d + 16 * 12345, h.size(), hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 64; ++i) {
            const uint32_t v = (uint32_t)(12345 + i) * 2654435761u;
            const uint32_t w[4] = {v, v ^ 1u, v ^ 2u, v ^ 3u};
            for (int b = 0; b < 16; ++b)
                if (h[16 * i + b] != (uint8_t)(w[b / 4] >> (8 * (b % 4)))) ++bad;
        }
        printf("{\"offset\": %d, \"GBps\": %.1f, \"bad_bytes\": %d}\n", offs[k], 5.0 * (1ull << 30) / (ms * 1e-3) / 1e9,
               bad);
    }
    hipFree(buf);
    return 0;
}
