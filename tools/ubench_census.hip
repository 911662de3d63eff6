// Diagnostic micro-benchmark (not part of the product): how many workgroups of one wave (and of
// 4 waves) are resident at once on the whole chip.  Every workgroup increments a live counter,
// records the maximum, holds ~200 us, then decrements; the peak / CUs is the residency per CU.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_census.hip -o tools/ubench_census
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int THREADS, int LDS>
__global__ __launch_bounds__(THREADS) void census(uint32_t *cnt) {
    __shared__ uint32_t pad[LDS / 4];
    if (threadIdx.x == 0) {
        const uint32_t now = atomicAdd(&cnt[0], 1u) + 1u;
        atomicMax(&cnt[1], now);
        pad[0] = now;
        const uint64_t t0 = wall_clock64();
        while (wall_clock64() - t0 < 20000) __builtin_amdgcn_s_sleep(10);  // 200 us at 100 MHz
        atomicSub(&cnt[0], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 1 && pad[0] == 0xffffffffu) cnt[2] = 1;
}

template <int THREADS, int LDS>
static void run(uint32_t *d, int cus) {
    hipMemset(d, 0, 16);
    const int blocks = cus * 64;
    census<THREADS, LDS><<<blocks, THREADS>>>(d);
    uint32_t h[4];
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("threads %4d  LDS %6d B: peak resident workgroups %6u = %.2f per CU (%.2f waves per CU)\n", THREADS, LDS,
           h[1], (double)h[1] / cus, (double)h[1] / cus * THREADS / 64);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    uint32_t *d;
    hipMalloc(&d, 16);
    run<64, 16>(d, cus);
    run<64, 4416>(d, cus);
    run<64, 6208>(d, cus);
    run<128, 16>(d, cus);
    run<256, 16>(d, cus);
    run<256, 17664>(d, cus);
    hipFree(d);
    return 0;
}
