// Diagnostic micro-benchmark (not part of the product): cost of workgroups that exit at once
// (a list kernel launched over more entries than its device-side count).  Each workgroup
// reads the count and returns; the kernels claim the LDS and VGPRs of the real encode /
// decode list kernels so that dispatch sees the same footprint.  Prints µs per launch and
// ns per empty workgroup.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_empty.hip -o tools/ubench_empty
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CLOBBER40 \
    "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", \
    "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", \
    "v33", "v34", "v35", "v36", "v37", "v38", "v39"
#define CLOBBER78 CLOBBER40, "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", \
    "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", \
    "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77"

template <int TEAM, int LDS>
__global__ __launch_bounds__(TEAM) void empty_kernel(const uint32_t *count, uint32_t *sink) {
    __shared__ uint8_t smem[LDS];
    if (blockIdx.x < *count) {
        asm volatile("" ::: CLOBBER78);
        smem[threadIdx.x] = (uint8_t)threadIdx.x;
        __syncthreads();
        sink[blockIdx.x] = smem[(threadIdx.x + 1) % TEAM];
    }
}

template <int TEAM, int LDS>
static void run(const char *name, uint32_t *cnt, uint32_t *sink) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (uint32_t n : {1u << 14, 1u << 16, 1u << 18, 1u << 20, 1u << 22}) {
        empty_kernel<TEAM, LDS><<<n, TEAM>>>(cnt, sink);  // warm
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r) empty_kernel<TEAM, LDS><<<n, TEAM>>>(cnt, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1000.0 / 5;
        printf("%-26s grid %8u: %9.1f us/launch  %6.3f ns/workgroup\n", name, n, us, us * 1000.0 / n);
    }
}

int main() {
    uint32_t *cnt, *sink;
    hipMalloc(&cnt, 4);
    hipMemset(cnt, 0, 4);
    hipMalloc(&sink, 4u << 22);
    run<512, 50816>("encode medium (512, 50 KB)", cnt, sink);
    run<64, 6304>("encode small (64, 6.3 KB)", cnt, sink);
    run<64, 6200>("decode (64, 6.2 KB)", cnt, sink);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
