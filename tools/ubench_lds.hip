// Diagnostic micro-benchmark (not part of the product): LDS instruction cost on gfx950 by
// access pattern, as the encode kernel's histogram / sweep / flush issue them.  Each wave runs
// ITER iterations of 16 LDS instructions; cost is printed per wave-instruction in CU cycles (at
// a nominal 2.4 GHz), with WPC waves per CU.  Also checks what an ds_add_u32 beyond the
// workgroup's LDS allocation does (the "oor" rows count what landed in the allocation).
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lds.hip -o tools/ubench_lds
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int ITER = 512;
constexpr int LDSW = 8192;  // dwords per workgroup (32 KiB)

// MODE: 0 ds_add conflict-free (lane-consecutive dwords), 1 ds_add 4 lanes per address
// (lane / 4), 2 ds_add random bins over 1 KiB x 4 copies (the H layout, nonzero values),
// 3 ds_add with 3/4 of the lanes exec-masked off, 4 ds_write_b16 lane-consecutive,
// 5 ds_write_b16 random within 8 KiB, 6 ds_read_u16 consecutive, 7 ds_read_b32 consecutive,
// 8 ds_add to an address past the allocation (all lanes), 9 ds_add 70 % of lanes past the
// allocation, 30 % conflict-free, 10 ds_write_b8 consecutive, 11 ds_read2st64_b32
template <int MODE>
__global__ __launch_bounds__(256) void kern(uint32_t *out, uint32_t seed, uint32_t *landed) {
    __shared__ uint32_t h[LDSW];
    for (int i = threadIdx.x; i < LDSW; i += 256) h[i] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = (seed ^ (threadIdx.x * 0x9E3779B9u)) * 0x85EBCA6Bu;
    x ^= x >> 13;
    uint32_t addr;
    const uint32_t base = w * 2048 * 4;  // each wave its own 8 KiB
    if constexpr (MODE == 0 || MODE == 3 || MODE == 4 || MODE == 6 || MODE == 7 || MODE == 10 || MODE == 11) addr = base + lane * 4;
    else if constexpr (MODE == 1) addr = base + (lane / 4) * 4;
    else if constexpr (MODE == 2) addr = base + (((x & 255) | 1) * 4 + (lane & 3)) * 4 % 4096;
    else if constexpr (MODE == 5) addr = base + ((x % 4096) * 2);
    else if constexpr (MODE == 8) addr = 0x10000u + lane * 4;
    else addr = (x % 10 < 7) ? 0x10000u + lane * 4 : base + lane * 4;
    uint32_t acc = 0;
    if constexpr (MODE == 3) {
        if ((lane & 3) == 0) {
            for (int i = 0; i < ITER; ++i)
                asm volatile("ds_add_u32 %0, %1\n ds_add_u32 %0, %1 offset:256\n ds_add_u32 %0, %1 offset:512\n ds_add_u32 %0, %1 offset:768\n"
                             "ds_add_u32 %0, %1 offset:1024\n ds_add_u32 %0, %1 offset:1280\n ds_add_u32 %0, %1 offset:1536\n ds_add_u32 %0, %1 offset:1792\n"
                             "ds_add_u32 %0, %1 offset:2048\n ds_add_u32 %0, %1 offset:2304\n ds_add_u32 %0, %1 offset:2560\n ds_add_u32 %0, %1 offset:2816\n"
                             "ds_add_u32 %0, %1 offset:3072\n ds_add_u32 %0, %1 offset:3328\n ds_add_u32 %0, %1 offset:3584\n ds_add_u32 %0, %1 offset:3840\n"
                             "s_waitcnt lgkmcnt(8)" ::"v"(addr), "v"(1u));
        }
    } else if constexpr (MODE == 0 || MODE == 1 || MODE == 2 || MODE == 8 || MODE == 9) {
        for (int i = 0; i < ITER; ++i)
            asm volatile("ds_add_u32 %0, %1\n ds_add_u32 %0, %1 offset:256\n ds_add_u32 %0, %1 offset:512\n ds_add_u32 %0, %1 offset:768\n"
                         "ds_add_u32 %0, %1 offset:1024\n ds_add_u32 %0, %1 offset:1280\n ds_add_u32 %0, %1 offset:1536\n ds_add_u32 %0, %1 offset:1792\n"
                         "ds_add_u32 %0, %1 offset:2048\n ds_add_u32 %0, %1 offset:2304\n ds_add_u32 %0, %1 offset:2560\n ds_add_u32 %0, %1 offset:2816\n"
                         "ds_add_u32 %0, %1 offset:3072\n ds_add_u32 %0, %1 offset:3328\n ds_add_u32 %0, %1 offset:3584\n ds_add_u32 %0, %1 offset:3840\n"
                         "s_waitcnt lgkmcnt(8)" ::"v"(addr), "v"(1u));
    } else if constexpr (MODE == 4 || MODE == 5) {
        for (int i = 0; i < ITER; ++i)
            asm volatile("ds_write_b16 %0, %1\n ds_write_b16 %0, %1 offset:256\n ds_write_b16 %0, %1 offset:512\n ds_write_b16 %0, %1 offset:768\n"
                         "ds_write_b16 %0, %1 offset:1024\n ds_write_b16 %0, %1 offset:1280\n ds_write_b16 %0, %1 offset:1536\n ds_write_b16 %0, %1 offset:1792\n"
                         "ds_write_b16 %0, %1 offset:2048\n ds_write_b16 %0, %1 offset:2304\n ds_write_b16 %0, %1 offset:2560\n ds_write_b16 %0, %1 offset:2816\n"
                         "ds_write_b16 %0, %1 offset:3072\n ds_write_b16 %0, %1 offset:3328\n ds_write_b16 %0, %1 offset:3584\n ds_write_b16 %0, %1 offset:3840\n"
                         "s_waitcnt lgkmcnt(8)" ::"v"(addr), "v"(x));
    } else if constexpr (MODE == 10) {
        for (int i = 0; i < ITER; ++i)
            asm volatile("ds_write_b8 %0, %1\n ds_write_b8 %0, %1 offset:256\n ds_write_b8 %0, %1 offset:512\n ds_write_b8 %0, %1 offset:768\n"
                         "ds_write_b8 %0, %1 offset:1024\n ds_write_b8 %0, %1 offset:1280\n ds_write_b8 %0, %1 offset:1536\n ds_write_b8 %0, %1 offset:1792\n"
                         "ds_write_b8 %0, %1 offset:2048\n ds_write_b8 %0, %1 offset:2304\n ds_write_b8 %0, %1 offset:2560\n ds_write_b8 %0, %1 offset:2816\n"
                         "ds_write_b8 %0, %1 offset:3072\n ds_write_b8 %0, %1 offset:3328\n ds_write_b8 %0, %1 offset:3584\n ds_write_b8 %0, %1 offset:3840\n"
                         "s_waitcnt lgkmcnt(8)" ::"v"(addr), "v"(x));
    } else if constexpr (MODE == 6 || MODE == 7 || MODE == 11) {
        uint32_t r0, r1, r2, r3;
        for (int i = 0; i < ITER; ++i) {
            if constexpr (MODE == 6)
                asm volatile("ds_read_u16 %0, %4\n ds_read_u16 %1, %4 offset:256\n ds_read_u16 %2, %4 offset:512\n ds_read_u16 %3, %4 offset:768\n"
                             "ds_read_u16 %0, %4 offset:1024\n ds_read_u16 %1, %4 offset:1280\n ds_read_u16 %2, %4 offset:1536\n ds_read_u16 %3, %4 offset:1792\n"
                             "ds_read_u16 %0, %4 offset:2048\n ds_read_u16 %1, %4 offset:2304\n ds_read_u16 %2, %4 offset:2560\n ds_read_u16 %3, %4 offset:2816\n"
                             "ds_read_u16 %0, %4 offset:3072\n ds_read_u16 %1, %4 offset:3328\n ds_read_u16 %2, %4 offset:3584\n ds_read_u16 %3, %4 offset:3840\n"
                             "s_waitcnt lgkmcnt(0)" : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3) : "v"(addr));
            else if constexpr (MODE == 7)
                asm volatile("ds_read_b32 %0, %4\n ds_read_b32 %1, %4 offset:256\n ds_read_b32 %2, %4 offset:512\n ds_read_b32 %3, %4 offset:768\n"
                             "ds_read_b32 %0, %4 offset:1024\n ds_read_b32 %1, %4 offset:1280\n ds_read_b32 %2, %4 offset:1536\n ds_read_b32 %3, %4 offset:1792\n"
                             "ds_read_b32 %0, %4 offset:2048\n ds_read_b32 %1, %4 offset:2304\n ds_read_b32 %2, %4 offset:2560\n ds_read_b32 %3, %4 offset:2816\n"
                             "ds_read_b32 %0, %4 offset:3072\n ds_read_b32 %1, %4 offset:3328\n ds_read_b32 %2, %4 offset:3584\n ds_read_b32 %3, %4 offset:3840\n"
                             "s_waitcnt lgkmcnt(0)" : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3) : "v"(addr));
            else {
                uint64_t q0, q1, q2, q3;
                asm volatile("ds_read2st64_b32 %0, %4 offset1:1\n ds_read2st64_b32 %1, %4 offset0:2 offset1:3\n ds_read2st64_b32 %2, %4 offset0:4 offset1:5\n ds_read2st64_b32 %3, %4 offset0:6 offset1:7\n"
                             "ds_read2st64_b32 %0, %4 offset0:8 offset1:9\n ds_read2st64_b32 %1, %4 offset0:10 offset1:11\n ds_read2st64_b32 %2, %4 offset0:12 offset1:13\n ds_read2st64_b32 %3, %4 offset0:14 offset1:15\n"
                             "ds_read2st64_b32 %0, %4 offset0:16 offset1:17\n ds_read2st64_b32 %1, %4 offset0:18 offset1:19\n ds_read2st64_b32 %2, %4 offset0:20 offset1:21\n ds_read2st64_b32 %3, %4 offset0:22 offset1:23\n"
                             "ds_read2st64_b32 %0, %4 offset0:24 offset1:25\n ds_read2st64_b32 %1, %4 offset0:26 offset1:27\n ds_read2st64_b32 %2, %4 offset0:28 offset1:29\n ds_read2st64_b32 %3, %4 offset0:30 offset1:31\n"
                             "s_waitcnt lgkmcnt(0)" : "=v"(q0), "=v"(q1), "=v"(q2), "=v"(q3) : "v"(addr & 0x3ff));
                r0 = (uint32_t)q0; r1 = (uint32_t)q1; r2 = (uint32_t)q2; r3 = (uint32_t)q3;
            }
            acc += r0 ^ r1 ^ r2 ^ r3;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)");
    __syncthreads();
    uint32_t s = 0;
    for (int i = threadIdx.x; i < LDSW; i += 256) s += h[i];
    if (MODE == 8 || MODE == 9) atomicAdd(landed, s);
    out[blockIdx.x * 256 + threadIdx.x] = s + acc;
}

static const char *names[] = {"ds_add conflict-free", "ds_add 4 lanes/address", "ds_add random bins x4 copies",
                              "ds_add 1/4 lanes active", "ds_write_b16 consecutive", "ds_write_b16 random",
                              "ds_read_u16 consecutive", "ds_read_b32 consecutive", "ds_add past allocation (all)",
                              "ds_add 70% past allocation", "ds_write_b8 consecutive", "ds_read2st64_b32"};

template <int MODE>
static void run(uint32_t *d, uint32_t *landed, int cus, int wgpc) {
    const int blocks = cus * wgpc;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<MODE><<<blocks, 256>>>(d, 1, landed);
    (void)hipMemset(landed, 0, 4);
    (void)hipEventRecord(e0);
    kern<MODE><<<blocks, 256>>>(d, 2, landed);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint32_t l = 0;
    (void)hipMemcpy(&l, landed, 4, hipMemcpyDeviceToHost);
    const double winst = (double)blocks * 4 * ITER * 16;
    const double cyc = ms * 1e-3 * 2.4e9;
    printf("%-32s waves/CU %2d %8.3f ms  %6.2f CU-cycles per wave-instr", names[MODE], 4 * wgpc, ms, cyc * cus / winst);
    if (MODE == 8 || MODE == 9) printf("   landed in allocation: %u of %.0f lane-adds", l, (double)blocks * 256 * ITER * 16);
    printf("\n");
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    uint32_t *d, *landed;
    (void)hipMalloc(&d, (size_t)cus * 8 * 256 * 4);
    (void)hipMalloc(&landed, 4);
    for (int wg : {2, 4}) {
        run<0>(d, landed, cus, wg);
        run<1>(d, landed, cus, wg);
        run<2>(d, landed, cus, wg);
        run<3>(d, landed, cus, wg);
        run<4>(d, landed, cus, wg);
        run<5>(d, landed, cus, wg);
        run<6>(d, landed, cus, wg);
        run<7>(d, landed, cus, wg);
        run<10>(d, landed, cus, wg);
        run<11>(d, landed, cus, wg);
    }
    run<8>(d, landed, cus, 4);
    run<9>(d, landed, cus, 4);
    (void)hipFree(d);
    (void)hipFree(landed);
    return 0;
}
