// Diagnostic micro-benchmark (not part of the product): issue cost on gfx950 of instruction
// forms the round-5 encode rework considers (SDWA byte selects, carry chains, cndmask on an SGPR
// mask, same-wave pairs of simple ops) and of LDS atomics by conflict degree.  Each wave runs
// ITER iterations of 8 independent chains (inline asm: the exact opcode is issued) unless the
// row says "dep"; the grid fills every SIMD with WPS waves.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu3.hip -o tools/ubench_valu3
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int ITER = 2048;

#define C8(ASM)                                                                              \
    for (int i = 0; i < ITER; ++i) {                                                         \
        asm volatile(ASM : "+v"(a0) : "v"(b)); asm volatile(ASM : "+v"(a1) : "v"(b));        \
        asm volatile(ASM : "+v"(a2) : "v"(b)); asm volatile(ASM : "+v"(a3) : "v"(b));        \
        asm volatile(ASM : "+v"(a4) : "v"(b)); asm volatile(ASM : "+v"(a5) : "v"(b));        \
        asm volatile(ASM : "+v"(a6) : "v"(b)); asm volatile(ASM : "+v"(a7) : "v"(b));        \
    }
// 8 instructions per iteration on ONE dependent chain
#define D8(ASM)                                                                              \
    for (int i = 0; i < ITER; ++i) {                                                         \
        asm volatile(ASM : "+v"(a0) : "v"(b)); asm volatile(ASM : "+v"(a0) : "v"(b));        \
        asm volatile(ASM : "+v"(a0) : "v"(b)); asm volatile(ASM : "+v"(a0) : "v"(b));        \
        asm volatile(ASM : "+v"(a0) : "v"(b)); asm volatile(ASM : "+v"(a0) : "v"(b));        \
        asm volatile(ASM : "+v"(a0) : "v"(b)); asm volatile(ASM : "+v"(a0) : "v"(b));        \
    }
// 4 chains, 2 instructions each (8 per iteration), given as one asm string of two lines
#define P4(ASM)                                                                              \
    for (int i = 0; i < ITER; ++i) {                                                         \
        asm volatile(ASM : "+v"(a0), "+v"(a1) : "v"(b)); asm volatile(ASM : "+v"(a2), "+v"(a3) : "v"(b)); \
        asm volatile(ASM : "+v"(a4), "+v"(a5) : "v"(b)); asm volatile(ASM : "+v"(a6), "+v"(a7) : "v"(b)); \
    }

#define NOPS 30
static const char *names[NOPS] = {
    "v_add_u32 (indep)",                 // 0
    "v_add_u32 (dep chain)",             // 1
    "v_perm_b32 (indep)",                // 2
    "add,add pairs + perm,perm",         // 3
    "v_mov_b32_sdwa dst BYTE_1 preserve",// 4
    "v_lshlrev_b32_sdwa src1 BYTE_1",    // 5
    "v_add_u32_sdwa src1 BYTE_2",        // 6
    "v_mul_u32_u24_sdwa src0 BYTE_1",    // 7
    "v_and_b32_sdwa src0 BYTE_3",        // 8
    "v_cndmask_b32 sgpr mask",           // 9
    "v_add_co_u32 vcc",                  // 10
    "v_addc_co_u32 (vcc in, sgpr out)",  // 11
    "v_bfi_b32",                         // 12
    "v_lshlrev_b32 vgpr shift",          // 13
    "v_lshrrev_b32 imm shift",           // 14
    "v_cmp_ne_u32 -> sgpr",              // 15
    "v_cmp_ne_u32_sdwa BYTE_1 -> sgpr",  // 16
    "v_not_b32",                         // 17
    "v_pk_sub_u16",                      // 18
    "v_sub_u32 (indep)",                 // 19
    "v_and_b32 imm",                     // 20
    "v_min_u32",                         // 21
    "v_lshl_add_u32",                    // 22
    "v_mad_u32_u24",                     // 23
    "v_bfe_u32",                         // 24
    "v_or_b32_sdwa dst WORD_1 preserve", // 25
    "and,perm pairs (dep-free)",         // 26
    "v_xad_u32",                         // 27
    "v_add_u32 dep + xor dep (2 chains)",// 28
    "v_cndmask_b32 vcc (vcc const)",     // 29
};

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7, b = seed * 3u + threadIdx.x;
    if constexpr (OP == 0) C8("v_add_u32 %0, %0, %1")
    if constexpr (OP == 1) D8("v_add_u32 %0, %0, %1")
    if constexpr (OP == 2) C8("v_perm_b32 %0, %0, %1, %1")
    if constexpr (OP == 3) P4("v_add_u32 %0, %0, %2\n v_add_u32 %1, %1, %2\n v_perm_b32 %0, %0, %2, %2\n v_perm_b32 %1, %1, %2, %2")
    if constexpr (OP == 4) C8("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2")
    if constexpr (OP == 5) C8("v_lshlrev_b32_sdwa %0, 6, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1")
    if constexpr (OP == 6) C8("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2")
    if constexpr (OP == 7) C8("v_mul_u32_u24_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD")
    if constexpr (OP == 8) C8("v_and_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD")
    if constexpr (OP == 9) C8("v_cndmask_b32_e64 %0, %0, %1, s[20:21]")
    if constexpr (OP == 10) C8("v_add_co_u32 %0, vcc, %0, %1")
    if constexpr (OP == 11) C8("v_addc_co_u32 %0, s[22:23], %0, %1, vcc")
    if constexpr (OP == 12) C8("v_bfi_b32 %0, %1, %0, %1")
    if constexpr (OP == 13) C8("v_lshlrev_b32 %0, %1, %0")
    if constexpr (OP == 14) C8("v_lshrrev_b32 %0, 3, %0")
    if constexpr (OP == 15) {
        for (int i = 0; i < ITER; ++i) {
            asm volatile("v_cmp_ne_u32 s[24:25], %0, %1\n v_cmp_ne_u32 s[26:27], %0, %1\n v_cmp_ne_u32 s[28:29], %0, %1\n v_cmp_ne_u32 s[30:31], %0, %1\n"
                         "v_cmp_ne_u32 s[32:33], %0, %1\n v_cmp_ne_u32 s[34:35], %0, %1\n v_cmp_ne_u32 s[36:37], %0, %1\n v_cmp_ne_u32 s[38:39], %0, %1"
                         :: "v"(a0), "v"(b) : "s24","s25","s26","s27","s28","s29","s30","s31","s32","s33","s34","s35","s36","s37","s38","s39");
        }
    }
    if constexpr (OP == 16) {
        for (int i = 0; i < ITER; ++i) {
            asm volatile("v_cmp_ne_u32_sdwa s[24:25], %0, %1 src0_sel:BYTE_1 src1_sel:DWORD\n v_cmp_ne_u32_sdwa s[26:27], %0, %1 src0_sel:BYTE_1 src1_sel:DWORD\n"
                         "v_cmp_ne_u32_sdwa s[28:29], %0, %1 src0_sel:BYTE_1 src1_sel:DWORD\n v_cmp_ne_u32_sdwa s[30:31], %0, %1 src0_sel:BYTE_1 src1_sel:DWORD\n"
                         "v_cmp_ne_u32_sdwa s[32:33], %0, %1 src0_sel:BYTE_1 src1_sel:DWORD\n v_cmp_ne_u32_sdwa s[34:35], %0, %1 src0_sel:BYTE_1 src1_sel:DWORD\n"
                         "v_cmp_ne_u32_sdwa s[36:37], %0, %1 src0_sel:BYTE_1 src1_sel:DWORD\n v_cmp_ne_u32_sdwa s[38:39], %0, %1 src0_sel:BYTE_1 src1_sel:DWORD"
                         :: "v"(a0), "v"(b) : "s24","s25","s26","s27","s28","s29","s30","s31","s32","s33","s34","s35","s36","s37","s38","s39");
        }
    }
    if constexpr (OP == 17) C8("v_not_b32 %0, %0")
    if constexpr (OP == 18) C8("v_pk_sub_u16 %0, %0, %1")
    if constexpr (OP == 19) C8("v_sub_u32 %0, %0, %1")
    if constexpr (OP == 20) C8("v_and_b32 %0, 0xff00ff, %0")
    if constexpr (OP == 21) C8("v_min_u32 %0, %0, %1")
    if constexpr (OP == 22) C8("v_lshl_add_u32 %0, %0, 1, %1")
    if constexpr (OP == 23) C8("v_mad_u32_u24 %0, %0, %1, %1")
    if constexpr (OP == 24) C8("v_bfe_u32 %0, %0, %1, 3")
    if constexpr (OP == 25) C8("v_or_b32_sdwa %0, %1, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:DWORD")
    if constexpr (OP == 26) P4("v_and_b32 %0, %0, %2\n v_perm_b32 %1, %1, %2, %2")
    if constexpr (OP == 27) C8("v_xad_u32 %0, %0, %1, %1")
    if constexpr (OP == 28) {
        for (int i = 0; i < ITER; ++i) {
            asm volatile("v_add_u32 %0, %0, %2\n v_xor_b32 %1, %1, %2\n v_add_u32 %0, %0, %2\n v_xor_b32 %1, %1, %2\n"
                         "v_add_u32 %0, %0, %2\n v_xor_b32 %1, %1, %2\n v_add_u32 %0, %0, %2\n v_xor_b32 %1, %1, %2"
                         : "+v"(a0), "+v"(a1) : "v"(b));
        }
    }
    if constexpr (OP == 29) C8("v_cndmask_b32 %0, %0, %1, vcc")
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// LDS atomics: 16 ds_add_u32 per iteration, lanes grouped so that K lanes of each 32-lane
// half share an address (K = 1: every lane its own bank-distinct dword).
template <int K>
__global__ __launch_bounds__(256) void kern_lds(uint32_t *out, uint32_t seed) {
    __shared__ uint32_t h[4096];
    for (int i = threadIdx.x; i < 4096; i += 256) h[i] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t addr = (w * 1024 + (lane / K) * 4 + (seed & 1)) * 4;  // (seed & 1) is 0
    for (int i = 0; i < ITER / 4; ++i) {
        asm volatile(
            "ds_add_u32 %0, %1\n ds_add_u32 %0, %1 offset:256\n ds_add_u32 %0, %1 offset:512\n ds_add_u32 %0, %1 offset:768\n"
            "ds_add_u32 %0, %1 offset:1024\n ds_add_u32 %0, %1 offset:1280\n ds_add_u32 %0, %1 offset:1536\n ds_add_u32 %0, %1 offset:1792\n"
            "ds_add_u32 %0, %1 offset:2048\n ds_add_u32 %0, %1 offset:2304\n ds_add_u32 %0, %1 offset:2560\n ds_add_u32 %0, %1 offset:2816\n"
            "ds_add_u32 %0, %1 offset:3072\n ds_add_u32 %0, %1 offset:3328\n ds_add_u32 %0, %1 offset:3584\n ds_add_u32 %0, %1 offset:3840\n"
            "s_waitcnt lgkmcnt(8)" ::"v"(addr), "v"(1u));
    }
    asm volatile("s_waitcnt lgkmcnt(0)");
    __syncthreads();
    out[blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x * 4];
}

template <class F>
static float timeit(F f) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    f();
    hipEventRecord(e0);
    f();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

template <int OP>
static void run(uint32_t *d, int cus, int wps, double ghz) {
    const int blocks = cus * wps;
    const float ms = timeit([&] { kern<OP><<<blocks, 256>>>(d, 1); });
    const double winst = (double)blocks * 4 * ITER * 8;
    const double cyc = ms * 1e-3 * ghz * 1e9;
    printf("%-38s wps %d %8.3f ms  %.2f cycles per wave-instr per SIMD\n", names[OP], wps, ms, cyc * 4 * cus / winst);
}
template <int K>
static void run_lds(uint32_t *d, int cus, int wps, double ghz) {
    const int blocks = cus * wps;
    const float ms = timeit([&] { kern_lds<K><<<blocks, 256>>>(d, 0); });
    const double winst = (double)blocks * 4 * (ITER / 4) * 16;
    const double cyc = ms * 1e-3 * ghz * 1e9;
    printf("ds_add_u32 %2d lanes per address     wps %d %8.3f ms  %.2f CU-cycles per wave-instr\n", K, wps, ms, cyc * cus / winst);
}

template <int... OPS>
static void run_all(uint32_t *d, int cus, int wps, double ghz, std::integer_sequence<int, OPS...>) {
    (run<OPS>(d, cus, wps, ghz), ...);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const double ghz = 2.4;
    printf("CUs %d, cycles at a nominal %.1f GHz\n", cus, ghz);
    uint32_t *d;
    hipMalloc(&d, (size_t)cus * 8 * 256 * 4);
    run_all(d, cus, 8, ghz, std::make_integer_sequence<int, NOPS>{});
    run<0>(d, cus, 2, ghz);
    run<4>(d, cus, 2, ghz);
    run<2>(d, cus, 2, ghz);
    run_lds<1>(d, cus, 6, ghz);
    run_lds<2>(d, cus, 6, ghz);
    run_lds<4>(d, cus, 6, ghz);
    run_lds<8>(d, cus, 6, ghz);
    run_lds<32>(d, cus, 6, ghz);
    hipFree(d);
    return 0;
}
