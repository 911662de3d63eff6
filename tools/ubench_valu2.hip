// Diagnostic micro-benchmark (not part of the product): issue cost on gfx950 of the SDWA byte
// selects, compare + select pairs and shift forms considered for the encode sweep (see
// tools/ubench_valu.hip for the method: 8 independent chains of one instruction per wave).
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu2.hip -o tools/ubench_valu2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITER = 4096;

#define CHAIN8(ASM)                                                                          \
    for (int i = 0; i < ITER; ++i) {                                                         \
        asm volatile(ASM : "+v"(a0) : "v"(b)); asm volatile(ASM : "+v"(a1) : "v"(b));        \
        asm volatile(ASM : "+v"(a2) : "v"(b)); asm volatile(ASM : "+v"(a3) : "v"(b));        \
        asm volatile(ASM : "+v"(a4) : "v"(b)); asm volatile(ASM : "+v"(a5) : "v"(b));        \
        asm volatile(ASM : "+v"(a6) : "v"(b)); asm volatile(ASM : "+v"(a7) : "v"(b));        \
    }
#define CHAIN8S(ASM)                                                                         \
    for (int i = 0; i < ITER; ++i) {                                                         \
        asm volatile(ASM : "+v"(a0) : "v"(b), "s"(sm)); asm volatile(ASM : "+v"(a1) : "v"(b), "s"(sm)); \
        asm volatile(ASM : "+v"(a2) : "v"(b), "s"(sm)); asm volatile(ASM : "+v"(a3) : "v"(b), "s"(sm)); \
        asm volatile(ASM : "+v"(a4) : "v"(b), "s"(sm)); asm volatile(ASM : "+v"(a5) : "v"(b), "s"(sm)); \
        asm volatile(ASM : "+v"(a6) : "v"(b), "s"(sm)); asm volatile(ASM : "+v"(a7) : "v"(b), "s"(sm)); \
    }

constexpr int NOPS = 12;
static const int kInstr[NOPS] = {1, 1, 1, 1, 1, 1, 2, 2, 1, 2, 2, 1};  // wave-instructions per asm statement
static const char *names[NOPS] = {"v_add_u32_sdwa byte1", "v_and_b32_sdwa byte2", "v_lshlrev_b32 vgpr amt",
                                  "v_lshrrev_b32 const 1", "v_bfi_b32", "v_cndmask_b32_e64 sgpr",
                                  "v_cmp_ne sdwa + cndmask", "v_cmp_ne e32 + cndmask vcc", "v_cndmask_b32 vcc",
                                  "bfe + lshl_add pair", "and + add pair", "v_sub_u32_sdwa word1"};

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7, b = seed * 3u + threadIdx.x;
    const uint64_t sm = __ballot(threadIdx.x & 1);
    if constexpr (OP == 0) CHAIN8("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1")
    if constexpr (OP == 1) CHAIN8("v_and_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2")
    if constexpr (OP == 2) CHAIN8("v_lshlrev_b32 %0, %1, %0")
    if constexpr (OP == 3) CHAIN8("v_lshrrev_b32 %0, 1, %0")
    if constexpr (OP == 4) CHAIN8("v_bfi_b32 %0, %1, %0, %1")
    if constexpr (OP == 5) CHAIN8S("v_cndmask_b32_e64 %0, %0, %1, %2")
    if constexpr (OP == 6) CHAIN8("v_cmp_ne_u32_sdwa vcc, %1, %0 src0_sel:BYTE_1 src1_sel:DWORD\n v_cndmask_b32 %0, %0, %1, vcc")
    if constexpr (OP == 7) CHAIN8("v_cmp_ne_u32 vcc, %1, %0\n v_cndmask_b32 %0, %0, %1, vcc")
    if constexpr (OP == 8) {
        asm volatile("v_cmp_ne_u32 vcc, 0, %0" ::"v"(b) : "vcc");
        CHAIN8("v_cndmask_b32 %0, %0, %1, vcc")
    }
    if constexpr (OP == 9) CHAIN8("v_bfe_u32 %0, %0, %1, 1\n v_lshl_add_u32 %0, %0, 1, %1")
    if constexpr (OP == 10) CHAIN8("v_and_b32 %0, %0, %1\n v_add_u32 %0, %0, %1")
    if constexpr (OP == 11) CHAIN8("v_sub_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1")
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int OP>
static void run(uint32_t *d, int cus, int wps, double clk_ghz) {
    const int blocks = cus * wps;  // 256 threads = 4 waves = one per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<OP><<<blocks, 256>>>(d, 1);
    hipEventRecord(e0);
    kern<OP><<<blocks, 256>>>(d, 2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double winst = (double)blocks * 4 * ITER * 8 * kInstr[OP];
    const double cyc = ms * 1e-3 * clk_ghz * 1e9;
    printf("%-28s waves/SIMD %2d  %8.3f ms  (%.2f cycles per wave-instr per SIMD at %.2f GHz)\n", names[OP], wps,
           ms, cyc * 4 * cus / winst, clk_ghz);
}

template <int... OPS>
static void all(uint32_t *d, int cus, double clk, std::integer_sequence<int, OPS...>) {
    (run<OPS>(d, cus, 8, clk), ...);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const double clk = p.clockRate / 1e6;
    uint32_t *d;
    hipMalloc(&d, (size_t)cus * 8 * 256 * 4);
    all(d, cus, clk, std::make_integer_sequence<int, NOPS>{});
    hipFree(d);
    return 0;
}
