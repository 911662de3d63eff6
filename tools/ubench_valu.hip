// Diagnostic micro-benchmark (not part of the product): issue throughput of the integer VALU
// instructions the codec kernels are made of, on gfx950.  Each wave runs ITER iterations of 8
// independent chains of one instruction (inline asm, so the exact opcode is issued); the grid
// fills every SIMD with WPS waves.  Prints wave-instructions per cycle per CU for each opcode.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o tools/ubench_valu
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

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7, b = seed * 3u + threadIdx.x;
    if constexpr (OP == 0) CHAIN8("v_add_u32 %0, %0, %1")
    if constexpr (OP == 1) CHAIN8("v_perm_b32 %0, %0, %1, %1")
    if constexpr (OP == 2) CHAIN8("v_and_b32 %0, %0, %1")
    if constexpr (OP == 3) CHAIN8("v_or_b32 %0, %0, %1")
    if constexpr (OP == 4) CHAIN8("v_xor_b32 %0, %0, %1")
    if constexpr (OP == 5) CHAIN8("v_lshlrev_b32 %0, 1, %0")
    if constexpr (OP == 6) CHAIN8("v_lshrrev_b32 %0, %1, %0")
    if constexpr (OP == 7) CHAIN8("v_min_u32 %0, %0, %1")
    if constexpr (OP == 8) CHAIN8("v_max_u32 %0, %0, %1")
    if constexpr (OP == 9) CHAIN8("v_sub_u32 %0, %0, %1")
    if constexpr (OP == 10) CHAIN8("v_mov_b32 %0, %1")
    if constexpr (OP == 11) CHAIN8("v_add3_u32 %0, %0, %1, %1")
    if constexpr (OP == 12) CHAIN8("v_or3_b32 %0, %0, %1, %1")
    if constexpr (OP == 13) CHAIN8("v_lshl_or_b32 %0, %0, 1, %1")
    if constexpr (OP == 14) CHAIN8("v_and_or_b32 %0, %0, %1, %1")
    if constexpr (OP == 15) CHAIN8("v_add_u32_e64 %0, %0, %1")
    if constexpr (OP == 16) CHAIN8("v_cndmask_b32 %0, %0, %1, vcc")
    if constexpr (OP == 17) CHAIN8("v_bfe_u32 %0, %0, %1, 3")
    if constexpr (OP == 18) CHAIN8("v_mad_u32_u24 %0, %0, %1, %1")
    if constexpr (OP == 19) CHAIN8("v_mul_u32_u24 %0, %0, %1")
    if constexpr (OP == 20) CHAIN8("v_pk_add_u16 %0, %0, %1")
    if constexpr (OP == 21) CHAIN8("v_max_u32_dpp %0, %0, %1 row_shr:1 bound_ctrl:0")
    if constexpr (OP == 22) CHAIN8("v_mov_b32_dpp %0, %1 row_shr:1 bound_ctrl:0")
    if constexpr (OP == 23) CHAIN8("v_lshl_add_u32 %0, %0, 1, %1")
    if constexpr (OP == 24) CHAIN8("v_bcnt_u32_b32 %0, %0, %1")
    if constexpr (OP == 25) CHAIN8("v_ffbh_u32 %0, %1")
    if constexpr (OP == 26) CHAIN8("v_alignbyte_b32 %0, %0, %1, 2")
    if constexpr (OP == 27) CHAIN8("v_pk_max_u16 %0, %0, %1")
    if constexpr (OP == 28) CHAIN8("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96")
    if constexpr (OP == 29) CHAIN8("v_add_u32 %0, %0, %1\n v_perm_b32 %0, %0, %1, %1")
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

static const char *names[] = {"v_add_u32", "v_perm_b32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_lshlrev_b32", "v_lshrrev_b32", "v_min_u32", "v_max_u32", "v_sub_u32", "v_mov_b32", "v_add3_u32", "v_or3_b32", "v_lshl_or_b32", "v_and_or_b32", "v_add_u32_e64", "v_cndmask_b32", "v_bfe_u32", "v_mad_u32_u24", "v_mul_u32_u24", "v_pk_add_u16", "v_max_u32_dpp", "v_mov_b32_dpp", "v_lshl_add_u32", "v_bcnt_u32_b32", "v_ffbh_u32", "v_alignbyte_b32", "v_pk_max_u16", "v_bitop3_b32", "add+perm pair"};

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
    const double winst = (double)blocks * 4 * ITER * 8 * (OP == 29 ? 2 : 1);  // wave-instructions
    const double cyc = ms * 1e-3 * clk_ghz * 1e9;
    printf("%-22s waves/SIMD %2d  %8.3f ms  %.3f wave-instr/cycle/CU  (%.2f cycles per wave-instr per SIMD)\n",
           names[OP], wps, ms, winst / cus / cyc, cyc * 4 * cus / winst);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const double clk = p.clockRate / 1e6;  // GHz (kHz in the property)
    printf("CUs %d, clock %.3f GHz (nominal; cycles below use it)\n", cus, clk);
    uint32_t *d;
    hipMalloc(&d, (size_t)cus * 8 * 256 * 4);
    for (int wps : {8}) {
        run<0>(d, cus, wps, clk);
        run<1>(d, cus, wps, clk);
        run<2>(d, cus, wps, clk);
        run<3>(d, cus, wps, clk);
        run<4>(d, cus, wps, clk);
        run<5>(d, cus, wps, clk);
        run<6>(d, cus, wps, clk);
        run<7>(d, cus, wps, clk);
        run<8>(d, cus, wps, clk);
        run<9>(d, cus, wps, clk);
        run<10>(d, cus, wps, clk);
        run<11>(d, cus, wps, clk);
        run<12>(d, cus, wps, clk);
        run<13>(d, cus, wps, clk);
        run<14>(d, cus, wps, clk);
        run<15>(d, cus, wps, clk);
        run<16>(d, cus, wps, clk);
        run<17>(d, cus, wps, clk);
        run<18>(d, cus, wps, clk);
        run<19>(d, cus, wps, clk);
        run<20>(d, cus, wps, clk);
        run<21>(d, cus, wps, clk);
        run<22>(d, cus, wps, clk);
        run<23>(d, cus, wps, clk);
        run<24>(d, cus, wps, clk);
        run<25>(d, cus, wps, clk);
        run<26>(d, cus, wps, clk);
        run<27>(d, cus, wps, clk);
        run<28>(d, cus, wps, clk);
        run<29>(d, cus, wps, clk);
    }
    hipFree(d);
    return 0;
}
