// tests/native/selftest.hip — hardware-semantics self-test of the device primitives in
// psyne_amd/csrc/tdt_device.h (DPP wave scans, team scans, SWAR run-start masks, v_perm /
// v_alignbyte operand order).  Test infrastructure: every access is within fixed-size
// buffers sized by the caller, so a wrong primitive shows up as a wrong value, never a fault.
#include "../../psyne_amd/csrc/tdt_device.h"

using namespace psy;

// in: 256 uint32; out layout (uint32):
//   [0,256)    wave inclusive add-scan (4 waves independently)
//   [256,512)  wave inclusive max-scan
//   [512,768)  team exclusive add-scan (W=4), [768] team total
//   [769,1025) team exclusive max-scan (W=4), [1025] total
//   [1026,1090) W=1 exclusive add-scan of the first 64 inputs, [1090] total
//   [1091,1155) neq_prev_mask4(in[l], in[l+64]) for lanes 0..63
//   [1155,1219) perm(in[l], in[l+64], sel[l%8])
//   [1219,1283) alignbyte(in[l], in[l+64], 3)
//   [1283,1347) wave_shift_up1(in[l])
//   [1347,1411) wave_shr1(in[l], 77)   [1411,1475) wave_shl1(in[l], 99)
//   [1475,1539) packed u16 max-scan     [1539,1603) ffbh_u32(in[l] >> (l % 33))
__global__ __launch_bounds__(256) void selftest_kernel(const uint32_t *in, uint32_t *out) {
    __shared__ uint32_t slots[2 * 4 * 4];
    const int t = threadIdx.x, lane = t & 63;
    const uint32_t x = in[t];
    out[t] = wave_incl_scan<OpAdd>(x);
    out[256 + t] = wave_incl_scan<OpMax>(x);
    uint32_t v[1] = {x}, tot[1];
    team_excl_scan<4, 1, OpAdd>(v, tot, slots);
    out[512 + t] = v[0];
    if (t == 0) out[768] = tot[0];
    uint32_t m[1] = {x}, mt[1];
    team_excl_scan<4, 1, OpMax>(m, mt, slots + 16);
    out[769 + t] = m[0];
    if (t == 0) out[1025] = mt[0];
    if (t < 64) {
        uint32_t w[1] = {x}, wt[1];
        team_excl_scan<1, 1, OpAdd>(w, wt, nullptr);
        out[1026 + t] = w[0];
        if (t == 0) out[1090] = wt[0];
        const uint32_t y = in[t + 64];
        out[1091 + t] = neq_prev_mask4(x, y);
        const uint32_t sels[8] = {0x03020100u, 0x07060504u, 0x0c0c0c0cu, 0x0400070cu,
                                  0x01050c02u, 0x0c0c0706u, 0x00000000u, 0x07070707u};
        out[1155 + t] = __builtin_amdgcn_perm(x, y, sels[lane & 7]);
        out[1219 + t] = __builtin_amdgcn_alignbyte(x, y, 3);
        out[1283 + t] = wave_shift_up1(x);
        out[1347 + t] = wave_shr1(x, 77u);
        out[1411 + t] = wave_shl1(x, 99u);
        out[1475 + t] = wave_incl_scan<OpPkMax>(x * 2654435761u);
        const uint32_t sh = (uint32_t)(t % 33);
        out[1539 + t] = ffbh_u32(sh == 32 ? 0u : (x >> sh));
    }
}

// Unaligned LDS stores/loads (ds_write_b16 at odd byte addresses, ds_read_b128 at 4-aligned
// ones): out[l] = the u32 read back at byte 4l of a buffer where lane l wrote u16 (0x100+l) at
// byte 2l+1, and out[64 + l] = the xor of the 4 dwords of a 16-byte read at byte 4l.
__global__ __launch_bounds__(64) void unaligned_lds_kernel(uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[512];
    const int l = threadIdx.x;
    for (int i = l; i < 512; i += 64) buf[i] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    uint8_t *pb = buf;
    *reinterpret_cast<uint16_t *>(pb + 2 * l + 1) = (uint16_t)(0x100 + l);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    out[l] = *reinterpret_cast<const uint32_t *>(buf + 4 * l);
    const uint4 q = *reinterpret_cast<const uint4 *>(pb + 4 * l);
    out[64 + l] = q.x ^ q.y ^ q.z ^ q.w;
}

extern "C" int selftest_unaligned_lds(uint32_t *d_out) {
    hipLaunchKernelGGL(unaligned_lds_kernel, dim3(1), dim3(64), 0, 0, d_out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

extern "C" int selftest_run(const uint32_t *d_in, uint32_t *d_out) {
    hipLaunchKernelGGL(selftest_kernel, dim3(1), dim3(256), 0, 0, d_in, d_out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

// ---------------------------------------------------------------------------------------
// Entropy arithmetic on the device, exactly as tdt_encode_kernel evaluates it (SURVEY.md §7
// hard part (i)): for c = 1..N, prob = (double)c / N, L = psy_log2_glibc(prob) with the
// glibc tables staged in LDS, and the entropy step fma(-prob, L, 0.0).  out: 2N doubles
// (L, step) per c.  The test compares them bitwise with the host's libm.
#include "../../psyne_amd/csrc/tdt_log2.h"

__constant__ __attribute__((aligned(16))) double st_log2_tab[128] = PSY_LOG2_TAB_INIT;
__constant__ __attribute__((aligned(16))) double st_log2_tab2[128] = PSY_LOG2_TAB2_INIT;

__global__ __launch_bounds__(256) void log2_sweep_kernel(uint32_t N, double *out) {
    __shared__ double tab[256];
    for (int i = threadIdx.x; i < 128; i += 256) {
        tab[i] = st_log2_tab[i];
        tab[128 + i] = st_log2_tab2[i];
    }
    __syncthreads();
    const uint32_t c = blockIdx.x * 256u + threadIdx.x + 1u;
    if (c > N) return;
    double prob, L;
    {
#pragma clang fp contract(off)
        prob = (double)c / (double)N;
        L = psy_log2_glibc(prob, tab, tab + 128);
    }
    out[2ull * (c - 1)] = L;
    out[2ull * (c - 1) + 1] = __builtin_fma(-prob, L, 0.0);
}

extern "C" int selftest_log2_sweep(uint32_t N, double *d_out) {
    if (N == 0) return 0;
    hipLaunchKernelGGL(log2_sweep_kernel, dim3((N + 255) / 256), dim3(256), 0, 0, N, d_out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

// Hardware log2 (v_log_f32) of (float)c — the encode's mapping fast path (tdt_encode.h, "E")
// bounds its error by 2^-18 per count: out[i] = log2f_hw((float)c_i) for the caller's counts.
__global__ __launch_bounds__(256) void hw_log2_kernel(const uint32_t *c, uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) out[i] = __builtin_amdgcn_logf((float)c[i]);
}

extern "C" int selftest_hw_log2(const uint32_t *d_c, uint32_t n, float *d_out) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(hw_log2_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, d_c, n, d_out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
