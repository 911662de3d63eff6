// tdt_log2.h — bit-exact restatement of the reference codec's mapping decision.
//
// Reference: include/psyne/protocol/tdt_compression.hpp
//   calculate_entropy  :470-480   entropy -= prob * std::log2(prob)  (count > 0 bins, bin order 0..255)
//   perform_clustering :507-525   mapping[b] = entropy[b] > accumulate(entropies, 0.0) / ws
//
// Two facts pin the arithmetic (both established in DESIGN.md §"Entropy bits"):
//  1. The reference build (g++ -std=c++20 -O3 -march=native on an FMA host) contracts
//     `entropy -= prob * log2(prob)` into one vfnmadd213sd, i.e.
//     entropy = fma(-prob, log2(prob), entropy) with a single rounding.  C++ keeps
//     -ffp-contract=fast even in ISO mode, so -std=c++20 and -std=gnu++20 agree.
//  2. std::log2 is glibc 2.35's log2 (ARM optimized-routines algorithm, 64-entry table),
//     and on x86_64 glibc ships only its non-FMA path (log2@@GLIBC_2.29 is plain SSE2).
//
// psy_log2_glibc() restates that non-FMA algorithm operation for operation, with the
// constants read from the system libm by tools/gen_glibc_log2.py.  Every operation below
// is a single IEEE double op, so the same source gives the same bits on x86 and gfx950 —
// provided nothing is contracted: HIP code gets `#pragma clang fp contract(off)`, host C
// is compiled with -ffp-contract=off.  tests/test_log2_restatement.py checks it against
// the system log2 bit for bit over every p = c/N the codec can produce for N <= 2^15,
// sampled N up to 2^20, and random doubles.
#pragma once
#include <stdint.h>
#include <string.h>
#include "glibc_log2_data.h"

#if defined(__HIPCC__) || defined(__HIP__)
#define PSY_HD __host__ __device__
#else
#define PSY_HD
#endif

static inline PSY_HD uint64_t psy_as_u64(double x) {
    uint64_t u;
    __builtin_memcpy(&u, &x, 8);
    return u;
}
static inline PSY_HD double psy_as_f64(uint64_t u) {
    double x;
    __builtin_memcpy(&x, &u, 8);
    return x;
}

// log2(x) for positive normal finite x, bit-identical to glibc 2.35 x86_64 log2.
// T  = { invc, logc } x 64, T2 = { chi, clo } x 64 (PSY_LOG2_TAB_INIT / PSY_LOG2_TAB2_INIT).
static inline PSY_HD double psy_log2_glibc(double x, const double *T, const double *T2) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    const double InvLn2hi = PSY_LOG2_INVLN2HI;
    const double InvLn2lo = PSY_LOG2_INVLN2LO;
    const double A[6] = PSY_LOG2_POLY_INIT;
    const double B[10] = PSY_LOG2_POLY1_INIT;
    const uint64_t ix = psy_as_u64(x);
    // LO = asuint64(1.0 - 0x1.5b51p-5), HI = asuint64(1.0 + 0x1.6ab2p-5)
    const uint64_t LO = 0x3feea4af00000000ULL, HI = 0x3ff0b55900000000ULL;
    if (ix - LO < HI - LO) {
        if (ix == 0x3ff0000000000000ULL) return 0.0;
        double r = x - 1.0;
        double rhi = psy_as_f64(psy_as_u64(r) & (~0ULL << 32));
        double rlo = r - rhi;
        double hi = rhi * InvLn2hi;
        double lo = rlo * InvLn2hi + r * InvLn2lo;
        double r2 = r * r;
        double r4 = r2 * r2;
        double p = r2 * (B[0] + r * B[1]);
        double y = hi + p;
        lo += hi - y + p;
        lo += r4 * (B[2] + r * B[3] + r2 * (B[4] + r * B[5]) +
                    r4 * (B[6] + r * B[7] + r2 * (B[8] + r * B[9])));
        y += lo;
        return y;
    }
    const uint64_t tmp = ix - 0x3fe6000000000000ULL;
    const int i = (int)((tmp >> 46) & 63);
    const int k = (int)((int64_t)tmp >> 52);
    const uint64_t iz = ix - (tmp & (0xfffULL << 52));
    const double invc = T[2 * i], logc = T[2 * i + 1];
    const double z = psy_as_f64(iz);
    const double kd = (double)k;
    double r = (z - T2[2 * i] - T2[2 * i + 1]) * invc;
    double rhi = psy_as_f64(psy_as_u64(r) & (~0ULL << 32));
    double rlo = r - rhi;
    double t1 = rhi * InvLn2hi;
    double t2 = rlo * InvLn2hi + r * InvLn2lo;
    double t3 = kd + logc;
    double hi = t3 + t1;
    double lo = t3 - hi + t1 + t2;
    double r2 = r * r;
    double r4 = r2 * r2;
    double p = A[0] + r * A[1] + r2 * (A[2] + r * A[3]) + r4 * (A[4] + r * A[5]);
    double y = lo + r2 * p + hi;
    return y;
}

// One step of calculate_entropy for a bin with count > 0 (tdt_compression.hpp:474-477),
// with the reference build's contraction: entropy = fma(-prob, log2(prob), entropy).
static inline PSY_HD double psy_entropy_step(double entropy, uint32_t count, double total,
                                             const double *T, const double *T2) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    const double prob = (double)count / total;
    return __builtin_fma(-prob, psy_log2_glibc(prob, T, T2), entropy);
}
