// Diagnostic micro-benchmark (not shipped): the achievable HBM rate on gfx950 for the access
// shapes the codec uses, to reconcile tools/ubench_copy.hip (5.36 TB/s) with the guide's
// 6.29 TB/s float4 copy, 6.0-6.1 TB/s read sweep and 6.0-6.2 TB/s plain stores
// (MI355X_MICROARCH.md:36,332,351).  Rows (bytes counted = bytes read + bytes written):
//   read   : dwordx4 loads, U in flight per lane, grid-stride, one store per lane at the end
//   write  : dwordx4 stores of a register value, U per lane per iteration, grid-stride
//   copy   : U loads then U stores per lane per iteration, grid-stride (ubench_copy's shape)
//   chunk  : one workgroup per CHUNK-byte piece, every load of the piece in flight before any
//            store (the resident encode/decode shape: read 64 KiB, write it back once)
//   mix    : chunk, but the workgroup writes `wfrac` of what it read (encode writes ~0.8 n)
// Each row: best and mean of REPS launches over BYTES (default 8 GiB per buffer, far past the
// 256 MiB Infinity Cache), workgroup sizes 256 / 512 / 1024, occupancy set by launch bounds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int B, int U, bool NT>
__global__ __launch_bounds__(B) void k_read(const u32x4 *__restrict__ src, u32x4 *__restrict__ sink, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * B * U;
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * B * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * B) : src[i + u * B];
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u];
    }
    if ((acc.x | acc.y | acc.z | acc.w) == 0x9e3779b9u) sink[threadIdx.x] = acc;  // (never: keeps the loads)
}

template <int B, int U, bool NT>
__global__ __launch_bounds__(B) void k_write(u32x4 *__restrict__ dst, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * B * U;
    const u32x4 v = {threadIdx.x, blockIdx.x, 1u, 2u};
    for (uint64_t i = (uint64_t)blockIdx.x * B * U + threadIdx.x; i < n16; i += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v, dst + i + u * B);
            else dst[i + u * B] = v;
        }
    }
}

template <int B, int U, bool NT, bool LNT = false>
__global__ __launch_bounds__(B) void k_copy(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * B * U;
    for (uint64_t i = (uint64_t)blockIdx.x * B * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = LNT ? __builtin_nontemporal_load(src + i + u * B) : src[i + u * B];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], dst + i + u * B);
            else dst[i + u * B] = v[u];
        }
    }
}

// one workgroup per piece of B*G*16 bytes (B=512, G=8: 64 KiB), all loads first; then the
// workgroup writes WN/8 of the piece (WN = 8: all of it)
template <int B, int G, int WN, bool NT, bool LNT = false>
__global__ __launch_bounds__(B) void k_chunk(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst) {
    const uint64_t base = (uint64_t)blockIdx.x * B * G;
    u32x4 v[G];
#pragma unroll
    for (int g = 0; g < G; ++g)
        v[g] = LNT ? __builtin_nontemporal_load(src + base + (uint64_t)g * B + threadIdx.x)
                   : src[base + (uint64_t)g * B + threadIdx.x];
    // (a little work, so the compiler cannot forward loads to stores; the pieces not stored are
    // folded into the first stored one so that every load stays live)
#pragma unroll
    for (int g = 0; g < G; ++g) v[g] = v[g] ^ (u32x4){(unsigned)g, 0u, 0u, 0u};
#pragma unroll
    for (int g = G * WN / 8; g < G; ++g) v[0] ^= v[g];
    const uint64_t ob = (uint64_t)blockIdx.x * B * G * WN / 8;
#pragma unroll
    for (int g = 0; g < G * WN / 8; ++g) {
        if (NT) __builtin_nontemporal_store(v[g], dst + ob + (uint64_t)g * B + threadIdx.x);
        else dst[ob + (uint64_t)g * B + threadIdx.x] = v[g];
    }
}

static uint64_t g_bytes;
static int g_reps = 8;

static void report(const char *row, const char *shape, int block, int grid, double bytes, const std::vector<float> &ms) {
    float best = *std::min_element(ms.begin(), ms.end());
    double mean = 0;
    for (float m : ms) mean += m;
    mean /= ms.size();
    std::printf("{\"row\": \"%s\", \"shape\": \"%s\", \"block\": %d, \"grid\": %d, \"GB\": %.3f, \"best_TBps\": %.3f, "
                "\"mean_TBps\": %.3f, \"best_ms\": %.4f}\n",
                row, shape, block, grid, bytes / 1e9, bytes / (best * 1e-3) / 1e12, bytes / (mean * 1e-3) / 1e12, best);
    std::fflush(stdout);
}

template <typename F>
static std::vector<float> timeit(F launch) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    launch();  // warm-up
    std::vector<float> out;
    for (int r = 0; r < g_reps; ++r) {
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        out.push_back(ms);
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return out;
}

int main(int argc, char **argv) {
    g_bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 8ull) << 30;
    const uint64_t n16 = g_bytes / 16;
    u32x4 *a, *b;
    if (hipMalloc(&a, g_bytes) != hipSuccess || hipMalloc(&b, g_bytes) != hipSuccess) return 1;
    hipMemset(a, 1, g_bytes);
    hipMemset(b, 0, g_bytes);
    hipDeviceSynchronize();
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    std::printf("{\"cus\": %d, \"bytes_per_buffer\": %llu}\n", cus, (unsigned long long)g_bytes);
    const double rw = 2.0 * g_bytes, r1 = 1.0 * g_bytes;
    if (argc > 2 && std::string(argv[2]) == "nt") {
        // non-temporal LOADS (the read row's best form) in the copy and chunk shapes
#define COPYL(BL, U, NT, G)                                                                                  \
    report("copy", "dwordx4 x" #U " ntload st" #NT, BL, G, rw,                                               \
           timeit([&] { k_copy<BL, U, NT, true><<<G, BL>>>(a, b, n16); }))
        for (int g : {cus * 8, cus * 16, cus * 32}) {
            COPYL(256, 4, true, g);
            COPYL(256, 8, true, g);
            COPYL(1024, 4, true, g);
            COPYL(256, 8, false, g);
        }
#define CHUNKL(BL, G, WN, NT)                                                                                \
    {                                                                                                        \
        const uint64_t piece = (uint64_t)BL * G * 16;                                                        \
        const int grid = (int)(g_bytes / piece);                                                             \
        const double by = (double)grid * piece * (1.0 + WN / 8.0);                                          \
        report(WN == 8 ? "chunk" : "mix", "piece " #BL "x" #G " w" #WN "/8 ntload st" #NT, BL, grid, by,      \
               timeit([&] { k_chunk<BL, G, WN, NT, true><<<grid, BL>>>(a, b); }));                           \
    }
        CHUNKL(512, 8, 8, true);
        CHUNKL(512, 8, 8, false);
        CHUNKL(512, 8, 6, true);
        CHUNKL(512, 8, 7, true);
        CHUNKL(512, 8, 4, true);
        CHUNKL(256, 8, 8, true);
        CHUNKL(1024, 4, 8, true);
        return 0;
    }

#define READ(BL, U, NT, G)                                                                                   \
    report("read", "dwordx4 x" #U #NT, BL, G, r1, timeit([&] { k_read<BL, U, NT><<<G, BL>>>(a, b, n16); }))
#define WRITE(BL, U, NT, G)                                                                                  \
    report("write", "dwordx4 x" #U #NT, BL, G, r1, timeit([&] { k_write<BL, U, NT><<<G, BL>>>(b, n16); }))
#define COPY(BL, U, NT, G)                                                                                   \
    report("copy", "dwordx4 x" #U #NT, BL, G, rw, timeit([&] { k_copy<BL, U, NT><<<G, BL>>>(a, b, n16); }))
    for (int g : {cus * 8, cus * 16, cus * 32, cus * 64}) {
        READ(256, 4, false, g);
        READ(256, 8, false, g);
        READ(512, 4, false, g);
        READ(512, 8, false, g);
        READ(1024, 4, false, g);
        READ(256, 8, true, g);
    }
    for (int g : {cus * 8, cus * 16, cus * 32, cus * 64}) {
        WRITE(256, 4, false, g);
        WRITE(256, 4, true, g);
        WRITE(512, 4, false, g);
        WRITE(1024, 2, false, g);
    }
    for (int g : {cus * 8, cus * 16, cus * 32, cus * 64}) {
        COPY(256, 4, false, g);
        COPY(256, 4, true, g);
        COPY(256, 8, false, g);
        COPY(256, 8, true, g);
        COPY(512, 4, false, g);
        COPY(512, 4, true, g);
        COPY(1024, 2, false, g);
        COPY(1024, 4, true, g);
    }
    // chunk shapes: one workgroup per piece, grid = pieces
#define CHUNK(BL, G, WN, NT)                                                                                 \
    {                                                                                                        \
        const uint64_t piece = (uint64_t)BL * G * 16;                                                        \
        const int grid = (int)(g_bytes / piece);                                                             \
        const double by = (double)grid * piece * (1.0 + WN / 8.0);                                          \
        report(WN == 8 ? "chunk" : "mix", "piece " #BL "x" #G " w" #WN "/8" #NT, BL, grid, by,                \
               timeit([&] { k_chunk<BL, G, WN, NT><<<grid, BL>>>(a, b); }));                                 \
    }
    CHUNK(512, 8, 8, false);
    CHUNK(512, 8, 8, true);
    CHUNK(256, 8, 8, true);
    CHUNK(1024, 4, 8, true);
    CHUNK(512, 4, 8, true);
    CHUNK(512, 8, 6, true);
    CHUNK(512, 8, 6, false);
    CHUNK(256, 16, 8, true);
    // hipMemcpyAsync DtoD beside them
    report("copy", "hipMemcpyAsync DtoD", 0, 0, rw,
           timeit([&] { hipMemcpyAsync(b, a, g_bytes, hipMemcpyDeviceToDevice, 0); }));
    return 0;
}
