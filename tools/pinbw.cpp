// tools/pinbw.cpp — diagnostic: one host thread's memcpy / memcmp throughput on pageable memory
// vs hipHostMalloc'd memory (default, non-coherent and write-combined flags) vs
// hipHostRegister'ed pageable memory — the CPU side of the substrate's socket copies and
// checks on pinned staging.  Not part of the product.
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double rate(void *dst, const void *src, size_t n, bool cmp) {
    const auto t0 = std::chrono::steady_clock::now();
    size_t done = 0;
    volatile int sink = 0;
    while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(300)) {
        if (cmp) sink += std::memcmp(dst, src, n);
        else std::memcpy(dst, src, n);
        done += n;
    }
    return done / std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 1e9;
}

int main() {
    const size_t n = 64ull << 20;
    std::vector<char> a(n, 1), b(n, 1);
    struct K { const char *name; unsigned flags; bool reg; };
    for (K k : {K{"hipHostMallocDefault", hipHostMallocDefault, false},
                K{"hipHostMallocNonCoherent", hipHostMallocNonCoherent, false},
                K{"hipHostMallocCoherent", hipHostMallocCoherent, false},
                K{"hipHostMallocWriteCombined", hipHostMallocWriteCombined, false},
                K{"hipHostRegister", 0, true}}) {
        void *p = nullptr;
        char *reg = nullptr;
        if (k.reg) {
            reg = static_cast<char *>(std::aligned_alloc(4096, n));
            std::memset(reg, 1, n);
            if (hipHostRegister(reg, n, hipHostRegisterDefault) != hipSuccess) { std::printf("register failed\n"); continue; }
            p = reg;
        } else if (hipHostMalloc(&p, n, k.flags) != hipSuccess) {
            std::printf("%s failed\n", k.name);
            continue;
        }
        std::memset(p, 1, n);
        std::printf("{\"mem\": \"%s\", \"to_pinned_GBps\": %.1f, \"from_pinned_GBps\": %.1f, \"memcmp_GBps\": %.1f, "
                    "\"pageable_memcpy_GBps\": %.1f}\n", k.name, rate(p, a.data(), n, false), rate(b.data(), p, n, false),
                    rate(p, a.data(), n, true), rate(b.data(), a.data(), n, false));
        if (k.reg) { (void)hipHostUnregister(reg); std::free(reg); }
        else (void)hipHostFree(p);
    }
    return 0;
}
