// tools/membw.cpp — diagnostic: host memcpy throughput with 1..16 threads (each copying between
// two private 64 MiB buffers for ~0.5 s), to size what the loopback harness's socket copies,
// staging copies and checks can draw from host memory.  Not part of the product.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

int main() {
    const size_t sz = 64ull << 20;
    for (int t : {1, 2, 4, 8, 16}) {
        std::atomic<uint64_t> bytes{0};
        std::vector<std::thread> th;
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < t; ++i)
            th.emplace_back([&] {
                std::vector<char> a(sz, 1), b(sz, 2);
                const auto s = std::chrono::steady_clock::now();
                uint64_t n = 0;
                while (std::chrono::steady_clock::now() - s < std::chrono::milliseconds(500)) {
                    std::memcpy(b.data(), a.data(), sz);
                    n += sz;
                }
                bytes += n;
            });
        for (auto &x : th) x.join();
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("{\"threads\": %d, \"memcpy_GBps\": %.1f}\n", t, bytes.load() / secs / 1e9);
    }
    return 0;
}
