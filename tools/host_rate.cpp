// tools/host_rate.cpp — diagnostic: host-path call rates of the C ABI (tdt_encode_host_v on
// pageable 1 MiB gradient messages, tdt_decode_host from pinned frames into pageable output) per
// sub-batch size, to size TdtSubstrate's pipeline.  Not part of the product.
#include <psyne_tdt.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include <cstdlib>

int main(int argc, char **argv) {
    tdt_config cfg;
    tdt_default_config(&cfg);
    cfg.sample_fraction = 1.0f;
    tdt_ctx *c = nullptr;
    if (tdt_ctx_create(0, &cfg, &c) != TDT_OK) return 1;
    tdt_ctx_set_metrics(c, 10.0, 1.0, 0.5);
    const size_t mb = 1 << 20, nmsg = 64;
    std::vector<std::vector<uint8_t>> msgs(nmsg, std::vector<uint8_t>(mb));
    std::mt19937 rng(1);
    std::normal_distribution<float> nd(0.f, 0.01f);
    std::uniform_real_distribution<float> u(0.f, 1.f);
    for (auto &m : msgs) {
        float *f = reinterpret_cast<float *>(m.data());
        for (size_t i = 0; i < mb / 4; ++i) f[i] = u(rng) < 0.7f ? 0.f : nd(rng);
    }
    std::vector<size_t> subs = {1, 2, 4, 8, 16, 32, 64};
    if (argc > 1) {  // sub-batch sizes to run (default: the sweep)
        subs.clear();
        for (int a = 1; a < argc; ++a) subs.push_back(std::strtoull(argv[a], nullptr, 10));
    }
    for (size_t sub : subs) {
        std::vector<const uint8_t *> p(sub);
        std::vector<uint64_t> sz(sub, mb), off(sub + 1);
        std::vector<int32_t> st(sub);
        void *pin = nullptr;
        const uint64_t cap = sub * tdt_encode_bound(mb, 4);
        tdt_host_alloc(cap, &pin);
        std::vector<uint8_t> back(sub * mb);
        void *pback = nullptr;
        tdt_host_alloc(sub * mb, &pback);
        std::vector<uint64_t> doff(sub + 1);
        std::vector<int32_t> dst(sub);
        double te = 0, td = 0, tp = 0;
        int reps = 0;
        for (int r = 0; r < 12; ++r) {
            for (size_t i = 0; i < sub; ++i) p[i] = msgs[(r * sub + i) % nmsg].data();
            auto t0 = std::chrono::steady_clock::now();
            if (tdt_encode_host_v(c, p.data(), sz.data(), (uint32_t)sub, (uint8_t *)pin, cap, off.data(), st.data()))
                return 2;
            auto t1 = std::chrono::steady_clock::now();
            if (tdt_decode_host(c, (uint8_t *)pin, off.data(), (uint32_t)sub, back.data(), back.size(), doff.data(),
                                dst.data()))
                return 3;
            auto t2 = std::chrono::steady_clock::now();
            if (tdt_decode_host(c, (uint8_t *)pin, off.data(), (uint32_t)sub, (uint8_t *)pback, sub * mb, doff.data(),
                                dst.data()))
                return 4;
            auto t3 = std::chrono::steady_clock::now();
            if (r >= 2) {
                te += std::chrono::duration<double>(t1 - t0).count();
                td += std::chrono::duration<double>(t2 - t1).count();
                tp += std::chrono::duration<double>(t3 - t2).count();
                ++reps;
            }
        }
        std::printf("{\"sub_msgs\": %zu, \"encode_v_GBps\": %.2f, \"decode_GBps\": %.2f, \"decode_pinned_GBps\": %.2f, "
                    "\"encode_us\": %.1f, \"decode_us\": %.1f, \"decode_pinned_us\": %.1f}\n",
                    sub, sub * mb * reps / te / 1e9, sub * mb * reps / td / 1e9, sub * mb * reps / tp / 1e9,
                    te / reps * 1e6, td / reps * 1e6, tp / reps * 1e6);
        tdt_host_free(pin);
        tdt_host_free(pback);
    }
    tdt_ctx_destroy(c);
    return 0;
}
