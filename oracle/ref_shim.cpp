// oracle/ref_shim.cpp — C-ABI shim over the REFERENCE codec, compiled where it lies.
//
// TEST INFRASTRUCTURE ONLY.  This file contains no codec logic: it #includes the
// reference's header-only codec from /root/reference (never copied into this repo) and
// exposes it through extern "C" so tests/ and bench.py's cpu_baseline leg can call the
// real reference.  Built by oracle/Makefile into oracle/_ref/libtdt_ref.so (git-ignored;
// it travels to the GPU box with the gpurun snapshot).  Nothing in psyne_amd/ links it.
//
// Reference symbols wrapped:
//   psyne::protocol::TDTConfig              include/psyne/protocol/tdt_compression.hpp:31-43
//   TDTCompressionProtocol::encode          :227-266
//   TDTCompressionProtocol::decode          :271-304
//   TDTCompressionProtocol::should_transform:186-201
//   TDTCompressionProtocol::update_*_metrics:309-319
//
// <functional> is included first because include/psyne/global/logger.hpp:347 uses
// std::function without including it; that is the only accommodation.
#include <functional>
#include <psyne/protocol/tdt_compression.hpp>

#include <pthread.h>
#include <sched.h>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

using psyne::protocol::TDTCompressionProtocol;
using psyne::protocol::TDTConfig;

namespace {
thread_local std::string g_last_error;

TDTConfig make_cfg(float sample_fraction, int word_size, size_t min_tensor_size) {
    TDTConfig c;
    c.sample_fraction = sample_fraction;
    c.word_size = word_size;
    c.min_tensor_size = min_tensor_size;
    return c;
}
} // namespace

extern "C" {

// Encode one message with a fresh protocol object.  bandwidth_mbps < 100 turns
// compression on (tdt_compression.hpp:200, :352).  Returns 0, or -2 if cap is too small.
int tdt_ref_encode(const uint8_t *data, size_t n, float sample_fraction, int word_size,
                   double bandwidth_mbps, double cpu_usage, size_t min_tensor_size,
                   uint8_t *out, size_t cap, size_t *out_len) {
    TDTCompressionProtocol p(make_cfg(sample_fraction, word_size, min_tensor_size));
    p.update_network_metrics(bandwidth_mbps, 1.0);
    p.update_system_metrics(cpu_usage);
    std::vector<uint8_t> blob = p.encode(const_cast<uint8_t *>(data), n);
    *out_len = blob.size();
    if (blob.size() > cap) return -2;
    std::memcpy(out, blob.data(), blob.size());
    return 0;
}

// Encode one message and report the reference's own transformation_ratio() (:329-331, set by
// compress_tdt :395-396 from encoded_size() :71-78) and whether processing_overhead_ms()
// (:332-334) changed (it does only on the compress path).
int tdt_ref_encode_ratio(const uint8_t *data, size_t n, float sample_fraction, int word_size,
                         double bandwidth_mbps, double *ratio, int *overhead_updated) {
    TDTCompressionProtocol p(make_cfg(sample_fraction, word_size, 1024));
    p.update_network_metrics(bandwidth_mbps, 1.0);
    const double before = p.processing_overhead_ms();
    std::vector<uint8_t> blob = p.encode(const_cast<uint8_t *>(data), n);
    *ratio = p.transformation_ratio();
    *overhead_updated = p.processing_overhead_ms() != before ? 1 : 0;
    return (int)blob.size();
}

int tdt_ref_should_transform(const uint8_t *data, size_t n, int word_size,
                             double bandwidth_mbps, double cpu_usage,
                             size_t min_tensor_size) {
    TDTCompressionProtocol p(make_cfg(0.3f, word_size, min_tensor_size));
    p.update_network_metrics(bandwidth_mbps, 1.0);
    p.update_system_metrics(cpu_usage);
    return p.should_transform(const_cast<uint8_t *>(data), n) ? 1 : 0;
}

// Decode one blob.  Returns 0, -1 on a reference exception (message via
// tdt_ref_last_error), -2 if cap is too small.  Callers must not pass blobs on which
// the reference has undefined behaviour (truncated headers/streams, bad mapping).
int tdt_ref_decode(const uint8_t *blob, size_t len, uint8_t *out, size_t cap,
                   size_t *out_len) {
    TDTCompressionProtocol p;
    std::vector<uint8_t> in(blob, blob + len);
    try {
        std::vector<uint8_t> r = p.decode(in);
        *out_len = r.size();
        if (r.size() > cap) return -2;
        if (!r.empty()) std::memcpy(out, r.data(), r.size());
        return 0;
    } catch (const std::exception &e) {
        g_last_error = e.what();
        *out_len = 0;
        return -1;
    }
}

const char *tdt_ref_last_error(void) { return g_last_error.c_str(); }

// A persistent protocol object (the loopback harness's CPU codec: one per endpoint, as a
// ProtocolChannel holds one, protocol_demo.cpp:105-216).
void *tdt_ref_new(float sample_fraction, int word_size, double bandwidth_mbps) {
    auto *p = new TDTCompressionProtocol(make_cfg(sample_fraction, word_size, 1024));
    p->update_network_metrics(bandwidth_mbps, 1.0);
    return p;
}
void tdt_ref_free(void *h) { delete static_cast<TDTCompressionProtocol *>(h); }
// Returns 0, -1 on a reference exception, -2 if cap is too small (out_len = needed).
int tdt_ref_encode_h(void *h, const uint8_t *data, size_t n, uint8_t *out, size_t cap, size_t *out_len) {
    std::vector<uint8_t> blob = static_cast<TDTCompressionProtocol *>(h)->encode(const_cast<uint8_t *>(data), n);
    *out_len = blob.size();
    if (blob.size() > cap) return -2;
    std::memcpy(out, blob.data(), blob.size());
    return 0;
}
int tdt_ref_decode_h(void *h, const uint8_t *blob, size_t len, uint8_t *out, size_t cap, size_t *out_len) {
    try {
        std::vector<uint8_t> r = static_cast<TDTCompressionProtocol *>(h)->decode(std::vector<uint8_t>(blob, blob + len));
        *out_len = r.size();
        if (r.size() > cap) return -2;
        if (!r.empty()) std::memcpy(out, r.data(), r.size());
        return 0;
    } catch (const std::exception &e) {
        g_last_error = e.what();
        *out_len = 0;
        return -1;
    }
}

// Timed CPU baseline: `threads` workers, one protocol object each (the reference object
// is not thread-safe, tdt_compression.hpp:349-360), messages statically interleaved.
// Each worker encodes then decodes every one of its messages `reps` times and checks
// the round trip.  Returns wall seconds (negative on a round-trip mismatch).
// cpus (optional, `threads` entries): worker t is pinned to CPU cpus[t] before it starts.
double tdt_ref_bench_pinned(const uint8_t *data, const uint64_t *off, uint32_t n_msgs,
                            float sample_fraction, int word_size, int threads, int reps,
                            uint64_t *encoded_bytes_out, const int *cpus) {
    if (threads < 1) threads = 1;
    std::vector<std::thread> pool;
    std::vector<uint64_t> enc_bytes(threads, 0);
    std::vector<int> bad(threads, 0);
    auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < threads; ++t) {
        pool.emplace_back([&, t]() {
            if (cpus) {
                cpu_set_t cs;
                CPU_ZERO(&cs);
                CPU_SET(cpus[t], &cs);
                pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
            }
            TDTCompressionProtocol p(make_cfg(sample_fraction, word_size, 1024));
            p.update_network_metrics(10.0, 1.0);
            for (int r = 0; r < reps; ++r) {
                for (uint32_t i = t; i < n_msgs; i += threads) {
                    size_t n = off[i + 1] - off[i];
                    uint8_t *m = const_cast<uint8_t *>(data + off[i]);
                    std::vector<uint8_t> blob = p.encode(m, n);
                    std::vector<uint8_t> back = p.decode(blob);
                    enc_bytes[t] += blob.size();
                    if (back.size() != n || std::memcmp(back.data(), m, n) != 0) bad[t] = 1;
                }
            }
        });
    }
    for (auto &th : pool) th.join();
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t tot = 0;
    int anybad = 0;
    for (int t = 0; t < threads; ++t) {
        tot += enc_bytes[t];
        anybad |= bad[t];
    }
    if (encoded_bytes_out) *encoded_bytes_out = tot;
    return anybad ? -s : s;
}

double tdt_ref_bench(const uint8_t *data, const uint64_t *off, uint32_t n_msgs,
                     float sample_fraction, int word_size, int threads, int reps,
                     uint64_t *encoded_bytes_out) {
    return tdt_ref_bench_pinned(data, off, n_msgs, sample_fraction, word_size, threads, reps,
                                encoded_bytes_out, nullptr);
}

} // extern "C"
