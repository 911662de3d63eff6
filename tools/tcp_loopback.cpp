// tcp_loopback.cpp — loopback TCP harness for the TDT substrate path (BASELINE.json configs[0]).
//
// Counterpart of the reference's benchmarks/tcp_tdt_benchmark.cpp (server :297-405, client
// :407-518): 1000 float32 "gradient" tensors of 256 Ki floats (1 MiB; 70 % exact zeros, the
// rest N(0, 0.01) — tcp_tdt_benchmark.cpp:52-66's GRADIENTS generator) cross a TCP connection
// on 127.0.0.1.  Here the sender and the receiver are two threads of one process, each with
// its own PosixTcpSubstrate end and its own GPU codec context:
//
//   --codec gpu   TdtSubstrate<PosixTcpSubstrate>: batches of --batch tensors are encoded by
//                 one tdt_encode_host call, sent as one frame per blob, received, decoded by one
//                 tdt_decode_host call and checked byte for byte against the originals
//   --codec none  the same frames without compression (the transport's own ceiling)
//
// Effective throughput = original bytes / wall time from the first send to the last verified
// receive (the reference's "Effective throughput ... MB/s (original)", :401-403).  One JSON
// line on stdout.
//
// build: g++ -std=c++20 -O2 -Iinclude tools/tcp_loopback.cpp -Lpsyne_amd -lpsyne_tdt -pthread
#include <psyne_amd/tdt_substrate.hpp>

#include <chrono>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

using namespace psyne_amd;

int main(int argc, char **argv) {
    size_t count = 1000, floats = 256 * 1024, batch = 50;
    int port = 18080;
    std::string codec = "gpu";
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i], v = argv[i + 1];
        if (k == "--count") count = std::stoul(v);
        else if (k == "--floats") floats = std::stoul(v);
        else if (k == "--batch") batch = std::stoul(v);
        else if (k == "--port") port = std::stoi(v);
        else if (k == "--codec") codec = v;
    }
    const size_t bytes = floats * 4;
    // payloads (GRADIENTS: 70 % zeros, N(0, 0.01) otherwise)
    std::vector<std::vector<uint8_t>> msgs(count, std::vector<uint8_t>(bytes));
    {
        std::mt19937_64 rng(0x5EED0001);
        std::normal_distribution<float> nd(0.0f, 0.01f);
        std::uniform_real_distribution<float> u(0.0f, 1.0f);
        for (auto &m : msgs) {
            float *f = reinterpret_cast<float *>(m.data());
            for (size_t i = 0; i < floats; ++i) f[i] = u(rng) < 0.7f ? 0.0f : nd(rng);
        }
    }
    const bool gpu = codec == "gpu";
    PosixTcpSubstrate server("127.0.0.1", (uint16_t)port, true);
    PosixTcpSubstrate client("127.0.0.1", (uint16_t)port, false);
    if (!server.wait_for_connection() || !client.wait_for_connection()) {
        std::fprintf(stderr, "connection failed\n");
        return 2;
    }
    TDTConfig cfg;
    cfg.sample_fraction = 1.0f;
    std::unique_ptr<HipTDTCompressionProtocol> enc_codec, dec_codec;
    std::unique_ptr<TdtSubstrate<PosixTcpSubstrate>> txp, rxp;
    if (gpu) {
        enc_codec = std::make_unique<HipTDTCompressionProtocol>(cfg);
        dec_codec = std::make_unique<HipTDTCompressionProtocol>(cfg);
        enc_codec->update_network_metrics(10.0, 1.0);  // slow link: compression on (:192-200)
        dec_codec->update_network_metrics(10.0, 1.0);
        txp = std::make_unique<TdtSubstrate<PosixTcpSubstrate>>(client, *enc_codec);
        rxp = std::make_unique<TdtSubstrate<PosixTcpSubstrate>>(server, *dec_codec);
    }

    size_t wire = 0, mismatches = 0;
    const auto t0 = std::chrono::steady_clock::now();
    std::thread receiver([&] {
        std::vector<uint8_t> out;
        std::vector<uint64_t> off;
        std::vector<uint8_t> raw(bytes + 64);
        for (size_t b = 0; b < count; b += batch) {
            const size_t nb = std::min(batch, count - b);
            if (gpu) {
                rxp->receive_batch(nb, bytes, out, off);
                for (size_t i = 0; i < nb; ++i)
                    if (off[i + 1] - off[i] != bytes || std::memcmp(out.data() + off[i], msgs[b + i].data(), bytes))
                        ++mismatches;
            } else {
                for (size_t i = 0; i < nb; ++i) {
                    server.transport_receive(raw.data(), raw.size());
                    if (server.last_received_size() != bytes || std::memcmp(raw.data(), msgs[b + i].data(), bytes))
                        ++mismatches;
                }
            }
        }
    });
    std::vector<const void *> ptrs(batch);
    std::vector<size_t> sizes(batch, bytes);
    for (size_t b = 0; b < count; b += batch) {
        const size_t nb = std::min(batch, count - b);
        if (gpu) {
            for (size_t i = 0; i < nb; ++i) ptrs[i] = msgs[b + i].data();
            wire += txp->send_batch(ptrs.data(), sizes.data(), nb);
        } else {
            for (size_t i = 0; i < nb; ++i) client.transport_send(msgs[b + i].data(), bytes);
            wire += nb * bytes;
        }
    }
    receiver.join();
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double orig = double(count) * double(bytes);
    std::printf("{\"harness\": \"tcp_loopback\", \"codec\": \"%s\", \"tensors\": %zu, \"tensor_bytes\": %zu, "
                "\"batch\": %zu, \"seconds\": %.4f, \"original_MB\": %.1f, \"wire_MB\": %.1f, "
                "\"compression_ratio\": %.4f, \"effective_MBps\": %.1f, \"network_MBps\": %.1f, "
                "\"mismatches\": %zu}\n",
                codec.c_str(), count, bytes, batch, secs, orig / 1e6, double(wire) / 1e6, orig / double(wire),
                orig / 1e6 / secs, double(wire) / 1e6 / secs, mismatches);
    return mismatches ? 1 : 0;
}
