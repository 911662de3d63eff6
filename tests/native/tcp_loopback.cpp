// tcp_loopback.cpp — loopback TCP harness for the TDT substrate path (BASELINE.json configs[0]).
// Test/measurement infrastructure (its --codec cpu mode calls the compiled reference).
//
// Counterpart of the reference's benchmarks/tcp_tdt_benchmark.cpp (server :297-405, client
// :407-518): float32 "gradient" tensors of 256 Ki floats (1 MiB; 70 % exact zeros, the rest
// N(0, 0.01) — tcp_tdt_benchmark.cpp:52-66's GRADIENTS generator) cross a TCP connection on
// 127.0.0.1 as u32-length frames (tcp_simple.hpp:68-150).  Sender and receiver are two threads
// of one process, each with its own substrate end; the payloads are generated before the
// clock starts (the reference times its generator inside the loop, :342-360):
//
//   --codec gpu   TdtSubstrate<PosixTcpSubstrate> on both ends (each owns its socket end and a
//                 GPU codec context): batches of --batch tensors go through send_batch (encoded
//                 in sub-batches by tdt_encode_host_v, sent by the decorator's sender thread while
//                 the next sub-batch is on the GPU); the receiver takes --batch frames per
//                 receive_batch_views (--rx views, default: payloads checked where the decoder
//                 left them, in pinned memory) or receive_batch (--rx copy: into a vector); its
//                 receiver and decoder threads read and decode ahead
//   --codec cpu   the REFERENCE codec (psyne::protocol::TDTCompressionProtocol compiled where
//                 it lies: oracle/_ref/libtdt_ref.so, loaded at run time), one protocol object
//                 per endpoint, one message per encode / decode — psyne's own CPU path
//   --codec none  the same frames without compression (the transport's own ceiling)
//
// Every received payload is compared with the original.  --dump DIR writes inputs.bin (the
// tensors back to back) and frames.bin (u32 length + bytes per sent frame) so that a test can
// check every wire blob against the oracle.  Effective throughput = original bytes / wall time
// from the first send to the last verified receive (the reference's "Effective throughput ...
// MB/s (original)", :401-403), after an untimed warm-up pass of --warm batches (default 2: the
// first calls of each end allocate its workspaces and pinned staging).  --mem pinned puts the
// tensors in pinned host memory (as a channel's message buffers could be) for every row.
// --procs 2 runs the receiving end in a child process forked before anything touches the GPU, so
// each end has its own process, HIP context and hardware queues, as the two hosts' ends of a link
// would (they still share this host's GPU, PCIe link and cores); the child reports its end time
// (CLOCK_MONOTONIC, shared by both processes) and its mismatch count through a pipe.  --passes P
// repeats the timed pass P times back to back on the same connection (each pass's clock runs from
// its first send to its last verified receive; the next pass starts after that), and reports
// every pass's rate with their median, minimum and maximum: one pass of C1 is ~0.1 s of traffic,
// too short to tell two rows apart.  One JSON line on stdout.
#include <dlfcn.h>
#include <sys/prctl.h>
#include <sys/wait.h>
#include <unistd.h>

#include <csignal>

#include <psyne_amd/tdt_substrate.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

using namespace psyne_amd;

namespace {

// oracle/_ref/libtdt_ref.so (oracle/ref_shim.cpp), resolved next to this binary's repo root
struct RefCodec {
    void *lib = nullptr;
    void *(*make)(float, int, double) = nullptr;
    void (*release)(void *) = nullptr;
    int (*enc)(void *, const uint8_t *, size_t, uint8_t *, size_t, size_t *) = nullptr;
    int (*dec)(void *, const uint8_t *, size_t, uint8_t *, size_t, size_t *) = nullptr;
    bool load(const std::string &root) {
        lib = dlopen((root + "/oracle/_ref/libtdt_ref.so").c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!lib) return false;
        make = reinterpret_cast<decltype(make)>(dlsym(lib, "tdt_ref_new"));
        release = reinterpret_cast<decltype(release)>(dlsym(lib, "tdt_ref_free"));
        enc = reinterpret_cast<decltype(enc)>(dlsym(lib, "tdt_ref_encode_h"));
        dec = reinterpret_cast<decltype(dec)>(dlsym(lib, "tdt_ref_decode_h"));
        return make && release && enc && dec;
    }
};

std::string repo_root(const char *argv0) {
    std::string p = argv0;
    const size_t k = p.rfind("/tests/native/");
    return k == std::string::npos ? std::string(".") : p.substr(0, k);
}

}  // namespace

int main(int argc, char **argv) {
    size_t count = 1000, floats = 256 * 1024, batch = 50, warm = 2;
    // diagnostics of the gpu row's two halves: --half tx (the receiver drains raw frames: no
    // decode, no check) or --half rx (the sender sends frames encoded before the clock starts)
    std::string half = "both";
    // gpu receiver: "views" (receive_batch_views: payloads checked in the pipeline's pinned
    // buffers, zero-copy) or "copy" (receive_batch into a std::vector)
    std::string rxmode = "views";
    // the tensors' memory, for every row: "pageable" (std::vector, default) or "pinned"
    // (tdt_host_alloc: the GPU row's encode DMAs them directly instead of staging them)
    std::string mem = "pageable";
    int port = 18080, procs = 1;
    size_t passes = 1;
    std::string codec = "gpu", dump;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i], v = argv[i + 1];
        if (k == "--count") count = std::stoul(v);
        else if (k == "--floats") floats = std::stoul(v);
        else if (k == "--batch") batch = std::stoul(v);
        else if (k == "--port") port = std::stoi(v);
        else if (k == "--codec") codec = v;
        else if (k == "--dump") dump = v;
        else if (k == "--warm") warm = std::stoul(v);
        else if (k == "--half") half = v;
        else if (k == "--rx") rxmode = v;
        else if (k == "--mem") mem = v;
        else if (k == "--procs") procs = std::stoi(v);
        else if (k == "--passes") passes = std::max<size_t>(1, std::stoul(v));
    }
    // --procs 2: fork before any thread exists and before anything touches the GPU (pinned
    // payloads included); role "tx" = the parent (sender), "rx" = the child (receiver)
    std::string role = "both";
    int rep[2] = {-1, -1};
    pid_t child = -1;
    if (procs == 2) {
        if (half != "both") {
            std::fprintf(stderr, "--procs 2 runs both halves (no --half)\n");
            return 2;
        }
        if (::pipe(rep) != 0) {
            std::perror("pipe");
            return 2;
        }
        std::fflush(nullptr);
        const pid_t parent = ::getpid();
        child = ::fork();
        if (child < 0) {
            std::perror("fork");
            return 2;
        }
        // the receiving end never outlives the sending one (a parent that fails must not leave a
        // child blocked on its socket, and holding the GPU)
        if (child == 0 && (::prctl(PR_SET_PDEATHSIG, SIGKILL) != 0 || ::getppid() != parent)) std::_Exit(7);
        role = child == 0 ? "rx" : "tx";
        ::close(child == 0 ? rep[0] : rep[1]);
    }
    const size_t bytes = floats * 4;
    // payloads (GRADIENTS: 70 % zeros, N(0, 0.01) otherwise)
    std::vector<std::vector<uint8_t>> pageable(mem == "pinned" ? 0 : count, std::vector<uint8_t>(bytes));
    PinnedBuffer pinned;
    if (mem == "pinned") pinned.reserve(count * bytes);
    struct Msg {
        uint8_t *p;
        uint8_t *data() const { return p; }
    };
    std::vector<Msg> msgs(count);
    for (size_t i = 0; i < count; ++i) msgs[i].p = mem == "pinned" ? pinned.data() + i * bytes : pageable[i].data();
    {
        std::mt19937_64 rng(0x5EED0001);
        std::normal_distribution<float> nd(0.0f, 0.01f);
        std::uniform_real_distribution<float> u(0.0f, 1.0f);
        for (auto &m : msgs) {
            float *f = reinterpret_cast<float *>(m.data());
            for (size_t i = 0; i < floats; ++i) f[i] = u(rng) < 0.7f ? 0.0f : nd(rng);
        }
    }
    TDTConfig cfg;
    cfg.sample_fraction = 1.0f;
    // slow link: compression on (tdt_compression.hpp:192-200) for every codec context
    TdtSubstrate<PosixTcpSubstrate>::defaults().bandwidth_mbps = 10.0;

    std::unique_ptr<PosixTcpSubstrate> raw_rx, raw_tx;
    std::unique_ptr<TdtSubstrate<PosixTcpSubstrate>> rx, tx;
    PosixTcpSubstrate *rx_inner = nullptr, *tx_inner = nullptr;
    const bool has_rx = role != "tx", has_tx = role != "rx";
    if (codec == "gpu") {
        if (has_rx) {
            rx = std::make_unique<TdtSubstrate<PosixTcpSubstrate>>(cfg, "127.0.0.1", (uint16_t)port, true);
            rx_inner = &rx->inner();
        }
        if (has_tx) {
            tx = std::make_unique<TdtSubstrate<PosixTcpSubstrate>>(cfg, "127.0.0.1", (uint16_t)port, false);
            tx_inner = &tx->inner();
        }
    } else {
        if (has_rx) raw_rx = std::make_unique<PosixTcpSubstrate>("127.0.0.1", (uint16_t)port, true);
        if (has_tx) raw_tx = std::make_unique<PosixTcpSubstrate>("127.0.0.1", (uint16_t)port, false);
        rx_inner = raw_rx.get();
        tx_inner = raw_tx.get();
    }
    // (two processes: the other end may still be generating its payloads or starting its GPU)
    const std::chrono::milliseconds cwait(procs == 2 ? 60000 : 5000);
    if ((rx_inner && !rx_inner->wait_for_connection(cwait)) || (tx_inner && !tx_inner->wait_for_connection(cwait))) {
        std::fprintf(stderr, "connection failed\n");
        return 2;
    }
    RefCodec ref;
    void *ref_tx = nullptr, *ref_rx = nullptr;
    if (codec == "cpu") {
        if (!ref.load(repo_root(argv[0]))) {
            std::fprintf(stderr, "oracle/_ref/libtdt_ref.so not found (make -C oracle in the build container)\n");
            return 3;
        }
        ref_tx = ref.make(1.0f, 4, 10.0);
        ref_rx = ref.make(1.0f, 4, 10.0);
    }
    FILE *frames = nullptr;
    if (!dump.empty() && has_tx) {
        FILE *f = std::fopen((dump + "/inputs.bin").c_str(), "wb");
        for (auto &m : msgs) std::fwrite(m.data(), 1, bytes, f);
        std::fclose(f);
        frames = std::fopen((dump + "/frames.bin").c_str(), "wb");
    }

    std::vector<const void *> ptrs(batch);
    std::vector<size_t> sizes(batch, bytes);
    // --half rx: every batch's frames encoded (by the sender's codec) before the clock starts
    std::vector<std::vector<uint8_t>> pre;
    std::vector<std::vector<uint64_t>> pre_off;
    if (codec == "gpu" && half == "rx") {
        for (size_t b = 0; b < count; b += batch) {
            const size_t nb = std::min(batch, count - b);
            std::vector<const uint8_t *> mp(nb);
            std::vector<uint64_t> ms(nb, bytes), eo(nb + 1, 0);
            for (size_t i = 0; i < nb; ++i) mp[i] = msgs[b + i].data();
            std::vector<uint8_t> enc(nb * tdt_encode_bound(bytes, 4));
            std::vector<int32_t> est(nb);
            if (tdt_encode_host_v(tx->codec().context(), mp.data(), ms.data(), (uint32_t)nb, enc.data(), enc.size(),
                                  eo.data(), est.data()) != TDT_OK) {
                std::fprintf(stderr, "pre-encode failed: %s\n", tdt_last_error());
                return 5;
            }
            enc.resize(eo[nb]);
            pre.push_back(std::move(enc));
            pre_off.push_back(std::move(eo));
        }
    }
    std::vector<uint8_t> blob(tdt_encode_bound(bytes, 4));
    size_t wire = 0, mismatches = 0;
    // One pass: tensors [0, n) sent in batches and verified on receipt.  The warm-up pass (not
    // timed: context workspaces, pinned staging and plan histories are set up by the first calls
    // of each end) precedes the timed pass over all `count` tensors.
    // the receiving end's part of a pass over tensors [0, n)
    auto recv_part = [&](size_t n) {
        std::vector<uint8_t> out;
        std::vector<uint64_t> off;
        std::vector<uint8_t> frame(tdt_encode_bound(bytes, 4) + 64), back(bytes);
        for (size_t b = 0; b < n; b += batch) {
            const size_t nb = std::min(batch, n - b);
            if (codec == "gpu" && half == "tx") {
                for (size_t i = 0; i < nb; ++i) {
                    size_t flen = 0;
                    while (!rx_inner->try_transport_receive(frame.data(), frame.size(), flen)) std::this_thread::yield();
                }
                continue;
            }
            if (codec == "gpu" && rxmode == "views") {
                const auto v = rx->receive_batch_views(nb, bytes);
                for (size_t i = 0; i < nb; ++i)
                    if (v[i].status != TDT_OK || v[i].size != bytes || std::memcmp(v[i].data, msgs[b + i].data(), bytes))
                        ++mismatches;
                continue;
            }
            if (codec == "gpu") {
                const std::vector<int32_t> st = rx->receive_batch(nb, bytes, out, off);
                for (size_t i = 0; i < nb; ++i)
                    if (st[i] != TDT_OK || off[i + 1] - off[i] != bytes ||
                        std::memcmp(out.data() + off[i], msgs[b + i].data(), bytes))
                        ++mismatches;
                continue;
            }
            for (size_t i = 0; i < nb; ++i) {
                size_t flen = 0;
                while (!rx_inner->try_transport_receive(frame.data(), frame.size(), flen)) {
                    if (!rx_inner->is_connected()) {
                        ++mismatches;
                        return;
                    }
                    std::this_thread::yield();
                }
                const uint8_t *got = frame.data();
                size_t glen = flen;
                if (codec == "cpu") {
                    if (ref.dec(ref_rx, frame.data(), flen, back.data(), back.size(), &glen) != 0) glen = 0;
                    got = back.data();
                }
                if (glen != bytes || std::memcmp(got, msgs[b + i].data(), bytes)) ++mismatches;
            }
        }
    };
    // the sending end's part
    auto send_part = [&](size_t n, FILE *frames) {
    if (codec == "gpu") tx->record_last_batch(frames != nullptr || half == "rx");
    for (size_t b = 0; b < n; b += batch) {
        const size_t nb = std::min(batch, n - b);
        if (codec == "gpu" && half == "rx") {
            const std::vector<uint8_t> &enc = pre[b / batch];
            const std::vector<uint64_t> &eo = pre_off[b / batch];
            for (size_t i = 0; i < nb; ++i) tx_inner->transport_send((void *)(enc.data() + eo[i]), eo[i + 1] - eo[i]);
            wire += eo[nb];
            continue;
        }
        if (codec == "gpu") {
            for (size_t i = 0; i < nb; ++i) ptrs[i] = msgs[b + i].data();
            wire += tx->send_batch(ptrs.data(), sizes.data(), nb);
            if (frames) {
                const std::vector<uint8_t> &enc = tx->last_batch();
                const std::vector<uint64_t> &eo = tx->last_batch_offsets();
                for (size_t i = 0; i < nb; ++i) {
                    const uint32_t l = (uint32_t)(eo[i + 1] - eo[i]);
                    std::fwrite(&l, 4, 1, frames);
                    std::fwrite(enc.data() + eo[i], 1, l, frames);
                }
            }
            continue;
        }
        for (size_t i = 0; i < nb; ++i) {
            uint8_t *p = msgs[b + i].data();
            size_t len = bytes;
            if (codec == "cpu") {
                if (ref.enc(ref_tx, p, bytes, blob.data(), blob.size(), &len) != 0) {
                    std::fprintf(stderr, "reference encode failed\n");
                    std::_Exit(4);
                }
                p = blob.data();
            }
            tx_inner->transport_send(p, len);
            if (frames) {
                const uint32_t l = (uint32_t)len;
                std::fwrite(&l, 4, 1, frames);
                std::fwrite(p, 1, len, frames);
            }
            wire += len;
        }
    }
    if (codec == "gpu" && half != "rx") tx->flush();  // every queued frame is on the wire
    };
    auto pass = [&](size_t n, FILE *frames) {
        if (!has_tx) return recv_part(n);
        if (!has_rx) return send_part(n, frames);
        std::thread receiver([&] { recv_part(n); });
        send_part(n, frames);
        receiver.join();
    };
    // child → parent reports (--procs 2)
    struct Report {
        int64_t t_ns;  // CLOCK_MONOTONIC (steady_clock) time of the report
        uint64_t mismatches;
    };
    auto now_ns = [] {
        return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch())
            .count();
    };
    auto send_report = [&] {
        const Report r{now_ns(), (uint64_t)mismatches};
        return ::write(rep[1], &r, sizeof(r)) == (ssize_t)sizeof(r);
    };
    auto read_report = [&](Report &r) {
        size_t got = 0;
        while (got < sizeof(r)) {
            const ssize_t k = ::read(rep[0], reinterpret_cast<char *>(&r) + got, sizeof(r) - got);
            if (k <= 0) return false;
            got += (size_t)k;
        }
        return true;
    };
    if (warm) {
        pass(std::min(count, warm * batch), nullptr);
        wire = 0;
    }
    using PS = TdtSubstrate<PosixTcpSubstrate>::PipeStats;
    PS tx0{}, rx0{};
    if (codec == "gpu") {
        if (tx) tx0 = tx->pipe_stats();
        if (rx) rx0 = rx->pipe_stats();
    }
    if (role == "rx") {
        // warm-up done (the parent starts its clock on this report), then the timed passes, each
        // ended by a report
        if (!send_report()) return 6;
        bool ok = true;
        for (size_t k = 0; k < passes && ok; ++k) {
            pass(count, nullptr);
            ok = send_report();
        }
        if (codec == "gpu") {
            const PS r = rx->pipe_stats();
            std::fprintf(stderr,
                         "{\"pipe_rx\": {\"recv\": %.4f, \"rx_sleep\": %.4f, \"rx_wait\": %.4f, \"decode\": %.4f, "
                         "\"decode_calls\": %llu, \"decode_MB\": %.1f, \"dec_wait\": %.4f, \"deliver_wait\": %.4f}}\n",
                         r.recv - rx0.recv, r.rx_sleep - rx0.rx_sleep, r.rx_wait - rx0.rx_wait, r.decode - rx0.decode,
                         (unsigned long long)(r.decode_calls - rx0.decode_calls),
                         double(r.decode_bytes - rx0.decode_bytes) / 1e6, r.dec_wait - rx0.dec_wait,
                         r.deliver_wait - rx0.deliver_wait);
        }
        ::close(rep[1]);
        return !ok ? 6 : mismatches ? 1 : 0;
    }
    Report rr{};
    auto reap = [&]() -> int {  // the child's exit code (-1: abnormal)
        int ws = 0;
        if (::waitpid(child, &ws, 0) != child || !WIFEXITED(ws)) return -1;
        return WEXITSTATUS(ws);
    };
    if (role == "tx" && !read_report(rr)) {
        std::fprintf(stderr, "receiver process ended during the warm-up (exit %d)\n", reap());
        return 6;
    }
    std::vector<double> pass_secs;
    for (size_t k = 0; k < passes; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        pass(count, k == 0 ? frames : nullptr);
        double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (role == "tx") {
            // the receiving end's last verified receive of the pass ends its clock
            if (!read_report(rr)) {
                std::fprintf(stderr, "receiver process ended without its report (exit %d)\n", reap());
                return 6;
            }
            secs = (double)(rr.t_ns - std::chrono::duration_cast<std::chrono::nanoseconds>(t0.time_since_epoch()).count()) *
                   1e-9;
            mismatches = (size_t)rr.mismatches;
        }
        pass_secs.push_back(secs);
    }
    double secs = 0;
    for (double x : pass_secs) secs += x;
    if (role == "tx") {
        const int code = reap();
        if (code != 0 && code != 1) {
            std::fprintf(stderr, "receiver process exit %d\n", code);
            return 6;
        }
    }
    if (frames) std::fclose(frames);
    if (ref_tx) ref.release(ref_tx);
    if (ref_rx) ref.release(ref_rx);
    const double orig1 = double(count) * double(bytes), orig = orig1 * double(passes);
    // per-pass rates, their median / min / max; effective_MBps is the median pass
    std::vector<double> rate;
    for (double x : pass_secs) rate.push_back(orig1 / 1e6 / x);
    std::vector<double> sorted = rate;
    std::sort(sorted.begin(), sorted.end());
    const size_t P = sorted.size();
    const double median = P % 2 ? sorted[P / 2] : 0.5 * (sorted[P / 2 - 1] + sorted[P / 2]);
    std::string rates = "[";
    for (size_t k = 0; k < P; ++k) rates += (k ? ", " : "") + std::to_string((long long)(rate[k] + 0.5));
    rates += "]";
    std::printf("{\"harness\": \"tcp_loopback\", \"codec\": \"%s\", \"tensors\": %zu, \"tensor_bytes\": %zu, "
                "\"batch\": %zu, \"passes\": %zu, \"seconds\": %.4f, \"original_MB\": %.1f, \"wire_MB\": %.1f, "
                "\"compression_ratio\": %.4f, \"effective_MBps\": %.1f, \"min_MBps\": %.1f, \"max_MBps\": %.1f, "
                "\"pass_MBps\": %s, \"network_MBps\": %.1f, "
                "\"mismatches\": %zu, \"warmup_tensors\": %zu, \"half\": \"%s\", \"rx\": \"%s\", \"mem\": \"%s\", "
                "\"procs\": %d}\n",
                codec.c_str(), count, bytes, codec == "gpu" ? batch : (size_t)1, P, secs, orig / 1e6,
                double(wire) / 1e6, orig / double(wire), median, sorted.front(), sorted.back(), rates.c_str(),
                double(wire) / 1e6 / secs, mismatches, warm ? std::min(count, warm * batch) : (size_t)0, half.c_str(),
                codec == "gpu" ? rxmode.c_str() : "-", mem.c_str(), procs == 2 ? 2 : 1);
    if (codec == "gpu" && role == "tx") {
        const PS t = tx->pipe_stats();
        std::fprintf(stderr,
                     "{\"pipe_tx\": {\"encode\": %.4f, \"encode_calls\": %llu, \"tx_wait\": %.4f, \"send\": %.4f}}\n",
                     t.encode - tx0.encode, (unsigned long long)(t.encode_calls - tx0.encode_calls), t.tx_wait - tx0.tx_wait,
                     t.send - tx0.send);
    } else if (codec == "gpu") {
        // where the pipeline threads spent the timed pass (seconds)
        const PS t = tx->pipe_stats(), r = rx->pipe_stats();
        std::fprintf(stderr,
                     "{\"pipe\": {\"encode\": %.4f, \"encode_calls\": %llu, \"tx_wait\": %.4f, \"send\": %.4f, "
                     "\"recv\": %.4f, \"rx_sleep\": %.4f, \"rx_wait\": %.4f, \"decode\": %.4f, \"decode_calls\": %llu, "
                     "\"decode_MB\": %.1f, \"dec_wait\": %.4f, \"deliver_wait\": %.4f}}\n",
                     t.encode - tx0.encode, (unsigned long long)(t.encode_calls - tx0.encode_calls), t.tx_wait - tx0.tx_wait,
                     t.send - tx0.send, r.recv - rx0.recv, r.rx_sleep - rx0.rx_sleep, r.rx_wait - rx0.rx_wait,
                     r.decode - rx0.decode, (unsigned long long)(r.decode_calls - rx0.decode_calls),
                     double(r.decode_bytes - rx0.decode_bytes) / 1e6, r.dec_wait - rx0.dec_wait,
                     r.deliver_wait - rx0.deliver_wait);
    }
    return mismatches ? 1 : 0;
}
