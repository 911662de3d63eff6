// tdt_substrate.hpp — the TCP substrate path with TDT payload compression on the GPU.
//
// psyne's network substrate (reference include/psyne/channel/substrate/tcp_simple.hpp) frames
// every message as a u32 length followed by the payload (transport_send :68-91,
// transport_receive :96-150, try_transport_receive :153-194); docs/tdt_attribution.md:62-75
// describes the intended TDT-over-IP substrate: payloads compressed before the socket and
// restored after it.  This header provides both halves for an MI355X host:
//
//   * PosixTcpSubstrate — SimpleTCP's public surface (allocate/deallocate slab,
//     transport_send/receive, try_transport_receive, identity, statistics, wait_for_connection)
//     over blocking POSIX sockets (the image has no Boost.Asio): byte-identical framing and the
//     reference's error texts.  Nothing beyond SimpleTCP's method set.
//   * TdtSubstrate<Inner, Base> — a substrate in the shape of psyne's SubstrateBehavior
//     (core/behaviors.hpp:32-48) that decorates any Inner with SimpleTCP's surface: it OWNS the
//     inner substrate and a GPU codec (HipTDTCompressionProtocol), is default-constructible as
//     ChannelBridge requires (behaviors.hpp:150: std::make_unique<SubstrateType>()),
//     transport_send encodes and sends one frame, transport_receive(void*, size_t) blocks until
//     one frame has arrived and decodes it into the buffer.  Frame lengths come from Inner's
//     try_transport_receive(buf, cap, received_size) (tcp_simple.hpp:153-194) — the only
//     receive that reports a length.  A frame is checked against the buffer BEFORE decoding:
//     its header's decoded size (UNCP: len - 4, TDT: original_size) must fit, so a crafted
//     header cannot make the receiver allocate or decode beyond buffer_size.
//     Base: the vtable to implement — psyne::behaviors::SubstrateBehavior in a psyne build
//     (every method here matches its signature, so it overrides), an empty struct otherwise.
//     send_batch / receive_batch move many messages per GPU call through the C ABI host
//     pipeline (tdt_encode_host_v / tdt_decode_host: chunked, H2D / kernel / D2H of neighbouring
//     chunks overlapped over four pipeline slots on two streams) with a sender and a receiver thread overlapping
//     the socket with the codec,
//     which is how the codec reaches the link's rate instead of per-message latency.
#pragma once

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <psyne_amd/hip_tdt_protocol.hpp>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace psyne_amd {

class PosixTcpSubstrate {
public:
    // host: bind address (server) or remote host (client); as SimpleTCP(host, port, is_server)
    explicit PosixTcpSubstrate(const std::string &host = "localhost", uint16_t port = 8080, bool is_server = false)
        : host_(host), port_(port), is_server_(is_server) {
        if (is_server_) {
            listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
            if (listen_fd_ < 0) throw std::runtime_error("TCP initialization failed: socket");
            int one = 1;
            ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
            sockaddr_in a{};
            a.sin_family = AF_INET;
            a.sin_port = htons(port_);
            a.sin_addr.s_addr = htonl(INADDR_ANY);
            if (::bind(listen_fd_, reinterpret_cast<sockaddr *>(&a), sizeof(a)) != 0 || ::listen(listen_fd_, 1) != 0) {
                ::close(listen_fd_);
                throw std::runtime_error("TCP initialization failed: bind/listen on port " + std::to_string(port_));
            }
            accept_thread_ = std::thread([this] {
                const int fd = ::accept(listen_fd_, nullptr, nullptr);
                if (fd >= 0) adopt(fd);
            });
        } else {
            connect_thread_ = std::thread([this] {
                for (int attempt = 0; attempt < 200 && !stop_.load(); ++attempt) {
                    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
                    sockaddr_in a{};
                    a.sin_family = AF_INET;
                    a.sin_port = htons(port_);
                    if (::inet_pton(AF_INET, host_ == "localhost" ? "127.0.0.1" : host_.c_str(), &a.sin_addr) == 1 &&
                        ::connect(fd, reinterpret_cast<sockaddr *>(&a), sizeof(a)) == 0) {
                        adopt(fd);
                        return;
                    }
                    ::close(fd);
                    std::this_thread::sleep_for(std::chrono::milliseconds(100));  // retry as :311-318
                }
            });
        }
    }
    ~PosixTcpSubstrate() { shutdown(); }
    PosixTcpSubstrate(const PosixTcpSubstrate &) = delete;
    PosixTcpSubstrate &operator=(const PosixTcpSubstrate &) = delete;

    // MEMORY OWNERSHIP (:47-62)
    void *allocate_memory_slab(size_t size_bytes) {
        void *p = std::aligned_alloc(64, (size_bytes + 63) / 64 * 64);
        if (!p) throw std::bad_alloc();
        slab_size_ = size_bytes;
        return p;
    }
    void deallocate_memory_slab(void *memory) { std::free(memory); }

    // TRANSPORT (:68-91): u32 length, then the bytes
    void transport_send(void *data, size_t size) {
        if (!is_connected()) throw std::runtime_error("TCP: Not connected");
        std::lock_guard<std::mutex> lk(smu_);
        const uint32_t hdr = static_cast<uint32_t>(size);
        if (!write_all(&hdr, sizeof(hdr)) || !write_all(data, size)) {
            connected_.store(false);
            throw std::runtime_error("TCP send failed: connection lost");
        }
        bytes_sent_ += size + sizeof(hdr);
        packets_sent_++;
    }

    // (:96-150) one frame into buffer (the caller learns no length: SubstrateBehavior's shape)
    void transport_receive(void *buffer, size_t buffer_size) {
        if (!is_connected()) throw std::runtime_error("TCP: Not connected");
        std::lock_guard<std::mutex> lk(rmu_);
        uint32_t hdr = 0;
        if (!read_all(&hdr, sizeof(hdr))) fail("TCP receive failed: connection lost");
        if (hdr == 0) throw std::runtime_error("TCP receive failed: TCP: Received empty message");
        if (hdr > buffer_size) {
            close_socket();
            throw std::runtime_error("TCP receive failed: TCP: Received message too large (" + std::to_string(hdr) +
                                     " > " + std::to_string(buffer_size) + ")");
        }
        if (hdr > kMaxReasonable) {
            close_socket();
            throw std::runtime_error("TCP receive failed: TCP: Suspicious message size detected");
        }
        if (!read_all(buffer, hdr)) fail("TCP receive failed: connection lost");
        bytes_received_ += hdr + sizeof(hdr);
        packets_received_++;
    }

    // The length word of the next frame, if it has arrived (nothing is consumed): lets a reader
    // size its buffer before try_transport_receive, which drops the connection on a frame
    // larger than the buffer it is given.
    bool peek_frame_length(size_t &len) {
        if (!is_connected()) return false;
        std::lock_guard<std::mutex> lk(rmu_);
        uint32_t hdr = 0;
        const ssize_t got = ::recv(fd_, &hdr, sizeof(hdr), MSG_PEEK | MSG_DONTWAIT);
        if (got < (ssize_t)sizeof(hdr)) return false;
        len = hdr;
        return true;
    }

    // (:153-194) non-blocking probe: a frame is read only when its length word has arrived;
    // like SimpleTCP it never throws (an oversized frame or a failed read drops the connection
    // and returns false)
    bool try_transport_receive(void *buffer, size_t buffer_size, size_t &received_size) {
        if (!is_connected()) return false;
        std::lock_guard<std::mutex> lk(rmu_);
        uint32_t hdr = 0;
        const ssize_t got = ::recv(fd_, &hdr, sizeof(hdr), MSG_PEEK | MSG_DONTWAIT);
        if (got < (ssize_t)sizeof(hdr)) return false;
        if (!read_all(&hdr, sizeof(hdr))) return fail_quiet();
        if (hdr > buffer_size) {  // "TCP: Received message too large for buffer", caught :189-191
            close_socket();
            return false;
        }
        if (!read_all(buffer, hdr)) return fail_quiet();
        received_size = hdr;
        bytes_received_ += hdr + sizeof(hdr);
        packets_received_++;
        return true;
    }

    // SUBSTRATE IDENTITY (:199-207)
    const char *substrate_name() const { return "PosixTCP"; }
    bool is_zero_copy() const { return false; }
    bool is_cross_process() const { return true; }

    bool is_connected() const { return connected_.load(); }
    bool wait_for_connection(std::chrono::milliseconds timeout = std::chrono::milliseconds(5000)) {
        const auto t0 = std::chrono::steady_clock::now();
        while (!is_connected() && std::chrono::steady_clock::now() - t0 < timeout)
            std::this_thread::sleep_for(std::chrono::milliseconds(10));
        return is_connected();
    }
    size_t get_bytes_sent() const { return bytes_sent_; }
    size_t get_bytes_received() const { return bytes_received_; }
    size_t get_packets_sent() const { return packets_sent_; }
    size_t get_packets_received() const { return packets_received_; }
    const std::string &get_host() const { return host_; }
    // shut the connection down (unblocks a thread inside a send or receive); the destructor joins
    void close() { close_socket(); }
    uint16_t get_port() const { return port_; }
    bool is_server_mode() const { return is_server_; }

private:
    static constexpr size_t kMaxReasonable = 100ull * 1024 * 1024;  // :127-134

    void adopt(int fd) {
        int one = 1;
        ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        int buf = 8 << 20;
        ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
        ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
        fd_ = fd;
        connected_.store(true);
    }
    bool write_all(const void *p, size_t n) {
        const char *c = static_cast<const char *>(p);
        while (n) {
            const ssize_t w = ::send(fd_, c, n, MSG_NOSIGNAL);
            if (w <= 0) return false;
            c += w;
            n -= (size_t)w;
        }
        return true;
    }
    bool read_all(void *p, size_t n) {
        char *c = static_cast<char *>(p);
        while (n) {
            const ssize_t r = ::recv(fd_, c, n, 0);
            if (r <= 0) return false;
            c += r;
            n -= (size_t)r;
        }
        return true;
    }
    [[noreturn]] void fail(const char *what) {
        connected_.store(false);
        throw std::runtime_error(what);
    }
    bool fail_quiet() {
        connected_.store(false);
        return false;
    }
    void close_socket() {
        connected_.store(false);
        if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
    }
    void shutdown() {
        stop_.store(true);
        connected_.store(false);
        if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
        if (listen_fd_ >= 0) ::shutdown(listen_fd_, SHUT_RDWR);
        if (accept_thread_.joinable()) accept_thread_.join();
        if (connect_thread_.joinable()) connect_thread_.join();
        if (fd_ >= 0) ::close(fd_);
        if (listen_fd_ >= 0) ::close(listen_fd_);
        fd_ = listen_fd_ = -1;
    }

    std::string host_;
    uint16_t port_;
    bool is_server_;
    int fd_ = -1, listen_fd_ = -1;
    std::thread accept_thread_, connect_thread_;
    std::atomic<bool> connected_{false}, stop_{false};
    std::mutex smu_, rmu_;  // one sender and one receiver at a time (the two directions are independent)
    size_t slab_size_ = 0;
    size_t bytes_sent_ = 0, bytes_received_ = 0, packets_sent_ = 0, packets_received_ = 0;
};

// Decoded size a blob's header claims (decode :271-304): UNCP → len - 4, TDT → original_size;
// -1 when the header is unreadable (the decode then reports the reference's error).
inline int64_t tdt_claimed_size(const uint8_t *blob, size_t len) {
    if (len < 4) return -1;
    uint32_t magic;
    std::memcpy(&magic, blob, 4);
    if (magic == 0x554E4350u) return (int64_t)len - 4;
    if (magic != 0x54445444u || len < 8) return -1;
    uint32_t orig;
    std::memcpy(&orig, blob + 4, 4);
    return (int64_t)orig;
}


struct NoSubstrateBase {};

// Pinned (page-locked) host buffer from the codec library (tdt_host_alloc): the host pipeline
// DMAs it directly (no staging copy).
class PinnedBuffer {
public:
    PinnedBuffer() = default;
    ~PinnedBuffer() { tdt_host_free(p_); }
    PinnedBuffer(const PinnedBuffer &) = delete;
    PinnedBuffer &operator=(const PinnedBuffer &) = delete;
    // (contents are not kept; a growth takes 1.5x and whole 2 MiB: pinning tens of MB costs
    // milliseconds, so a buffer should grow rarely)
    void reserve(size_t bytes) {
        if (bytes <= cap_) return;
        const size_t want = std::max(bytes, cap_ + cap_ / 2);
        const size_t cap = (want + (2u << 20) - 1) & ~size_t((2u << 20) - 1);
        tdt_host_free(p_);
        p_ = nullptr;
        cap_ = 0;
        void *q = nullptr;
        if (tdt_host_alloc(cap, &q) != TDT_OK) throw std::bad_alloc();
        p_ = static_cast<uint8_t *>(q);
        cap_ = cap;
    }
    uint8_t *data() { return p_; }
    size_t capacity() const { return cap_; }

private:
    uint8_t *p_ = nullptr;
    size_t cap_ = 0;
};

// Decorator: TDT payload compression on the GPU between the channel and a framed substrate.
//
// Batches are pipelined (docs/tdt_attribution.md:62-75's intent; tcp_simple.hpp:68-91 framing):
//  * send_batch encodes its messages in sub-batches (tdt_encode_host_v: the caller's buffers are
//    gathered straight into pinned staging, no packing copy) into a ring of pinned output
//    buffers; a sender thread writes each finished sub-batch's frames to Inner while the next
//    sub-batch is on the GPU.  It returns once its messages are encoded (the caller may reuse
//    them); frames leave in order; flush() waits until every queued frame is on the wire.
//  * receiving runs as three stages once receive_batch has started them: a receiver thread reads
//    frames from Inner into a ring of pinned buffers (sealing one when it is full or the socket
//    has nothing more for now), a decoder thread decodes each sealed buffer on the GPU (direct
//    H2D from the pinned frames, D2H into a pinned payload buffer), and receive_batch hands the
//    decoded payloads to the caller (parallel copy) — socket, GPU and the caller's copy overlap.
template <class Inner, class Base = NoSubstrateBase>
class TdtSubstrate : public Base {
public:
    // Codec configuration of default-constructed decorators (ChannelBridge builds its substrate
    // with `std::make_unique<SubstrateType>()`); the reference's own defaults otherwise
    // (bandwidth 100 Mbps = passthrough, tdt_compression.hpp:39-40, :352).
    struct Defaults {
        TDTConfig config{};
        double bandwidth_mbps = 100.0;
        double latency_ms = 1.0;
        int device = 0;
    };
    static Defaults &defaults() {
        static Defaults d;
        return d;
    }

    TdtSubstrate() : TdtSubstrate(defaults().config) {}
    // inner_args: Inner's constructor arguments (SimpleTCP(host, port, is_server))
    template <class... InnerArgs>
    explicit TdtSubstrate(const TDTConfig &cfg, InnerArgs &&...inner_args)
        : inner_(std::forward<InnerArgs>(inner_args)...), codec_(cfg, defaults().device) {
        codec_.update_network_metrics(defaults().bandwidth_mbps, defaults().latency_ms);
        name_ = std::string("TDT+") + inner_.substrate_name();
    }
    ~TdtSubstrate() {
        // queued frames get a bounded wait to leave (a peer that stopped reading would otherwise
        // block the destructor for ever); then Inner is closed, which ends a send stuck inside it
        try {
            if (tx_thread_.joinable()) {
                std::unique_lock<std::mutex> lk(tx_mu_);
                tx_cv_.wait_for(lk, std::chrono::seconds(5), [&] { return tx_queue_.empty() && !tx_busy_; });
            }
        } catch (...) {
        }
        {
            std::lock_guard<std::mutex> lk(tx_mu_);
            tx_stop_ = true;
        }
        tx_cv_.notify_all();
        {
            std::lock_guard<std::mutex> lk(rx_mu_);
            rx_stop_ = true;
        }
        rx_cv_.notify_all();
        if constexpr (requires(Inner &s) { s.close(); }) {
            // (the receiver may sit inside a read, the sender inside a write)
            if (rx_thread_.joinable() || tx_thread_.joinable()) inner_.close();
        }
        if (tx_thread_.joinable()) tx_thread_.join();
        if (rx_thread_.joinable()) rx_thread_.join();
        if (dec_thread_.joinable()) dec_thread_.join();
    }
    TdtSubstrate(const TdtSubstrate &) = delete;
    TdtSubstrate &operator=(const TdtSubstrate &) = delete;

    Inner &inner() { return inner_; }
    HipTDTCompressionProtocol &codec() { return codec_; }

    // MEMORY OWNERSHIP
    void *allocate_memory_slab(size_t n) { return inner_.allocate_memory_slab(n); }
    void deallocate_memory_slab(void *p) { inner_.deallocate_memory_slab(p); }

    // TRANSPORT: one message = one frame (UNCP when the policy is off, exactly as
    // TDTCompressionProtocol::encode :227-266); after any queued batch frames
    void transport_send(void *data, size_t size) {
        if (tx_thread_.joinable()) flush();
        std::vector<uint8_t> blob = codec_.encode(data, size);
        inner_.transport_send(blob.data(), blob.size());
        raw_sent_ += size;
        wire_sent_ += blob.size();
    }

    // Blocks until one frame has arrived, decodes it into buffer (its decoded size:
    // last_received_size()).  Throws the reference's decode errors (:274-276, :127-129), the
    // inner substrate's "TCP: Not connected", or "TDT: decoded message larger than the buffer".
    void transport_receive(void *buffer, size_t buffer_size) {
        size_t got = 0;
        auto pause = std::chrono::microseconds(1);
        while (!try_transport_receive(buffer, buffer_size, got)) {
            if constexpr (requires(Inner &s) { s.is_connected(); }) {
                if (!inner_.is_connected() && !frames_pending()) throw std::runtime_error("TCP: Not connected");
            }
            std::this_thread::sleep_for(pause);
            if (pause < std::chrono::microseconds(200)) pause *= 2;
        }
    }

    // (tcp_simple.hpp:153-194 shape) false when no frame is waiting; otherwise one frame is
    // taken (from Inner, or from the receive pipeline once receive_batch started it), checked,
    // decoded into buffer, and its decoded size returned.
    bool try_transport_receive(void *buffer, size_t buffer_size, size_t &received_size) {
        if (rx_thread_.joinable()) {
            release_views();
            std::unique_lock<std::mutex> lk(rx_mu_);
            // (an error is reported once every frame that arrived before it is delivered)
            if (rx_err_ && rx_drained()) std::rethrow_exception(rx_err_);
            RxBuf *b = rx_front_decoded();
            if (!b) return false;
            const size_t k = b->used;
            rx_consume(1);  // (the frame's payload stays put until its buffer is refilled: see rx_consume)
            const int64_t claimed = b->claim[k];
            int32_t st = b->st[k];
            uint64_t n = b->doff[k + 1] - b->doff[k];
            if (claimed > (int64_t)buffer_size) {
                rx_release_if_done(b);
                lk.unlock();
                rx_cv_.notify_all();
                throw std::runtime_error("TDT: decoded message larger than the buffer");
            }
            if (claimed > (int64_t)b->lim) {
                // over the decoder's limit (the largest max_msg of a receive_batch call) but
                // within this caller's buffer: decoded now, as receive_batch does
                const uint64_t fo[2] = {b->off[k], b->off[k + 1]};
                uint64_t oo[2] = {0, 0};
                st = TDT_OK;
                const int rc = tdt_decode_host(codec_.context(), b->mem.data(), fo, 1, static_cast<uint8_t *>(buffer),
                                               (uint64_t)buffer_size, oo, &st);
                n = oo[1];
                rx_release_if_done(b);
                lk.unlock();
                rx_cv_.notify_all();
                if (rc != TDT_OK) throw std::runtime_error(std::string("TDT: GPU decode failed: ") + tdt_last_error());
                if (st != TDT_OK) throw std::runtime_error(tdt_status_string(st));
                received_size = n;
                last_received_ = n;
                return true;
            }
            if (st == TDT_OK && n) std::memcpy(buffer, b->dec.data() + b->doff[k], n);
            rx_release_if_done(b);
            lk.unlock();
            rx_cv_.notify_all();
            if (st != TDT_OK) throw std::runtime_error(tdt_status_string(st));
            received_size = n;
            last_received_ = n;
            return true;
        }
        stage_.resize(frame_capacity(buffer_size));
        size_t flen = 0;
        if (!inner_.try_transport_receive(stage_.data(), stage_.size(), flen)) return false;
        const int64_t claimed = tdt_claimed_size(stage_.data(), flen);
        if (claimed > (int64_t)buffer_size) throw std::runtime_error("TDT: decoded message larger than the buffer");
        // decode straight into the caller's buffer (GPU, C-ABI host path); no allocation sized by the frame
        const uint64_t off[2] = {0, flen};
        uint64_t ooff[2] = {0, 0};
        int32_t st = 0;
        if (tdt_decode_host(codec_.context(), stage_.data(), off, 1, static_cast<uint8_t *>(buffer), buffer_size,
                            ooff, &st) != TDT_OK)
            throw std::runtime_error(std::string("TDT: GPU decode failed: ") + tdt_last_error());
        if (st != TDT_OK) throw std::runtime_error(tdt_status_string(st));
        received_size = ooff[1];
        last_received_ = received_size;
        return true;
    }

    // SUBSTRATE IDENTITY
    const char *substrate_name() const { return name_.c_str(); }
    bool is_zero_copy() const { return false; }
    bool is_cross_process() const { return inner_.is_cross_process(); }

    // EXTENSIONS ----------------------------------------------------------------------------
    size_t last_received_size() const { return last_received_; }
    // wire bytes / payload bytes sent so far
    double wire_ratio() const { return raw_sent_ ? double(wire_sent_) / double(raw_sent_) : 1.0; }
    // keep a copy of each send_batch's blobs for last_batch() (tests; off by default)
    void record_last_batch(bool on) { record_last_ = on; }

    // Where the pipeline's threads spent their time (seconds, cumulative; diagnostics).
    struct PipeStats {
        double encode = 0, tx_wait = 0;             // caller: encode calls / waiting for a tx buffer
        double send = 0;                            // sender thread: socket writes
        double recv = 0, rx_sleep = 0, rx_wait = 0; // receiver thread: filling / polling pauses / no free buffer
        double decode = 0, dec_wait = 0;            // decoder thread: decode calls / idle
        double deliver_wait = 0;                    // caller: waiting for decoded frames
        uint64_t encode_calls = 0, decode_calls = 0, decode_bytes = 0;
    };
    PipeStats pipe_stats() {
        std::lock_guard<std::mutex> a(tx_mu_), b(rx_mu_);
        return st_;
    }
    // Test hook: the receive pipeline's decoder thread fails on its next buffer, as a failed GPU
    // decode call does (tests/cpp/test_substrate.cpp: the error must reach the caller).
    void fail_next_decode_for_test() { fail_decoder_.store(true); }

    // Many messages per GPU call: the batch is encoded in sub-batches and queued for the sender
    // thread (one frame per blob, in order).  Returns the wire bytes of this batch.
    size_t send_batch(const void *const *data, const size_t *sizes, size_t n) {
        static_assert(sizeof(size_t) == sizeof(uint64_t), "size_t is 64-bit");
        if (n == 0) return 0;
        rethrow_tx();
        if (!tx_thread_.joinable()) {
            // every ring buffer pinned up front for the first sub-batch's size (not one by one
            // inside later, timed sends)
            uint64_t cap = 0, payload = 0;
            for (size_t i = 0; i < n && (i == 0 || payload + sizes[i] <= kSubBytes) && i < kSubFrames; ++i) {
                payload += sizes[i];
                cap += tdt_encode_bound(sizes[i], codec_.word_size());
            }
            for (auto &t : tx_ring_) t.mem.reserve(cap);
            tx_thread_ = std::thread([this] { tx_loop(); });
        }
        const auto *msgs = reinterpret_cast<const uint8_t *const *>(data);
        const auto *sz = reinterpret_cast<const uint64_t *>(sizes);
        if (record_last_) {
            enc_.clear();
            eoff_.assign(1, 0);
        }
        size_t wire = 0;
        for (size_t i = 0; i < n;) {
            size_t m = 0;
            uint64_t payload = 0, cap = 0;
            while (i + m < n && (m == 0 || (payload + sz[i + m] <= kSubBytes && m < kSubFrames))) {
                payload += sz[i + m];
                cap += tdt_encode_bound(sz[i + m], codec_.word_size());
                ++m;
            }
            auto t0 = Clock::now();
            TxBuf &b = tx_acquire();
            auto t1 = Clock::now();
            b.mem.reserve(cap);
            b.off.assign(m + 1, 0);
            b.st.assign(m, 0);
            if (tdt_encode_host_v(codec_.context(), msgs + i, sz + i, (uint32_t)m, b.mem.data(), cap, b.off.data(),
                                  b.st.data()) != TDT_OK) {
                tx_release_unused(b);
                throw std::runtime_error(std::string("TDT: GPU batch encode failed: ") + tdt_last_error());
            }
            for (size_t k = 0; k < m; ++k)
                if (b.st[k] != TDT_OK) {
                    tx_release_unused(b);
                    throw std::runtime_error(tdt_status_string(b.st[k]));
                }
            b.n = m;
            {
                std::lock_guard<std::mutex> lk(tx_mu_);
                st_.tx_wait += std::chrono::duration<double>(t1 - t0).count();
                st_.encode += since(t1);
                ++st_.encode_calls;
            }
            if (record_last_) {
                const uint64_t base = enc_.size();
                enc_.insert(enc_.end(), b.mem.data(), b.mem.data() + b.off[m]);
                for (size_t k = 1; k <= m; ++k) eoff_.push_back(base + b.off[k]);
            }
            raw_sent_ += payload;
            wire_sent_ += b.off[m];
            wire += b.off[m];
            tx_submit(b);
            i += m;
        }
        return wire;
    }

    // Every frame queued by send_batch is on the wire (rethrows a send error).
    void flush() {
        std::unique_lock<std::mutex> lk(tx_mu_);
        tx_cv_.wait(lk, [&] { return tx_queue_.empty() && !tx_busy_; });
        lk.unlock();
        rethrow_tx();
    }

    // The blobs of the last send_batch when record_last_batch(true) (frame i =
    // last_batch()[offsets[i] .. offsets[i+1])).
    const std::vector<uint8_t> &last_batch() const { return enc_; }
    const std::vector<uint64_t> &last_batch_offsets() const { return eoff_; }

    // Receive n frames (each expected to decode to <= max_msg bytes) and decode them; out /
    // out_off (n+1) receive the payloads back to back.  Returns the per-message status: a frame
    // whose header claims more than max_msg is not decoded (TDT_E_CAPACITY, empty payload) and
    // does not affect the others; decode errors keep their own status.
    std::vector<int32_t> receive_batch(size_t n, size_t max_msg, std::vector<uint8_t> &out,
                                       std::vector<uint64_t> &out_off) {
        release_views();
        std::vector<int32_t> st(n, TDT_OK);
        out_off.assign(n + 1, 0);
        if (n == 0) return st;
        start_rx(max_msg);
        size_t done = 0;
        uint64_t cur = 0;
        while (done < n) {
            RxBuf *b = wait_front();
            // (only this thread consumes: the buffer's frames and payloads stay put until released)
            const size_t k0 = b->used, k1 = std::min(b->n, k0 + (n - done));
            uint64_t total = 0;
            for (size_t k = k0; k < k1; ++k)
                if (b->claim[k] <= (int64_t)max_msg) total += b->claim[k] > 0 ? (uint64_t)b->claim[k] : 0u;
            if (out.size() < cur + total) out.resize(cur + total);
            // payloads decoded ahead are contiguous in b->dec: runs of them leave in one parallel
            // copy; a frame over this call's max_msg is not delivered; one the decoder skipped
            // (over its limit at the time, within this call's) is decoded now
            size_t run0 = k0;
            auto copy_run = [&](size_t e) {
                const uint64_t a0 = b->doff[run0], len = b->doff[e] - a0;
                if (len && tdt_host_copy(codec_.context(), out.data() + cur, b->dec.data() + a0, len) != TDT_OK)
                    throw std::runtime_error(std::string("TDT: host copy failed: ") + tdt_last_error());
                for (size_t k = run0; k < e; ++k) out_off[done + (k - k0) + 1] = cur + (b->doff[k + 1] - a0);
                cur += len;
            };
            for (size_t k = k0; k < k1; ++k) {
                const size_t j = done + (k - k0);
                const int64_t c = b->claim[k];
                if (c <= (int64_t)max_msg && c <= (int64_t)b->lim) {
                    st[j] = b->st[k];
                    continue;
                }
                copy_run(k);
                run0 = k + 1;
                if (c > (int64_t)max_msg) {
                    st[j] = TDT_E_CAPACITY;
                } else {
                    const uint64_t fo[2] = {b->off[k], b->off[k + 1]};
                    uint64_t oo[2] = {0, 0};
                    if (tdt_decode_host(codec_.context(), b->mem.data(), fo, 1, out.data() + cur, (uint64_t)c, oo,
                                        &st[j]) != TDT_OK)
                        throw std::runtime_error(std::string("TDT: GPU decode failed: ") + tdt_last_error());
                    cur += oo[1];
                }
                out_off[j + 1] = cur;
            }
            copy_run(k1);
            done += k1 - k0;
            {
                std::lock_guard<std::mutex> lk(rx_mu_);
                rx_consume(k1 - k0);
                rx_release_if_done(b);
            }
            rx_cv_.notify_all();
        }
        out.resize(cur);
        return st;
    }

    // Zero-copy receive: views of the next n decoded payloads in the pipeline's pinned buffers,
    // valid until the next receive call on this substrate (or release_views()).  Statuses as
    // receive_batch.
    struct FrameView {
        const uint8_t *data;
        uint64_t size;
        int32_t status;
    };
    std::vector<FrameView> receive_batch_views(size_t n, size_t max_msg) {
        release_views();
        std::vector<FrameView> v(n, FrameView{nullptr, 0, TDT_OK});
        if (n == 0) return v;
        start_rx(max_msg);
        size_t done = 0;
        while (done < n) {
            // a consumer holding too many buffers would starve the receiver: move the held
            // payloads out (one copy) and give their buffers back
            if (rx_held_.size() >= kRxMax / 2) migrate_views(v);
            RxBuf *b = wait_front();
            const size_t k0 = b->used, k1 = std::min(b->n, k0 + (n - done));
            holds_.push_back(Hold{b, done, done + (k1 - k0), k0});
            for (size_t k = k0; k < k1; ++k) {
                FrameView &f = v[done + (k - k0)];
                const int64_t c = b->claim[k];
                if (c > (int64_t)max_msg) {
                    f.status = TDT_E_CAPACITY;
                } else if (c > (int64_t)b->lim) {  // skipped by the decoder: decoded now
                    late_.emplace_back((size_t)std::max<int64_t>(c, 1));
                    const uint64_t fo[2] = {b->off[k], b->off[k + 1]};
                    uint64_t oo[2] = {0, 0};
                    if (tdt_decode_host(codec_.context(), b->mem.data(), fo, 1, late_.back().data(), (uint64_t)c, oo,
                                        &f.status) != TDT_OK)
                        throw std::runtime_error(std::string("TDT: GPU decode failed: ") + tdt_last_error());
                    f.data = late_.back().data();
                    f.size = oo[1];
                } else {
                    f.data = b->dec.data() + b->doff[k];
                    f.size = b->doff[k + 1] - b->doff[k];
                    f.status = b->st[k];
                }
            }
            done += k1 - k0;
            {
                std::lock_guard<std::mutex> lk(rx_mu_);
                rx_consume(k1 - k0);
                if (b->used == b->n) {  // consumed: held (not reused) while the views live
                    rx_order_.erase(rx_order_.begin());
                    rx_held_.push_back(b);
                }
            }
            rx_cv_.notify_all();
        }
        return v;
    }
    // The views of the last receive_batch_views are no longer used: their buffers return to
    // the pipeline.  (Every receive call does this first.)
    void release_views() {
        {
            std::lock_guard<std::mutex> lk(rx_mu_);
            for (RxBuf *b : rx_held_) b->free = true;
            rx_held_.clear();
        }
        late_.clear();
        holds_.clear();
        rx_cv_.notify_all();
    }

private:
    // sub-batch bounds of send_batch (payload bytes, frames) and receive ring buffers: a host
    // pipeline call costs ~0.3 ms however small (tools/host_rate.cpp: 8 MiB per call runs at
    // 10 GB/s, 32 MiB at 17, 64 MiB at 21), so calls are made large and the threads overlap
    // whole calls with the socket
    static constexpr uint64_t kSubBytes = 64ull << 20;
    static constexpr size_t kSubFrames = 16384;
    static constexpr size_t kRing = 3;
    static constexpr uint64_t kRxBytes = 32ull << 20;
    static constexpr size_t kRxFrames = 16384;
    static constexpr size_t kRxMax = 16;  // receive buffers at most (32 MiB of frames each)
    static constexpr uint64_t kRxEager = 4ull << 20;  // an idle decoder gets a buffer once it holds this much
    static constexpr size_t kMaxFrame = 100ull * 1024 * 1024;  // the reference's frame cap (tcp_simple.hpp:127-134)

    using Clock = std::chrono::steady_clock;
    static double since(Clock::time_point t) { return std::chrono::duration<double>(Clock::now() - t).count(); }

    // largest frame a <= payload-byte message can arrive as (TDT bound or UNCP n + 4)
    size_t frame_capacity(size_t payload) const { return tdt_encode_bound(payload, codec_.word_size()) + 64; }

    // ---- sender ring
    struct TxBuf {
        PinnedBuffer mem;
        std::vector<uint64_t> off;
        std::vector<int32_t> st;
        size_t n = 0;
        bool free = true;
    };
    TxBuf &tx_acquire() {
        std::unique_lock<std::mutex> lk(tx_mu_);
        for (;;) {
            if (tx_err_) {
                lk.unlock();
                rethrow_tx();
            }
            for (auto &b : tx_ring_)
                if (b.free) {
                    b.free = false;
                    return b;
                }
            tx_cv_.wait(lk);
        }
    }
    void tx_release_unused(TxBuf &b) {
        std::lock_guard<std::mutex> lk(tx_mu_);
        b.free = true;
    }
    void tx_submit(TxBuf &b) {
        {
            std::lock_guard<std::mutex> lk(tx_mu_);
            tx_queue_.push_back(&b);
        }
        tx_cv_.notify_all();
    }
    void rethrow_tx() {
        std::exception_ptr e;
        {
            std::lock_guard<std::mutex> lk(tx_mu_);
            e = tx_err_;
            tx_err_ = nullptr;
        }
        if (e) std::rethrow_exception(e);
    }
    void tx_loop() {
        for (;;) {
            TxBuf *b = nullptr;
            {
                std::unique_lock<std::mutex> lk(tx_mu_);
                tx_cv_.wait(lk, [&] { return tx_stop_ || !tx_queue_.empty(); });
                if (tx_queue_.empty()) return;  // (stop)
                b = tx_queue_.front();
                tx_queue_.erase(tx_queue_.begin());
                tx_busy_ = true;
            }
            auto t0 = Clock::now();
            try {
                for (size_t k = 0; k < b->n; ++k)
                    inner_.transport_send(b->mem.data() + b->off[k], b->off[k + 1] - b->off[k]);
            } catch (...) {
                std::lock_guard<std::mutex> lk(tx_mu_);
                tx_err_ = std::current_exception();
                for (TxBuf *q : tx_queue_) q->free = true;  // frames after a failed send are dropped
                tx_queue_.clear();
            }
            {
                std::lock_guard<std::mutex> lk(tx_mu_);
                st_.send += since(t0);
                b->free = true;
                tx_busy_ = false;
            }
            tx_cv_.notify_all();
        }
    }

    // ---- receive pipeline: ring buffers move free -> filling -> sealed -> decoded -> free
    struct RxBuf {
        PinnedBuffer mem;              // frames back to back
        std::vector<uint64_t> off{0};  // frame k = mem[off[k] .. off[k+1])
        PinnedBuffer dec;              // decoded payloads back to back
        std::vector<uint64_t> doff;    // payload k = dec[doff[k] .. doff[k+1])
        std::vector<int64_t> claim;    // decoded size each frame's header claims (-1: unreadable)
        std::vector<int32_t> st;
        size_t n = 0, used = 0;        // frames received / consumed
        uint64_t lim = 0;              // frames claiming more were not decoded (the decoder's limit)
        bool sealed = false, decoded = false, free = true;
    };
    // the oldest decoded buffer with unconsumed frames (rx_mu_ held), or null
    RxBuf *rx_front_decoded() {
        if (rx_order_.empty()) return nullptr;
        RxBuf *b = rx_order_.front();
        return b->decoded && b->used < b->n ? b : nullptr;
    }
    // nothing decoded or still to decode is waiting (rx_mu_ held); once the decoder thread has
    // failed, a sealed buffer it never decoded counts as drained, so its error reaches the caller
    // instead of every receive waiting forever for those frames
    bool rx_drained() {
        for (RxBuf *b : rx_order_)
            if (b->sealed && b->used < b->n && (b->decoded || !dec_dead_)) return false;
        return true;
    }
    bool frames_ready() {
        if (!rx_thread_.joinable()) return false;
        std::lock_guard<std::mutex> lk(rx_mu_);
        return rx_front_decoded() != nullptr;
    }
    // frames that arrived and are not yet delivered, decoded or not
    bool frames_pending() {
        if (!rx_thread_.joinable()) return false;
        std::lock_guard<std::mutex> lk(rx_mu_);
        return !rx_drained();
    }
    // k frames of the front buffer consumed (rx_mu_ held)
    void rx_consume(size_t k) { rx_order_.front()->used += k; }
    // a fully consumed buffer returns to the ring (rx_mu_ held)
    void rx_release_if_done(RxBuf *b) {
        if (b->used == b->n && !rx_order_.empty() && rx_order_.front() == b) {
            rx_order_.erase(rx_order_.begin());
            b->free = true;
        }
    }
    // views [j0, j1) of the current receive_batch_views call point into buffer b (frames from k0)
    struct Hold {
        RxBuf *b;
        size_t j0, j1, k0;
    };
    std::vector<Hold> holds_;
    // copy the payloads of every fully consumed buffer the current views hold into late_ and
    // return those buffers to the pipeline
    template <class V>
    void migrate_views(V &v) {
        std::vector<RxBuf *> moved;
        {
            std::lock_guard<std::mutex> lk(rx_mu_);
            moved = rx_held_;
        }
        for (Hold &h : holds_) {
            RxBuf *b = h.b;
            if (!b || std::find(moved.begin(), moved.end(), b) == moved.end()) continue;
            const uint64_t a0 = b->doff[h.k0], len = b->doff[h.k0 + (h.j1 - h.j0)] - a0;
            late_.emplace_back(std::max<uint64_t>(len, 1));
            if (len) std::memcpy(late_.back().data(), b->dec.data() + a0, len);
            const uint8_t *lo = b->dec.data() + a0, *hi = lo + len;
            for (size_t j = h.j0; j < h.j1; ++j)
                if (v[j].data >= lo && v[j].data < hi) v[j].data = late_.back().data() + (v[j].data - lo);
            h.b = nullptr;
        }
        std::lock_guard<std::mutex> lk(rx_mu_);
        for (RxBuf *b : moved) b->free = true;
        rx_held_.erase(std::remove_if(rx_held_.begin(), rx_held_.end(),
                                      [&](RxBuf *b) { return std::find(moved.begin(), moved.end(), b) != moved.end(); }),
                       rx_held_.end());
        rx_cv_.notify_all();
    }
    void start_rx(size_t max_msg) {
        {
            std::lock_guard<std::mutex> lk(rx_mu_);
            rx_frame_cap_ = std::max(rx_frame_cap_, frame_capacity(max_msg));
            rx_max_msg_ = std::max<uint64_t>(rx_max_msg_, max_msg);
        }
        if (!rx_thread_.joinable()) {
            // the read-ahead ring, plus two buffers for the views a consumer holds, pinned up
            // front (frames and payloads of a full buffer at a 1.5x decoded/wire ratio; larger
            // payloads grow a buffer once): pinning one mid-run stalled the receiver for ~8 ms
            const uint64_t fcap = frame_capacity(max_msg);
            while (rx_pool_.size() < kRing + 3) {
                rx_pool_.push_back(std::make_unique<RxBuf>());
                rx_pool_.back()->mem.reserve(std::max<uint64_t>(kRxBytes + fcap, 2 * fcap));
                rx_pool_.back()->dec.reserve(kRxBytes + kRxBytes / 2);
            }
            dec_thread_ = std::thread([this] { dec_loop(); });
            rx_thread_ = std::thread([this] { rx_loop(); });
        }
    }
    // the front buffer once decoded (waits); rethrows the pipeline's error when nothing is left
    RxBuf *wait_front() {
        std::unique_lock<std::mutex> lk(rx_mu_);
        const auto t0 = Clock::now();
        rx_cv_.wait(lk, [&] { return rx_front_decoded() != nullptr || (rx_err_ && rx_drained()); });
        st_.deliver_wait += since(t0);
        RxBuf *b = rx_front_decoded();
        if (!b) std::rethrow_exception(rx_err_);
        return b;
    }

    void rx_loop() {
        for (;;) {
            RxBuf *b = nullptr;
            size_t fcap;
            {
                std::unique_lock<std::mutex> lk(rx_mu_);
                // a free buffer of the pool, or a new one while the pool is below kRxMax (a
                // consumer holding views can keep many buffers at once)
                auto pick = [&]() -> RxBuf * {
                    for (auto &q : rx_pool_)
                        if (q->free) return q.get();
                    // read-ahead is kRing + 1 buffers; beyond that only what views hold (each
                    // new buffer is a pinned allocation)
                    if (rx_pool_.size() < std::min(kRxMax, kRing + 1 + rx_held_.size())) {
                        rx_pool_.push_back(std::make_unique<RxBuf>());
                        return rx_pool_.back().get();
                    }
                    return nullptr;
                };
                const auto tw = Clock::now();
                rx_cv_.wait(lk, [&] {
                    if (rx_stop_ || rx_err_) return true;
                    return (b = pick()) != nullptr;
                });
                st_.rx_wait += since(tw);
                if (rx_stop_ || rx_err_) return;
                b->free = false;
                b->sealed = b->decoded = false;
                b->n = b->used = 0;
                b->off.assign(1, 0);
                rx_order_.push_back(b);
                fcap = rx_frame_cap_;
            }
            auto pause = std::chrono::microseconds(1);
            auto last = std::chrono::steady_clock::now();
            const auto tf = Clock::now();
            double slept = 0;
            try {
                b->mem.reserve(std::max<uint64_t>(kRxBytes + fcap, 2 * fcap));
            } catch (...) {
                rx_fail(b);
                return;
            }
            for (;;) {
                size_t flen = 0;
                bool got = false;
                try {
                    // a frame larger than the current capacity (a later call's larger messages)
                    // is received into a buffer grown for it alone instead of reaching Inner with
                    // too small a buffer, which drops the connection: the filling
                    // buffer is sealed first if it holds frames, and the pool's capacity for
                    // later buffers is not raised (one 100 MB frame used to make
                    // every buffer reserve 200 MB of pinned memory).  Frames above the
                    // reference's 100 MB cap are left to Inner, which refuses them as the
                    // reference does
                    if constexpr (requires(Inner &s, size_t &l) { s.peek_frame_length(l); }) {
                        size_t l = 0;
                        if (inner_.peek_frame_length(l) && l > fcap && l <= kMaxFrame) {
                            fcap = l;  // (b->n > 0: the capacity test below seals b)
                            if (b->n == 0) b->mem.reserve(fcap);
                        }
                    }
                    if (b->mem.capacity() - b->off[b->n] >= fcap)
                        got = inner_.try_transport_receive(b->mem.data() + b->off[b->n], fcap, flen);
                } catch (...) {
                    rx_fail(b);
                    return;
                }
                if (got) {
                    b->off.push_back(b->off[b->n] + flen);
                    ++b->n;
                    pause = std::chrono::microseconds(1);
                    last = std::chrono::steady_clock::now();
                    if (b->n < kRxFrames && b->off[b->n] < kRxBytes) continue;
                }
                if (b->n > 0) {
                    // full, or the decoder waits for work and either enough has collected or
                    // the socket has been quiet for a moment: publish (frames keep collecting
                    // otherwise: larger decode calls)
                    std::lock_guard<std::mutex> lk(rx_mu_);
                    const bool full = b->n >= kRxFrames || b->off[b->n] >= kRxBytes ||
                                      b->mem.capacity() - b->off[b->n] < fcap;
                    const bool quiet = std::chrono::steady_clock::now() - last > std::chrono::microseconds(20);
                    if (full || (dec_idle_ && (b->off[b->n] >= kRxEager || quiet))) {
                        b->sealed = true;
                        st_.recv += since(tf) - slept;
                        st_.rx_sleep += slept;
                        break;
                    }
                }
                bool stop;
                {
                    std::lock_guard<std::mutex> lk(rx_mu_);
                    stop = rx_stop_;
                    if constexpr (requires(Inner &s) { s.is_connected(); }) {
                        if (!stop && !inner_.is_connected())
                            rx_err_ = std::make_exception_ptr(std::runtime_error("TCP: Not connected"));
                    }
                    stop = stop || rx_err_ != nullptr;
                    if (stop) {
                        if (b->n > 0) {
                            b->sealed = true;  // what arrived before the end is still delivered
                        } else {
                            rx_order_.pop_back();
                            b->free = true;
                        }
                    }
                }
                if (stop) {
                    rx_cv_.notify_all();
                    return;
                }
                const auto ts = Clock::now();
                std::this_thread::sleep_for(pause);
                slept += since(ts);
                if (pause < std::chrono::microseconds(100)) pause *= 2;
            }
            rx_cv_.notify_all();
        }
    }
    // the receiver's own failure (allocation, a throwing Inner): recorded for the consumers, what
    // arrived before it still delivered
    void rx_fail(RxBuf *b) {
        {
            std::lock_guard<std::mutex> lk(rx_mu_);
            if (!rx_err_) rx_err_ = std::current_exception();
            if (b->n > 0) {
                b->sealed = true;
            } else {
                rx_order_.pop_back();
                b->free = true;
            }
        }
        rx_cv_.notify_all();
    }
    // decoder thread: each sealed buffer's frames on the GPU, in arrival order
    void dec_loop() {
        for (;;) {
            RxBuf *b = nullptr;
            uint64_t lim;
            {
                std::unique_lock<std::mutex> lk(rx_mu_);
                auto next = [&]() -> RxBuf * {
                    for (RxBuf *q : rx_order_)
                        if (q->sealed && !q->decoded) return q;
                    return nullptr;
                };
                dec_idle_ = next() == nullptr;
                const auto tw = Clock::now();
                rx_cv_.wait(lk, [&] { return rx_stop_ || next() != nullptr; });
                st_.dec_wait += since(tw);
                dec_idle_ = false;
                if (rx_stop_) return;
                b = next();
                lim = rx_max_msg_;
            }
            const auto td = Clock::now();
            try {
                if (fail_decoder_.exchange(false)) throw std::runtime_error("TDT: GPU batch decode failed: injected");
                b->claim.resize(b->n);
                b->st.assign(b->n, TDT_OK);
                b->doff.assign(b->n + 1, 0);
                uint64_t total = 0;
                for (size_t k = 0; k < b->n; ++k) {
                    b->claim[k] = tdt_claimed_size(b->mem.data() + b->off[k], b->off[k + 1] - b->off[k]);
                    if (b->claim[k] > 0 && b->claim[k] <= (int64_t)lim) total += (uint64_t)b->claim[k];
                }
                b->dec.reserve(std::max<uint64_t>(total, 1));
                // runs of frames within the limit: one decode call each (a frame claiming more is
                // never decoded: TDT_E_CAPACITY, no payload)
                uint64_t o = 0;
                for (size_t a = 0; a < b->n;) {
                    if (b->claim[a] > (int64_t)lim) {
                        b->st[a] = TDT_E_CAPACITY;
                        b->doff[a + 1] = o;
                        ++a;
                        continue;
                    }
                    size_t e = a;
                    uint64_t t = 0;
                    while (e < b->n && b->claim[e] <= (int64_t)lim) {
                        if (b->claim[e] > 0) t += (uint64_t)b->claim[e];
                        ++e;
                    }
                    dec_off_.assign(e - a + 1, 0);
                    if (tdt_decode_host(codec_.context(), b->mem.data(), b->off.data() + a, (uint32_t)(e - a),
                                        b->dec.data() + o, t, dec_off_.data(), b->st.data() + a) != TDT_OK)
                        throw std::runtime_error(std::string("TDT: GPU batch decode failed: ") + tdt_last_error());
                    for (size_t k = a; k < e; ++k) b->doff[k + 1] = o + dec_off_[k - a + 1];
                    o += dec_off_[e - a];
                    a = e;
                }
            } catch (...) {
                std::lock_guard<std::mutex> lk(rx_mu_);
                rx_err_ = std::current_exception();
                dec_dead_ = true;  // (this buffer and every later one stay undecoded: rx_drained)
                rx_cv_.notify_all();
                return;
            }
            {
                std::lock_guard<std::mutex> lk(rx_mu_);
                st_.decode += since(td);
                ++st_.decode_calls;
                st_.decode_bytes += b->off[b->n];
                b->lim = lim;
                b->decoded = true;
            }
            rx_cv_.notify_all();
        }
    }

    Inner inner_;
    HipTDTCompressionProtocol codec_;
    std::string name_;
    std::vector<uint8_t> stage_, enc_;
    std::vector<uint64_t> eoff_, dec_off_;
    size_t raw_sent_ = 0, wire_sent_ = 0, last_received_ = 0;
    PipeStats st_;  // (tx fields under tx_mu_, rx fields under rx_mu_)
    bool record_last_ = false;

    std::mutex tx_mu_;
    std::condition_variable tx_cv_;
    TxBuf tx_ring_[kRing];
    std::vector<TxBuf *> tx_queue_;
    bool tx_busy_ = false, tx_stop_ = false;
    std::exception_ptr tx_err_;
    std::thread tx_thread_;

    std::mutex rx_mu_;
    std::condition_variable rx_cv_;
    std::vector<std::unique_ptr<RxBuf>> rx_pool_;
    std::vector<RxBuf *> rx_held_;            // consumed buffers whose payloads the last views reference
    std::vector<std::vector<uint8_t>> late_;  // payloads decoded at delivery for the last views
    std::vector<RxBuf *> rx_order_;  // buffers in arrival order (the one being filled last)
    size_t rx_frame_cap_ = 0;
    uint64_t rx_max_msg_ = 0;        // largest max_msg of a receive_batch call: the decoder's limit
    bool rx_stop_ = false, dec_idle_ = true, dec_dead_ = false;
    std::atomic<bool> fail_decoder_{false};
    std::exception_ptr rx_err_;
    std::thread rx_thread_, dec_thread_;
};

}  // namespace psyne_amd
