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
//     pipeline (tdt_encode_host / tdt_decode_host: chunked, H2D / kernel / D2H overlapped on two
//     streams), which is how the codec reaches PCIe rates instead of per-message latency.
#pragma once

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <psyne_amd/hip_tdt_protocol.hpp>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
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
        std::lock_guard<std::mutex> lk(mu_);
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
        std::lock_guard<std::mutex> lk(mu_);
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

    // (:153-194) non-blocking probe: a frame is read only when its length word has arrived;
    // like SimpleTCP it never throws (an oversized frame or a failed read drops the connection
    // and returns false)
    bool try_transport_receive(void *buffer, size_t buffer_size, size_t &received_size) {
        if (!is_connected()) return false;
        std::lock_guard<std::mutex> lk(mu_);
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
    std::mutex mu_;
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

// Decorator: TDT payload compression on the GPU between the channel and a framed substrate.
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
    TdtSubstrate(const TdtSubstrate &) = delete;
    TdtSubstrate &operator=(const TdtSubstrate &) = delete;

    Inner &inner() { return inner_; }
    HipTDTCompressionProtocol &codec() { return codec_; }

    // MEMORY OWNERSHIP
    void *allocate_memory_slab(size_t n) { return inner_.allocate_memory_slab(n); }
    void deallocate_memory_slab(void *p) { inner_.deallocate_memory_slab(p); }

    // TRANSPORT: one message = one frame (UNCP when the policy is off, exactly as
    // TDTCompressionProtocol::encode :227-266)
    void transport_send(void *data, size_t size) {
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
                if (!inner_.is_connected()) throw std::runtime_error("TCP: Not connected");
            }
            std::this_thread::sleep_for(pause);
            if (pause < std::chrono::microseconds(200)) pause *= 2;
        }
    }

    // (tcp_simple.hpp:153-194 shape) false when no frame is waiting; otherwise one frame is
    // taken from Inner, checked, decoded into buffer, and its decoded size returned.
    bool try_transport_receive(void *buffer, size_t buffer_size, size_t &received_size) {
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

    // Many messages per GPU call: pack → tdt_encode_host (one pipelined batch) → one frame per
    // blob, in order.  Returns the wire bytes.
    size_t send_batch(const void *const *data, const size_t *sizes, size_t n) {
        if (n == 0) return 0;
        std::vector<uint64_t> off(n + 1, 0);
        for (size_t i = 0; i < n; ++i) off[i + 1] = off[i] + sizes[i];
        pack_.resize(off[n]);
        for (size_t i = 0; i < n; ++i) std::memcpy(pack_.data() + off[i], data[i], sizes[i]);
        uint64_t cap = 0;
        for (size_t i = 0; i < n; ++i) cap += tdt_encode_bound(sizes[i], codec_.word_size());
        enc_.resize(cap);
        std::vector<uint64_t> &eoff = eoff_;
        eoff.assign(n + 1, 0);
        std::vector<int32_t> st(n);
        if (tdt_encode_host(codec_.context(), pack_.data(), off.data(), (uint32_t)n, enc_.data(), cap, eoff.data(),
                            st.data()) != TDT_OK)
            throw std::runtime_error(std::string("TDT: GPU batch encode failed: ") + tdt_last_error());
        for (size_t i = 0; i < n; ++i) {
            if (st[i] != TDT_OK) throw std::runtime_error(tdt_status_string(st[i]));
            inner_.transport_send(enc_.data() + eoff[i], eoff[i + 1] - eoff[i]);
        }
        raw_sent_ += off[n];
        wire_sent_ += eoff[n];
        return eoff[n];
    }

    // The blobs of the last send_batch (frame i = last_batch()[offsets[i] .. offsets[i+1])).
    const std::vector<uint8_t> &last_batch() const { return enc_; }
    const std::vector<uint64_t> &last_batch_offsets() const { return eoff_; }

    // Receive n frames (each expected to decode to <= max_msg bytes) and decode them in one GPU
    // call; out / out_off (n+1) receive the payloads back to back.  Returns the per-message
    // status: a frame whose header claims more than max_msg is not decoded (TDT_E_CAPACITY,
    // empty payload) and does not affect the others; decode errors keep their own status.
    std::vector<int32_t> receive_batch(size_t n, size_t max_msg, std::vector<uint8_t> &out,
                                       std::vector<uint64_t> &out_off) {
        const size_t fcap = frame_capacity(max_msg);
        std::vector<uint64_t> boff(n + 1, 0);
        std::vector<int32_t> st(n, TDT_OK);
        std::vector<bool> rejected(n, false);
        pack_.resize(n * fcap + 4);
        uint64_t decoded = 0;
        for (size_t i = 0; i < n; ++i) {
            size_t flen = 0;
            auto pause = std::chrono::microseconds(1);
            while (!inner_.try_transport_receive(pack_.data() + boff[i], fcap, flen)) {
                if constexpr (requires(Inner &s) { s.is_connected(); }) {
                    if (!inner_.is_connected()) throw std::runtime_error("TCP: Not connected");
                }
                std::this_thread::sleep_for(pause);
                if (pause < std::chrono::microseconds(200)) pause *= 2;
            }
            const int64_t claimed = tdt_claimed_size(pack_.data() + boff[i], flen);
            if (claimed > (int64_t)max_msg) {  // replace by an empty UNCP blob
                static const uint8_t kEmpty[4] = {0x50, 0x43, 0x4E, 0x55};
                std::memcpy(pack_.data() + boff[i], kEmpty, 4);
                flen = 4;
                rejected[i] = true;
            } else if (claimed > 0) {
                decoded += (uint64_t)claimed;
            }
            boff[i + 1] = boff[i] + flen;
        }
        out.resize(decoded ? decoded : 1);
        out_off.assign(n + 1, 0);
        if (tdt_decode_host(codec_.context(), pack_.data(), boff.data(), (uint32_t)n, out.data(), decoded,
                            out_off.data(), st.data()) != TDT_OK)
            throw std::runtime_error(std::string("TDT: GPU batch decode failed: ") + tdt_last_error());
        for (size_t i = 0; i < n; ++i)
            if (rejected[i]) st[i] = TDT_E_CAPACITY;
        out.resize(out_off[n]);
        return st;
    }

private:
    // largest frame a <= payload-byte message can arrive as (TDT bound or UNCP n + 4)
    size_t frame_capacity(size_t payload) const { return tdt_encode_bound(payload, codec_.word_size()) + 64; }

    Inner inner_;
    HipTDTCompressionProtocol codec_;
    std::string name_;
    std::vector<uint8_t> stage_, pack_, enc_;
    std::vector<uint64_t> eoff_;
    size_t raw_sent_ = 0, wire_sent_ = 0, last_received_ = 0;
};

}  // namespace psyne_amd
