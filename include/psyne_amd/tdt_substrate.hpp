// tdt_substrate.hpp — the TCP substrate path with TDT payload compression on the GPU.
//
// psyne's network substrate (reference include/psyne/channel/substrate/tcp_simple.hpp) frames
// every message as a u32 length followed by the payload (transport_send :68-91,
// transport_receive :96-150, try_transport_receive :153-194).  docs/tdt_attribution.md:62-75
// describes the intended TDT-over-IP substrate: payloads compressed before the socket and
// restored after it.  This header provides both halves for an MI355X host:
//
//   * PosixTcpSubstrate — SimpleTCP's SubstrateBehavior surface (allocate/deallocate slab,
//     transport_send/receive, try_transport_receive, identity, statistics, wait_for_connection)
//     over blocking POSIX sockets (the image has no Boost.Asio), byte-identical framing and
//     the reference's error texts.
//   * TdtSubstrate<Inner> — a decorator over any substrate with that surface: transport_send
//     encodes the payload with the GPU codec (HipTDTCompressionProtocol: UNCP passthrough when
//     the policy says so, exactly like the reference codec) and sends the blob through Inner's
//     framing; transport_receive takes one frame from Inner and decodes it.  send_batch /
//     receive_batch move many messages per GPU call through the C ABI host pipeline
//     (tdt_encode_host / tdt_decode_host: chunked, H2D / kernel / D2H overlapped on two
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
#include <vector>

namespace psyne_amd {

class PosixTcpSubstrate {
public:
    // host: bind address (server) or remote host (client); as SimpleTCP(host, port, is_server)
    explicit PosixTcpSubstrate(const std::string &host = "127.0.0.1", uint16_t port = 8080, bool is_server = false)
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

    // (:96-150) one frame into buffer; its size is last_received_size()
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
        last_received_ = hdr;
        bytes_received_ += hdr + sizeof(hdr);
        packets_received_++;
    }

    // (:153-194) non-blocking probe: a frame is read only when its length word has arrived
    bool try_transport_receive(void *buffer, size_t buffer_size, size_t &received_size) {
        if (!is_connected()) return false;
        std::lock_guard<std::mutex> lk(mu_);
        uint32_t hdr = 0;
        const ssize_t got = ::recv(fd_, &hdr, sizeof(hdr), MSG_PEEK | MSG_DONTWAIT);
        if (got < (ssize_t)sizeof(hdr)) return false;
        if (!read_all(&hdr, sizeof(hdr))) return fail_quiet();
        if (hdr > buffer_size) throw std::runtime_error("TCP: Received message too large for buffer");
        if (!read_all(buffer, hdr)) return fail_quiet();
        received_size = hdr;
        last_received_ = hdr;
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
    size_t last_received_size() const { return last_received_; }
    const std::string &get_host() const { return host_; }
    uint16_t get_port() const { return port_; }
    bool is_server_mode() const { return is_server_; }

private:
    static constexpr size_t kMaxReasonable = 100ull * 1024 * 1024;  // :132-140

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
    size_t slab_size_ = 0, last_received_ = 0;
    size_t bytes_sent_ = 0, bytes_received_ = 0, packets_sent_ = 0, packets_received_ = 0;
};

// Decorator: TDT payload compression on the GPU between the channel and a framed substrate.
template <class Inner>
class TdtSubstrate {
public:
    TdtSubstrate(Inner &inner, HipTDTCompressionProtocol &codec) : inner_(inner), codec_(codec) {}

    void *allocate_memory_slab(size_t n) { return inner_.allocate_memory_slab(n); }
    void deallocate_memory_slab(void *p) { inner_.deallocate_memory_slab(p); }

    // One message: encode (UNCP when the policy is off, as TDTCompressionProtocol::encode
    // :227-266) and send the blob as one frame.
    void transport_send(void *data, size_t size) {
        std::vector<uint8_t> blob = codec_.encode(data, size);
        inner_.transport_send(blob.data(), blob.size());
        raw_sent_ += size;
        wire_sent_ += blob.size();
    }

    // One frame → decode → buffer; returns the decoded size (the reference throws on a
    // malformed blob: decode :271-304).
    size_t transport_receive(void *buffer, size_t buffer_size) {
        stage_.resize(tdt_encode_bound(buffer_size, 4) + 64);
        inner_.transport_receive(stage_.data(), stage_.size());
        std::vector<uint8_t> blob(stage_.begin(), stage_.begin() + (ptrdiff_t)inner_.last_received_size());
        std::vector<uint8_t> out = codec_.decode(blob);
        if (out.size() > buffer_size) throw std::runtime_error("TDT: decoded message larger than the buffer");
        std::memcpy(buffer, out.data(), out.size());
        return out.size();
    }

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
        std::vector<uint64_t> eoff(n + 1);
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

    // Receive n frames (each decoding to <= max_msg bytes) and decode them in one GPU call.
    // out / out_off (n+1) receive the payloads back to back.
    void receive_batch(size_t n, size_t max_msg, std::vector<uint8_t> &out, std::vector<uint64_t> &out_off) {
        const size_t fcap = tdt_encode_bound(max_msg, codec_.word_size()) + 64;
        std::vector<uint64_t> boff(n + 1, 0);
        pack_.resize(n * fcap);
        uint64_t decoded = 0;
        for (size_t i = 0; i < n; ++i) {
            inner_.transport_receive(pack_.data() + boff[i], fcap);
            boff[i + 1] = boff[i] + inner_.last_received_size();
            decoded += max_msg;
        }
        out.resize(decoded ? decoded : 1);
        out_off.assign(n + 1, 0);
        std::vector<int32_t> st(n);
        if (tdt_decode_host(codec_.context(), pack_.data(), boff.data(), (uint32_t)n, out.data(), out.size(),
                            out_off.data(), st.data()) != TDT_OK)
            throw std::runtime_error(std::string("TDT: GPU batch decode failed: ") + tdt_last_error());
        for (size_t i = 0; i < n; ++i)
            if (st[i] != TDT_OK) throw std::runtime_error(tdt_status_string(st[i]));
        out.resize(out_off[n]);
    }

    const char *substrate_name() const { return "TDT+PosixTCP"; }
    bool is_zero_copy() const { return false; }
    bool is_cross_process() const { return inner_.is_cross_process(); }
    // wire bytes / payload bytes sent so far
    double wire_ratio() const { return raw_sent_ ? double(wire_sent_) / double(raw_sent_) : 1.0; }

private:
    Inner &inner_;
    HipTDTCompressionProtocol &codec_;
    std::vector<uint8_t> stage_, pack_, enc_;
    size_t raw_sent_ = 0, wire_sent_ = 0;
};

}  // namespace psyne_amd
