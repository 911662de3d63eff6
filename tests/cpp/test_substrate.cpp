// tests/cpp/test_substrate.cpp — TdtSubstrate<PosixTcpSubstrate> over 127.0.0.1 (GPU codec):
//   * frames round-trip through transport_send / transport_receive(void*, size_t) (psyne's
//     SubstrateBehavior shape, lengths taken from the inner try_transport_receive);
//   * a 24-byte TDT frame whose header claims original_size = 0xFFFFFFF0 is rejected BEFORE
//     decoding ("TDT: decoded message larger than the buffer"), and the connection stays usable;
//   * in receive_batch one oversized frame gets TDT_E_CAPACITY while its neighbours decode;
//   * reference decode errors keep the reference's text ("Invalid TDT magic number");
//   * after receive_batch started the pipeline with a small max_msg, a frame larger than its
//     buffers (and than the decoder's limit) still reaches transport_receive intact (ADVICE r04:
//     the receiver used to hand Inner a too-small buffer, which drops the connection);
//   * a failed decoder thread surfaces as an exception from transport_receive, not a hang.
// Prints "cpp substrate OK" on success.
#include <psyne_amd/tdt_substrate.hpp>

#include <cstdio>
#include <random>

using namespace psyne_amd;

static std::vector<uint8_t> grad(std::mt19937 &rng, size_t floats) {
    std::normal_distribution<float> nd(0.f, 0.01f);
    std::uniform_real_distribution<float> u(0.f, 1.f);
    std::vector<float> g(floats);
    for (auto &x : g) x = u(rng) < 0.7f ? 0.f : nd(rng);
    const uint8_t *p = reinterpret_cast<const uint8_t *>(g.data());
    return std::vector<uint8_t>(p, p + floats * 4);
}

#define CHECK(c, msg)                                   \
    do {                                                \
        if (!(c)) {                                     \
            std::printf("FAILED: %s\n", msg);           \
            return 1;                                   \
        }                                               \
    } while (0)

int main() {
    TdtSubstrate<PosixTcpSubstrate>::defaults().bandwidth_mbps = 10.0;  // compression on
    TDTConfig cfg;
    cfg.sample_fraction = 1.0f;
    TdtSubstrate<PosixTcpSubstrate> rx(cfg, "127.0.0.1", (uint16_t)18201, true);
    PosixTcpSubstrate raw("127.0.0.1", (uint16_t)18201, false);  // a plain peer: sends any frame
    CHECK(rx.inner().wait_for_connection() && raw.wait_for_connection(), "connect");
    std::mt19937 rng(11);
    std::vector<uint8_t> buf(1 << 20);

    // 1. a frame encoded by a second decorator's codec, sent raw, received and decoded
    std::vector<uint8_t> msg = grad(rng, 16384);
    std::vector<uint8_t> blob = rx.codec().encode(msg.data(), msg.size());
    CHECK(blob.size() < msg.size(), "compressed");
    raw.transport_send(blob.data(), blob.size());
    rx.transport_receive(buf.data(), buf.size());
    CHECK(rx.last_received_size() == msg.size() && std::memcmp(buf.data(), msg.data(), msg.size()) == 0, "round trip");

    // 2. crafted header claiming 0xFFFFFFF0 decoded bytes: rejected without decoding
    uint8_t evil[24] = {0x44, 0x54, 0x44, 0x54, 0xF0, 0xFF, 0xFF, 0xFF, 1, 0, 0, 0, 4, 0, 0, 0, 4, 0, 0, 0, 0, 0, 0, 0};
    raw.transport_send(evil, sizeof(evil));
    bool threw = false;
    try {
        rx.transport_receive(buf.data(), buf.size());
    } catch (const std::runtime_error &e) {
        threw = std::string(e.what()) == "TDT: decoded message larger than the buffer";
    }
    CHECK(threw, "oversized claim rejected");
    raw.transport_send(blob.data(), blob.size());  // the connection is still usable
    rx.transport_receive(buf.data(), buf.size());
    CHECK(std::memcmp(buf.data(), msg.data(), msg.size()) == 0, "after rejection");

    // 3. reference decode error text
    uint8_t bad[12] = {'X', 'Y', 'Z', 'W', 0, 0, 0, 0, 0, 0, 0, 0};
    raw.transport_send(bad, sizeof(bad));
    threw = false;
    try {
        rx.transport_receive(buf.data(), buf.size());
    } catch (const std::runtime_error &e) {
        threw = std::string(e.what()) == "Invalid TDT magic number";
    }
    CHECK(threw, "bad magic text");

    // 4. batch: frames 0 and 2 valid, frame 1 claims too much
    std::vector<uint8_t> m2 = grad(rng, 8192);
    std::vector<uint8_t> b2 = rx.codec().encode(m2.data(), m2.size());
    raw.transport_send(blob.data(), blob.size());
    raw.transport_send(evil, sizeof(evil));
    raw.transport_send(b2.data(), b2.size());
    std::vector<uint8_t> out;
    std::vector<uint64_t> off;
    const std::vector<int32_t> st = rx.receive_batch(3, 1 << 16, out, off);
    CHECK(st[0] == TDT_OK && st[1] == TDT_E_CAPACITY && st[2] == TDT_OK, "batch statuses");
    CHECK(off[1] - off[0] == msg.size() && std::memcmp(out.data() + off[0], msg.data(), msg.size()) == 0, "batch 0");
    CHECK(off[2] == off[1], "batch 1 empty");
    CHECK(off[3] - off[2] == m2.size() && std::memcmp(out.data() + off[2], m2.data(), m2.size()) == 0, "batch 2");

    // 4b. a frame larger than the pipeline's buffers and its decoder's limit (64 KiB above),
    //     then a small one: both arrive, the connection stays up
    std::vector<uint8_t> big = grad(rng, 131072);  // 512 KiB payload, ~410 KB frame
    std::vector<uint8_t> bigb = rx.codec().encode(big.data(), big.size());
    raw.transport_send(bigb.data(), bigb.size());
    raw.transport_send(b2.data(), b2.size());
    rx.transport_receive(buf.data(), buf.size());
    CHECK(rx.last_received_size() == big.size() && std::memcmp(buf.data(), big.data(), big.size()) == 0,
          "large frame after a small receive_batch");
    rx.transport_receive(buf.data(), buf.size());
    CHECK(rx.last_received_size() == m2.size() && std::memcmp(buf.data(), m2.data(), m2.size()) == 0,
          "frame after the large one");
    CHECK(rx.inner().is_connected(), "connection kept");

    // 5. default construction (ChannelBridge: std::make_unique<SubstrateType>())
    static_assert(std::is_default_constructible_v<TdtSubstrate<PosixTcpSubstrate>>);

    // 6. (last: it stops the pipeline) the decoder thread fails on the next buffer, as a failed
    //    GPU decode call does: transport_receive throws the decoder's error instead of waiting
    //    forever for the frames it never decoded
    rx.fail_next_decode_for_test();
    raw.transport_send(blob.data(), blob.size());
    raw.transport_send(b2.data(), b2.size());
    threw = false;
    {
        const auto t0 = std::chrono::steady_clock::now();
        try {
            rx.transport_receive(buf.data(), buf.size());
        } catch (const std::runtime_error &e) {
            threw = std::string(e.what()).find("injected") != std::string::npos;
        }
        CHECK(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10), "decoder failure reported promptly");
    }
    CHECK(threw, "decoder failure reaches transport_receive");
    std::printf("cpp substrate OK name=%s\n", rx.substrate_name());
    return 0;
}
