// tests/cpp/test_protocol.cpp — the C++ drop-in used the way psyne's ProtocolChannel uses
// a Protocol (examples/protocols/protocol_demo.cpp:135-189 in the reference):
// analyze_data → should_transform → encode → (transport) → decode, through the concept.
#include <psyne_amd/hip_tdt_protocol.hpp>
#include <psyne_amd/protocol_stack.hpp>

#include <cstdio>
#include <random>

template <psyne_amd::concepts::Protocol P>
static int roundtrip(P &p, std::vector<uint8_t> &msg, bool expect_compressed) {
    p.analyze_data(msg.data(), msg.size());
    const bool t = p.should_transform(msg.data(), msg.size());
    std::vector<uint8_t> wire = p.encode(msg.data(), msg.size());
    uint32_t magic;
    std::memcpy(&magic, wire.data(), 4);
    const bool compressed = magic == 0x54445444u;
    std::vector<uint8_t> back = p.decode(wire);
    if (back != msg) return 1;
    if (compressed != expect_compressed || t != expect_compressed) return 2;
    return 0;
}

int main() {
    psyne_amd::TDTConfig cfg;
    cfg.sample_fraction = 1.0f;
    psyne_amd::HipTDTCompressionProtocol p(cfg);
    std::mt19937 rng(7);
    std::normal_distribution<float> nd(0.f, 0.01f);
    std::uniform_real_distribution<float> u(0.f, 1.f);
    std::vector<float> g(16384);
    for (auto &x : g) x = u(rng) < 0.7f ? 0.f : nd(rng);
    std::vector<uint8_t> msg(reinterpret_cast<uint8_t *>(g.data()), reinterpret_cast<uint8_t *>(g.data()) + 65536);
    int rc = roundtrip(p, msg, false);  // default 100 Mbps: passthrough (:200, :352)
    if (rc) { std::printf("passthrough rc=%d\n", rc); return 1; }
    p.update_network_metrics(25.0, 15.0);  // protocol_demo.cpp:335 forces compression
    rc = roundtrip(p, msg, true);
    if (rc) { std::printf("compressed rc=%d\n", rc); return 1; }
    if (!(p.transformation_ratio() > 1.0) || !(p.get_average_entropy() > 0.0)) { std::printf("metrics\n"); return 1; }
    try {
        p.decode(std::vector<uint8_t>{1, 2});
        return 1;
    } catch (const std::runtime_error &e) {
        if (std::string(e.what()) != "TDT: Invalid encoded data size") return 1;
    }
    try {
        p.decode(std::vector<uint8_t>{'X', 'Y', 'Z', 'W', 0, 0, 0, 0});
        return 1;
    } catch (const std::runtime_error &e) {
        if (std::string(e.what()) != "Invalid TDT magic number") return 1;
    }
    // ProtocolStack (protocol_concepts.hpp:55-69): TDT then identity; decode in reverse order
    psyne_amd::ProtocolStack stack;
    stack.push_protocol<psyne_amd::HipTDTCompressionProtocol>(cfg);
    stack.push_protocol();  // the concept's nullary push: an identity layer
    stack.update_network_metrics(10.0, 1.0);
    std::vector<uint8_t> wire = stack.encode_stack(msg.data(), msg.size());
    if (wire != p.encode(msg.data(), msg.size())) { std::printf("stack encode\n"); return 1; }
    if (stack.decode_stack(wire) != msg) { std::printf("stack decode\n"); return 1; }
    if (std::string(stack.stack_name()) != "TDT-Compression -> Identity") { std::printf("stack name\n"); return 1; }
    auto *tdt = stack.layer<psyne_amd::HipTDTCompressionProtocol>(0);
    if (!tdt || stack.total_overhead_ms() != tdt->processing_overhead_ms() || !(stack.total_overhead_ms() > 0.0)) {
        std::printf("stack overhead\n");
        return 1;
    }
    std::printf("cpp protocol OK ratio=%.4f entropy=%.6f stack=%s\n", p.transformation_ratio(), p.get_average_entropy(),
                stack.stack_name());
    return 0;
}
