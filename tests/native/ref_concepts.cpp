// tests/native/ref_concepts.cpp — compile-only check of the drop-in boundary against the
// REFERENCE's own contracts (build container only: tests/test_reference_concepts.py compiles it
// with -I/root/reference/include; nothing of the reference is copied or linked):
//   * psyne::concepts::Protocol      (include/psyne/concepts/protocol_concepts.hpp:22-47)
//     holds for psyne_amd::HipTDTCompressionProtocol and psyne_amd::IdentityProtocol;
//   * psyne::concepts::ProtocolStack (:55-69) holds for psyne_amd::ProtocolStack;
//   * psyne_amd::TdtSubstrate over an inner substrate that has exactly SimpleTCP's public
//     method set (tcp_simple.hpp:26-361 — no last_received_size()) and derives from
//     psyne::behaviors::SubstrateBehavior (core/behaviors.hpp:32-48) is itself a complete
//     SubstrateBehavior, default-constructible, and instantiates psyne's own
//     ChannelBridge<Msg, Substrate, Pattern> (behaviors.hpp:142-265) with SimpleSPSC.
// <cstdint> and <functional> first: protocol_concepts.hpp uses uint8_t and logger.hpp std::function
// without including them (the only accommodation)
#include <cstdint>
#include <functional>
#include <psyne/concepts/protocol_concepts.hpp>
#include <psyne/core/behaviors.hpp>
#include <psyne/core/simple_patterns.hpp>

#include <psyne_amd/hip_tdt_protocol.hpp>
#include <psyne_amd/protocol_stack.hpp>
#include <psyne_amd/tdt_substrate.hpp>

#include <type_traits>

static_assert(psyne::concepts::Protocol<psyne_amd::HipTDTCompressionProtocol>);
static_assert(psyne::concepts::Protocol<psyne_amd::IdentityProtocol>);
static_assert(psyne::concepts::ProtocolStack<psyne_amd::ProtocolStack>);

// SimpleTCP's public surface, nothing more (tcp_simple.hpp:26-257), as a SubstrateBehavior.
class RefShapedTCP : public psyne::behaviors::SubstrateBehavior {
public:
    explicit RefShapedTCP(const std::string &host = "localhost", uint16_t port = 8080, bool is_server = false);
    ~RefShapedTCP();
    void *allocate_memory_slab(size_t size_bytes) override;
    void deallocate_memory_slab(void *memory) override;
    void transport_send(void *data, size_t size) override;
    void transport_receive(void *buffer, size_t buffer_size) override;
    bool try_transport_receive(void *buffer, size_t buffer_size, size_t &received_size);
    const char *substrate_name() const override;
    bool is_zero_copy() const override;
    bool is_cross_process() const override;
    bool is_connected() const;
    bool wait_for_connection(std::chrono::milliseconds timeout = std::chrono::milliseconds(5000));
    size_t get_bytes_sent() const;
    size_t get_bytes_received() const;
    size_t get_packets_sent() const;
    size_t get_packets_received() const;
    const std::string &get_host() const;
    uint16_t get_port() const;
    bool is_server_mode() const;
};

using TdtOverRef = psyne_amd::TdtSubstrate<RefShapedTCP, psyne::behaviors::SubstrateBehavior>;
static_assert(std::is_default_constructible_v<TdtOverRef>);
static_assert(std::is_base_of_v<psyne::behaviors::SubstrateBehavior, TdtOverRef>);
static_assert(!std::is_abstract_v<TdtOverRef>, "every SubstrateBehavior pure virtual is implemented");

// and over this repo's POSIX substrate (no virtual base)
using TdtOverPosix = psyne_amd::TdtSubstrate<psyne_amd::PosixTcpSubstrate>;
static_assert(std::is_default_constructible_v<TdtOverPosix>);

struct TensorMsg {
    float values[256];
};
// psyne's own channel over the decorated substrate
template class psyne::behaviors::ChannelBridge<TensorMsg, TdtOverRef, psyne::simple_patterns::SimpleSPSC>;

int main() { return 0; }
