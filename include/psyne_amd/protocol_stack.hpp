// protocol_stack.hpp — psyne's ProtocolStack contract (reference
// include/psyne/concepts/protocol_concepts.hpp:55-69: push_protocol, encode_stack,
// decode_stack, stack_name, total_overhead_ms), never implemented by the reference.
//
// A stack owns an ordered list of layers, each any type satisfying the Protocol concept
// (protocol_concepts.hpp:22-47).  encode_stack runs the layers' encode in push order (each
// layer decides passthrough itself, as TDTCompressionProtocol::encode does with its UNCP
// marker); decode_stack runs their decode in reverse order.  The "Composable Usage" example
// of the reference (:105-110, "TDT Compression -> AES Encryption -> Checksum -> Substrate") is
// push_protocol<HipTDTCompressionProtocol>(cfg) followed by the other layers.
//
// The concept calls push_protocol() with no argument; here that pushes an IdentityProtocol
// layer (a Protocol that returns its input), and push_protocol<P>(args...) pushes a P built
// from args in place.
#pragma once

#include <psyne_amd/hip_tdt_protocol.hpp>

#include <concepts>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace psyne_amd {

namespace concepts {
// Restatement of psyne::concepts::ProtocolStack (protocol_concepts.hpp:55-69).
template <typename PS>
concept ProtocolStack = requires(PS stack, void *data, size_t size) {
    { stack.push_protocol() } -> std::same_as<void>;
    { stack.encode_stack(data, size) } -> std::convertible_to<std::vector<uint8_t>>;
    { stack.decode_stack(std::declval<const std::vector<uint8_t> &>()) } -> std::convertible_to<std::vector<uint8_t>>;
    { stack.stack_name() } -> std::convertible_to<const char *>;
    { stack.total_overhead_ms() } -> std::same_as<double>;
};
}  // namespace concepts

// A Protocol that changes nothing (ratio 1, lossless, no overhead).
class IdentityProtocol {
public:
    bool should_transform(void *, size_t) { return false; }
    void analyze_data(void *, size_t) {}
    std::vector<uint8_t> encode(void *data, size_t size) {
        const uint8_t *p = static_cast<const uint8_t *>(data);
        return std::vector<uint8_t>(p, p + size);
    }
    std::vector<uint8_t> decode(const std::vector<uint8_t> &encoded) { return encoded; }
    void update_network_metrics(double, double) {}
    void update_system_metrics(double) {}
    const char *protocol_name() const { return "Identity"; }
    bool is_lossless() const { return true; }
    double transformation_ratio() const { return 1.0; }
    double processing_overhead_ms() const { return 0.0; }
};
static_assert(concepts::Protocol<IdentityProtocol>);

class ProtocolStack {
public:
    ProtocolStack() = default;
    ProtocolStack(const ProtocolStack &) = delete;
    ProtocolStack &operator=(const ProtocolStack &) = delete;

    // Push a layer P built in place from args (default: an IdentityProtocol).
    template <concepts::Protocol P = IdentityProtocol, class... Args>
    void push_protocol(Args &&...args) {
        auto h = std::make_unique<Holder<P>>(std::forward<Args>(args)...);
        if (!layers_.empty()) name_ += " -> ";
        name_ += h->p.protocol_name();
        layers_.push_back(std::move(h));
    }

    // Layers' encode in push order (an empty stack copies the input).
    std::vector<uint8_t> encode_stack(void *data, size_t size) {
        if (layers_.empty()) return IdentityProtocol().encode(data, size);
        std::vector<uint8_t> buf = layers_[0]->encode(data, size);
        for (size_t i = 1; i < layers_.size(); ++i) buf = layers_[i]->encode(buf.data(), buf.size());
        return buf;
    }

    // Layers' decode in reverse order.
    std::vector<uint8_t> decode_stack(const std::vector<uint8_t> &encoded) {
        std::vector<uint8_t> buf = encoded;
        for (size_t i = layers_.size(); i-- > 0;) buf = layers_[i]->decode(buf);
        return buf;
    }

    const char *stack_name() const { return name_.c_str(); }

    // Σ processing_overhead_ms() of the layers (:332-334 per layer).
    double total_overhead_ms() const {
        double t = 0.0;
        for (const auto &l : layers_) t += l->overhead_ms();
        return t;
    }

    // Forward update_network_metrics / update_system_metrics to every layer.
    void update_network_metrics(double bandwidth_mbps, double latency_ms) {
        for (auto &l : layers_) l->network(bandwidth_mbps, latency_ms);
    }
    void update_system_metrics(double cpu_usage) {
        for (auto &l : layers_) l->system(cpu_usage);
    }

    size_t size() const { return layers_.size(); }
    // Layer i as a P (nullptr if it is another type).
    template <class P>
    P *layer(size_t i) {
        auto *h = dynamic_cast<Holder<P> *>(layers_.at(i).get());
        return h ? &h->p : nullptr;
    }

private:
    struct Layer {
        virtual ~Layer() = default;
        virtual std::vector<uint8_t> encode(void *data, size_t size) = 0;
        virtual std::vector<uint8_t> decode(const std::vector<uint8_t> &encoded) = 0;
        virtual double overhead_ms() const = 0;
        virtual void network(double bw, double lat) = 0;
        virtual void system(double cpu) = 0;
    };
    template <class P>
    struct Holder final : Layer {
        template <class... Args>
        explicit Holder(Args &&...args) : p(std::forward<Args>(args)...) {}
        std::vector<uint8_t> encode(void *data, size_t size) override { return p.encode(data, size); }
        std::vector<uint8_t> decode(const std::vector<uint8_t> &e) override { return p.decode(e); }
        double overhead_ms() const override { return p.processing_overhead_ms(); }
        void network(double bw, double lat) override { p.update_network_metrics(bw, lat); }
        void system(double cpu) override { p.update_system_metrics(cpu); }
        P p;
    };
    std::vector<std::unique_ptr<Layer>> layers_;
    std::string name_;
};
static_assert(concepts::ProtocolStack<ProtocolStack>);

}  // namespace psyne_amd
