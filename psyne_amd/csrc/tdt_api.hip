// tdt_api.hip — C ABI (include/psyne_tdt.h) over the gfx950 TDT kernels.
//
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC (psyne_amd/build.py).
// The library never falls back to a CPU path: every entry point launches a HIP kernel or
// fails with TDT_E_HIP.
#include "../../include/psyne_tdt.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <sched.h>
#include <string>
#include <vector>

#include "tdt_copypool.h"
#include "tdt_decode.h"
#include "tdt_encode.h"
#include "tdt_slots.h"

// The encode kernels live in tdt_enc_ws.hip (one translation unit per word size); diagnostic
// builds (word size 4 only, phase profiling) instantiate them here instead.
#if !defined(PSY_FAST_BUILD) && !(defined(PSY_PROF) && PSY_PROF) && !defined(PSY_SINGLE_TU)
#define PSY_ENC_EXT(WS, T, G, M, L, TL, PS, PA) \
    extern template __global__ void psy::tdt_encode_kernel<WS, T, G, psy::M, L, TL, PS, PA>(psy::EncodeArgs);
#define PSY_ENC_EXT_WS(WS)                 \
    PSY_ENC_INSTANCES(PSY_ENC_EXT, WS)     \
    extern template __global__ void psy::tdt_encode_lscan_kernel<WS>(psy::EncodeArgs, const uint32_t *, uint32_t);
PSY_ENC_EXT_WS(1)
PSY_ENC_EXT_WS(2)
PSY_ENC_EXT_WS(4)
PSY_ENC_EXT_WS(8)
PSY_ENC_EXT_WS(16)
#endif

namespace {

thread_local std::string g_err;

int set_err(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return set_err(TDT_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_));    \
    } while (0)

bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
}
// A workspace must grow: not possible while the stream is being captured (the allocator and
// the implicit synchronisation of a free are not capturable) — warm the context with one eager
// call of the batch first.
int no_growth_in_capture(hipStream_t s) {
    if (!capturing(s)) return TDT_OK;
    return set_err(TDT_E_CAPTURE, "workspace too small for this batch under stream capture: issue one eager call "
                                  "of the same batch size on this context before capturing");
}

}  // namespace

// Counts of an earlier plan (the slotted calls size their main grids from them; no call ever
// waits for them).  Each call's plan counters are copied into pinned memory behind the plan
// kernel; a later call takes them once that copy has completed.
struct CountHist {
    uint32_t *pin = nullptr;  // pinned: the plan's 8 u64 counters
    hipEvent_t ev = nullptr;
    bool pending = false, valid = false;
    uint32_t v[32] = {};
    uint32_t n = 0, n_pending = 0;  // messages in the snapshot's batch
    // fold the newest completed snapshot in (never waits)
    void refresh() {
        if (pending && hipEventQuery(ev) == hipSuccess) {
            std::memcpy(v, pin, sizeof(v));
            n = n_pending;
            valid = true;
            pending = false;
        }
    }
    void release() {
        if (ev) (void)hipEventDestroy(ev);
        if (pin) (void)hipHostFree(pin);
        ev = nullptr;
        pin = nullptr;
        pending = valid = false;
    }
};

// Workspace of the slotted calls' plan (message classes / large-message state).  One per
// stream user: the context's own, and one per host-pipeline slot (those run concurrently).
struct PlanWS {
    uint8_t *buf = nullptr;  // counters | lists (grows with the batch)
    size_t bytes = 0;
    // large-message state, allocated at a small budget and grown (to the counts a plan reported)
    // when a batch had more large messages than the budget held
    uint8_t *elarge = nullptr;  // encode: LMeta | tile entries | tile records | span entries | span bins
    uint32_t e_lcap = 0, e_tcap = 0;
    uint8_t *dlarge = nullptr;  // decode: DMeta | block entries | block sums | tile entries | tile blocks
    uint32_t d_lcap = 0, d_bcap = 0, d_tcap = 0;
    CountHist eh, dh;  // encode / decode plan counts
    // buffers replaced by a larger one: a graph captured on the context before the growth may
    // still point at them, so they are freed only with the workspace
    std::vector<void *> retired;
    // the large-message pipeline runs on `side` beside the medium/small lists (fork/join events)
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    // host-pipeline slots run without the side stream: their chunks already overlap one another,
    // and every extra stream shares HIP's few hardware queues with the other slots (and with the
    // other end's context in a one-process loopback: C1's encode 6.2 -> 4.0 ms per 50 MiB call)
    bool no_side = false;
    void release() {
        if (join) (void)hipEventDestroy(join);
        if (fork) (void)hipEventDestroy(fork);
        if (side) (void)hipStreamDestroy(side);
        side = nullptr;
        fork = join = nullptr;
        if (buf) (void)hipFree(buf);
        if (elarge) (void)hipFree(elarge);
        if (dlarge) (void)hipFree(dlarge);
        for (void *p : retired) (void)hipFree(p);
        retired.clear();
        buf = elarge = dlarge = nullptr;
        e_lcap = e_tcap = d_lcap = d_bcap = d_tcap = 0;
        eh.release();
        dh.release();
        bytes = 0;
    }
};

// host pipeline slots (chunks in flight per tdt_encode_host / tdt_decode_host call)
constexpr int kHostSlots = 4;

struct tdt_ctx {
    int device = 0;
    tdt_config cfg{};
    std::atomic<double> bandwidth{100.0};  // reference defaults :352-354
    std::atomic<double> latency{1.0};
    std::atomic<double> cpu{0.5};
    std::atomic<uint64_t> size_hint{65536};
    std::mutex mu;
    // workspace: [0..64) counters (ticket, timeout), then one u64 look-back word per message
    uint8_t *ws = nullptr;
    // device buffers a captured graph may still reference after a growth (ws, slot_sums): freed
    // at tdt_ctx_destroy, never while the context lives
    std::vector<void *> retired;
    std::vector<void *> retired_host;  // pinned host-pipeline buffers replaced by larger ones
    size_t ws_bytes = 0;
    // per-chunk sums of tdt_decode_slots' two-pass scan (one u64 per 8192 messages; stream-ordered
    // like `ws`: one slotted decode per context at a time)
    uint64_t *slot_sums = nullptr;
    uint32_t slot_sums_n = 0;
    // host-path device buffers and stream (tdt_analyze_host)
    uint8_t *h_dev = nullptr;
    size_t h_dev_bytes = 0;
    hipStream_t astream = nullptr;
    // host pipeline (tdt_encode_host / tdt_decode_host): kHostSlots slots, each with its own stream,
    // device buffer (input, offsets, output, status, look-back workspace) and pinned offsets
    struct HostSlot {
        hipStream_t stream = nullptr;
        hipEvent_t ev = nullptr;
        uint8_t *dev = nullptr;
        size_t dev_bytes = 0;
        uint64_t *pin = nullptr;  // pinned: in_off (n+1) | out_off (n+1) | status (n, int32 pairs)
        size_t pin_words = 0;
        uint32_t *flag = nullptr;  // pinned: the last chunk's device error flags
        uint8_t *stage_in = nullptr, *stage_out = nullptr;  // pinned staging for pageable callers
        size_t sin_bytes = 0, sout_bytes = 0;
        hipEvent_t evc = nullptr;  // after the chunk's output copy (orders the next chunk's)
        hipEvent_t evi = nullptr;  // after the chunk's input copy (orders the next chunk's)
        PlanWS pw;
    } hs[kHostSlots];
    // the host pipeline's two streams (chunk buffers stay per slot): every input copy on `hin`, in
    // chunk order; every kernel and read-back on `hex`.  Per-slot streams (PSYNE_TDT_SLOT_STREAMS=1,
    // round 4) outnumber the HIP runtime's default 4 hardware queues together with the caller's
    // streams: streams sharing a queue serialised the chunks (profiles/r05_diag/host_decode/)
    hipStream_t hin = nullptr, hex = nullptr;
    bool slot_streams = false;
    // one-message fast path (tdt_encode_host / tdt_decode_host with one message of at most
    // kOneMax bytes: the per-call Protocol::encode / decode of the drop-in class): a mapped pinned
    // block holding the call's offsets, list, status, input and output, read and written by ONE
    // class kernel in place (zero-copy), so a call is two host memcpys, one launch and one sync
    uint8_t *one = nullptr;
    size_t one_bytes = 0;
    hipStream_t one_stream = nullptr;
    std::shared_ptr<CopyPool> pool;  // host threads of the staging copies (shared: tdt_host_copy)
    uint64_t *hbases = nullptr;      // host_encode: device-side running output base per chunk
    size_t hbases_n = 0;
    int copy_threads = 8;
    std::mutex hmu;
    // error flags of the host pipeline's chunks, OR-ed since the context was created
    std::atomic<uint32_t> host_flags{0};
    PlanWS pw;                        // the slotted calls' plan workspace
    // two-phase compacted encode (batches with messages > 64 KiB): slotted blobs, their slots
    // and lengths, then a scan and a gather into the caller's compacted buffer
    uint8_t *cp_buf = nullptr;
    size_t cp_bytes = 0;
    uint64_t *cp_idx = nullptr;  // slots (n + 1) | lengths (n) | flag
    size_t cp_idx_n = 0;
    uint64_t large_min = 256 * 1024;  // messages (decode: decoded blobs) above this take the tiled path
    uint32_t tile_cap = ~0u;          // lower tile budget (tests)
    // diagnostic knobs (read once at tdt_ctx_create from the environment, or tdt_ctx_set_option)
    bool no_side = false;       // PSYNE_TDT_NO_SIDE: no side stream for the tile pipeline
    bool small_main = false;    // PSYNE_TDT_SMALL_MAIN: small lists on the caller's stream
    bool no_two_phase = false;  // PSYNE_TDT_NO_TWO_PHASE: compacted calls take the one-pass kernels
    bool no_one = false;        // PSYNE_TDT_NO_ONE: one-message host calls take the pipeline too
    bool one_wave = false;      // PSYNE_TDT_ONE_WAVE=1: one-message decode as one wave (round-4 path)
    uint64_t one_wave_max = 4096;  // one-message decode: outputs up to this size take the one-wave kernel
    bool dout_sdma = false;     // PSYNE_TDT_DOUT_SDMA=1: host_decode's output by hipMemcpyAsync (round 4)
    bool one_spin = true;       // PSYNE_TDT_ONE_SPIN=0: one-message calls wait in hipStreamSynchronize
    uint32_t one_seq = 0;
    uint32_t copy_wgs = 8;      // PSYNE_TDT_COPY_WGS: copy-list workgroups per CU
    // PSYNE_TDT_DSMALL_MAX: blobs decoding to at most this many bytes take the one-round-window
    // list on the side stream (C4 decode 11.80 -> 11.42 ms at 8 KiB against 1 KiB; 16-64 KiB
    // gave 11.6-11.8, profiles/r03_dsm2/ab.txt)
    uint64_t dsmall_max = 8192;
    uint64_t dbig_min = 128 * 1024;  // PSYNE_TDT_DBIG_MIN: one-wave blobs above this are dispatched first
    int cus = 256;              // compute units (overflow grids)
};

namespace {

constexpr size_t kCounterBytes = 64;

int ensure_ws(tdt_ctx *c, uint32_t n_msgs, hipStream_t s) {
    const size_t need = kCounterBytes + 8ull * (n_msgs + 1);
    if (need > c->ws_bytes) {
        if (int st = no_growth_in_capture(s)) return st;
        if (c->ws) c->retired.push_back(c->ws);  // (a graph captured earlier may use it)
        c->ws = nullptr;
        size_t cap = std::max<size_t>(need, c->ws_bytes * 2);
        HIPCHK(hipMalloc(&c->ws, cap));
        c->ws_bytes = cap;
    }
    return TDT_OK;
}

bool ws_supported(int ws) { return ws == 1 || ws == 2 || ws == 4 || ws == 8 || ws == 16; }

bool policy_on(const tdt_ctx *c) {
    // should_transform :192-200 (the size / tensor-shape terms are evaluated per message on
    // the device)
    return !(c->cpu.load() > c->cfg.cpu_usage_threshold) &&
           c->bandwidth.load() < c->cfg.bandwidth_threshold_mbps;
}

template <int WS, int TEAM, int G, int MODE, int LB, int PATH = psy::PATH_BOTH>
int launch_encode_t(psy::EncodeArgs a, hipStream_t s) {
    // one workgroup per message; a launch holds < 2^32 threads, so very large batches take
    // several (message ids come from the ticket, so the look-back order spans them)
    const uint32_t maxb = 0xffffffffu / TEAM;
    for (uint32_t b = 0; b < a.n_msgs; b += maxb)
        hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, TEAM, G, MODE, LB, 0, 0, PATH>), dim3(std::min(maxb, a.n_msgs - b)),
                           dim3(TEAM), 0, s, a);
    return TDT_OK;
}

// ---------------------------------------------------------------------------------------
// Passthrough copies (UNCP): messages that stay UNCP (encode :227-266: below min_tensor_size, the
// policy off, or a size that is not a whole number of words) and UNCP blobs (decode :271-304) get
// a copy list of their own.  Sixteen lanes per entry, 16 entries per 256-lane workgroup,
// grid-stride over the list (its length is device data); a one-wave team per 64-byte message
// cost a whole wave's launch, LDS and header work.
template <int GL>
__device__ __forceinline__ void lanes_copy_any(uint8_t *dst, const uint8_t *src, uint64_t len, uint32_t l) {
    // 16-byte aligned stores on dst; each 16-byte chunk read as aligned dwords and funnel-shifted
    // by the source misalignment
    uint64_t head = (16 - ((uintptr_t)dst & 15)) & 15;
    if (head > len) head = len;
    if (l < head) dst[l] = src[l];
    const uint64_t nb = (len - head) / 16;
    const uint8_t *s0 = src + head;
    const uint32_t sh = (uint32_t)((uintptr_t)s0 & 3) * 8;
    const uint32_t *sw = reinterpret_cast<const uint32_t *>((uintptr_t)s0 & ~(uintptr_t)3);
    uint4 *dv = reinterpret_cast<uint4 *>(dst + head);
    for (uint64_t k = l; k < nb; k += GL) {
        const uint32_t *q = sw + 4 * k;
        const uint32_t w0 = psy::gload<uint32_t>(q), w1 = psy::gload<uint32_t>(q + 1), w2 = psy::gload<uint32_t>(q + 2),
                       w3 = psy::gload<uint32_t>(q + 3);
        const uint32_t w4 = sh ? psy::gload<uint32_t>(q + 4) : 0u;  // (only when misaligned: inside src)
        dv[k] = make_uint4((uint32_t)((((uint64_t)w1 << 32) | w0) >> sh), (uint32_t)((((uint64_t)w2 << 32) | w1) >> sh),
                           (uint32_t)((((uint64_t)w3 << 32) | w2) >> sh), (uint32_t)((((uint64_t)w4 << 32) | w3) >> sh));
    }
    for (uint64_t k = head + 16 * nb + l; k < len; k += GL) dst[k] = src[k];
}

// encode: blob = "UNCP" + payload in the message's slot (slotted batches)
__global__ __launch_bounds__(256) void tdt_encode_copy_kernel(psy::EncodeArgs a) {
    const uint32_t n = __builtin_amdgcn_readfirstlane(*a.list_count);
    const uint32_t q = threadIdx.x >> 4, l = threadIdx.x & 15u;
    for (uint32_t i = blockIdx.x * 16u + q; i < n; i += gridDim.x * 16u) {
        const uint32_t msg = a.list[i];
        const uint64_t off0 = a.in_off[msg], len = a.in_off[msg + 1] - off0;
        const uint64_t sb = a.slot_off[msg], E = len + 4;
        const bool fits = E <= a.slot_off[msg + 1] - sb;
        if (l == 0) {
            if (a.status) a.status[msg] = fits ? psy::ST_OK : psy::ST_CAPACITY;
            if (a.out_len) a.out_len[msg] = fits ? E : 0;
        }
        if (!fits) continue;
        uint8_t *dst = a.out + sb;
        if (l < 4) dst[l] = (uint8_t)(psy::kMagicUNCP >> (8 * l));
        lanes_copy_any<16>(dst + 4, a.in + off0, len, l);
    }
}

// decode: payload of a UNCP blob into its slot
__global__ __launch_bounds__(256) void tdt_decode_copy_kernel(psy::DecodeArgs a) {
    const uint32_t n = __builtin_amdgcn_readfirstlane(*a.list_count);
    const uint32_t q = threadIdx.x >> 4, l = threadIdx.x & 15u;
    for (uint32_t i = blockIdx.x * 16u + q; i < n; i += gridDim.x * 16u) {
        const uint32_t msg = a.list[i];
        const uint64_t boff = a.in_off[msg];
        const uint64_t len = a.in_len ? a.in_len[msg] : a.in_off[msg + 1] - boff;  // >= 4 (the plan)
        const uint64_t ob = a.slot_off[msg], osize = len - 4;
        const bool fits = osize <= a.slot_off[msg + 1] - ob;
        if (l == 0) {
            if (a.out_len) a.out_len[msg] = fits ? osize : 0;
            if (a.status) a.status[msg] = fits ? psy::ST_OK : psy::ST_CAPACITY;
        }
        if (fits) lanes_copy_any<16>(a.out + ob, a.in + boff + 4, osize, l);
    }
}

// ---------------------------------------------------------------------------------------
// Slotted encode (the hot path): a plan kernel sorts the messages into classes — large
// messages as 64 KiB tiles (histogram + mapping, count, scan, emit), medium messages one
// 512-lane team each, small ones one wave each — into lists whose lengths stay in device
// memory.  The host never reads them: each class kernel is launched twice, a main launch of
// one workgroup per entry whose grid comes from an EARLIER call's counts (CountHist: slack on
// top; the batch size before any count is known), and an overflow launch that walks the
// entries past that grid (grid-stride; it exits at once when there are none).  A class that
// an earlier plan found empty is switched off in the plan (its messages join the medium list,
// which takes any size), so repeated batches of one shape launch exactly what they need.
// Calls are therefore asynchronous and capturable (hipGraphs).
constexpr uint64_t kSmallMax = 4096;  // one-wave teams up to this size
// medium messages above this (the streaming body: more than 8 resident rounds per wave) are
// dispatched first
constexpr uint64_t kBigMin = 65536;
// 256-lane teams (4 waves, 8 resident rounds each: 32 KiB) above kSmallMax up to this size: a
// message-sized 512-lane team would give each wave at most four rounds, and the per-wave fixed
// work (entropy share, flush set-up, header) would weigh twice as much per byte
constexpr uint64_t kMidMax = 32768;
constexpr uint32_t kLmax = 1u << 16;   // large messages per batch (full budget)
// tiles per batch at the full budget: 256 MiB of span histograms (WS KiB per 512 KiB span) —
// 32 GiB of large messages at word size 4 (C4's 4 Mi-message Zipf batch holds 12 GiB of them);
// further large messages in the batch stay medium (one 512-lane team each, streaming)
uint32_t tile_cap_of(int ws) { return (262144u / (uint32_t)ws) * psy::kSpanTiles; }
// the budget a context starts with (512 MiB of large messages); plans that claim more grow it
constexpr uint32_t kL0 = 1024, kT0 = 8192;
size_t elarge_bytes(uint32_t lcap, uint32_t tcap, int ws) {
    const size_t sc = tcap / psy::kSpanTiles;
    // LMeta | tile entries | tile records | span entries | span bins | count-pass tile list
    return (size_t)lcap * sizeof(psy::LMeta) + (size_t)tcap * (8 + sizeof(psy::TileRec)) + sc * 8 + sc * ws * 1024 +
           (size_t)tcap * 8;
}
uint32_t pow2_at_least(uint64_t x, uint32_t lo, uint32_t hi) {
    uint64_t p = lo;
    while (p < x && p < hi) p *= 2;
    return (uint32_t)std::min<uint64_t>(p, hi);
}

int ensure_plan(PlanWS &w, uint32_t n, hipStream_t s) {
    const size_t need = 256 + 20ull * n;  // counters | small | medium | mid-sized | big | copy lists
    if (need > w.bytes) {
        if (int st = no_growth_in_capture(s)) return st;
        if (w.buf) w.retired.push_back(w.buf);  // (a graph captured earlier may use it)
        w.buf = nullptr;
        const size_t cap = std::max(need, w.bytes * 2);
        HIPCHK(hipMalloc(&w.buf, cap));
        w.bytes = cap;
    }
    return TDT_OK;
}

// Small device → pinned-host copies (plan counters, a host chunk's lengths / statuses / error
// flags) as one kernel's stores over PCIe rather than DMA commands: a DMA read-back queued behind
// a chunk's kernels held up the next chunks' input DMAs behind it (profiles/r05_diag/host_decode/)
struct SmallCopies {
    const uint32_t *src[3];
    uint32_t *dst[3];
    uint32_t words[3];
};
__global__ __launch_bounds__(256) void small_copy_kernel(SmallCopies a) {
    for (int k = 0; k < 3; ++k)
        for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < a.words[k]; i += gridDim.x * 256) a.dst[k][i] = a.src[k][i];
}
int small_copies(hipStream_t s, const void *s0, void *d0, size_t b0, const void *s1 = nullptr, void *d1 = nullptr,
                 size_t b1 = 0, const void *s2 = nullptr, void *d2 = nullptr, size_t b2 = 0) {
    SmallCopies a{{static_cast<const uint32_t *>(s0), static_cast<const uint32_t *>(s1), static_cast<const uint32_t *>(s2)},
                  {static_cast<uint32_t *>(d0), static_cast<uint32_t *>(d1), static_cast<uint32_t *>(d2)},
                  {(uint32_t)(b0 / 4), (uint32_t)(b1 / 4), (uint32_t)(b2 / 4)}};
    const size_t mx = std::max(b0, std::max(b1, b2)) / 4;
    hipLaunchKernelGGL(small_copy_kernel, dim3((uint32_t)std::min<size_t>(64, mx / 1024 + 1)), dim3(256), 0, s, a);
    HIPCHK(hipGetLastError());
    return TDT_OK;
}

// The plan counters of this call → pinned snapshot (not under stream capture).
int record_counts(CountHist &h, const void *dcnt, uint32_t n_msgs, hipStream_t s) {
    if (!h.pin) {
        HIPCHK(hipHostMalloc(&h.pin, 128, hipHostMallocDefault));
        HIPCHK(hipEventCreateWithFlags(&h.ev, hipEventDisableTiming));
    }
    if (int st = small_copies(s, dcnt, h.pin, 128)) return st;
    HIPCHK(hipEventRecord(h.ev, s));
    h.n_pending = n_msgs;
    h.pending = true;
    return TDT_OK;
}

// Main-launch grid of a class: the earlier count plus slack (capped), or `dflt` before any.
uint32_t guess(const CountHist &h, int idx, uint32_t bound, uint32_t dflt) {
    if (!h.valid) return std::min(dflt, bound);
    const uint64_t x = h.v[idx];
    return (uint32_t)std::min<uint64_t>(x + x / 8 + 64, bound);
}

// fork `s` onto the side stream (high priority: the tile pipeline is a chain of dependent
// kernels; the independent medium/small lists fill the CUs it leaves idle at each boundary)
int fork_side(PlanWS &w, hipStream_t s) {
    if (!w.side) {
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&w.side, hipStreamNonBlocking, hi));
        HIPCHK(hipEventCreateWithFlags(&w.fork, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&w.join, hipEventDisableTiming));
    }
    HIPCHK(hipEventRecord(w.fork, s));
    HIPCHK(hipStreamWaitEvent(w.side, w.fork, 0));
    return TDT_OK;
}
int join_side(PlanWS &w, hipStream_t s) {
    HIPCHK(hipEventRecord(w.join, w.side));
    HIPCHK(hipStreamWaitEvent(s, w.join, 0));
    return TDT_OK;
}

// Large-message budget: allocated on the first batch that may hold large messages, grown to
// what an earlier plan claimed.
int ensure_elarge(PlanWS &w, int ws, hipStream_t s) {
    uint32_t lc = w.e_lcap ? w.e_lcap : kL0, tc = w.e_tcap ? w.e_tcap : kT0;
    if (w.eh.valid) {
        lc = std::max(lc, pow2_at_least(w.eh.v[4], kL0, kLmax));
        tc = std::max(tc, pow2_at_least(std::max<uint64_t>(w.eh.v[6], (uint64_t)w.eh.v[8] * psy::kSpanTiles), kT0,
                                        tile_cap_of(ws)));
    }
    if (w.elarge && lc == w.e_lcap && tc == w.e_tcap) return TDT_OK;
    if (w.elarge) {
        // retired, not freed: earlier calls still queued, or a graph captured on the warm
        // context, may use the old records (their launches carry the old budgets)
        w.retired.push_back(w.elarge);
        w.elarge = nullptr;
        w.e_lcap = w.e_tcap = 0;
    }
    const size_t b = elarge_bytes(lc, tc, ws);
    HIPCHK(hipMalloc(&w.elarge, b));
    HIPCHK(hipMemsetAsync(w.elarge, 0, b, s));
    w.e_lcap = lc;
    w.e_tcap = tc;
    return TDT_OK;
}

// grid of one list-driven launch of TEAM-lane workgroups over `count` entries (launches of
// < 2^32 threads each)
template <class F>
void launch_list(uint32_t count, uint32_t team, F &&launch) {
    const uint32_t mx = 0xffffffffu / team;
    for (uint32_t b = 0; b < count; b += mx) launch(b, std::min(mx, count - b));
}

template <int WS>
int launch_slotted(tdt_ctx *c, PlanWS &pw, psy::EncodeArgs a, hipStream_t s) {
    using psy::MODE_ENCODE;
    const uint32_t n = a.n_msgs;
    int st = ensure_plan(pw, n, s);
    if (st) return st;
    const bool capturing = ::capturing(s);
    CountHist &H = pw.eh;
    if (!capturing) H.refresh();  // (event queries are not capturable)
    // classes an earlier plan found empty are off (their messages, if any, go medium)
    const bool small_on = !H.valid || H.v[10] > 0;  // (counter 5: small messages, listed or not)
    const bool mid_on = !H.valid || H.v[14] > 0;    // (counter 7: mid-sized messages, listed or not)
    const bool copy_on = !H.valid || H.v[18] > 0;   // (counter 9: UNCP messages)
    bool tiles_on = !H.valid || H.v[4] > 0;
    if (tiles_on && !capturing) {
        st = ensure_elarge(pw, WS, s);
        if (st) return st;
    }
    tiles_on = tiles_on && pw.elarge;
    auto *cnt64 = reinterpret_cast<unsigned long long *>(pw.buf);
    auto *cnt = reinterpret_cast<uint32_t *>(pw.buf);  // cnt[2k]: the low word of counter k
    uint32_t *slist = reinterpret_cast<uint32_t *>(pw.buf + 256), *mlist = slist + n, *qlist = mlist + n,
             *blist = qlist + n, *clist = blist + n;
    const uint32_t lcap = tiles_on ? pw.e_lcap : 0u;
    const uint32_t tcap = tiles_on ? std::min(pw.e_tcap, std::max(c->tile_cap, psy::kSpanTiles)) : 0u;
    const uint32_t scap = tcap / psy::kSpanTiles;
    auto *lmeta = reinterpret_cast<psy::LMeta *>(pw.elarge);
    auto *tiles = reinterpret_cast<uint64_t *>(pw.elarge + (size_t)pw.e_lcap * sizeof(psy::LMeta));
    auto *trec = reinterpret_cast<psy::TileRec *>(reinterpret_cast<uint8_t *>(tiles) + 8ull * pw.e_tcap);
    auto *spans =
        reinterpret_cast<uint64_t *>(reinterpret_cast<uint8_t *>(trec) + sizeof(psy::TileRec) * pw.e_tcap);
    auto *shist = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(spans) + 8ull * (pw.e_tcap / psy::kSpanTiles));
    auto *rtiles = reinterpret_cast<uint64_t *>(shist + (size_t)(pw.e_tcap / psy::kSpanTiles) * WS * 256);
    HIPCHK(hipMemsetAsync(cnt, 0, 128, s));
    psy::PlanArgs p{a.in,      a.in_off,  n,       cnt64,   slist,          mlist,              qlist,
                    blist,     clist,   tiles,   spans,          lmeta,              lcap,
                    tcap,      kSmallMax, kMidMax, kBigMin,      c->large_min,       small_on ? 1u : 0u,
                    mid_on ? 1u : 0u, a.min_tensor, (uint32_t)a.policy_on, (uint32_t)WS, copy_on ? 1u : 0u};
    const uint32_t per = psy::kPlanThreads * psy::kPlanPer;
    hipLaunchKernelGGL(psy::tdt_encode_plan_kernel, dim3((uint32_t)(((uint64_t)n + per - 1) / per)),
                       dim3(psy::kPlanThreads), 0, s, p);
    HIPCHK(hipGetLastError());
    // (with tiles, the snapshot follows the map pass instead: it also holds the count pass's list length)
    if (!capturing && !tiles_on && (st = record_counts(H, cnt, n, s))) return st;
    a.pcnt = cnt;
    const uint32_t ovf512 = (uint32_t)c->cus * 3, ovf256 = (uint32_t)c->cus * 6, ovf64 = (uint32_t)c->cus * 24;
    // main launch over [0, g) + overflow launch over [g, count) of one class
    auto both = [&](uint32_t g, uint32_t bound, uint32_t ovf, auto &&main, auto &&over) {
        if (g) main(0u, g);
        if (g < bound) over(g, std::min(ovf, bound - g));
    };
    bool forked = false;
    hipStream_t ts = s;  // the tile pipeline's (and the small / mid-sized lists') stream
    // the side stream carries the tile pipeline and the small / mid-sized lists beside the medium
    // list (queued behind it on one stream they would run alone in its tail)
    const bool medium_on = !H.valid || H.v[2] + H.v[16] > 0;  // (counters 1 and 8)
    if (tiles_on || ((small_on || mid_on || copy_on) && medium_on && !c->small_main)) {
        const int fr = c->no_side || pw.no_side ? -1 : fork_side(pw, s);
        if (fr > 0) return fr;
        forked = fr == TDT_OK;
        if (forked) ts = pw.side;
    }
    if (tiles_on) {
        a.tiles = tiles;
        a.spans = spans;
        a.lmeta = lmeta;
        a.trec = trec;
        a.shist = shist;
        a.rtiles = rtiles;
        a.rcount = cnt64 + 11;
        a.lcap = lcap;
        a.tcap = tcap;
#define PSY_TILE_STEP(TL, IDX, BOUND)                                                                           \
        both(guess(H, IDX, BOUND, 0), BOUND, ovf512,                                                            \
             [&](uint32_t b, uint32_t g) {                                                                      \
                 a.list_base = b;                                                                               \
                 hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 512, 8, MODE_ENCODE, 0, TL, 0>), dim3(g), dim3(512), \
                                    0, ts, a);                                                                  \
             },                                                                                                 \
             [&](uint32_t b, uint32_t g) {                                                                      \
                 a.list_base = b;                                                                               \
                 hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 512, 8, MODE_ENCODE, 0, TL, 1>), dim3(g), dim3(512), \
                                    0, ts, a);                                                                  \
             })
        PSY_TILE_STEP(1, 8, scap);  // span histograms (and counts under the speculated mapping)
        PSY_TILE_STEP(4, 4, lcap);  // mapping per large message; lists the tiles to count again
        if (!capturing && (st = record_counts(H, cnt, n, ts))) return st;
        PSY_TILE_STEP(2, 22, tcap);  // per-tile counts of the listed tiles
        hipLaunchKernelGGL((psy::tdt_encode_lscan_kernel<WS>), dim3(std::max(1u, std::min(lcap, 1024u))), dim3(64), 0,
                           ts, a, cnt + 4, lcap);
        PSY_TILE_STEP(3, 6, tcap);  // emit
#undef PSY_TILE_STEP
    }
    // medium messages: one workgroup per list entry — the big list first (longer or unaligned
    // messages: the streaming-only kernel; a long team started last would run alone in the
    // kernel's tail), then the medium list (resident-only kernel)
    a.list2 = nullptr;
    {
        // (always launched: messages of a class switched off join it; the overflow launch ends at
        // once when the list is empty)
        a.list = blist;
        a.list_count = cnt + 16;
        both(H.valid ? (H.v[16] ? guess(H, 16, n, n) : 0u) : n, n, ovf512,
             [&](uint32_t b, uint32_t g) {
                 launch_list(g, 512, [&](uint32_t b2, uint32_t g2) {
                     a.list_base = b + b2;
                     hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 512, 8, MODE_ENCODE, 0, 0, 0, psy::PATH_STREAM>),
                                        dim3(g2), dim3(512), 0, s, a);
                 });
             },
             [&](uint32_t b, uint32_t g) {
                 a.list_base = b;
                 hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 512, 8, MODE_ENCODE, 0, 0, 1, psy::PATH_STREAM>), dim3(g),
                                    dim3(512), 0, s, a);
             });
    }
    a.list = mlist;
    a.list_count = cnt + 2;
    const uint32_t gmed = H.valid ? guess(H, 2, n, n) : n;
    both(gmed, n, ovf512,
         [&](uint32_t b, uint32_t g) {
             launch_list(g, 512, [&](uint32_t b2, uint32_t g2) {
                 a.list_base = b + b2;
                 hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 512, 8, MODE_ENCODE, 0, 0, 0, psy::PATH_RES>), dim3(g2),
                                    dim3(512), 0, s, a);
             });
         },
         [&](uint32_t b, uint32_t g) {
             a.list_base = b;
             hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 512, 8, MODE_ENCODE, 0, 0, 1, psy::PATH_RES>), dim3(g),
                                dim3(512), 0, s, a);
         });
    // small messages behind the tile pipeline on the side stream (the two streams' loads balance
    // better: C4's tile pipeline is shorter than its medium list)
    if (small_on) {
        const hipStream_t ss = forked && !c->small_main ? pw.side : s;
        a.list = slist;
        a.list_count = cnt;
        both(guess(H, 0, n, n), n, ovf64,
             [&](uint32_t b, uint32_t g) {
                 launch_list(g, 64, [&](uint32_t b2, uint32_t g2) {
                     a.list_base = b + b2;
                     hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 64, 4, MODE_ENCODE, 0, 0, 0>), dim3(g2), dim3(64),
                                        0, ss, a);
                 });
             },
             [&](uint32_t b, uint32_t g) {
                 a.list_base = b;
                 hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 64, 4, MODE_ENCODE, 0, 0, 1>), dim3(g), dim3(64), 0,
                                    ss, a);
             });
    }
    // passthrough copies on the small list's stream
    if (copy_on) {
        a.list = clist;
        a.list_count = cnt + 20;
        hipLaunchKernelGGL(tdt_encode_copy_kernel, dim3(std::max(1u, std::min((uint32_t)c->cus * c->copy_wgs, (n + 15) / 16))),
                           dim3(256), 0, forked && !c->small_main ? pw.side : s, a);
    }
    // mid-sized messages (256-lane teams) on the small list's stream
    if (mid_on) {
        const hipStream_t qs = forked && !c->small_main ? pw.side : s;
        a.list = qlist;
        a.list_count = cnt + 12;
        both(guess(H, 12, n, n), n, ovf256,
             [&](uint32_t b, uint32_t g) {
                 launch_list(g, 256, [&](uint32_t b2, uint32_t g2) {
                     a.list_base = b + b2;
                     hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 256, 8, MODE_ENCODE, 0, 0, 0>), dim3(g2),
                                        dim3(256), 0, qs, a);
                 });
             },
             [&](uint32_t b, uint32_t g) {
                 a.list_base = b;
                 hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 256, 8, MODE_ENCODE, 0, 0, 1>), dim3(g), dim3(256), 0,
                                    qs, a);
             });
    }
    if (forked) return join_side(pw, s);
    return TDT_OK;
}

int launch_slotted_any(tdt_ctx *c, PlanWS &pw, psy::EncodeArgs a, hipStream_t s) {
    switch (c->cfg.word_size) {
#ifdef PSY_FAST_BUILD
        case 4: return launch_slotted<4>(c, pw, a, s);
#else
        case 1: return launch_slotted<1>(c, pw, a, s);
        case 2: return launch_slotted<2>(c, pw, a, s);
        case 4: return launch_slotted<4>(c, pw, a, s);
        case 8: return launch_slotted<8>(c, pw, a, s);
        case 16: return launch_slotted<16>(c, pw, a, s);
#endif
    }
    return set_err(TDT_E_UNSUPPORTED, "word_size not supported on the GPU path");
}

// messages > 4 KiB: TEAM threads per message, G resident rounds per wave (64 KiB resident)
#ifndef PSY_BIG_TEAM
#define PSY_BIG_TEAM 512
#define PSY_BIG_G 8
#endif

// res: every message is aligned, a whole number of 16-byte groups and at most 64 KiB (the
// caller checked): the resident-only kernel (without the streaming body's live registers; the
// one-pass compacted C3 encode 9.58 ms with both bodies)
template <int WS, int MODE, int LB>
int launch_encode_ws(psy::EncodeArgs a, bool small, bool res, hipStream_t s) {
    if (small) return launch_encode_t<WS, 64, 4, MODE, LB>(a, s);
    if constexpr (MODE == psy::MODE_ENCODE && LB == 1 && PSY_BIG_TEAM == 512 && PSY_BIG_G == 8)
        if (res) return launch_encode_t<WS, 512, 8, MODE, LB, psy::PATH_RES>(a, s);
    return launch_encode_t<WS, PSY_BIG_TEAM, PSY_BIG_G, MODE, LB>(a, s);
}

// LB: compacted output (look-back) vs slotted output
// Team shape of a one-pass (look-back) launch when the caller does not know the batch's sizes:
// one-wave teams when most messages of this context's latest slotted plan were small (<= 4 KiB),
// the size hint only before any plan has been observed.
bool lb_small_teams(tdt_ctx *c, hipStream_t s) {
    CountHist &H = c->pw.eh;
    if (!capturing(s)) H.refresh();
    if (H.valid && H.n) return 2ull * ((uint64_t)H.v[10] + H.v[18]) > H.n;  // (counters 5, 9: small, UNCP)
    return c->size_hint.load() <= kSmallMax;
}

// small_teams: -1 from the context's history, 0 message-sized teams, 1 one-wave teams, 2
// message-sized resident-only teams (see launch_encode_ws)
template <int MODE, int LB>
int launch_encode(tdt_ctx *c, psy::EncodeArgs a, hipStream_t s, int small_teams) {
    const bool small = small_teams < 0 ? lb_small_teams(c, s) : small_teams == 1;
    const bool res = small_teams == 2;
    switch (c->cfg.word_size) {
#ifdef PSY_FAST_BUILD  // diagnostic builds: word_size 4 only
        case 4: return launch_encode_ws<4, MODE, LB>(a, small, res, s);
#else
        case 1: return launch_encode_ws<1, MODE, LB>(a, small, res, s);
        case 2: return launch_encode_ws<2, MODE, LB>(a, small, res, s);
        case 4: return launch_encode_ws<4, MODE, LB>(a, small, res, s);
        case 8: return launch_encode_ws<8, MODE, LB>(a, small, res, s);
        case 16: return launch_encode_ws<16, MODE, LB>(a, small, res, s);
#endif
    }
    return set_err(TDT_E_UNSUPPORTED, "word_size not supported on the GPU path");
}

// Zero the counters + look-back words of a batch; `wsp` = an explicit workspace (host
// pipeline slots) or null for the context's own.  Slotted batches (no look-back, message id =
// block index) only need the counter block for the error flags, zeroed once per context.
int prep(tdt_ctx *c, uint32_t n_msgs, hipStream_t s, uint8_t *&wsp, bool lookback = true) {
    HIPCHK(hipSetDevice(c->device));
    if (!wsp) {
        const bool fresh = c->ws == nullptr;
        int st = ensure_ws(c, lookback ? n_msgs : 0, s);
        if (st) return st;
        wsp = c->ws;
        if (!lookback) {
            if (fresh) HIPCHK(hipMemsetAsync(wsp, 0, kCounterBytes, s));
            return TDT_OK;
        }
    } else if (!lookback) {
        HIPCHK(hipMemsetAsync(wsp, 0, kCounterBytes, s));  // pipeline chunk: fresh error flags
        return TDT_OK;
    }
    HIPCHK(hipMemsetAsync(wsp, 0, kCounterBytes + 8ull * n_msgs, s));
    return TDT_OK;
}

int encode_common(tdt_ctx *c, int mode, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs,
                  const int32_t *d_mapping, uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off,
                  int32_t *d_status, uint32_t *d_hist, double *d_ent, int32_t *d_map, void *stream,
                  const uint64_t *d_slot_off = nullptr, uint64_t *d_out_len = nullptr, uint8_t *wsp = nullptr,
                  PlanWS *pws = nullptr, int small_teams = -1) {
    if (!c) return set_err(TDT_E_ARG, "null context");
    if (n_msgs == 0) return TDT_OK;
    if (!d_in_off) return set_err(TDT_E_ARG, "null input offsets");  // d_in may be null: all-empty batch
    const bool slotted = d_slot_off != nullptr;
    if (mode != psy::MODE_ANALYZE && (!d_out || (!slotted && !d_out_off))) return set_err(TDT_E_ARG, "null output");
    if (mode == psy::MODE_MAPPED && !d_mapping) return set_err(TDT_E_ARG, "null mapping");
    hipStream_t s = (hipStream_t)stream;
    std::unique_lock<std::mutex> lk(c->mu, std::defer_lock);
    if (!wsp) lk.lock();  // pipeline slots own their workspace
    int st = prep(c, n_msgs, s, wsp, !slotted);
    if (st) return st;
    psy::EncodeArgs a{};
    a.in = d_in;
    a.in_off = d_in_off;
    a.n_msgs = n_msgs;
    a.out = d_out;
    a.out_cap = out_cap;
    a.out_off = d_out_off;
    a.status = d_status;
    a.mapping_in = d_mapping;
    a.hist_out = d_hist;
    a.ent_out = d_ent;
    a.map_out = d_map;
    a.ticket = reinterpret_cast<uint32_t *>(wsp);
    a.errflags = reinterpret_cast<uint32_t *>(wsp) + 1;
    a.lookback = reinterpret_cast<uint64_t *>(wsp + kCounterBytes);
    a.min_tensor = c->cfg.min_tensor_size;
    a.policy_on = policy_on(c) ? 1 : 0;
    a.slot_off = d_slot_off;
    a.out_len = d_out_len;
    if (mode == psy::MODE_ENCODE) {
        st = slotted ? launch_slotted_any(c, pws ? *pws : c->pw, a, s)
                     : launch_encode<psy::MODE_ENCODE, 1>(c, a, s, small_teams);
    } else if (mode == psy::MODE_MAPPED) {
        st = launch_encode<psy::MODE_MAPPED, 1>(c, a, s, small_teams);
    } else {
        st = launch_encode<psy::MODE_ANALYZE, 1>(c, a, s, small_teams);
    }
    if (st) return st;
    HIPCHK(hipGetLastError());
    return TDT_OK;
}

// Slotted decode: a plan kernel separates the large blobs (decoded size > large_min and
// > 1/4096 of the batch) and the blobs decoding to <= 1 KiB from the rest; the rest decode one
// wave each, the small ones one wave each with one-round windows, the large ones through the
// prep / block / scan / tile passes (tdt_decode.h).  As for encode, the list lengths stay on
// the device: main grids from an earlier call's counts, overflow launches past them.
constexpr uint32_t kDLmax = 1u << 16, kDBcap = 1u << 23, kDTcap = 1u << 20;  // full budgets
constexpr uint32_t kDL0 = 1024, kDB0 = 1u << 16, kDT0 = 8192;                 // starting budgets
size_t dlarge_bytes(uint32_t lcap, uint32_t bcap, uint32_t tcap) {
    return (size_t)lcap * sizeof(psy::DMeta) + 8ull * bcap + 4ull * tcap + 8ull * tcap;
}

int ensure_dlarge(PlanWS &w) {
    uint32_t lc = w.d_lcap ? w.d_lcap : kDL0, bc = w.d_bcap ? w.d_bcap : kDB0, tc = w.d_tcap ? w.d_tcap : kDT0;
    if (w.dh.valid) {
        lc = std::max(lc, pow2_at_least(w.dh.v[2], kDL0, kDLmax));
        tc = std::max(tc, pow2_at_least(w.dh.v[4], kDT0, kDTcap));
        bc = std::max(bc, pow2_at_least(w.dh.v[6], kDB0, kDBcap));
    }
    if (w.dlarge && lc == w.d_lcap && bc == w.d_bcap && tc == w.d_tcap) return TDT_OK;
    if (w.dlarge) {
        w.retired.push_back(w.dlarge);  // (as ensure_elarge)
        w.dlarge = nullptr;
        w.d_lcap = w.d_bcap = w.d_tcap = 0;
    }
    HIPCHK(hipMalloc(&w.dlarge, dlarge_bytes(lc, bc, tc)));
    w.d_lcap = lc;
    w.d_bcap = bc;
    w.d_tcap = tc;
    return TDT_OK;
}

int launch_decode_slotted(tdt_ctx *c, PlanWS &pw, psy::DecodeArgs a, hipStream_t s) {
    const uint32_t n = a.n_msgs;
    int st = ensure_plan(pw, n, s);
    if (st) return st;
    const bool capturing = ::capturing(s);
    CountHist &H = pw.dh;
    if (!capturing) H.refresh();
    const bool small_on = !H.valid || H.v[10] > 0;  // counter 5: small blobs, listed or not
    const bool copy_on = !H.valid || H.v[14] > 0;   // counter 7: UNCP blobs
    bool large_on = !H.valid || H.v[2] > 0;
    if (large_on && !capturing) {
        st = ensure_dlarge(pw);
        if (st) return st;
    }
    large_on = large_on && pw.dlarge;
    auto *cnt = reinterpret_cast<unsigned long long *>(pw.buf);
    auto *cnt32 = reinterpret_cast<uint32_t *>(pw.buf);
    auto *list = reinterpret_cast<uint32_t *>(pw.buf + 256);
    uint32_t *slist = list + n, *blist = slist + n, *clist = blist + n;
    const uint32_t lcap = large_on ? pw.d_lcap : 0u, bcap = large_on ? pw.d_bcap : 0u,
                   tcap = large_on ? pw.d_tcap : 0u;
    auto *dmeta = reinterpret_cast<psy::DMeta *>(pw.dlarge);
    auto *bent = reinterpret_cast<uint32_t *>(pw.dlarge + (size_t)pw.d_lcap * sizeof(psy::DMeta));
    uint32_t *bsum = bent + pw.d_bcap, *tent = bsum + pw.d_bcap, *tblk = tent + pw.d_tcap;
    HIPCHK(hipMemsetAsync(cnt, 0, 128, s));
    psy::DPlanArgs p{a.in, a.in_off, a.in_len, n, cnt, list, slist, c->dsmall_max, blist, c->dbig_min, clist, dmeta,
                     bent, tent, lcap, bcap, tcap, c->large_min, small_on ? 1u : 0u, copy_on ? 1u : 0u};
    hipLaunchKernelGGL(psy::tdt_decode_plan_kernel, dim3((uint32_t)(((uint64_t)n + 4095) / 4096)), dim3(1024), 0, s, p);
    HIPCHK(hipGetLastError());
    if (!capturing && (st = record_counts(H, cnt, n, s))) return st;
    a.dmeta = dmeta;
    a.bent = bent;
    a.bsum = bsum;
    a.tent = tent;
    a.tblk = tblk;
    a.pcnt = cnt32;
    a.lcap = lcap;
    a.bcap = bcap;
    a.tcap = tcap;
    const uint32_t ovf = (uint32_t)c->cus * 32;
    // one-wave list kernels: main launch over [0, g), overflow launch over [g, count)
    auto lists = [&](uint32_t g, hipStream_t ls, auto main_k, auto over_k) {
        if (g) launch_list(g, 64, [&](uint32_t b, uint32_t k) {
            a.list_base = b;
            hipLaunchKernelGGL(main_k, dim3(k), dim3(64), 0, ls, a);
        });
        if (g < n) {
            a.list_base = g;
            hipLaunchKernelGGL(over_k, dim3(std::min(ovf, n - g)), dim3(64), 0, ls, a);
        }
    };
    bool forked = false;
    hipStream_t ts = s;
    // the side stream carries the large-blob pipeline and the small-blob list beside the main
    // list (the small list queued behind the main list ran alone in its tail: C4 1.6 ms)
    const bool main_on = !H.valid || H.v[0] + H.v[12] > 0;  // (counters 0 and 6)
    if (large_on || ((small_on || copy_on) && main_on && !c->small_main)) {
        const int fr = c->no_side || pw.no_side ? -1 : fork_side(pw, s);
        if (fr > 0) return fr;
        forked = fr == TDT_OK;
        if (forked) ts = pw.side;
    }
    if (large_on) {
        const uint32_t gl = std::max(1u, std::min(lcap, 1024u));
        hipLaunchKernelGGL(psy::tdt_decode_lprep_kernel, dim3(gl), dim3(256), 0, ts, a);
        hipLaunchKernelGGL(psy::tdt_decode_lblock_kernel, dim3(std::max(1u, std::min((bcap + 3) / 4, ovf / 4))),
                           dim3(256), 0, ts, a);
        hipLaunchKernelGGL(psy::tdt_decode_lscan_kernel, dim3(gl, 2), dim3(64), 0, ts, a);
        const uint32_t gt = guess(H, 4, tcap, 0);
        if (gt) {
            a.list_base = 0;
            hipLaunchKernelGGL(psy::tdt_decode_ltile_kernel<0>, dim3(gt), dim3(64), 0, ts, a);
        }
        if (gt < tcap) {
            a.list_base = gt;
            hipLaunchKernelGGL(psy::tdt_decode_ltile_kernel<1>, dim3(std::min(ovf, tcap - gt)), dim3(64), 0, ts, a);
        }
    }
    a.list = list;
    a.list_count = cnt32;
    a.blist = blist;
    a.blist_count = cnt32 + 12;
    const uint32_t gmain = H.valid ? std::min<uint32_t>(n, guess(H, 0, n, n) + guess(H, 12, n, n)) : n;
    lists(gmain, s, psy::tdt_decode_kernel<0, psy::kDecWR, 0>, psy::tdt_decode_kernel<0, psy::kDecWR, 1>);
    a.blist = nullptr;
    // passthrough copies beside the main list
    if (copy_on) {
        a.list = clist;
        a.list_count = cnt32 + 16;
        hipLaunchKernelGGL(tdt_decode_copy_kernel, dim3(std::max(1u, std::min((uint32_t)c->cus * c->copy_wgs, (n + 15) / 16))),
                           dim3(256), 0, forked && !c->small_main ? pw.side : s, a);
    }
    // small blobs: one-round windows (a third less LDS per wave: more blobs in flight per CU)
    if (small_on) {
        a.list = slist;
        a.list_count = cnt32 + 8;
        lists(guess(H, 8, n, n), forked && !c->small_main ? pw.side : s, psy::tdt_decode_kernel<0, 1, 0>,
              psy::tdt_decode_kernel<0, 1, 1>);
    }
    if (forked) return join_side(pw, s);
    return TDT_OK;
}

int decode_common(tdt_ctx *c, bool sizes_only, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs,
                  uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off, uint64_t *d_sizes, int32_t *d_status,
                  void *stream, const uint64_t *d_slot_off = nullptr, uint64_t *d_out_len = nullptr,
                  const uint64_t *d_in_len = nullptr, uint8_t *wsp = nullptr, PlanWS *pws = nullptr) {
    if (!c) return set_err(TDT_E_ARG, "null context");
    if (n_msgs == 0) return TDT_OK;
    if (!d_in_off) return set_err(TDT_E_ARG, "null input offsets");
    const bool slotted = d_slot_off != nullptr;
    if (!sizes_only && !slotted && !d_out_off) return set_err(TDT_E_ARG, "null output offsets");
    if (sizes_only && !d_sizes) return set_err(TDT_E_ARG, "null sizes");
    hipStream_t s = (hipStream_t)stream;
    std::unique_lock<std::mutex> lk(c->mu, std::defer_lock);
    if (!wsp) lk.lock();
    int st = prep(c, n_msgs, s, wsp, !(slotted || sizes_only));
    if (st) return st;
    psy::DecodeArgs a{};
    a.in = d_in;
    a.in_off = d_in_off;
    a.n_msgs = n_msgs;
    a.out = d_out;
    a.out_cap = out_cap;
    a.out_off = d_out_off;
    a.status = d_status;
    a.sizes_out = d_sizes;
    a.ticket = reinterpret_cast<uint32_t *>(wsp);
    a.errflags = reinterpret_cast<uint32_t *>(wsp) + 1;
    a.lookback = reinterpret_cast<uint64_t *>(wsp + kCounterBytes);
    a.slot_off = d_slot_off;
    a.out_len = d_out_len;
    a.in_len = d_in_len;
    if (sizes_only) {
        hipLaunchKernelGGL(psy::tdt_decode_sizes_kernel, dim3((n_msgs + 255) / 256), dim3(256), 0, s, a);
    } else if (slotted) {
        st = launch_decode_slotted(c, pws ? *pws : c->pw, a, s);
        if (st) return st;
    } else {
        launch_list(n_msgs, 64, [&](uint32_t, uint32_t g) {  // ids from the ticket
            hipLaunchKernelGGL((psy::tdt_decode_kernel<1>), dim3(g), dim3(64), 0, s, a);
        });
    }
    HIPCHK(hipGetLastError());
    return TDT_OK;
}

int ensure_host_dev(tdt_ctx *c, size_t bytes) {
    if (bytes > c->h_dev_bytes) {
        if (c->h_dev) HIPCHK(hipFree(c->h_dev));
        c->h_dev = nullptr;
        size_t cap = std::max(bytes, c->h_dev_bytes * 2);
        HIPCHK(hipMalloc(&c->h_dev, cap));
        c->h_dev_bytes = cap;
    }
    return TDT_OK;
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------------------
// Host pipeline (the TCP socket-buffer case: SimpleTCP sends from and receives into host
// memory, tcp_simple.hpp:68-91, :153-194).  The batch is cut into chunks of whole messages
// (<= kHostChunk input bytes); chunk c runs on slot c % kHostSlots — its own stream, device
// buffer, plan workspace and pinned buffers — as H2D → batch kernels → D2H, and the host finishes
// chunk c - 3 (its output) while chunks c - 2 .. c are on the GPU: with two slots the next H2D
// waited for the D2H of the chunk before (the pinned 50 x 1 MiB decode moved its bytes one PCIe
// direction at a time: 22.6 GB/s, profiles/r04_hp1).  Caller buffers that are not pinned
// (std::vector socket buffers, numpy arrays) are staged through the slot's pinned buffers by a
// pool of host threads (parallel memcpy: one thread's memcpy is far below the PCIe rate);
// pinned caller buffers are DMA'd directly.  Every device → host copy lands in pinned memory,
// so no copy blocks the host behind the kernels.
constexpr uint64_t kHostChunk = 64ull << 20;

bool is_pinned(const void *p) {
    hipPointerAttribute_t at{};
    if (!p || hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

int ensure_slot(tdt_ctx *c, int k, size_t dev_bytes, size_t pin_words, size_t sin, size_t sout) {
    auto &h = c->hs[k];
    if (!c->hin) {
        HIPCHK(hipStreamCreateWithFlags(&c->hin, hipStreamNonBlocking));
        HIPCHK(hipStreamCreateWithFlags(&c->hex, hipStreamNonBlocking));
    }
    if (!h.stream) {
        h.pw.no_side = true;
        HIPCHK(hipStreamCreateWithFlags(&h.stream, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&h.ev, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&h.evc, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&h.evi, hipEventDisableTiming));
        HIPCHK(hipHostMalloc(&h.flag, 4, hipHostMallocDefault));
        *h.flag = 0;
    }
    // growth takes 1.5x (whole MiB) and retires the old buffer until tdt_ctx_destroy instead of
    // freeing it: a hipFree waits for the whole device (every stream, the other contexts' of
    // the process too: a C1 loopback end stalled the other end's pipeline for milliseconds), and
    // pinning host memory costs milliseconds, so buffers sized by the chunks of varying calls
    // settle after a few (the retired ones sum to less than twice the last)
    auto grown = [](size_t need, size_t have) {
        return (std::max(need, have + have / 2) + (1u << 20) - 1) & ~size_t((1u << 20) - 1);
    };
    if (dev_bytes > h.dev_bytes) {
        const size_t cap = grown(dev_bytes, h.dev_bytes);
        if (h.dev) c->retired.push_back(h.dev);  // (the slot's earlier chunks are done: synced)
        h.dev = nullptr;
        h.dev_bytes = 0;
        HIPCHK(hipMalloc(&h.dev, cap));
        h.dev_bytes = cap;
    }
    auto pinned = [&](uint8_t *&buf, size_t &have, size_t need) -> int {
        if (need <= have) return TDT_OK;
        const size_t cap = grown(need, have);
        if (buf) c->retired_host.push_back(buf);
        buf = nullptr;
        have = 0;
        HIPCHK(hipHostMalloc(&buf, cap, hipHostMallocDefault));
        have = cap;
        return TDT_OK;
    };
    uint8_t *pw = reinterpret_cast<uint8_t *>(h.pin);
    size_t pb = 8 * h.pin_words;
    int st = pinned(pw, pb, 8 * pin_words);
    if (st) return st;
    h.pin = reinterpret_cast<uint64_t *>(pw);
    h.pin_words = pb / 8;
    if ((st = pinned(h.stage_in, h.sin_bytes, sin)) || (st = pinned(h.stage_out, h.sout_bytes, sout))) return st;
    return TDT_OK;
}

// every host-pipeline stream idle (an error mid-pipeline: copies and kernels may still touch the
// caller's buffers)
void drain_host(tdt_ctx *c) {
    for (auto &h : c->hs)
        if (h.stream) (void)hipStreamSynchronize(h.stream);
    if (c->hin) (void)hipStreamSynchronize(c->hin);
    if (c->hex) (void)hipStreamSynchronize(c->hex);
}

// Once a slot's last chunk is done: fold its device error flags into the context.
int sync_slot(tdt_ctx *c, tdt_ctx::HostSlot &h) {
    // (the slot's last command is its chunk's h.ev record; never recorded: complete)
    HIPCHK(c->slot_streams ? hipStreamSynchronize(h.stream) : hipEventSynchronize(h.ev));
    if (h.flag) {
        c->host_flags.fetch_or(*h.flag);
        *h.flag = 0;
    }
    return TDT_OK;
}

struct Chunk {
    uint32_t m0 = 0, n = 0;
    uint64_t in_bytes = 0, cap = 0, base = 0;
    uint64_t scap = 0;  // encode through the slotted kernels: the blobs' slot bytes (Σ bounds)
    // device layout: input | in_off (n+1), slots (n+1) | out (cap) | out_off (n+1) | status (n)
    // | workspace | lengths (n) | slotted blobs (scap)
    size_t o_off = 0, o_out = 0, o_ooff = 0, o_st = 0, o_ws = 0, o_len = 0, o_sbuf = 0, end = 0;
};

// Chunk size of a call: an eighth of its input (with four slots in flight the H2D of later
// chunks, the kernels of one and the D2H of earlier ones overlap even for a socket-sized batch
// of tens of MiB), between 2 and 64 MiB.
uint64_t host_chunk_bytes(const uint64_t *h_in_off, uint32_t n_msgs) {
    const uint64_t total = h_in_off[n_msgs] - h_in_off[0];
    return std::min<uint64_t>(kHostChunk, std::max<uint64_t>(2ull << 20, (total / 8 + 4095) & ~4095ull));
}

Chunk plan_chunk(const uint64_t *h_in_off, uint32_t m0, uint32_t n_msgs, bool encode, bool slotted, int ws,
                 const uint64_t *dec_sizes, uint64_t chunk_bytes) {
    Chunk k;
    k.m0 = m0;
    uint32_t m = m0;
    uint64_t cap = 0;
    while (m < n_msgs) {
        const uint64_t len = h_in_off[m + 1] - h_in_off[m];
        if (m > m0 && h_in_off[m + 1] - h_in_off[m0] > chunk_bytes) break;
        cap += encode ? tdt_encode_bound(len, ws) : dec_sizes[m];
        ++m;
    }
    k.n = m - m0;
    k.in_bytes = h_in_off[m] - h_in_off[m0];
    k.cap = cap;
    k.scap = encode && slotted ? cap : 0;
    k.o_off = align_up(k.in_bytes, 256);
    k.o_out = align_up(k.o_off + 16ull * (k.n + 1), 256);
    // (the slotted encode writes its blobs into the slot buffer at o_sbuf: no compacted region)
    k.o_ooff = align_up(k.o_out + (k.scap ? 1ull : std::max<uint64_t>(cap, 1)), 256);
    k.o_st = align_up(k.o_ooff + 8ull * (k.n + 1), 256);
    k.o_ws = align_up(k.o_st + 4ull * k.n, 256);
    k.o_len = align_up(k.o_ws + kCounterBytes + 8ull * (k.n + 1), 256);
    k.o_sbuf = align_up(k.o_len + 8ull * k.n, 256);
    k.end = k.o_sbuf + (k.scap ? k.scap + 16 : 0);  // (+16: the gather's funnel reads past a blob)
    return k;
}

size_t chunk_dev_bytes(const Chunk &k) { return k.end; }
// pinned words of a slot: in_off (n+1) | slots (n+1) | out_off or lengths (n+1) | status (n int32)
size_t chunk_pin_words(const Chunk &k) { return 3ull * k.n + 3 + (k.n + 1) / 2; }
uint64_t *pin_slots(tdt_ctx::HostSlot &h, const Chunk &k) { return h.pin + (k.n + 1); }
uint64_t *pin_back(tdt_ctx::HostSlot &h, const Chunk &k) { return h.pin + 2ull * (k.n + 1); }
int32_t *pin_status(tdt_ctx::HostSlot &h, const Chunk &k) { return reinterpret_cast<int32_t *>(h.pin + 3ull * k.n + 3); }

// decode: the decoded size of every blob from its header (the kernel validates; a blob it
// rejects gets 0 and its bytes are dropped when the output is compacted)
uint64_t host_decoded_size(const uint8_t *b, uint64_t len) {
    if (len < 4) return 0;
    uint32_t magic;
    std::memcpy(&magic, b, 4);
    if (magic == psy::kMagicUNCP) return len - 4;
    if (magic != psy::kMagicTDT || len < 8) return 0;
    uint32_t orig;
    std::memcpy(&orig, b + 4, 4);
    return orig;
}

// One wave copies `len` bytes: 16-byte aligned stores; each 16-byte chunk read as five aligned
// dwords and funnel-shifted by the (constant) source misalignment — compacted offsets have any
// alignment, so a byte loop would be the common case otherwise.
__device__ __forceinline__ void wave_copy_any(uint8_t *dst, const uint8_t *src, uint64_t len) {
    const uint32_t lane = (uint32_t)psy::lane_id();
    uint64_t head = (16 - ((uintptr_t)dst & 15)) & 15;
    if (head > len) head = len;
    if (lane < head) dst[lane] = src[lane];
    const uint64_t nb = (len - head) / 16;
    const uint8_t *s0 = src + head;
    const uint32_t sh = (uint32_t)((uintptr_t)s0 & 3) * 8;
    const uint32_t *sw = reinterpret_cast<const uint32_t *>((uintptr_t)s0 & ~(uintptr_t)3);
    uint4 *dv = reinterpret_cast<uint4 *>(dst + head);
    for (uint64_t k = lane; k < nb; k += 64) {
        const uint32_t *q = sw + 4 * k;
        const uint32_t w0 = psy::gload<uint32_t>(q), w1 = psy::gload<uint32_t>(q + 1), w2 = psy::gload<uint32_t>(q + 2),
                       w3 = psy::gload<uint32_t>(q + 3);
        // (the fifth dword only when misaligned: it may lie past the source's end otherwise)
        const uint32_t w4 = sh ? psy::gload<uint32_t>(q + 4) : 0u;
        dv[k] = make_uint4((uint32_t)((((uint64_t)w1 << 32) | w0) >> sh), (uint32_t)((((uint64_t)w2 << 32) | w1) >> sh),
                           (uint32_t)((((uint64_t)w3 << 32) | w2) >> sh), (uint32_t)((((uint64_t)w4 << 32) | w3) >> sh));
    }
    for (uint64_t k = head + 16 * nb + lane; k < len; k += 64) dst[k] = src[k];
}

// Chunk ci's compacted output → host memory, issued behind the encode kernel so that no host
// wait sits between a chunk's kernel and its copy (the length is device-side: the chunk's last
// offset).  dst: the slot's pinned staging (direct = 0), or the caller's pinned buffer at the
// running base (direct = 1; bases[ci] = the totals of the chunks before, written by the previous
// chunk's launch, which this one follows by an event).  Past out_cap nothing is copied (the host
// reports TDT_E_CAPACITY).  Stores are 16-byte aligned on dst; the source is read as aligned
// dwords and funnel-shifted.
// total bytes src → d (host memory over PCIe, or device): 16-byte stores at d's alignment, the
// source read as aligned dwords and shifted (src + total + 4 must be readable)
__device__ __forceinline__ void grid_copy_out(uint8_t *d, const uint8_t *src, uint64_t total) {
    const uint64_t gtid = (uint64_t)blockIdx.x * 256 + threadIdx.x, gsz = (uint64_t)gridDim.x * 256;
    uint64_t head = (16 - ((uintptr_t)d & 15)) & 15;
    if (head > total) head = total;
    if (gtid < head) d[gtid] = src[gtid];
    const uint64_t nb = (total - head) / 16;
    const uint8_t *s0 = src + head;
    const uint32_t sh = (uint32_t)((uintptr_t)s0 & 3) * 8;
    const uint32_t *sw = reinterpret_cast<const uint32_t *>((uintptr_t)s0 & ~(uintptr_t)3);
    uint4 *dv = reinterpret_cast<uint4 *>(d + head);
    for (uint64_t k = gtid; k < nb; k += gsz) {
        const uint32_t *q = sw + 4 * k;
        const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
        const uint32_t w4 = sh ? q[4] : 0u;  // (inside the chunk buffer's slack)
        dv[k] = make_uint4((uint32_t)((((uint64_t)w1 << 32) | w0) >> sh), (uint32_t)((((uint64_t)w2 << 32) | w1) >> sh),
                           (uint32_t)((((uint64_t)w3 << 32) | w2) >> sh), (uint32_t)((((uint64_t)w4 << 32) | w3) >> sh));
    }
    for (uint64_t k = head + 16 * nb + gtid; k < total; k += gsz) d[k] = src[k];
}

__global__ __launch_bounds__(256) void host_out_kernel(const uint8_t *src, const uint64_t *chunk_off, uint32_t n,
                                                       uint8_t *dst, uint64_t *bases, uint32_t ci, uint64_t cap,
                                                       int direct) {
    const uint64_t total = chunk_off[n];
    const uint64_t base = bases[ci];
    if (blockIdx.x == 0 && threadIdx.x == 0) bases[ci + 1] = base + total;
    if (base + total > cap || total == 0) return;
    grid_copy_out(direct ? dst + base : dst, src, total);
}

// host_decode: a chunk's slotted output → the caller's pinned buffer (or the pinned staging)
__global__ __launch_bounds__(256) void host_dout_kernel(const uint8_t *src, uint8_t *dst, uint64_t total) {
    grid_copy_out(dst, src, total);
}

// A slotted chunk's blob lengths → exclusive offsets (total at [n]): one workgroup, 4096
// lengths per step (a chunk holds at most kHostChunk bytes of messages).
__global__ __launch_bounds__(1024) void host_scan_kernel(const uint64_t *len, uint64_t *out_off, uint32_t n) {
    __shared__ uint64_t wsum[16];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint64_t carry = 0;
    for (uint32_t b = 0; b < n; b += 4096) {
        uint64_t v[4], s = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = b + 4u * (uint32_t)t + (uint32_t)k;
            v[k] = i < n ? len[i] : 0ull;
            s += v[k];
        }
        uint64_t x = s;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        uint64_t pre = carry, tot = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            const uint64_t q = wsum[w];
            pre += w < wv ? q : 0ull;
            tot += q;
        }
        uint64_t e = pre + x - s;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = b + 4u * (uint32_t)t + (uint32_t)k;
            if (i < n) out_off[i] = e;
            e += v[k];
        }
        carry += tot;
        __syncthreads();  // wsum is reused
    }
    if (t == 0) out_off[n] = carry;
}

// A slotted chunk's blobs → host memory at their compacted places (the output copy of
// host_out_kernel, gathering from the slots): P waves per blob, each a contiguous part; the
// running base is chained as there.
__global__ __launch_bounds__(256) void host_gather_kernel(const uint8_t *src, const uint64_t *slot, const uint64_t *len,
                                                          const uint64_t *out_off, uint32_t n, uint32_t P, uint8_t *dst,
                                                          uint64_t *bases, uint32_t ci, uint64_t cap, int direct) {
    const uint64_t total = out_off[n];
    const uint64_t base = bases[ci];
    if (blockIdx.x == 0 && threadIdx.x == 0) bases[ci + 1] = base + total;
    if (base + total > cap || total == 0) return;
    uint8_t *d = direct ? dst + base : dst;
    const uint64_t nw = (uint64_t)n * P;
    for (uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); w < nw; w += (uint64_t)gridDim.x * 4) {
        const uint32_t i = (uint32_t)(w / P), p = (uint32_t)(w % P);
        const uint64_t l = len[i], a = l * p / P, e = l * (p + 1) / P;
        if (e > a) wave_copy_any(d + out_off[i] + a, src + slot[i] + a, e - a);
    }
}

// The issue / finish loop of a host call: chunk ci is issued on slot ci % kHostSlots once that
// slot's previous chunk is done, and finished (its outputs and statuses read back) kHostSlots - 1
// chunks later, so that up to kHostSlots chunks are in flight.
template <class I, class F>
int host_loop(size_t nc, I &&issue, F &&finish) {
    constexpr size_t L = kHostSlots - 1;
    for (size_t ci = 0; ci < nc; ++ci) {
        int st = issue(ci);
        if (!st && ci >= L) st = finish(ci - L);
        if (st) return st;
    }
    for (size_t ci = nc > L ? nc - L : 0; ci < nc; ++ci)
        if (int st = finish(ci)) return st;
    return TDT_OK;
}

// msgs / sizes (gather input, tdt_encode_host_v): message i = msgs[i][0 .. sizes[i]); h_in is then
// unused and h_in_off holds the prefix sums of sizes
int host_encode(tdt_ctx *c, const uint8_t *h_in, const uint64_t *h_in_off, uint32_t n_msgs, uint8_t *h_out,
                uint64_t out_cap, uint64_t *h_out_off, int32_t *h_status, const uint8_t *const *msgs = nullptr,
                const uint64_t *sizes = nullptr) {
    const int ws = c->cfg.word_size;
    const bool pin_in = !msgs && is_pinned(h_in + h_in_off[0]);
    // gather input from pinned caller buffers (a channel's pinned message memory): DMA'd run by
    // run of adjacent messages instead of staged by the copy pool.  A pointer-attribute query per
    // message (~1 µs): only for calls of up to 4096 messages whose first message is pinned (a
    // pageable first message — the common case — costs one query)
    bool msgs_pinned = msgs && n_msgs <= 4096;
    for (uint32_t i = 0; i < n_msgs && msgs_pinned; ++i) msgs_pinned = sizes[i] == 0 || is_pinned(msgs[i]);
    // a pinned caller buffer receives the chunks' output straight from the copy kernels
    uint8_t *d_out = nullptr;
    if (is_pinned(h_out) && hipHostGetDevicePointer(reinterpret_cast<void **>(&d_out), h_out, 0) != hipSuccess) {
        (void)hipGetLastError();
        d_out = nullptr;
    }
    const bool pin_out = d_out != nullptr;
    // one pass with the look-back when every message is <= 64 KiB and they average >= 16 KiB (as
    // tdt_encode_batch); otherwise the slotted message-class kernels (a 1 MiB message spreads over
    // 64 KiB tiles instead of running in one workgroup) and a gather into the host buffer
    bool lb = h_in_off[n_msgs] - h_in_off[0] >= 16384ull * n_msgs;
    for (uint32_t i = 0; i < n_msgs && lb; ++i) lb = h_in_off[i + 1] - h_in_off[i] <= kBigMin;
    std::vector<Chunk> ch;
    const uint64_t cb = host_chunk_bytes(h_in_off, n_msgs);
    for (uint32_t m = 0; m < n_msgs;) {
        ch.push_back(plan_chunk(h_in_off, m, n_msgs, true, !lb, ws, nullptr, cb));
        m += ch.back().n;
    }
    if (ch.size() + 1 > c->hbases_n) {
        if (c->hbases) HIPCHK(hipFree(c->hbases));
        c->hbases = nullptr;
        HIPCHK(hipMalloc(&c->hbases, 8 * (ch.size() + 1)));
        c->hbases_n = ch.size() + 1;
    }
    uint64_t base = 0;  // output bytes of the chunks finished so far
    bool capacity = false;
    auto issue = [&](size_t ci) -> int {
        const Chunk &k = ch[ci];
        const int si = (int)(ci % kHostSlots);
        auto &h = c->hs[si];
        int st = ensure_slot(c, si, chunk_dev_bytes(k), chunk_pin_words(k), pin_in || msgs_pinned ? 0 : k.in_bytes,
                             pin_out ? 0 : k.cap);
        if (st) return st;
        st = sync_slot(c, h);  // the slot's previous chunk is done with its buffers
        if (st) return st;
        uint64_t *pin_in_off = h.pin, *pin_slot = pin_slots(h, k);
        const uint64_t b0 = h_in_off[k.m0];
        uint64_t acc = 0;
        for (uint32_t i = 0; i <= k.n; ++i) {
            pin_in_off[i] = h_in_off[k.m0 + i] - b0;
            if (k.scap) {
                pin_slot[i] = acc;
                if (i < k.n) acc += tdt_encode_bound(h_in_off[k.m0 + i + 1] - h_in_off[k.m0 + i], ws);
            }
        }
        const uint8_t *src = msgs ? nullptr : h_in + b0;
        if (msgs && !msgs_pinned) {
            c->pool->gather(h.stage_in, msgs + k.m0, sizes + k.m0, k.n);
            src = h.stage_in;
        } else if (!msgs && !pin_in) {
            c->pool->copy(h.stage_in, src, k.in_bytes);
            src = h.stage_in;
        }
        uint8_t *d = h.dev;
        auto *doff = reinterpret_cast<uint64_t *>(d + k.o_off);
        auto *dslot = doff + (k.n + 1);
        auto *dooff = reinterpret_cast<uint64_t *>(d + k.o_ooff);
        auto *dst = reinterpret_cast<int32_t *>(d + k.o_st);
        auto *dlen = reinterpret_cast<uint64_t *>(d + k.o_len);
        const hipStream_t s_in = c->slot_streams ? h.stream : c->hin, s_ex = c->slot_streams ? h.stream : c->hex;
        if (src) {
            HIPCHK(hipMemcpyAsync(d, src, k.in_bytes, hipMemcpyHostToDevice, s_in));
        } else {
            for (uint32_t i = 0; i < k.n;) {
                const uint8_t *p0 = msgs[k.m0 + i];
                uint64_t len = sizes[k.m0 + i];
                uint32_t j = i + 1;
                while (j < k.n && msgs[k.m0 + j] == p0 + len) len += sizes[k.m0 + j++];
                if (len) HIPCHK(hipMemcpyAsync(d + pin_in_off[i], p0, len, hipMemcpyHostToDevice, s_in));
                i = j;
            }
        }
        // in_off and (slotted) the slots: one copy
        HIPCHK(hipMemcpyAsync(doff, pin_in_off, (k.scap ? 16ull : 8ull) * (k.n + 1), hipMemcpyHostToDevice, s_in));
        if (s_in != s_ex) {
            HIPCHK(hipEventRecord(h.evi, s_in));
            HIPCHK(hipStreamWaitEvent(s_ex, h.evi, 0));
        }
        if (k.scap) {
            st = encode_common(c, psy::MODE_ENCODE, d, doff, k.n, nullptr, d + k.o_sbuf, k.scap, nullptr, dst, nullptr,
                               nullptr, nullptr, s_ex, dslot, dlen, d + k.o_ws, &h.pw);
            if (st) return st;
            hipLaunchKernelGGL(host_scan_kernel, dim3(1), dim3(1024), 0, s_ex, dlen, dooff, k.n);
            HIPCHK(hipGetLastError());
        } else {
            st = encode_common(c, psy::MODE_ENCODE, d, doff, k.n, nullptr, d + k.o_out, k.cap, dooff, dst, nullptr,
                               nullptr, nullptr, s_ex, nullptr, nullptr, d + k.o_ws, nullptr,
                               k.in_bytes <= kSmallMax * k.n ? 1 : 0);  // (the chunk's sizes are host data)
            if (st) return st;
        }
        // the output, in chunk order (each copy follows the previous chunk's: the running base)
        if (ci == 0) HIPCHK(hipMemsetAsync(c->hbases, 0, 8, s_ex));
        else if (c->slot_streams) HIPCHK(hipStreamWaitEvent(s_ex, c->hs[(ci - 1) % kHostSlots].evc, 0));
        uint8_t *odst = pin_out ? d_out : h.stage_out;
        if (k.scap) {
            const uint32_t P = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(1, k.in_bytes / k.n / 16384));
            const uint32_t grid = (uint32_t)std::min<uint64_t>(2048, ((uint64_t)k.n * P + 3) / 4);
            hipLaunchKernelGGL(host_gather_kernel, dim3(grid), dim3(256), 0, s_ex, d + k.o_sbuf, dslot, dlen, dooff,
                               k.n, P, odst, c->hbases, (uint32_t)ci, out_cap, pin_out ? 1 : 0);
        } else {
            const uint32_t grid = (uint32_t)std::min<uint64_t>(1024, k.cap / 4096 + 1);
            hipLaunchKernelGGL(host_out_kernel, dim3(grid), dim3(256), 0, s_ex, d + k.o_out, dooff, k.n, odst,
                               c->hbases, (uint32_t)ci, out_cap, pin_out ? 1 : 0);
        }
        HIPCHK(hipGetLastError());
        if (c->slot_streams) HIPCHK(hipEventRecord(h.evc, s_ex));
        if ((st = small_copies(s_ex, d + k.o_ws + 4, h.flag, 4, dooff, pin_back(h, k), 8ull * (k.n + 1), dst,
                               pin_status(h, k), 4ull * k.n)))
            return st;
        HIPCHK(hipEventRecord(h.ev, s_ex));
        return TDT_OK;
    };
    // chunk ci's compacted size is known once its event fires; then its output comes back
    auto finish = [&](size_t ci) -> int {
        const Chunk &k = ch[ci];
        auto &h = c->hs[ci % kHostSlots];
        HIPCHK(hipEventSynchronize(h.ev));
        const uint64_t *pin_out_off = pin_back(h, k);
        const uint64_t total = pin_out_off[k.n];
        if (capacity || base + total > out_cap) capacity = true;
        for (uint32_t i = 0; i < k.n; ++i) h_out_off[k.m0 + i] = base + (capacity ? 0 : pin_out_off[i]);
        if (h_status) std::memcpy(h_status + k.m0, pin_status(h, k), 4ull * k.n);
        // (the copy kernel has written the output: into h_out directly, or into the staging)
        if (!capacity && total && !pin_out) c->pool->copy(h_out + base, h.stage_out, total);
        if (!capacity) base += total;
        return TDT_OK;
    };
    int st = host_loop(ch.size(), issue, finish);
    if (st) return st;
    for (auto &h : c->hs)
        if (h.stream && (st = sync_slot(c, h))) return st;
    h_out_off[n_msgs] = base;
    if (capacity) return set_err(TDT_E_CAPACITY, "host output capacity exceeded");
    return TDT_OK;
}

int host_decode(tdt_ctx *c, const uint8_t *h_in, const uint64_t *h_in_off, uint32_t n_msgs, uint8_t *h_out,
                uint64_t out_cap, uint64_t *h_out_off, int32_t *h_status) {
    // decoded sizes from the headers → every chunk's output offsets are known up front: the
    // decode is slotted at those offsets
    std::vector<uint64_t> dsz(n_msgs);
    uint64_t need = 0;
    for (uint32_t i = 0; i < n_msgs; ++i) {
        dsz[i] = host_decoded_size(h_in + h_in_off[i], h_in_off[i + 1] - h_in_off[i]);
        need += dsz[i];
    }
    if (need > out_cap) return set_err(TDT_E_CAPACITY, "host output capacity exceeded");
    const bool pin_in = is_pinned(h_in + h_in_off[0]), pin_out = is_pinned(h_out);
    // the device's view of a pinned caller buffer (registered memory may map elsewhere)
    uint8_t *d_hout = nullptr;
    if (pin_out && hipHostGetDevicePointer(reinterpret_cast<void **>(&d_hout), h_out, 0) != hipSuccess) {
        (void)hipGetLastError();
        d_hout = nullptr;
    }
    const bool dma_out = c->dout_sdma || (pin_out && !d_hout);
    std::vector<Chunk> ch;
    uint64_t base = 0;
    const uint64_t cb = host_chunk_bytes(h_in_off, n_msgs);
    for (uint32_t m = 0; m < n_msgs;) {
        ch.push_back(plan_chunk(h_in_off, m, n_msgs, false, false, c->cfg.word_size, dsz.data(), cb));
        ch.back().base = base;
        base += ch.back().cap;
        m += ch.back().n;
    }
    std::vector<uint64_t> lens(n_msgs);
    std::vector<int32_t> stv(n_msgs);
    auto issue = [&](size_t ci) -> int {
        const Chunk &k = ch[ci];
        const int si = (int)(ci % kHostSlots);
        auto &h = c->hs[si];
        int st = ensure_slot(c, si, chunk_dev_bytes(k), chunk_pin_words(k), pin_in ? 0 : k.in_bytes, pin_out ? 0 : k.cap);
        if (st) return st;
        st = sync_slot(c, h);
        if (st) return st;
        uint64_t *pin_in_off = h.pin, *pin_slot = pin_slots(h, k);
        const uint64_t b0 = h_in_off[k.m0];
        uint64_t acc = 0;
        for (uint32_t i = 0; i <= k.n; ++i) {
            pin_in_off[i] = h_in_off[k.m0 + i] - b0;
            pin_slot[i] = acc;
            if (i < k.n) acc += dsz[k.m0 + i];
        }
        const uint8_t *src = h_in + b0;
        if (!pin_in) {
            c->pool->copy(h.stage_in, src, k.in_bytes);
            src = h.stage_in;
        }
        uint8_t *d = h.dev;
        auto *doff = reinterpret_cast<uint64_t *>(d + k.o_off);
        auto *dslot = doff + (k.n + 1);
        auto *dst = reinterpret_cast<int32_t *>(d + k.o_st);
        auto *dlen = reinterpret_cast<uint64_t *>(d + k.o_len);
        // input copies in chunk order, each after the previous chunk's: concurrent copies of
        // several slots share the link and all land late, the earliest-needed one included
        // (decode 31 -> 37 GiB/s pinned; the same ordering cost host_encode 44 -> 36 GiB/s,
        // profiles/r05_diag/host_decode/)
        const hipStream_t s_in = c->slot_streams ? h.stream : c->hin, s_ex = c->slot_streams ? h.stream : c->hex;
        if (ci > 0 && c->slot_streams) HIPCHK(hipStreamWaitEvent(s_in, c->hs[(ci - 1) % kHostSlots].evi, 0));
        HIPCHK(hipMemcpyAsync(d, src, k.in_bytes, hipMemcpyHostToDevice, s_in));
        HIPCHK(hipMemcpyAsync(doff, pin_in_off, 16ull * (k.n + 1), hipMemcpyHostToDevice, s_in));  // offsets + slots
        HIPCHK(hipEventRecord(h.evi, s_in));
        if (s_in != s_ex) HIPCHK(hipStreamWaitEvent(s_ex, h.evi, 0));
        st = decode_common(c, false, d, doff, k.n, d + k.o_out, 0, nullptr, nullptr, dst, s_ex, dslot, dlen,
                           nullptr, d + k.o_ws, &h.pw);
        if (st) return st;
        if (acc && dma_out) {
            HIPCHK(hipMemcpyAsync(pin_out ? h_out + k.base : h.stage_out, d + k.o_out, acc, hipMemcpyDeviceToHost,
                                  s_ex));
        } else if (acc) {
            // the output crosses PCIe as a copy kernel's stores (as host_encode's), not a DMA: the
            // DMA engines then carry only the H2D direction
            hipLaunchKernelGGL(host_dout_kernel, dim3((uint32_t)std::min<uint64_t>(1024, acc / 4096 + 1)), dim3(256), 0,
                               s_ex, d + k.o_out, pin_out ? d_hout + k.base : h.stage_out, acc);
            HIPCHK(hipGetLastError());
        }
        if ((st = small_copies(s_ex, d + k.o_ws + 4, h.flag, 4, dlen, pin_back(h, k), 8ull * k.n, dst,
                               pin_status(h, k), 4ull * k.n)))
            return st;
        HIPCHK(hipEventRecord(h.ev, s_ex));
        return TDT_OK;
    };
    auto finish = [&](size_t ci) -> int {
        const Chunk &k = ch[ci];
        auto &h = c->hs[ci % kHostSlots];
        HIPCHK(hipEventSynchronize(h.ev));
        if (!pin_out && k.cap) c->pool->copy(h_out + k.base, h.stage_out, k.cap);
        std::memcpy(lens.data() + k.m0, pin_back(h, k), 8ull * k.n);
        std::memcpy(stv.data() + k.m0, pin_status(h, k), 4ull * k.n);
        return TDT_OK;
    };
    int st = host_loop(ch.size(), issue, finish);
    if (st) return st;
    for (auto &h : c->hs) {
        st = h.stream ? sync_slot(c, h) : TDT_OK;
        if (st) return st;
    }
    // offsets; blobs the kernel rejected (status != OK, length 0) leave a gap: compact it
    uint64_t w = 0, r = 0;
    for (uint32_t i = 0; i < n_msgs; ++i) {
        h_out_off[i] = w;
        if (lens[i] && w != r) std::memmove(h_out + w, h_out + r, lens[i]);
        w += lens[i];
        r += dsz[i];
        if (h_status) h_status[i] = stv[i];
    }
    h_out_off[n_msgs] = w;
    return TDT_OK;
}

// ---------------------------------------------------------------------------------------
// One-message fast path.  Block layout (`one`, mapped pinned memory): [0, 256) argument words,
// then the input at kOneIn, then the output.  The class kernel of the message's size runs as a
// single workgroup on a one-entry list; every argument, the input and the output live in host
// memory the kernel reads and writes over PCIe.
constexpr uint64_t kOneMax = 256 * 1024;  // largest message (encode) / decoded message the path takes
constexpr size_t kOneIn = 256;
struct OneArgs {
    uint64_t off[2];   // input offsets
    uint64_t slot[2];  // output slot
    uint64_t len;      // output length
    int32_t status;
    uint32_t list, cnt, flags;
    uint32_t done, pad;  // completion word (one_spin: written by the stream after the kernel)
};

int ensure_one(tdt_ctx *c, size_t bytes) {
    if (!c->one_stream) HIPCHK(hipStreamCreateWithFlags(&c->one_stream, hipStreamNonBlocking));
    if (bytes <= c->one_bytes) return TDT_OK;
    if (c->one) HIPCHK(hipHostFree(c->one));
    c->one = nullptr;
    c->one_bytes = 0;
    const size_t cap = std::max<size_t>(bytes, 64 * 1024);
    // coherent (fine-grained, uncached on the device): the kernel's result stores reach host
    // memory before the stream writes the completion word the host spins on, with no cache
    // write-back to order; the block is read and written once per call anyway
    HIPCHK(hipHostMalloc(&c->one, cap, hipHostMallocCoherent));
    c->one_bytes = cap;
    return TDT_OK;
}

template <int WS>
void launch_one_encode(const psy::EncodeArgs &a, uint64_t n, hipStream_t s) {
    using psy::MODE_ENCODE;
    if (n <= kSmallMax)
        hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 64, 4, MODE_ENCODE, 0, 0, 0>), dim3(1), dim3(64), 0, s, a);
    else if (n <= kMidMax)
        hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 256, 8, MODE_ENCODE, 0, 0, 0>), dim3(1), dim3(256), 0, s, a);
    else if (n <= 65536 && (n & 15) == 0)  // (the block's input is 16-byte aligned: resident)
        hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 512, 8, MODE_ENCODE, 0, 0, 0, psy::PATH_RES>), dim3(1),
                           dim3(512), 0, s, a);
    else
        hipLaunchKernelGGL((psy::tdt_encode_kernel<WS, 512, 8, MODE_ENCODE, 0, 0, 0, psy::PATH_STREAM>), dim3(1),
                           dim3(512), 0, s, a);
}

// returns TDT_OK, an error, or -1: not taken (the pipeline serves the call)
int host_one(tdt_ctx *c, bool encode, const uint8_t *h_in, const uint64_t *h_in_off, uint8_t *h_out,
             uint64_t out_cap, uint64_t *h_out_off, int32_t *h_status) {
    const uint64_t len = h_in_off[1] - h_in_off[0];
    const uint8_t *src = h_in + h_in_off[0];
    uint64_t osize;
    if (encode) {
        if (len > kOneMax) return -1;
        osize = tdt_encode_bound(len, c->cfg.word_size);
    } else {
        osize = host_decoded_size(src, len);
        if (osize > kOneMax || len > 2 * kOneMax + 1024) return -1;
        if (osize > out_cap) return set_err(TDT_E_CAPACITY, "host output capacity exceeded");
    }
    const size_t o_out = kOneIn + align_up(std::max<uint64_t>(len, 1), 256);
    int st = ensure_one(c, o_out + align_up(std::max<uint64_t>(osize, 1), 256) + 256);
    if (st) return st;
    uint8_t *hb = c->one;
    uint8_t *db = nullptr;
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&db), hb, 0));
    OneArgs *A = reinterpret_cast<OneArgs *>(hb);
    const OneArgs *dA = reinterpret_cast<const OneArgs *>(db);
    A->off[0] = 0;
    A->off[1] = len;
    A->slot[0] = 0;
    A->slot[1] = osize;
    A->len = 0;
    A->status = -1;
    A->list = 0;
    A->cnt = 1;
    A->flags = 0;
    A->done = 0;
    if (len) std::memcpy(hb + kOneIn, src, len);
    hipStream_t s = c->one_stream;
    if (encode) {
        psy::EncodeArgs a{};
        a.in = db + kOneIn;
        a.in_off = dA->off;
        a.n_msgs = 1;
        a.out = db + o_out;
        a.slot_off = dA->slot;
        a.out_len = const_cast<uint64_t *>(&dA->len);
        a.status = const_cast<int32_t *>(&dA->status);
        a.errflags = const_cast<uint32_t *>(&dA->flags);
        a.min_tensor = c->cfg.min_tensor_size;
        a.policy_on = policy_on(c) ? 1 : 0;
        a.list = &dA->list;
        a.list_count = &dA->cnt;
        switch (c->cfg.word_size) {
#ifdef PSY_FAST_BUILD
            case 4: launch_one_encode<4>(a, len, s); break;
#else
            case 1: launch_one_encode<1>(a, len, s); break;
            case 2: launch_one_encode<2>(a, len, s); break;
            case 4: launch_one_encode<4>(a, len, s); break;
            case 8: launch_one_encode<8>(a, len, s); break;
            case 16: launch_one_encode<16>(a, len, s); break;
#endif
            default: return set_err(TDT_E_UNSUPPORTED, "word_size not supported on the GPU path");
        }
    } else {
        psy::DecodeArgs a{};
        a.in = db + kOneIn;
        // (blobs are read in place over PCIe: staging them into HBM first, in the kernel or by a
        // copy, measured no faster — profiles/r05_diag/one_message/)
        const bool one_wave = c->one_wave || osize <= c->one_wave_max;
        a.in_off = dA->off;
        a.n_msgs = 1;
        a.out = db + o_out;
        a.slot_off = dA->slot;
        a.out_len = const_cast<uint64_t *>(&dA->len);
        a.status = const_cast<int32_t *>(&dA->status);
        a.errflags = const_cast<uint32_t *>(&dA->flags);
        a.list = &dA->list;
        a.list_count = &dA->cnt;
        if (one_wave)
            hipLaunchKernelGGL((psy::tdt_decode_kernel<0, psy::kDecWR, 0>), dim3(1), dim3(64), 0, s, a);
        else  // a workgroup of kOneWaves waves: tiles of the blob (tdt_decode_one_kernel)
            hipLaunchKernelGGL((psy::tdt_decode_one_kernel<psy::kOneWaves>), dim3(1), dim3(64 * psy::kOneWaves), 0,
                               s, a);
    }
    HIPCHK(hipGetLastError());
    bool done = false;
    if (c->one_spin) {
        // the stream writes `done` after the kernel; the host spins on it (1 ms at most, then the
        // stream sync, which also reports a failed kernel)
        const uint32_t seq = ++c->one_seq ? c->one_seq : ++c->one_seq;
        HIPCHK(hipStreamWriteValue32(s, const_cast<uint32_t *>(&dA->done), seq, 0));
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t k = 1;; ++k) {
            if (__atomic_load_n(&A->done, __ATOMIC_ACQUIRE) == seq) {
                done = true;
                break;
            }
            __builtin_ia32_pause();
            if ((k & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(1)) break;
        }
    }
    if (!done) HIPCHK(hipStreamSynchronize(s));
    c->host_flags.fetch_or(A->flags);
    const uint64_t olen = A->len;
    const int32_t ost = A->status;
    if (h_status) h_status[0] = ost;
    h_out_off[0] = 0;
    if (encode && olen > out_cap) {
        h_out_off[1] = 0;
        return set_err(TDT_E_CAPACITY, "host output capacity exceeded");
    }
    if (olen) std::memcpy(h_out, hb + o_out, olen);
    h_out_off[1] = olen;
    return TDT_OK;
}

int host_path(tdt_ctx *c, bool encode, const uint8_t *h_in, const uint64_t *h_in_off, uint32_t n_msgs,
              uint8_t *h_out, uint64_t out_cap, uint64_t *h_out_off, int32_t *h_status) {
    if (!c) return set_err(TDT_E_ARG, "null context");
    if (n_msgs == 0) {
        if (h_out_off) h_out_off[0] = 0;
        return TDT_OK;
    }
    if (!h_in_off || !h_out_off) return set_err(TDT_E_ARG, "null offsets");
    HIPCHK(hipSetDevice(c->device));
    std::lock_guard<std::mutex> lk(c->hmu);  // the pipeline slots belong to the context
    if (n_msgs == 1 && !c->no_one) {
        const int st1 = host_one(c, encode, h_in, h_in_off, h_out, out_cap, h_out_off, h_status);
        if (st1 >= 0) return st1;
    }
    if (!c->pool) c->pool.reset(new CopyPool(c->copy_threads));
    const int st = encode ? host_encode(c, h_in, h_in_off, n_msgs, h_out, out_cap, h_out_off, h_status)
                          : host_decode(c, h_in, h_in_off, n_msgs, h_out, out_cap, h_out_off, h_status);
    if (st != TDT_OK) {
        // an error mid-pipeline: the other slot's copies and kernels may still read the caller's
        // input or write its output — drain both slots before the caller gets its buffers back
        drain_host(c);
        (void)hipGetLastError();
    }
    return st;
}

}  // namespace

namespace {
// any message longer than `lim` bytes → *flag = 1 (one atomic per workgroup)
// any message longer than `lim` bytes → *flag |= 1; any message that the resident-only kernel
// cannot hold (unaligned start, a partial 16-byte group, over 64 KiB) → *flag |= 2 (one atomic
// per workgroup and bit)
__global__ __launch_bounds__(256) void cp_big_kernel(const uint8_t *in, const uint64_t *in_off, uint32_t n,
                                                     uint64_t lim, uint64_t *flag) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint64_t len = i < n ? in_off[i + 1] - in_off[i] : 0;
    const bool big = i < n && len > lim;
    const bool nonres = i < n && (len > 65536 || (len & 15) != 0 || (((uintptr_t)in + in_off[i]) & 15) != 0);
    const bool any_big = __syncthreads_or(big), any_nonres = __syncthreads_or(nonres);
    if (threadIdx.x == 0 && (any_big || any_nonres))
        atomicOr(reinterpret_cast<unsigned long long *>(flag), (any_big ? 1ull : 0ull) | (any_nonres ? 2ull : 0ull));
}
// lengths → the scan's input (in place in out_off)
__global__ __launch_bounds__(256) void cp_len_kernel(const uint64_t *len, uint64_t *out_off, uint32_t n) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out_off[i] = len[i];
}
// blob i (one wave each, four per workgroup): slot → its compacted place (capacity: the
// TDT_E_CAPACITY of the look-back path; out_off keeps the full prefix sum either way)
__global__ __launch_bounds__(256) void cp_gather_kernel(const uint8_t *src, const uint64_t *slot, const uint64_t *len,
                                                      uint8_t *dst, const uint64_t *out_off, uint64_t cap,
                                                      int32_t *status, uint32_t n) {
    const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const uint64_t o = out_off[i], l = len[i];
    if (o + l > cap) {
        if ((threadIdx.x & 63) == 0 && status && status[i] == 0) status[i] = TDT_E_CAPACITY;
        return;
    }
    wave_copy_any(dst + o, src + slot[i], l);
}
}  // namespace

static int scan_sizes(tdt_ctx *ctx, uint64_t *d_off, uint32_t n_msgs, hipStream_t stream);
// The two-phase compaction reads a few bytes back to choose its path: not under stream capture
// (the one-pass kernels need no read-back), nor with the no-two-phase knob.
static bool two_phase_ok(const tdt_ctx *ctx, void *stream) {
    if (ctx->no_two_phase) return false;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &cap) != hipSuccess) return false;
    return cap == hipStreamCaptureStatusNone;
}

// tdt_copy_device (include/psyne_tdt.h): one 512-lane workgroup per 64 KiB piece, its eight
// 16-byte loads per lane in flight before the non-temporal stores (tools/ubench_hbm.hip "chunk"
// row: the fastest hand-written copy shape measured on the box).  Both pointers 16-byte aligned;
// the caller handles any ragged head / tail.
constexpr uint32_t kCopyPiece = 512u * 8u * 16u;
__global__ __launch_bounds__(512) void hbm_copy_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                       uint64_t n16) {
    const uint64_t base = (uint64_t)blockIdx.x * (kCopyPiece / 16u) + threadIdx.x;
    if (base + 7u * 512u < n16) {
        uint4 v[8];
#pragma unroll
        for (int g = 0; g < 8; ++g) v[g] = src[base + (uint64_t)g * 512u];
#pragma unroll
        for (int g = 0; g < 8; ++g) psy::st16_nt(dst + base + (uint64_t)g * 512u, v[g]);
    } else {
        for (int g = 0; g < 8; ++g)
            if (base + (uint64_t)g * 512u < n16) dst[base + (uint64_t)g * 512u] = src[base + (uint64_t)g * 512u];
    }
}
__global__ __launch_bounds__(256) void byte_copy_kernel(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                        uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) dst[i] = src[i];
}

extern "C" {

int tdt_copy_device(void *d_dst, const void *d_src, uint64_t bytes, void *hip_stream) {
    if (bytes == 0) return TDT_OK;
    if (!d_dst || !d_src) return set_err(TDT_E_ARG, "null buffer");
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    uint8_t *dst = static_cast<uint8_t *>(d_dst);
    const uint8_t *src = static_cast<const uint8_t *>(d_src);
    if ((((uintptr_t)dst ^ (uintptr_t)src) & 15u) != 0) {
        // different 16-byte phases: a byte copy (no caller of the codec needs this form fast)
        const uint64_t g = std::min<uint64_t>((bytes + 255) / 256, 65536);
        hipLaunchKernelGGL(byte_copy_kernel, dim3((uint32_t)g), dim3(256), 0, s, src, dst, bytes);
        HIPCHK(hipGetLastError());
        return TDT_OK;
    }
    const uint64_t head = std::min<uint64_t>((16u - ((uintptr_t)dst & 15u)) & 15u, bytes);
    if (head) hipLaunchKernelGGL(byte_copy_kernel, dim3(1), dim3(256), 0, s, src, dst, head);
    const uint64_t n16 = (bytes - head) / 16u, tail = bytes - head - 16u * n16;
    if (n16) {
        const uint64_t pieces = (n16 * 16u + kCopyPiece - 1) / kCopyPiece;
        if (pieces >= (1ull << 31)) return set_err(TDT_E_ARG, "copy too large");
        hipLaunchKernelGGL(hbm_copy_kernel, dim3((uint32_t)pieces), dim3(512), 0, s,
                           reinterpret_cast<const uint4 *>(src + head), reinterpret_cast<uint4 *>(dst + head), n16);
    }
    if (tail) hipLaunchKernelGGL(byte_copy_kernel, dim3(1), dim3(256), 0, s, src + head + 16u * n16,
                                 dst + head + 16u * n16, tail);
    HIPCHK(hipGetLastError());
    return TDT_OK;
}

void tdt_default_config(tdt_config *cfg) {
    cfg->sample_fraction = 0.3f;
    cfg->word_size = 4;
    cfg->bandwidth_threshold_mbps = 100.0;
    cfg->cpu_usage_threshold = 0.8;
    cfg->min_tensor_size = 1024;
}

int tdt_ctx_create(int device, const tdt_config *cfg, tdt_ctx **out) {
    if (!out) return set_err(TDT_E_ARG, "null out");
    *out = nullptr;
    tdt_config c;
    if (cfg) c = *cfg;
    else tdt_default_config(&c);
    if (c.word_size <= 0) return set_err(TDT_E_CONFIG, "word_size must be positive");
    if (!ws_supported(c.word_size)) return set_err(TDT_E_UNSUPPORTED, "GPU encoder supports word_size 1,2,4,8,16");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return set_err(TDT_E_ARG, "bad device");
    tdt_ctx *x = new tdt_ctx();
    x->device = device;
    x->cfg = c;
    // tuning / test overrides, read once here (tdt_ctx_set_option changes them later): the
    // tiled-path threshold, a lower tile budget (fallback tests), the diagnostic stream knobs
    if (const char *e = std::getenv("PSYNE_TDT_LARGE_MIN")) x->large_min = std::strtoull(e, nullptr, 10);
    if (const char *e = std::getenv("PSYNE_TDT_TILE_CAP")) x->tile_cap = (uint32_t)std::strtoul(e, nullptr, 10);
    auto flag = [](const char *name) {
        const char *e = std::getenv(name);
        return e && *e == '1';
    };
    x->no_side = flag("PSYNE_TDT_NO_SIDE");
    x->small_main = flag("PSYNE_TDT_SMALL_MAIN");
    x->no_two_phase = flag("PSYNE_TDT_NO_TWO_PHASE");
    x->no_one = flag("PSYNE_TDT_NO_ONE");
    x->one_wave = flag("PSYNE_TDT_ONE_WAVE");
    x->dout_sdma = flag("PSYNE_TDT_DOUT_SDMA");
    x->slot_streams = flag("PSYNE_TDT_SLOT_STREAMS");
    if (const char *e = std::getenv("PSYNE_TDT_ONE_SPIN")) x->one_spin = *e == '1';
    if (const char *e = std::getenv("PSYNE_TDT_DBIG_MIN")) x->dbig_min = std::strtoull(e, nullptr, 10);
    if (const char *e = std::getenv("PSYNE_TDT_DSMALL_MAX")) x->dsmall_max = std::strtoull(e, nullptr, 10);
    if (const char *e = std::getenv("PSYNE_TDT_COPY_WGS")) x->copy_wgs = std::max(1ul, std::strtoul(e, nullptr, 10));
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        x->cus = cus;
    // staging-copy threads: up to 16, within this process's CPU affinity (PSYNE_TDT_COPY_THREADS)
    cpu_set_t cs;
    CPU_ZERO(&cs);
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) x->copy_threads = std::max(1, std::min(16, CPU_COUNT(&cs)));
    if (const char *e = std::getenv("PSYNE_TDT_COPY_THREADS"))
        x->copy_threads = std::max(1, std::min(64, (int)std::strtol(e, nullptr, 10)));
    *out = x;
    return TDT_OK;
}

void tdt_ctx_destroy(tdt_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->slot_sums) (void)hipFree(ctx->slot_sums);
    if (ctx->cp_buf) (void)hipFree(ctx->cp_buf);
    if (ctx->cp_idx) (void)hipFree(ctx->cp_idx);
    for (void *p : ctx->retired) (void)hipFree(p);
    for (void *p : ctx->retired_host) (void)hipHostFree(p);
    ctx->pw.release();
    if (ctx->hbases) (void)hipFree(ctx->hbases);
    if (ctx->one_stream) (void)hipStreamSynchronize(ctx->one_stream);
    if (ctx->one) (void)hipHostFree(ctx->one);
    if (ctx->one_stream) (void)hipStreamDestroy(ctx->one_stream);
    if (ctx->astream) (void)hipStreamSynchronize(ctx->astream);
    if (ctx->h_dev) (void)hipFree(ctx->h_dev);
    if (ctx->astream) (void)hipStreamDestroy(ctx->astream);
    for (auto &h : ctx->hs) {
        if (h.stream) (void)hipStreamSynchronize(h.stream);
        if (h.dev) (void)hipFree(h.dev);
        if (h.pin) (void)hipHostFree(h.pin);
        if (h.flag) (void)hipHostFree(h.flag);
        if (h.stage_in) (void)hipHostFree(h.stage_in);
        if (h.stage_out) (void)hipHostFree(h.stage_out);
        h.pw.release();
        if (h.ev) (void)hipEventDestroy(h.ev);
        if (h.evc) (void)hipEventDestroy(h.evc);
        if (h.evi) (void)hipEventDestroy(h.evi);
        if (h.stream) (void)hipStreamDestroy(h.stream);
    }
    if (ctx->hin) (void)hipStreamSynchronize(ctx->hin);
    if (ctx->hex) (void)hipStreamSynchronize(ctx->hex);
    if (ctx->hin) (void)hipStreamDestroy(ctx->hin);
    if (ctx->hex) (void)hipStreamDestroy(ctx->hex);
    delete ctx;
}

void tdt_ctx_set_metrics(tdt_ctx *ctx, double bandwidth_mbps, double latency_ms, double cpu_usage) {
    ctx->bandwidth.store(bandwidth_mbps);
    ctx->latency.store(latency_ms);
    ctx->cpu.store(cpu_usage);
}

void tdt_ctx_get_metrics(const tdt_ctx *ctx, double *bandwidth_mbps, double *latency_ms, double *cpu_usage) {
    if (bandwidth_mbps) *bandwidth_mbps = ctx->bandwidth.load();
    if (latency_ms) *latency_ms = ctx->latency.load();
    if (cpu_usage) *cpu_usage = ctx->cpu.load();
}

void tdt_ctx_set_size_hint(tdt_ctx *ctx, uint64_t bytes) { ctx->size_hint.store(bytes); }

int tdt_ctx_set_option(tdt_ctx *ctx, int option, uint64_t value) {
    if (!ctx) return set_err(TDT_E_ARG, "null context");
    if (option == TDT_OPT_COPY_THREADS) {
        // the copy pool belongs to the host pipeline (hmu); lock order everywhere: hmu, then mu
        std::lock_guard<std::mutex> hl(ctx->hmu);
        ctx->copy_threads = (int)std::max<uint64_t>(1, std::min<uint64_t>(value, 64));
        ctx->pool.reset();
        return TDT_OK;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    switch (option) {
        case TDT_OPT_LARGE_MIN: ctx->large_min = value; return TDT_OK;
        case TDT_OPT_TILE_CAP: ctx->tile_cap = (uint32_t)std::min<uint64_t>(value, 0xffffffffu); return TDT_OK;
        case TDT_OPT_NO_SIDE_STREAM: ctx->no_side = value != 0; return TDT_OK;
        case TDT_OPT_SMALL_ON_CALLER_STREAM: ctx->small_main = value != 0; return TDT_OK;
        case TDT_OPT_NO_TWO_PHASE: ctx->no_two_phase = value != 0; return TDT_OK;
    }
    return set_err(TDT_E_ARG, "unknown option");
}

int tdt_should_transform(const tdt_ctx *ctx, uint64_t n) {
    if (n < ctx->cfg.min_tensor_size) return 0;
    if (ctx->cpu.load() > ctx->cfg.cpu_usage_threshold) return 0;
    if (!((n % 4 == 0) && (n >= 64))) return 0;
    return ctx->bandwidth.load() < ctx->cfg.bandwidth_threshold_mbps ? 1 : 0;
}

uint64_t tdt_encode_bound(uint64_t n, int32_t word_size) {
    const uint64_t w = word_size > 0 ? (uint64_t)word_size : 4;
    const uint64_t tdt = 20 + 4 * w + 8 + 2 * n;
    return std::max<uint64_t>(tdt, n + 4);
}


// Compacted encode.  Batches of medium messages (none over 64 KiB, >= 16 KiB on average): one
// pass, offsets by the kernels' decoupled look-back.  Batches with longer messages: a message's
// size is known only after its whole analysis, and those take far longer than the rest, so
// successors waiting in the look-back would stall every CU (head-of-line blocking); batches of
// small messages: the per-message ticket / look-back chain bounds the rate.  Both are encoded
// slotted (the message-class kernels), then the lengths are scanned and the blobs gathered.
int tdt_encode_batch(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs, uint8_t *d_out,
                     uint64_t out_cap, uint64_t *d_out_off, int32_t *d_status, void *stream) {
    if (!ctx || n_msgs == 0 || !d_in_off || !d_out || !d_out_off || !two_phase_ok(ctx, stream))
        return encode_common(ctx, psy::MODE_ENCODE, d_in, d_in_off, n_msgs, nullptr, d_out, out_cap, d_out_off,
                             d_status, nullptr, nullptr, nullptr, stream);
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(ctx->device));
    uint64_t h3[3];
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        const size_t need = 2ull * n_msgs + 2;
        if (need > ctx->cp_idx_n) {
            if (ctx->cp_idx) HIPCHK(hipFree(ctx->cp_idx));
            ctx->cp_idx = nullptr;
            HIPCHK(hipMalloc(&ctx->cp_idx, 8 * need));
            ctx->cp_idx_n = need;
        }
        uint64_t *flag = ctx->cp_idx + 2ull * n_msgs + 1;
        HIPCHK(hipMemsetAsync(flag, 0, 8, s));
        hipLaunchKernelGGL(cp_big_kernel, dim3((n_msgs + 255) / 256), dim3(256), 0, s, d_in, d_in_off, n_msgs,
                           (uint64_t)65536, flag);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(&h3[0], flag, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&h3[1], d_in_off, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&h3[2], d_in_off + n_msgs, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    // one pass with the look-back for batches of medium messages (all <= 64 KiB, 16 KiB or more
    // on average); small messages make the per-message ticket and look-back chain the limit
    // (C2: 12 ms for 1 Mi x 1 KiB), long ones stall it — both take the two phases
    if (!(h3[0] & 1) && (h3[2] - h3[1]) >= 16384ull * n_msgs)  // (16 KiB on average: 512-lane teams)
        return encode_common(ctx, psy::MODE_ENCODE, d_in, d_in_off, n_msgs, nullptr, d_out, out_cap, d_out_off,
                             d_status, nullptr, nullptr, nullptr, stream, nullptr, nullptr, nullptr, nullptr,
                             (h3[0] & 2) ? 0 : 2);
    uint64_t *slot = ctx->cp_idx, *len = ctx->cp_idx + n_msgs + 1;
    // Σ encode bounds <= 2·(input bytes) + n·(28 + 4·ws) (and >= n + 4 per message)
    const uint64_t bound = 2 * (h3[2] - h3[1]) + (uint64_t)n_msgs * (28 + 4ull * (uint64_t)ctx->cfg.word_size + 4);
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (bound > ctx->cp_bytes) {
            if (ctx->cp_buf) HIPCHK(hipFree(ctx->cp_buf));
            ctx->cp_buf = nullptr;
            HIPCHK(hipMalloc(&ctx->cp_buf, bound));
            ctx->cp_bytes = bound;
        }
    }
    int st = tdt_encode_slots(ctx, d_in_off, n_msgs, slot, stream);
    if (st) return st;
    st = tdt_encode_batch_into(ctx, d_in, d_in_off, n_msgs, ctx->cp_buf, slot, len, d_status, stream);
    if (st) return st;
    hipLaunchKernelGGL(cp_len_kernel, dim3((n_msgs + 255) / 256), dim3(256), 0, s, len, d_out_off, n_msgs);
    HIPCHK(hipGetLastError());
    st = scan_sizes(ctx, d_out_off, n_msgs, s);  // exclusive, total at [n]
    if (st) return st;
    hipLaunchKernelGGL(cp_gather_kernel, dim3((n_msgs + 3) / 4), dim3(256), 0, s, ctx->cp_buf, slot, len, d_out,
                       d_out_off, out_cap, d_status, n_msgs);
    HIPCHK(hipGetLastError());
    return TDT_OK;
}

int tdt_encode_with_mapping_batch(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs,
                                  const int32_t *d_mapping, uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off,
                                  int32_t *d_status, void *stream) {
    return encode_common(ctx, psy::MODE_MAPPED, d_in, d_in_off, n_msgs, d_mapping, d_out, out_cap, d_out_off,
                         d_status, nullptr, nullptr, nullptr, stream);
}

int tdt_analyze_batch(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs, uint32_t *d_hist,
                      double *d_entropy, int32_t *d_mapping, int32_t *d_status, void *stream) {
    return encode_common(ctx, psy::MODE_ANALYZE, d_in, d_in_off, n_msgs, nullptr, nullptr, 0, nullptr, d_status,
                         d_hist, d_entropy, d_mapping, stream);
}

// Compacted decode.  Decoded sizes are in the headers, so the output offsets are computed
// first (sizes + scan) and the blobs decoded by the slotted message-class kernels straight into
// their compacted places (no copy; and no look-back, whose successors stall behind long blobs);
// batches whose total exceeds out_cap take the look-back kernel, which assigns
// TDT_E_CAPACITY per blob.
int tdt_decode_batch(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs, uint8_t *d_out,
                     uint64_t out_cap, uint64_t *d_out_off, int32_t *d_status, void *stream) {
    if (ctx && n_msgs && d_in_off && d_out && d_out_off && two_phase_ok(ctx, stream)) {
        hipStream_t s = (hipStream_t)stream;
        HIPCHK(hipSetDevice(ctx->device));
        int st = tdt_decode_slots(ctx, d_in, d_in_off, nullptr, n_msgs, d_out_off, d_status, stream);
        if (st) return st;
        uint64_t total = 0;
        {
            std::lock_guard<std::mutex> lk(ctx->mu);
            const size_t need = 2ull * n_msgs + 2;
            if (need > ctx->cp_idx_n) {
                if (ctx->cp_idx) HIPCHK(hipFree(ctx->cp_idx));
                ctx->cp_idx = nullptr;
                HIPCHK(hipMalloc(&ctx->cp_idx, 8 * need));
                ctx->cp_idx_n = need;
            }
            HIPCHK(hipMemcpyAsync(&total, d_out_off + n_msgs, 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        if (total <= out_cap)
            return tdt_decode_batch_into(ctx, d_in, d_in_off, nullptr, n_msgs, d_out, d_out_off, ctx->cp_idx, d_status,
                                         stream);
    }
    return decode_common(ctx, false, d_in, d_in_off, n_msgs, d_out, out_cap, d_out_off, nullptr, d_status, stream);
}

int tdt_decoded_sizes_batch(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs,
                            uint64_t *d_sizes, int32_t *d_status, void *stream) {
    return decode_common(ctx, true, d_in, d_in_off, n_msgs, nullptr, 0, nullptr, d_sizes, d_status, stream);
}

int tdt_encode_batch_into(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs,
                          uint8_t *d_out, const uint64_t *d_slot_off, uint64_t *d_out_len, int32_t *d_status,
                          void *stream) {
    if (n_msgs && !d_slot_off) return set_err(TDT_E_ARG, "null slot offsets");
    return encode_common(ctx, psy::MODE_ENCODE, d_in, d_in_off, n_msgs, nullptr, d_out, 0, nullptr, d_status, nullptr,
                         nullptr, nullptr, stream, d_slot_off, d_out_len);
}

int tdt_decode_batch_into(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, const uint64_t *d_in_len,
                          uint32_t n_msgs, uint8_t *d_out, const uint64_t *d_slot_off, uint64_t *d_out_len,
                          int32_t *d_status, void *stream) {
    if (n_msgs && !d_slot_off) return set_err(TDT_E_ARG, "null slot offsets");
    return decode_common(ctx, false, d_in, d_in_off, n_msgs, d_out, 0, nullptr, nullptr, d_status, stream, d_slot_off,
                         d_out_len, d_in_len);
}

int tdt_encode_slots(tdt_ctx *ctx, const uint64_t *d_in_off, uint32_t n_msgs, uint64_t *d_slot_off, void *stream) {
    if (!ctx) return set_err(TDT_E_ARG, "null context");
    if (!d_slot_off || (n_msgs && !d_in_off)) return set_err(TDT_E_ARG, "null offsets");
    HIPCHK(hipSetDevice(ctx->device));
    if (n_msgs == 0) {  // d_in_off may be null for an empty batch
        HIPCHK(hipMemsetAsync(d_slot_off, 0, 8, (hipStream_t)stream));
        return TDT_OK;
    }
    hipLaunchKernelGGL(psy::tdt_encode_slots_kernel, dim3((n_msgs + 256) / 256), dim3(256), 0, (hipStream_t)stream,
                       d_in_off, d_slot_off, n_msgs, (uint32_t)ctx->cfg.word_size);
    HIPCHK(hipGetLastError());
    return TDT_OK;
}

int tdt_decode_slots(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, const uint64_t *d_in_len,
                     uint32_t n_msgs, uint64_t *d_slot_off, int32_t *d_status, void *stream) {
    if (!ctx) return set_err(TDT_E_ARG, "null context");
    if (!d_slot_off) return set_err(TDT_E_ARG, "null offsets");
    if (n_msgs) {
        int st = decode_common(ctx, true, d_in, d_in_off, n_msgs, nullptr, 0, nullptr, d_slot_off, d_status, stream,
                               nullptr, nullptr, d_in_len);
        if (st) return st;
    }
    HIPCHK(hipSetDevice(ctx->device));
    return scan_sizes(ctx, d_slot_off, n_msgs, (hipStream_t)stream);
}


int tdt_encode_host(tdt_ctx *ctx, const uint8_t *h_in, const uint64_t *h_in_off, uint32_t n_msgs, uint8_t *h_out,
                    uint64_t out_cap, uint64_t *h_out_off, int32_t *h_status) {
    return host_path(ctx, true, h_in, h_in_off, n_msgs, h_out, out_cap, h_out_off, h_status);
}

int tdt_decode_host(tdt_ctx *ctx, const uint8_t *h_in, const uint64_t *h_in_off, uint32_t n_msgs, uint8_t *h_out,
                    uint64_t out_cap, uint64_t *h_out_off, int32_t *h_status) {
    return host_path(ctx, false, h_in, h_in_off, n_msgs, h_out, out_cap, h_out_off, h_status);
}

int tdt_encode_host_v(tdt_ctx *ctx, const uint8_t *const *msgs, const uint64_t *sizes, uint32_t n_msgs, uint8_t *h_out,
                      uint64_t out_cap, uint64_t *h_out_off, int32_t *h_status) {
    if (!ctx) return set_err(TDT_E_ARG, "null context");
    if (n_msgs == 0) {
        if (h_out_off) h_out_off[0] = 0;
        return TDT_OK;
    }
    if (!msgs || !sizes || !h_out_off) return set_err(TDT_E_ARG, "null argument");
    if (n_msgs == 1) {
        const uint64_t off[2] = {0, sizes[0]};
        return host_path(ctx, true, msgs[0], off, 1, h_out, out_cap, h_out_off, h_status);
    }
    std::vector<uint64_t> voff(n_msgs + 1, 0);
    for (uint32_t i = 0; i < n_msgs; ++i) voff[i + 1] = voff[i] + sizes[i];
    HIPCHK(hipSetDevice(ctx->device));
    std::lock_guard<std::mutex> lk(ctx->hmu);
    if (!ctx->pool) ctx->pool.reset(new CopyPool(ctx->copy_threads));
    const int st = host_encode(ctx, nullptr, voff.data(), n_msgs, h_out, out_cap, h_out_off, h_status, msgs, sizes);
    if (st != TDT_OK) {
        drain_host(ctx);
        (void)hipGetLastError();
    }
    return st;
}

int tdt_host_alloc(uint64_t bytes, void **ptr) {
    if (!ptr) return set_err(TDT_E_ARG, "null argument");
    *ptr = nullptr;
    HIPCHK(hipHostMalloc(ptr, std::max<uint64_t>(bytes, 1), hipHostMallocDefault));
    return TDT_OK;
}

void tdt_host_free(void *ptr) {
    if (ptr) (void)hipHostFree(ptr);
}

int tdt_host_copy(tdt_ctx *ctx, void *dst, const void *src, uint64_t bytes) {
    if (!ctx || (bytes && (!dst || !src))) return set_err(TDT_E_ARG, "null argument");
    std::shared_ptr<CopyPool> pool;
    {
        std::lock_guard<std::mutex> lk(ctx->hmu);  // (the pool is created and replaced under hmu)
        if (!ctx->pool) ctx->pool.reset(new CopyPool(ctx->copy_threads));
        pool = ctx->pool;
    }
    pool->copy(dst, src, bytes);  // (outside hmu: CopyPool::copy serialises concurrent callers itself)
    return TDT_OK;
}

int tdt_ctx_error_flags(tdt_ctx *ctx, void *stream, uint32_t *flags) {
    if (!ctx || !flags) return set_err(TDT_E_ARG, "null argument");
    *flags = ctx->host_flags.load();
    if (!ctx->ws) return TDT_OK;
    HIPCHK(hipSetDevice(ctx->device));
    // stream-ordered read of the flag word: waits for the batches issued on `stream` only
    uint32_t f = 0;
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(&f, ctx->ws + 4, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *flags |= f;
    return TDT_OK;
}

int tdt_analyze_host(tdt_ctx *ctx, const uint8_t *h_in, const uint64_t *h_in_off, uint32_t n_msgs, double *h_entropy,
                     int32_t *h_mapping, int32_t *h_status) {
    if (!ctx) return set_err(TDT_E_ARG, "null context");
    if (n_msgs == 0) return TDT_OK;
    HIPCHK(hipSetDevice(ctx->device));
    const uint64_t in_bytes = h_in_off[n_msgs] - h_in_off[0];
    const size_t ws = (size_t)ctx->cfg.word_size;
    const size_t o_off = align_up(in_bytes, 256);
    const size_t o_ent = align_up(o_off + 8ull * (n_msgs + 1), 256);
    const size_t o_map = align_up(o_ent + 8ull * n_msgs * ws, 256);
    const size_t o_st = align_up(o_map + 4ull * n_msgs * ws, 256);
    const size_t total = align_up(o_st + 4ull * n_msgs, 256);
    // h_dev and astream belong to the host paths (hmu, held for the whole call, so a second
    // caller cannot reallocate h_dev under this one); encode_common then takes mu: the lock
    // order everywhere is hmu, then mu
    std::lock_guard<std::mutex> hl(ctx->hmu);
    int st = ensure_host_dev(ctx, total);
    if (st) return st;
    uint8_t *d = ctx->h_dev;
    std::vector<uint64_t> tmp(n_msgs + 1);
    for (uint32_t i = 0; i <= n_msgs; ++i) tmp[i] = h_in_off[i] - h_in_off[0];
    // on the context's own stream (synchronising that stream only, not the device)
    if (!ctx->astream) HIPCHK(hipStreamCreateWithFlags(&ctx->astream, hipStreamNonBlocking));
    hipStream_t s = ctx->astream;
    HIPCHK(hipMemcpyAsync(d, h_in + h_in_off[0], in_bytes, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d + o_off, tmp.data(), 8ull * (n_msgs + 1), hipMemcpyHostToDevice, s));
    st = encode_common(ctx, psy::MODE_ANALYZE, d, reinterpret_cast<uint64_t *>(d + o_off), n_msgs, nullptr, nullptr,
                       0, nullptr, reinterpret_cast<int32_t *>(d + o_st), nullptr,
                       reinterpret_cast<double *>(d + o_ent), reinterpret_cast<int32_t *>(d + o_map), s, nullptr,
                       nullptr, nullptr, nullptr, in_bytes <= kSmallMax * n_msgs ? 1 : 0);
    if (st) return st;
    if (h_entropy) HIPCHK(hipMemcpyAsync(h_entropy, d + o_ent, 8ull * n_msgs * ws, hipMemcpyDeviceToHost, s));
    if (h_mapping) HIPCHK(hipMemcpyAsync(h_mapping, d + o_map, 4ull * n_msgs * ws, hipMemcpyDeviceToHost, s));
    if (h_status) HIPCHK(hipMemcpyAsync(h_status, d + o_st, 4ull * n_msgs, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return TDT_OK;
}

const char *tdt_last_error(void) { return g_err.c_str(); }

const char *tdt_status_string(int status) {
    switch (status) {
        case TDT_OK: return "OK";
        case TDT_E_SHORT: return "TDT: Invalid encoded data size";
        case TDT_E_MAGIC: return "Invalid TDT magic number";
        case TDT_E_TRUNCATED: return "TDT: truncated blob";
        case TDT_E_BAD_MAPPING: return "TDT: invalid cluster mapping";
        case TDT_E_CAPACITY: return "TDT: output capacity exceeded";
        case TDT_E_UNSUPPORTED: return "TDT: word size not supported on the GPU path";
        case TDT_E_BAD_HEADER: return "TDT: word size 0";
        case TDT_E_CONFIG: return "TDT: invalid configuration";
        case TDT_E_HIP: return "TDT: HIP runtime error";
        case TDT_E_CAPTURE: return "TDT: workspace growth needed under stream capture";
        case TDT_E_ARG: return "TDT: invalid argument";
    }
    return "TDT: unknown status";
}

#if defined(PSY_PROF) && PSY_PROF
// diagnostic builds only: read and clear the phase-cycle counters
int tdt_prof_read(uint64_t *out32) {
    if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(psy::psy_prof), 32 * sizeof(uint64_t)) != hipSuccess) return TDT_E_HIP;
    static const uint64_t zero[32] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(psy::psy_prof), zero, sizeof(zero)) != hipSuccess) return TDT_E_HIP;
    return TDT_OK;
}
#endif
}  // extern "C"

// In-place exclusive scan of n sizes (u64) at d_off; d_off[n] = the total.
static int scan_sizes(tdt_ctx *ctx, uint64_t *d_slot_off, uint32_t n_msgs, hipStream_t stream) {
    const uint32_t nb = (n_msgs + psy::kSlotChunk - 1) / psy::kSlotChunk;
    if (nb > 1) {
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (nb > ctx->slot_sums_n) {
            if (int st = no_growth_in_capture(stream)) return st;
            if (ctx->slot_sums) ctx->retired.push_back(ctx->slot_sums);  // (a captured graph may use it)
            ctx->slot_sums = nullptr;
            HIPCHK(hipMalloc(&ctx->slot_sums, 8ull * nb));
            ctx->slot_sums_n = nb;
        }
        hipLaunchKernelGGL(psy::tdt_slot_sums_kernel, dim3(nb - 1), dim3(psy::kSlotThreads), 0, (hipStream_t)stream,
                           d_slot_off, ctx->slot_sums, n_msgs);
        HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(psy::tdt_slot_scan_kernel, dim3(nb ? nb : 1), dim3(psy::kSlotThreads), 0, (hipStream_t)stream,
                       d_slot_off, nb > 1 ? ctx->slot_sums : nullptr, n_msgs);
    HIPCHK(hipGetLastError());
    return TDT_OK;
}

