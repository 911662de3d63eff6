/* psyne_tdt.h — C ABI of the MI355X TDT payload codec (libpsyne_tdt.so).
 *
 * Drop-in boundary for psyne's TDT protocol (include/psyne/protocol/tdt_compression.hpp
 * in the reference).  The reference exposes the codec through the C++ `Protocol` concept
 * (include/psyne/concepts/protocol_concepts.hpp:22-47), one message per call, host
 * vectors in and out.  This ABI is what a binding of that concept for the GPU binds:
 * plain pointers and sizes, batches of independent messages, device-resident buffers,
 * asynchronous on a caller-supplied hipStream_t (passed as void*).  The header-only C++
 * class psyne_amd::HipTDTCompressionProtocol (include/psyne_amd/hip_tdt_protocol.hpp)
 * layers the reference's exact Protocol surface on top of it.
 *
 * Which reference interface each entry point replaces:
 *   tdt_ctx_create / tdt_ctx_destroy  TDTCompressionProtocol(const TDTConfig&)   :178-179
 *   tdt_ctx_set_metrics               update_network_metrics / update_system_metrics :309-319
 *   tdt_should_transform              should_transform                            :186-201
 *   tdt_encode_batch                  encode                                      :227-266
 *   tdt_encode_with_mapping_batch     encode with a given cluster mapping (parity hook for
 *                                     blobs made in the reference's random-sample mode)
 *   tdt_decode_batch                  decode                                      :271-304
 *   tdt_decoded_sizes_batch           the output size decode would produce (header parse)
 *   tdt_encode_batch_into /           encode / decode into caller slots (one vector per
 *   tdt_decode_batch_into             message, as the reference returns them)
 *   tdt_analyze_batch                 analyze_data / extract_features / perform_clustering
 *                                     :206-222, :434-525 (full-sample histograms, entropies,
 *                                     mapping per message)
 *   tdt_encode_bound                  worst-case blob size (sizing out buffers)
 *   tdt_last_error                    the reference's exception text (:128, :275)
 *
 * Wire format: identical bytes to the reference: UNCP marker
 * 0x554E4350 + payload, or TDT header | mapping | (u32 len, RLE pairs) per stream.
 *
 * Batch layout: message i occupies in[in_off[i] .. in_off[i+1]) (in_off has n+1
 * entries, device memory).  Outputs are either SLOTTED (the *_into entry points, below) or
 * COMPACTED (tdt_encode_batch / tdt_decode_batch): message i's result is written at
 * out[out_off[i] .. out_off[i+1]) and the kernel fills out_off (n+1 entries, device
 * memory) itself with a single-pass decoupled look-back, so the caller never needs the
 * sizes up front.  Per-message status codes go to status[i] if status != NULL.
 *
 * Determinism: the reference chooses the byte-plane mapping from a random 30% sample
 * (mt19937 seeded by random_device).  This codec always analyses every word — the
 * reference's sample_fraction = 1.0 behaviour — so its output is deterministic and
 * byte-identical to the reference configured that way; tdt_encode_with_mapping_batch
 * reproduces default-mode blobs given their mapping.
 */
#ifndef PSYNE_TDT_H
#define PSYNE_TDT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSYNE_TDT_ABI_VERSION 1

/* Status codes (per call and per message). */
#define TDT_OK 0
#define TDT_E_SHORT 1         /* blob < 4 bytes: "TDT: Invalid encoded data size" (:274-276) */
#define TDT_E_MAGIC 2         /* neither UNCP nor TDT magic: "Invalid TDT magic number" (:127-129) */
#define TDT_E_TRUNCATED 3     /* header or stream runs past the blob (reference: UB) */
#define TDT_E_BAD_MAPPING 4   /* mapping shorter than word_size or value >= num_streams (reference: UB) */
#define TDT_E_CAPACITY 5      /* output buffer too small for this message */
#define TDT_E_UNSUPPORTED 6   /* word_size this build does not implement on the GPU */
#define TDT_E_BAD_HEADER 7    /* word_size == 0 in a blob (reference: division by zero) */
#define TDT_E_CONFIG 8        /* invalid tdt_config */
#define TDT_E_HIP 10          /* HIP runtime error (tdt_last_error has the text) */
#define TDT_E_ARG 11          /* invalid argument */
#define TDT_E_CAPTURE 12      /* a workspace must grow while the stream is captured: make one eager
                                 call of the batch on this context before capturing it */

/* TDTConfig (:31-43).  Fields the reference declares but never reads
 * (auto_detect_clusters, max_clusters, enable_simd) are omitted. */
typedef struct tdt_config {
    float sample_fraction;           /* accepted; the GPU always uses the full sample (1.0) */
    int32_t word_size;               /* 1, 2, 4, 8 or 16 */
    double bandwidth_threshold_mbps; /* default 100.0 */
    double cpu_usage_threshold;      /* default 0.8 */
    uint64_t min_tensor_size;        /* default 1024 */
} tdt_config;

typedef struct tdt_ctx tdt_ctx;

void tdt_default_config(tdt_config *cfg);

/* Create a codec context bound to HIP device `device`.
 *
 * Streams: a context owns one device workspace (look-back words, error flags, slot-scan
 * sums), so its *_batch / *_slots calls must be issued on ONE stream at a time (stream order
 * keeps consecutive batches apart); use one context per stream for concurrent batches.  The
 * host calls (tdt_*_host) run on the context's own two pipeline streams and are serialised by
 * the context; they do not touch the caller's streams. */
int tdt_ctx_create(int device, const tdt_config *cfg, tdt_ctx **out);
void tdt_ctx_destroy(tdt_ctx *ctx);

/* update_network_metrics(bandwidth, latency) + update_system_metrics(cpu) (:309-319).
 * Defaults match the reference: bandwidth 100 Mbps (compression OFF), cpu 0.5. */
void tdt_ctx_set_metrics(tdt_ctx *ctx, double bandwidth_mbps, double latency_ms, double cpu_usage);
void tdt_ctx_get_metrics(const tdt_ctx *ctx, double *bandwidth_mbps, double *latency_ms, double *cpu_usage);

/* Seed for the team shape of one-pass launches whose message sizes the host does not know
 * (tdt_encode_with_mapping_batch, tdt_analyze_batch, and tdt_encode_batch under stream
 * capture): one 64-lane wave per message up to 4 KiB, a 512-lane workgroup otherwise.  Once a
 * slotted plan of this context has completed, its class counts decide instead; the slotted
 * calls, tdt_encode_batch outside capture and the host pipeline never use it.  Optional; any
 * size encodes correctly with either shape. */
void tdt_ctx_set_size_hint(tdt_ctx *ctx, uint64_t typical_message_bytes);

/* should_transform (:186-201) for a message of n bytes under the current metrics. */
int tdt_should_transform(const tdt_ctx *ctx, uint64_t n);

/* Worst-case encoded size of one n-byte message: max(n + 4, 28 + 4*ws + 2n). */
uint64_t tdt_encode_bound(uint64_t n, int32_t word_size);

/* Encode a batch.  out_cap: bytes available at d_out (use the sum of tdt_encode_bound).
 * Messages whose compressed blob would overflow out_cap get TDT_E_CAPACITY.
 * Returns TDT_OK or an argument/HIP error; per-message results go to d_status. */
int tdt_encode_batch(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs,
                     uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off, int32_t *d_status,
                     void *hip_stream);

/* Encode with a caller-chosen mapping: d_mapping holds n_msgs * word_size int32 values in
 * {0, 1} (e.g. read from reference blobs at bytes 20 .. 20 + 4*ws). */
int tdt_encode_with_mapping_batch(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off,
                                  uint32_t n_msgs, const int32_t *d_mapping, uint8_t *d_out,
                                  uint64_t out_cap, uint64_t *d_out_off, int32_t *d_status,
                                  void *hip_stream);

/* Decode a batch of blobs (any mix of UNCP and TDT).  Output compacted by decoded size. */
int tdt_decode_batch(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs,
                     uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off, int32_t *d_status,
                     void *hip_stream);

/* SLOTTED batches — the hot path.  No dependency between messages: blob i goes to
 * out[slot_off[i] ..) with capacity slot_off[i+1] - slot_off[i] (slot_off: n+1 entries,
 * device memory, chosen by the caller — tdt_encode_slots gives the prefix sum of the encode
 * bounds, tdt_decode_slots the prefix sum of the decoded sizes); its length goes to
 * out_len[i] (0 with status TDT_E_CAPACITY if the slot is too small).  This is the layout of
 * the reference's API — one independent vector per message (:227-266, :271-304) — and of
 * batched GPU codecs generally: each blob is sent as its own frame. */
int tdt_encode_batch_into(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs,
                          uint8_t *d_out, const uint64_t *d_slot_off, uint64_t *d_out_len, int32_t *d_status,
                          void *hip_stream);
/* Decode input: blob i = in[in_off[i] .. in_off[i] + in_len[i]) when d_in_len != NULL (e.g. the
 * slots and lengths tdt_encode_batch_into produced), else in[in_off[i] .. in_off[i+1]). */
int tdt_decode_batch_into(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, const uint64_t *d_in_len,
                          uint32_t n_msgs, uint8_t *d_out, const uint64_t *d_slot_off, uint64_t *d_out_len,
                          int32_t *d_status, void *hip_stream);
/* d_slot_off (n+1 entries) = exclusive prefix sum of tdt_encode_bound(size_i, word_size). */
int tdt_encode_slots(tdt_ctx *ctx, const uint64_t *d_in_off, uint32_t n_msgs, uint64_t *d_slot_off,
                     void *hip_stream);
/* d_slot_off (n+1 entries) = exclusive prefix sum of the decoded sizes (header parse). */
int tdt_decode_slots(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, const uint64_t *d_in_len,
                     uint32_t n_msgs, uint64_t *d_slot_off, int32_t *d_status, void *hip_stream);

/* Decoded size of each blob (0 for blobs with an error status). */
int tdt_decoded_sizes_batch(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off,
                            uint32_t n_msgs, uint64_t *d_sizes, int32_t *d_status, void *hip_stream);

/* Full-sample analysis of each message (n must be a non-zero multiple of word_size):
 * d_hist n*ws*256 uint32, d_entropy n*ws double, d_mapping n*ws int32 (any may be NULL). */
int tdt_analyze_batch(tdt_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, uint32_t n_msgs,
                      uint32_t *d_hist, double *d_entropy, int32_t *d_mapping, int32_t *d_status,
                      void *hip_stream);

/* Host-memory path (the TCP socket-buffer case).  The batch runs as chunks (an eighth of the
 * call's input, 2-64 MiB) through four pipeline slots (device buffers) on two streams, one for
 * the input DMAs and one for the kernels and the output: H2D, kernel and D2H of neighbouring
 * chunks overlap.  Pinned caller buffers are DMA'd
 * directly; pageable ones (std::vector, numpy) are staged through the context's pinned buffers
 * by a pool of host threads (TDT_OPT_COPY_THREADS).  h_out must hold the sum of
 * tdt_encode_bound (encode) or of the decoded sizes (decode); h_out_off receives n+1 offsets.
 * Blocks the calling thread until the results are in h_out. */
int tdt_encode_host(tdt_ctx *ctx, const uint8_t *h_in, const uint64_t *h_in_off, uint32_t n_msgs,
                    uint8_t *h_out, uint64_t out_cap, uint64_t *h_out_off, int32_t *h_status);
int tdt_decode_host(tdt_ctx *ctx, const uint8_t *h_in, const uint64_t *h_in_off, uint32_t n_msgs,
                    uint8_t *h_out, uint64_t out_cap, uint64_t *h_out_off, int32_t *h_status);
/* tdt_encode_host over n messages that are NOT contiguous (message i = msgs[i][0 .. sizes[i])),
 * as a substrate's send path holds them (one buffer per message, transport_send(void*, size_t),
 * tcp_simple.hpp:68-91): the pool copies them straight into the pinned staging, no packing
 * copy.  Replaces a loop of TDTCompressionProtocol::encode (tdt_compression.hpp:227-266). */
int tdt_encode_host_v(tdt_ctx *ctx, const uint8_t *const *msgs, const uint64_t *sizes, uint32_t n_msgs,
                      uint8_t *h_out, uint64_t out_cap, uint64_t *h_out_off, int32_t *h_status);
/* Pinned (page-locked, device-mapped) host memory for callers that keep their socket buffers in
 * it: the host paths DMA such buffers directly instead of staging them.  Returns TDT_OK. */
int tdt_host_alloc(uint64_t bytes, void **ptr);
void tdt_host_free(void *ptr);
/* dst[0, bytes) = src[0, bytes) on the context's staging-copy threads (a parallel memcpy: one
 * thread's copy is below what a socket pipeline needs).  Host memory only. */
int tdt_host_copy(tdt_ctx *ctx, void *dst, const void *src, uint64_t bytes);
/* d_dst[0, bytes) = d_src[0, bytes) between device buffers, asynchronously on hip_stream (NULL:
 * the null stream), by the codec's hand-written HBM copy: one 512-lane workgroup per 64 KiB piece,
 * every load of the piece in flight before its non-temporal stores — the access shape of the
 * resident encode / decode, and the best hand-written copy measured on MI355X (tools/ubench_hbm.hip:
 * 5.6-5.8 TB/s read + write).  bench.py times it as roofline.copy_ceiling.  Any sizes and
 * alignments; the buffers must not overlap. */
int tdt_copy_device(void *d_dst, const void *d_src, uint64_t bytes, void *hip_stream);

/* Device-side invariant flags: bit0 look-back timeout, bit1 staging-index guard, bit2
 * flush-bound guard.  Always 0 for a correct build; the guards turn a logic error into a flag
 * instead of a wild write.  Reads the flag word in stream order on `hip_stream` (the stream
 * the context's batches were issued on) and synchronises that stream only.  Scope: the most
 * recent compacted (look-back) batch on the context's workspace, OR-ed with every slotted
 * batch since then (slotted calls do not clear the word) and with every host-pipeline chunk
 * since the context was created (sticky). */
int tdt_ctx_error_flags(tdt_ctx *ctx, void *hip_stream, uint32_t *flags);

/* Tuning / diagnostic options (tdt_ctx_create reads the same from the environment once:
 * PSYNE_TDT_LARGE_MIN, PSYNE_TDT_TILE_CAP, PSYNE_TDT_NO_SIDE, PSYNE_TDT_SMALL_MAIN,
 * PSYNE_TDT_NO_TWO_PHASE, PSYNE_TDT_COPY_THREADS).  Not needed for correct results: every setting encodes and decodes
 * the same bytes. */
#define TDT_OPT_LARGE_MIN 1               /* messages above this many bytes take the tiled path */
#define TDT_OPT_TILE_CAP 2                /* lower tile budget per batch (tests of the fallback) */
#define TDT_OPT_NO_SIDE_STREAM 3          /* 1: the tile pipeline runs on the caller's stream */
#define TDT_OPT_SMALL_ON_CALLER_STREAM 4  /* 1: small-message lists stay on the caller's stream */
#define TDT_OPT_NO_TWO_PHASE 5            /* 1: compacted calls always take the one-pass kernels */
#define TDT_OPT_COPY_THREADS 6            /* host threads staging pageable buffers (default <= 16) */
int tdt_ctx_set_option(tdt_ctx *ctx, int option, uint64_t value);

/* Host-memory analyze (analyze_data :206-222): h_entropy n*ws doubles, h_mapping n*ws int32
 * (either may be NULL).  Blocks the calling thread. */
int tdt_analyze_host(tdt_ctx *ctx, const uint8_t *h_in, const uint64_t *h_in_off, uint32_t n_msgs,
                     double *h_entropy, int32_t *h_mapping, int32_t *h_status);

/* Text of the last error on this thread ("" if none). */
const char *tdt_last_error(void);
/* Human-readable status name; for TDT_E_SHORT / TDT_E_MAGIC the reference's exception text. */
const char *tdt_status_string(int status);

#ifdef __cplusplus
}
#endif
#endif
