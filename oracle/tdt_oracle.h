/* oracle/tdt_oracle.h — CPU restatement of the reference TDT codec.
 *
 * TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the CHECKER.  The product path (psyne_amd/) never links or calls it.
 *
 * Restates include/psyne/protocol/tdt_compression.hpp (reference, read-only) in plain C.
 * Parity is pinned by tests/golden/ fixtures generated from the compiled reference header
 * (oracle/_ref/libtdt_ref.so, see oracle/Makefile and tests/golden/make_golden.py).
 *
 * Determinism: the reference samples words with std::shuffle(mt19937(random_device))
 * (:419-432).  The restatement covers the deterministic case, sample count == word count
 * (sample_fraction >= 1, or word_count <= 100), which is what the GPU path implements.
 * A caller-supplied mapping covers blobs made in the reference's default (random) mode.
 */
#ifndef PSYNE_TDT_ORACLE_H
#define PSYNE_TDT_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes: identical values to include/psyne_tdt.h. */
#define TDT_ORACLE_OK 0
#define TDT_ORACLE_E_SHORT 1        /* blob < 4 bytes          (:274-276) */
#define TDT_ORACLE_E_MAGIC 2        /* not UNCP and not TDT    (:127-129) */
#define TDT_ORACLE_E_TRUNCATED 3    /* header/stream past end  (reference: UB) */
#define TDT_ORACLE_E_BAD_MAPPING 4  /* mapping short or value >= num_streams (reference: UB) */
#define TDT_ORACLE_E_CAPACITY 5     /* output buffer too small */
#define TDT_ORACLE_E_BAD_HEADER 7   /* word_size == 0 (reference: division by zero) */
#define TDT_ORACLE_E_CONFIG 8       /* word_size <= 0 in the encoder config */
#define TDT_ORACLE_E_NONDETERMINISTIC 9 /* sample count < word count and no mapping given */

typedef struct {
    float sample_fraction;          /* TDTConfig :32 */
    int32_t word_size;              /* :33 */
    double bandwidth_threshold_mbps;/* :39-40 */
    double cpu_usage_threshold;     /* :41 */
    uint64_t min_tensor_size;       /* :42 */
} tdt_oracle_config;

void tdt_oracle_default_config(tdt_oracle_config *cfg);

/* should_transform :186-201 with is_tensor_data :409-413. */
int tdt_oracle_should_transform(uint64_t n, const tdt_oracle_config *cfg,
                                double bandwidth_mbps, double cpu_usage);

/* Worst-case encoded size: max(UNCP n+4, TDT 20 + 4*ws + 8 + 2n). */
uint64_t tdt_oracle_encode_bound(uint64_t n, int32_t word_size);

/* Histograms (ws x 256, full sample), entropies (ws) and mapping (ws) of one message:
 * extract_features :434-468, calculate_entropy :470-480, perform_clustering :507-525. */
int tdt_oracle_analyze(const uint8_t *data, uint64_t n, int32_t word_size,
                       uint32_t *hist, double *entropy, int32_t *mapping);

/* encode :227-266.  mapping == NULL: computed from full-sample histograms (deterministic
 * case only); else used as given (values must be >= 0 and < 2 * word_size). */
int tdt_oracle_encode(const uint8_t *data, uint64_t n, const tdt_oracle_config *cfg,
                      double bandwidth_mbps, double cpu_usage, const int32_t *mapping,
                      uint8_t *out, uint64_t cap, uint64_t *out_len);

/* decode :271-304 (deserialize :119-170, decompress :584-612, recombine :614-637).
 * Where the reference has undefined behaviour the restatement returns an error code. */
int tdt_oracle_decode(const uint8_t *blob, uint64_t len, uint8_t *out, uint64_t cap,
                      uint64_t *out_len);

/* Size the decode would produce (0 on error). */
int tdt_oracle_decoded_size(const uint8_t *blob, uint64_t len, uint64_t *out_len);

/* Batch helpers used by tests and bench (threads >= 1; one codec state per thread). */
int tdt_oracle_encode_batch(const uint8_t *in, const uint64_t *in_off, uint32_t n_msgs,
                            const tdt_oracle_config *cfg, double bandwidth_mbps,
                            double cpu_usage, uint8_t *out, const uint64_t *slot_off,
                            uint64_t *out_len, int32_t *status);
int tdt_oracle_encode_batch_mt(const uint8_t *in, const uint64_t *in_off, uint32_t n_msgs,
                               const tdt_oracle_config *cfg, double bandwidth_mbps,
                               double cpu_usage, uint8_t *out, const uint64_t *slot_off,
                               uint64_t *out_len, int32_t *status, int threads);
int tdt_oracle_decode_batch(const uint8_t *in, const uint64_t *in_off, uint32_t n_msgs,
                            uint8_t *out, const uint64_t *slot_off, uint64_t *out_len,
                            int32_t *status);

#ifdef __cplusplus
}
#endif
#endif
