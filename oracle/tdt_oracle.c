/* oracle/tdt_oracle.c — plain-C restatement of the reference TDT codec.
 *
 * TEST INFRASTRUCTURE ONLY (see tdt_oracle.h).  Every function cites the reference lines
 * in include/psyne/protocol/tdt_compression.hpp that it restates.
 *
 * Build: gcc -O2 -ffp-contract=off (oracle/Makefile).  The entropy update is written as an
 * explicit fma() because the reference build contracts it (vfnmadd213sd, DESIGN.md
 * §"Entropy bits"); log2 is the system glibc log2, i.e. the same function the reference
 * calls.
 */
#include "tdt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define MAGIC_TDT 0x54445444u  /* :85 */
#define MAGIC_UNCP 0x554E4350u /* :233 */

static uint32_t rd32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
static void wr32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }

void tdt_oracle_default_config(tdt_oracle_config *cfg) {
    /* TDTConfig defaults :31-43 */
    cfg->sample_fraction = 0.3f;
    cfg->word_size = 4;
    cfg->bandwidth_threshold_mbps = 100.0;
    cfg->cpu_usage_threshold = 0.8;
    cfg->min_tensor_size = 1024;
}

/* should_transform :186-201; is_tensor_data :409-413 ignores word_size. */
int tdt_oracle_should_transform(uint64_t n, const tdt_oracle_config *cfg,
                                double bandwidth_mbps, double cpu_usage) {
    if (n < cfg->min_tensor_size) return 0;
    if (cpu_usage > cfg->cpu_usage_threshold) return 0;
    if (!((n % 4 == 0) && (n >= 64))) return 0;
    return bandwidth_mbps < cfg->bandwidth_threshold_mbps;
}

uint64_t tdt_oracle_encode_bound(uint64_t n, int32_t ws) {
    uint64_t uncp = n + 4;
    uint64_t w = ws > 0 ? (uint64_t)ws : 4;
    uint64_t tdt = 20 + 4 * w + 8 + 2 * n;
    return tdt > uncp ? tdt : uncp;
}

/* generate_sample_indices :419-432 — the sample count, with the float product of :421. */
static uint64_t sample_count(uint64_t wc, float sf) {
    uint64_t c = (uint64_t)((float)wc * sf);
    if (c < 100) c = 100;
    if (c > wc) c = wc;
    return c;
}

/* extract_features :434-468 (histogram over all words), calculate_entropy :470-480,
 * perform_clustering :507-525. */
int tdt_oracle_analyze(const uint8_t *data, uint64_t n, int32_t ws, uint32_t *hist,
                       double *entropy, int32_t *mapping) {
    if (ws <= 0 || n == 0 || n % (uint64_t)ws) return TDT_ORACLE_E_CONFIG;
    uint64_t wc = n / (uint64_t)ws;
    memset(hist, 0, sizeof(uint32_t) * 256 * (size_t)ws);
    for (uint64_t w = 0; w < wc; ++w)
        for (int32_t b = 0; b < ws; ++b) hist[b * 256 + data[w * ws + b]]++;
    const double total = (double)wc;
    double sum = 0.0;
    for (int32_t b = 0; b < ws; ++b) {
        double e = 0.0;
        for (int v = 0; v < 256; ++v) {
            uint32_t c = hist[b * 256 + v];
            if (c > 0) {
                double prob = (double)c / total;
                e = fma(-prob, log2(prob), e); /* entropy -= prob*log2(prob), contracted */
            }
        }
        entropy[b] = e;
        sum += e; /* std::accumulate(..., 0.0) :516-518 */
    }
    double threshold = sum / (double)ws;
    for (int32_t b = 0; b < ws; ++b) mapping[b] = entropy[b] > threshold ? 1 : 0;
    return TDT_ORACLE_OK;
}

/* encode :227-266 → compress_tdt :363-399 → serialize :81-117. */
int tdt_oracle_encode(const uint8_t *data, uint64_t n, const tdt_oracle_config *cfg,
                      double bandwidth_mbps, double cpu_usage, const int32_t *mapping_in,
                      uint8_t *out, uint64_t cap, uint64_t *out_len) {
    const int32_t ws = cfg->word_size;
    if (ws <= 0) return TDT_ORACLE_E_CONFIG;
    int compress = tdt_oracle_should_transform(n, cfg, bandwidth_mbps, cpu_usage);
    /* compress_tdt throws on n == 0 || n % ws (:364-367) → UNCP fallback (:256-265). */
    if (compress && (n == 0 || n % (uint64_t)ws)) compress = 0;
    if (!compress) {
        *out_len = n + 4;
        if (n + 4 > cap) return TDT_ORACLE_E_CAPACITY;
        wr32(out, MAGIC_UNCP);
        memcpy(out + 4, data, n);
        return TDT_ORACLE_OK;
    }
    const uint64_t wc = n / (uint64_t)ws;
    int32_t mapping[64];
    if (ws > 64) return TDT_ORACLE_E_CONFIG;
    if (mapping_in) {
        for (int32_t b = 0; b < ws; ++b) {
            if (mapping_in[b] < 0 || mapping_in[b] >= 2 * ws) return TDT_ORACLE_E_BAD_MAPPING;
            mapping[b] = mapping_in[b];
        }
    } else {
        if (sample_count(wc, cfg->sample_fraction) != wc) return TDT_ORACLE_E_NONDETERMINISTIC;
        uint32_t *hist = (uint32_t *)malloc(sizeof(uint32_t) * 256 * (size_t)ws);
        double ent[64];
        tdt_oracle_analyze(data, n, ws, hist, ent, mapping);
        free(hist);
    }
    /* separate_byte_streams :527-549: streams = max(mapping) + 1. */
    int32_t ns = 0;
    for (int32_t b = 0; b < ws; ++b)
        if (mapping[b] + 1 > ns) ns = mapping[b] + 1;
    uint64_t hdr = 20 + 4 * (uint64_t)ws;
    /* First pass: RLE lengths per stream (simple_rle_compress :557-582). */
    uint64_t pos = hdr;
    for (int32_t c = 0; c < ns; ++c) {
        uint64_t pairs = 0;
        int have = 0;
        uint8_t cur = 0, cnt = 0;
        for (uint64_t w = 0; w < wc; ++w)
            for (int32_t b = 0; b < ws; ++b) {
                if (mapping[b] != c) continue;
                uint8_t x = data[w * ws + b];
                if (!have) {
                    cur = x;
                    cnt = 1;
                    have = 1;
                } else if (x == cur && cnt < 255) {
                    cnt++;
                } else {
                    pairs++;
                    cur = x;
                    cnt = 1;
                }
            }
        if (have) pairs++;
        pos += 4 + 2 * pairs;
    }
    *out_len = pos;
    if (pos > cap) return TDT_ORACLE_E_CAPACITY;
    wr32(out + 0, MAGIC_TDT);
    wr32(out + 4, (uint32_t)n); /* static_cast<uint32_t>(original_size) :88 */
    wr32(out + 8, (uint32_t)ns);
    wr32(out + 12, (uint32_t)ws);
    wr32(out + 16, (uint32_t)ws);
    for (int32_t b = 0; b < ws; ++b) wr32(out + 20 + 4 * b, (uint32_t)mapping[b]);
    uint64_t o = hdr;
    for (int32_t c = 0; c < ns; ++c) {
        uint64_t len_at = o;
        o += 4;
        uint64_t start = o;
        int have = 0;
        uint8_t cur = 0, cnt = 0;
        for (uint64_t w = 0; w < wc; ++w)
            for (int32_t b = 0; b < ws; ++b) {
                if (mapping[b] != c) continue;
                uint8_t x = data[w * ws + b];
                if (!have) {
                    cur = x;
                    cnt = 1;
                    have = 1;
                } else if (x == cur && cnt < 255) {
                    cnt++;
                } else {
                    out[o++] = cnt;
                    out[o++] = cur;
                    cur = x;
                    cnt = 1;
                }
            }
        if (have) {
            out[o++] = cnt;
            out[o++] = cur;
        }
        wr32(out + len_at, (uint32_t)(o - start));
    }
    return TDT_ORACLE_OK;
}

/* Header checks of deserialize :119-170, plus the bounds checks the reference lacks. */
static int parse_and_size(const uint8_t *blob, uint64_t len, uint64_t *out_len,
                          int *is_uncp) {
    *is_uncp = 0;
    if (len < 4) return TDT_ORACLE_E_SHORT; /* :274-276 */
    uint32_t magic = rd32(blob);
    if (magic == MAGIC_UNCP) { /* :280-283 */
        *is_uncp = 1;
        *out_len = len - 4;
        return TDT_ORACLE_OK;
    }
    if (len < 8) return magic == MAGIC_TDT ? TDT_ORACLE_E_TRUNCATED : TDT_ORACLE_E_MAGIC;
    if (magic != MAGIC_TDT) return TDT_ORACLE_E_MAGIC; /* :127-129 */
    if (len < 20) return TDT_ORACLE_E_TRUNCATED;
    uint32_t orig = rd32(blob + 4), ns = rd32(blob + 8), wsu = rd32(blob + 12),
             msize = rd32(blob + 16);
    int32_t ws = (int32_t)wsu;
    uint64_t off = 20 + 4 * (uint64_t)msize;
    if (off > len) return TDT_ORACLE_E_TRUNCATED;
    for (uint32_t s = 0; s < ns; ++s) {
        if (off + 4 > len) return TDT_ORACLE_E_TRUNCATED;
        uint32_t sl = rd32(blob + off);
        off += 4;
        if (off + sl > len) return TDT_ORACLE_E_TRUNCATED;
        off += sl;
    }
    if (ws == 0) return TDT_ORACLE_E_BAD_HEADER; /* original_size / 0 :618 */
    /* word_count = original_size / word_size with word_size converted to size_t (:618): a
     * negative int word_size becomes huge, so word_count = 0 and the mapping is unused. */
    uint64_t wc = ws > 0 ? orig / (uint64_t)ws : 0;
    if (wc > 0) {
        if (msize < (uint32_t)ws) return TDT_ORACLE_E_BAD_MAPPING;
        for (int32_t b = 0; b < ws; ++b) {
            int32_t m = (int32_t)rd32(blob + 20 + 4 * (uint64_t)b);
            if (m < 0 || (uint32_t)m >= ns) return TDT_ORACLE_E_BAD_MAPPING;
        }
    }
    *out_len = orig;
    return TDT_ORACLE_OK;
}

int tdt_oracle_decoded_size(const uint8_t *blob, uint64_t len, uint64_t *out_len) {
    int u;
    *out_len = 0;
    int st = parse_and_size(blob, len, out_len, &u);
    if (st) *out_len = 0;
    return st;
}

/* decode :271-304. */
int tdt_oracle_decode(const uint8_t *blob, uint64_t len, uint8_t *out, uint64_t cap,
                      uint64_t *out_len) {
    int is_uncp;
    uint64_t olen = 0;
    *out_len = 0;
    int st = parse_and_size(blob, len, &olen, &is_uncp);
    if (st) return st;
    *out_len = olen;
    if (olen > cap) return TDT_ORACLE_E_CAPACITY;
    if (is_uncp) {
        memcpy(out, blob + 4, olen);
        return TDT_ORACLE_OK;
    }
    const uint32_t orig = rd32(blob + 4), ns = rd32(blob + 8), msize = rd32(blob + 16);
    const int32_t ws = (int32_t)rd32(blob + 12);
    memset(out, 0, olen); /* std::vector<uint8_t> result(original_size) :617 */
    const uint64_t wc = ws > 0 ? orig / (uint64_t)ws : 0;
    if (wc == 0) return TDT_ORACLE_OK;
    /* Locate streams. */
    uint64_t *soff = (uint64_t *)malloc(sizeof(uint64_t) * (ns ? ns : 1));
    uint64_t *slen = (uint64_t *)malloc(sizeof(uint64_t) * (ns ? ns : 1));
    uint64_t off = 20 + 4 * (uint64_t)msize;
    for (uint32_t s = 0; s < ns; ++s) {
        slen[s] = rd32(blob + off);
        soff[s] = off + 4;
        off += 4 + slen[s];
    }
    /* decompress_streams :584-612 lazily: per stream a cursor over (count, value) pairs;
     * recombine :614-637 consumes decompressed bytes in word-major order. */
    uint64_t *pair_i = (uint64_t *)calloc(ns, sizeof(uint64_t)); /* byte index of pair */
    uint32_t *left = (uint32_t *)calloc(ns, sizeof(uint32_t));   /* bytes left in pair */
    uint8_t *val = (uint8_t *)calloc(ns, 1);
    for (uint64_t w = 0; w < wc; ++w) {
        for (int32_t b = 0; b < ws; ++b) {
            int32_t c = (int32_t)rd32(blob + 20 + 4 * (uint64_t)b);
            /* advance to a pair with bytes left: pairs need i + 1 < len (:600-601),
             * count 0 emits nothing. */
            while (left[c] == 0 && pair_i[c] + 1 < slen[c]) {
                left[c] = blob[soff[c] + pair_i[c]];
                val[c] = blob[soff[c] + pair_i[c] + 1];
                pair_i[c] += 2;
            }
            if (left[c] > 0) { /* stream_positions[c] < streams[c].size() :628 */
                out[w * ws + b] = val[c];
                left[c]--;
            }
        }
    }
    free(soff);
    free(slen);
    free(pair_i);
    free(left);
    free(val);
    return TDT_ORACLE_OK;
}

int tdt_oracle_encode_batch(const uint8_t *in, const uint64_t *in_off, uint32_t n_msgs,
                            const tdt_oracle_config *cfg, double bandwidth_mbps,
                            double cpu_usage, uint8_t *out, const uint64_t *slot_off,
                            uint64_t *out_len, int32_t *status) {
    int any = 0;
    for (uint32_t i = 0; i < n_msgs; ++i) {
        uint64_t n = in_off[i + 1] - in_off[i];
        status[i] = tdt_oracle_encode(in + in_off[i], n, cfg, bandwidth_mbps, cpu_usage, NULL,
                                      out + slot_off[i], slot_off[i + 1] - slot_off[i],
                                      &out_len[i]);
        any |= status[i];
    }
    return any ? 1 : 0;
}

int tdt_oracle_decode_batch(const uint8_t *in, const uint64_t *in_off, uint32_t n_msgs,
                            uint8_t *out, const uint64_t *slot_off, uint64_t *out_len,
                            int32_t *status) {
    int any = 0;
    for (uint32_t i = 0; i < n_msgs; ++i) {
        status[i] = tdt_oracle_decode(in + in_off[i], in_off[i + 1] - in_off[i],
                                      out + slot_off[i], slot_off[i + 1] - slot_off[i],
                                      &out_len[i]);
        any |= status[i];
    }
    return any ? 1 : 0;
}

/* Threaded batch encode into caller slots (tests of 10^5..10^6 messages): `threads` workers,
 * message i on worker i % threads.  Same per-message semantics as tdt_oracle_encode_batch. */
typedef struct {
    const uint8_t *in;
    const uint64_t *in_off;
    uint32_t n_msgs, t, threads;
    const tdt_oracle_config *cfg;
    double bw, cpu;
    uint8_t *out;
    const uint64_t *slot_off;
    uint64_t *out_len;
    int32_t *status;
} enc_job;

static void *enc_worker(void *arg) {
    enc_job *j = (enc_job *)arg;
    for (uint32_t i = j->t; i < j->n_msgs; i += j->threads)
        j->status[i] = tdt_oracle_encode(j->in + j->in_off[i], j->in_off[i + 1] - j->in_off[i], j->cfg, j->bw,
                                         j->cpu, NULL, j->out + j->slot_off[i],
                                         j->slot_off[i + 1] - j->slot_off[i], &j->out_len[i]);
    return NULL;
}

int tdt_oracle_encode_batch_mt(const uint8_t *in, const uint64_t *in_off, uint32_t n_msgs,
                               const tdt_oracle_config *cfg, double bandwidth_mbps, double cpu_usage,
                               uint8_t *out, const uint64_t *slot_off, uint64_t *out_len, int32_t *status,
                               int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    enc_job jobs[256];
    for (int t = 0; t < threads; ++t) {
        enc_job j = {in, in_off, n_msgs, (uint32_t)t, (uint32_t)threads, cfg, bandwidth_mbps, cpu_usage,
                     out, slot_off, out_len, status};
        jobs[t] = j;
        pthread_create(&tid[t], NULL, enc_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    for (uint32_t i = 0; i < n_msgs; ++i)
        if (status[i]) return 1;
    return 0;
}
