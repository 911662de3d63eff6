// Host check of the decode recombine forms (tdt_decode.h make_rec_layout / decode_fast): for every
// word-size-4 mapping (16 of them) and random stream words S, the output dwords built by the
// form the layout selects (rkind 1-4: segments 12+4, 4+12, 8+8, one stream; 0: the generic two
// v_perm + or) must hold output byte i = the stream byte the reference's recombine puts there
// (include/psyne/protocol/tdt_compression.hpp recombine_byte_streams :615-637: byte b of word w
// comes from stream mapping[b], at that stream's position w·k + rank of b among the bytes mapped
// to it).  v_perm is emulated for the selector bytes the tables use (0-7: a byte of {hi, lo};
// 0x0c: zero).  Built by tests/test_recombine_layout.py with hipcc (host code only; nothing runs
// on a GPU).
#include "../../psyne_amd/csrc/tdt_decode.h"

#include <cstdio>
#include <random>

static uint32_t hperm(uint32_t hi, uint32_t lo, uint32_t sel) {
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int j = 0; j < 4; ++j) {
        const uint32_t s = (sel >> (8 * j)) & 0xffu;
        uint32_t b;
        if (s < 8) b = (uint32_t)(v >> (8 * s)) & 0xffu;
        else if (s == 0x0c) b = 0;
        else return 0xdeadbeefu;  // a selector byte the tables never hold
        r |= b << (8 * j);
    }
    return r;
}

int main() {
    std::mt19937 rng(7);
    int bad = 0, kinds[5] = {0, 0, 0, 0, 0};
    for (uint32_t mb = 0; mb < 16; ++mb) {
        const psy::RecLayout G = psy::make_rec_layout<4>(mb);
        uint32_t k[2] = {0, 0};
        for (int b = 0; b < 4; ++b) k[(mb >> b) & 1u]++;
        const uint32_t m0 = mb & 1u;  // the stream of first use holds mapping[0]'s value
        if (G.rkind > 4) {
            std::printf("mb %u: rkind %u out of range\n", mb, G.rkind);
            return 1;
        }
        for (int trial = 0; trial < 500; ++trial) {
            uint32_t S[4];
            uint8_t Sb[16];
            for (int d = 0; d < 4; ++d) {
                S[d] = rng();
                for (int j = 0; j < 4; ++j) Sb[4 * d + j] = (S[d] >> (8 * j)) & 0xffu;
            }
            uint8_t want[16];
            for (uint32_t i = 0; i < 16; ++i) {
                const uint32_t b = i % 4, v = (mb >> b) & 1u;
                uint32_t rank = 0;
                for (uint32_t bb = 0; bb < b; ++bb) rank += ((mb >> bb) & 1u) == v ? 1u : 0u;
                want[i] = Sb[(v == m0 ? 0u : G.seg0) + (i / 4) * k[v] + rank];
            }
            const uint32_t *OA = G.OA, *OB = G.OB;
            uint32_t o[4];
            if (G.rkind == 1) {
                o[0] = hperm(S[3], S[0], OA[0]);
                o[1] = hperm(S[3], hperm(S[1], S[0], OB[1]), OA[1]);
                o[2] = hperm(S[3], hperm(S[2], S[1], OB[2]), OA[2]);
                o[3] = hperm(S[3], S[2], OA[3]);
            } else if (G.rkind == 3) {
                o[0] = hperm(S[2], S[0], OA[0]);
                o[1] = hperm(S[2], S[0], OA[1]);
                o[2] = hperm(S[3], S[1], OA[2]);
                o[3] = hperm(S[3], S[1], OA[3]);
            } else if (G.rkind == 2) {
                o[0] = hperm(S[0], S[1], OA[0]);
                o[1] = hperm(S[0], hperm(S[2], S[1], OB[1]), OA[1]);
                o[2] = hperm(S[0], hperm(S[3], S[2], OB[2]), OA[2]);
                o[3] = hperm(S[0], S[3], OA[3]);
            } else if (G.rkind == 4) {
                for (int q = 0; q < 4; ++q) o[q] = S[q];
            } else {
                for (int q = 0; q < 4; ++q) o[q] = hperm(S[1], S[0], OA[q]) | hperm(S[3], S[2], OB[q]);
            }
            for (int i = 0; i < 16; ++i)
                if (((o[i >> 2] >> (8 * (i & 3))) & 0xffu) != want[i]) {
                    ++bad;
                    break;
                }
        }
        kinds[G.rkind]++;
        std::printf("mapping %2u: segments %2u + %2u, form %u\n", mb, G.seg0, G.seg1, G.rkind);
    }
    std::printf("mismatches %d; forms 0-4: %d %d %d %d %d\n", bad, kinds[0], kinds[1], kinds[2], kinds[3], kinds[4]);
    return bad != 0;
}
