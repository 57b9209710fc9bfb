// xor_cse.hpp -- compile-time common-subexpression elimination for the bit-sliced RS folds.
//
// A fold adds one node's 8 bit-planes into the 32 accumulator planes of the q RS rows: output
// plane (p, bo) ^= XOR of the input planes selected by the 8 x 8 bit matrix of the generator
// coefficient g[p][node] (bitslice.hpp plane_mask).  Done row by row that is one 3-input XOR per
// two selected planes.  Rows of the same node share many pairs and triples of input planes, so a
// greedy (Paar-style) search at compile time factors the most profitable ones out into
// temporaries first (cost model: a row of w operands costs ceil(w / 2) 3-input XORs; a
// temporary costs one).  (10,4) generator: 652 -> ~470 XOR instructions per 10-node layer pass.
#pragma once

#include <stdint.h>

namespace clay {
namespace bs {

constexpr int kCseMaxT = 14;

struct XorCse {
    int nt;
    uint8_t t[kCseMaxT][3];  // operands of temporary k (0..7 inputs, 8 + j temporary j); [2] = 255: two-input
    uint32_t row[32];        // per output row: operand mask over 0 .. 8 + nt - 1
};

constexpr int cse_popc(uint32_t v) {
    int n = 0;
    for (; v; v &= v - 1) n++;
    return n;
}
constexpr int cse_cost(int w) { return w <= 0 ? 0 : (w + 1) / 2; }

// NIN input operands (8 bit-planes of one node, or 16 for a PFT pair)
template <int NR, int NIN = 8>
constexpr XorCse make_xor_cse(const uint32_t (&in)[NR]) {
    static_assert(NIN + kCseMaxT <= 32 && NR <= 32, "operand masks are 32 bits");
    XorCse c{};
    for (int r = 0; r < NR; r++) c.row[r] = in[r];
    int nops = NIN;
    while (c.nt < kCseMaxT) {
        int best = 0, bi = -1, bj = -1, bk = -1;
        for (int i = 0; i < nops; i++)
            for (int j = i + 1; j < nops; j++) {
                const uint32_t m2 = (1u << i) | (1u << j);
                int sav = -1, n2 = 0;
                for (int r = 0; r < NR; r++)
                    if ((c.row[r] & m2) == m2) {
                        const int w = cse_popc(c.row[r]);
                        sav += cse_cost(w) - cse_cost(w - 1);
                        n2++;
                    }
                if (sav > best) {
                    best = sav;
                    bi = i, bj = j, bk = -1;
                }
                if (n2 < 2) continue;  // a triple containing (i, j) is in at most as many rows
                for (int k = j + 1; k < nops; k++) {
                    const uint32_t m3 = m2 | (1u << k);
                    int s3 = -1;
                    for (int r = 0; r < NR; r++)
                        if ((c.row[r] & m3) == m3) {
                            const int w = cse_popc(c.row[r]);
                            s3 += cse_cost(w) - cse_cost(w - 2);
                        }
                    if (s3 > best) {
                        best = s3;
                        bi = i, bj = j, bk = k;
                    }
                }
            }
        if (best <= 0) break;
        const uint32_t m = (1u << bi) | (1u << bj) | (bk >= 0 ? (1u << bk) : 0u);
        c.t[c.nt][0] = uint8_t(bi);
        c.t[c.nt][1] = uint8_t(bj);
        c.t[c.nt][2] = uint8_t(bk >= 0 ? bk : 255);
        for (int r = 0; r < NR; r++)
            if ((c.row[r] & m) == m) c.row[r] = (c.row[r] & ~m) | (1u << nops);
        nops++;
        c.nt++;
    }
    return c;
}

// acc[o] (^)= the CSE program F::C applied to the 8 input planes u, outputs o < NOUT
// (ACC = false: the first fold into uninitialised accumulators).  Needs bitslice.hpp (sfor,
// xor3, xor_sel) included first.
template <class F, int NOUT, bool ACC, int NIN = 8>
__device__ __forceinline__ void cse_fold(const uint32_t (&u)[NIN], uint32_t *acc) {
    uint32_t ext[NIN + kCseMaxT];
#pragma unroll
    for (int w = 0; w < NIN; w++) ext[w] = u[w];
    sfor<kCseMaxT>([&](auto kc) __attribute__((always_inline)) {
        constexpr int k = decltype(kc)::value;
        if constexpr (k < F::C.nt) {
            constexpr int o0 = F::C.t[k][0], o1 = F::C.t[k][1], o2 = F::C.t[k][2];
            if constexpr (o2 == 255) ext[NIN + k] = ext[o0] ^ ext[o1];
            else ext[NIN + k] = xor3(ext[o0], ext[o1], ext[o2]);
        }
    });
    sfor<NOUT>([&](auto oc) __attribute__((always_inline)) {
        constexpr int o = decltype(oc)::value;
        constexpr uint64_t mk = F::C.row[o];
        acc[o] = xor_sel<mk, ACC>(acc[o], ext);
    });
}

}  // namespace bs
}  // namespace clay
