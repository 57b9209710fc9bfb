// encode_math.hpp -- the bit-sliced GF(2^8) math of the (10,4,13) / (9,4,12) streaming encode
// (stream_encode.hpp): the RS generator fold of one data node and the PFT pair, as compile-time
// XOR networks over 8 bit-planes (a plane = one uint32 = 32 byte positions, bitslice.hpp).
//
//  * fold: parity p (4 x 8 planes) += g[p][node] * U(node) for one node of a data y-section; the
//    32 output rows over the node's 8 input planes are factored into common subexpressions at
//    compile time (xor_cse.hpp): 652 -> ~470 XORs per 10-node layer pass.
//  * PFT pair (transforms.rs:108-125): C = det^-1 (U + gamma U*) for both members of a pair of
//    the parity section, the 16 rows over 16 planes factored the same way (60 -> ~20 XORs).
//  * Hold: the U values of earlier groups that later PFT pairs need (at most four 8-plane sets).
#pragma once

#include "bitslice.hpp"
#include "xor_cse.hpp"

namespace clay {
namespace bs {

template <int KD>
struct EncMath {
    using S = Shape<KD, 4>;
    static constexpr int Q = S::Q, T = S::T, ALPHA = S::ALPHA;
    static_assert(Q == 4 && T == 4 && ALPHA == 256 && KD <= 12, "q = 4, t = 4 (alpha 256)");

    template <int BO>
    static constexpr uint64_t pft_mask() {
        return plane_mask(S::DINV, BO, 0) | plane_mask(gm(S::DINV, 2), BO, 8);
    }

    // the fold's 32 output rows for node (Y, X), CSE-factored at compile time (xor_cse.hpp)
    template <int Y, int X>
    struct FoldCse {
        static constexpr XorCse make() {
            uint32_t rows[Q * 8] = {};
            for (int p = 0; p < Q; p++)
                for (int bo = 0; bo < 8; bo++) rows[p * 8 + bo] = uint32_t(plane_mask(S::RS.g[p][Y * Q + X], bo, 0));
            return make_xor_cse(rows);
        }
        static constexpr XorCse C = make();
    };
    // bit transpose + RS fold of U[x] into the accumulators, through the CSE temporaries
    template <int Y, int X>
    __device__ static void fold_x_cse(uint32_t (&u)[8], uint32_t (&acc)[Q * 8]) {
        transpose8(u);
        cse_fold<FoldCse<Y, X>, Q * 8, (Y > 0 || X > 0)>(u, acc);
    }
    // bit transpose + RS fold of U[x] into the accumulators.
    template <int Y, int X>
    __device__ static void fold_x(uint32_t (&u)[8], uint32_t (&acc)[Q * 8]) {
        transpose8(u);
        sfor<Q>([&](auto pc_) BS_INL {
            constexpr int p = decltype(pc_)::value;
            sfor<8>([&](auto bc) BS_INL {
                constexpr int bo = decltype(bc)::value;
                constexpr uint64_t mk = plane_mask(S::RS.g[p][Y * Q + X], bo, 0);
                acc[p * 8 + bo] = xor_sel<mk, (Y > 0 || X > 0)>(acc[p * 8 + bo], u);
            });
        });
    }
    // both PFT outputs of a pair at once: c[0..7] = pft(u, us), c[8..15] = pft(us, u), the 16
    // rows over the 16 input planes factored by xor_cse.hpp (60 -> ~20 XOR instructions)
    struct PftCse {
        static constexpr XorCse make() {
            uint32_t rows[16] = {};
            for (int bo = 0; bo < 8; bo++) {
                rows[bo] = uint32_t(pft_mask_of(bo, 0));
                rows[8 + bo] = uint32_t(pft_mask_of(bo, 8));
            }
            return make_xor_cse<16, 16>(rows);
        }
        static constexpr XorCse C = make();
    };
    // mask of output plane bo of pft(first, second) over (u at bits 0-7, us at 8-15); base 8:
    // the swapped pair pft(us, u)
    static constexpr uint64_t pft_mask_of(int bo, int base) {
        return base == 0 ? (plane_mask(S::DINV, bo, 0) | plane_mask(gm(S::DINV, 2), bo, 8))
                         : (plane_mask(S::DINV, bo, 8) | plane_mask(gm(S::DINV, 2), bo, 0));
    }
    __device__ static void pft_pair(const uint32_t *u, const uint32_t *us, uint32_t (&c)[16]) {
        uint32_t in[16];
#pragma unroll
        for (int w = 0; w < 8; w++) {
            in[w] = u[w];
            in[8 + w] = us[w];
        }
        cse_fold<PftCse, 16, false, 16>(in, c);
    }
    // PFT pair: C = det^-1 (u + gamma * ustar)
    __device__ static void pft(const uint32_t *u, const uint32_t *us, uint32_t (&cv)[8]) {
        uint32_t in[16];
#pragma unroll
        for (int w = 0; w < 8; w++) { in[w] = u[w]; in[8 + w] = us[w]; }
        sfor<8>([&](auto bc) BS_INL {
            cv[decltype(bc)::value] = xor_sel<pft_mask<decltype(bc)::value>(), false>(0u, in);
        });
    }

    // U[p][z(h)] values later PFT pairs need, in four rotating 8-plane registers sets
    // (never more than four live): after group 0 R0 = U[1][z0], R1 = U[2][z0],
    // R2 = U[3][z0]; after group 1 R0 = U[2][z1], R3 = U[3][z1]; after group 2 R1 = U[3][z2].
    struct Hold {
        uint32_t r[4][8];
    };

};

}  // namespace bs
}  // namespace clay
