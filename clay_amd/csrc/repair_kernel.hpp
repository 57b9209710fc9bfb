// repair_kernel.hpp -- bit-sliced single-launch repair for codes with q = m (d = k + m - 1),
// e.g. the BASELINE (9,3,11), when every other node is a helper (no aloof nodes).
//
// The reference (repair.rs:299-418), per layer z of the repair plane (digit y0 of z = x0, the
// lost node (y0, x0)):
//   phase 1  U of every node outside section y0: red -> C, else the PRT pair with its
//            companion, which lies in the plane too (transforms.rs:42-89; both are helpers)
//   phase 2  RS reconstruct of section y0's q U values from the K others (decode.rs:332-408:
//            exactly K shards are present, so the result is THE codeword through them)
//   phase 3  C(lost, z) = U(lost, z) (red); for x != x0: C(lost, z[y0:=x]) =
//            (U(y0,x,z) + C(y0,x,z)) * gamma^-1 (compute_cstar_from_c_and_u, decode.rs:566-576)
// Phase 2's map is fixed by y0: U_y0 = R * U_others with R = H_y0^-1 H_others over the parity
// check H = [G | I] of the RS generator, computed at compile time -> XOR networks, as in the
// bit-sliced encode (bitslice.hpp).  x0 only moves addresses.
//
// Lane = (plane layer j, part): 32 positions of one plane layer; a workgroup covers every plane
// layer of W = 32 * PARTS positions, so the PRT companions (other plane layers of the same
// positions) are read by lanes of the same workgroup and come from L1/L2.  Helper rows are
// read with plain (unaligned) global loads: sub-chunks need not be 8-byte aligned.
#pragma once

#include "bitslice.hpp"
#include "kernels.hpp"

namespace clay {
namespace bs {

struct RepArgs {
    const uint8_t *h[16];  // internal node -> its helper buffer (nullptr: shortened, zero)
    uint8_t *out;          // the lost node's chunk
    uint64_t sc;
    uint32_t x0;           // lost node = (Y0, x0)
    uint32_t full;         // 1: helper buffers are whole chunks (layer z at z * sc);
                           // 0: the beta plane layers in ascending order (layer j at j * sc)
    uint32_t ntiles, per_xcd;
};

template <int Q>
struct SmallMat {
    uint8_t a[Q][Q];
};

template <int KD, int M, int Y0>
struct BsRepair {
    using S = Shape<KD, M>;
    static constexpr int Q = S::Q, T = S::T, ALPHA = S::ALPHA, K = S::K, NI = Q * T;
    static_assert(Q == M && Y0 >= 0 && Y0 < T, "repair kernel: q = m codes");
    static constexpr int P = ALPHA / Q;  // plane layers (beta)
    static_assert(P <= 256, "plane fits a workgroup");
    static constexpr int PARTS = 256 / P;
    static constexpr int BLOCK = 256, LANES = P * PARTS, W = 32 * PARTS;

    static constexpr uint8_t H(int p, int i) { return i < K ? S::RS.g[p][i] : uint8_t(i - K == p ? 1 : 0); }
    // H restricted to section Y0's q columns, inverted (Gauss-Jordan at compile time)
    static constexpr SmallMat<Q> hinv() {
        uint8_t a[Q][Q] = {}, inv[Q][Q] = {};
        for (int r = 0; r < Q; r++)
            for (int c = 0; c < Q; c++) {
                a[r][c] = H(r, Y0 * Q + c);
                inv[r][c] = r == c ? 1 : 0;
            }
        for (int c = 0; c < Q; c++) {
            int piv = c;
            while (a[piv][c] == 0) piv++;
            for (int j = 0; j < Q; j++) {
                uint8_t t = a[c][j];
                a[c][j] = a[piv][j];
                a[piv][j] = t;
                t = inv[c][j];
                inv[c][j] = inv[piv][j];
                inv[piv][j] = t;
            }
            const uint8_t s = ginv(a[c][c]);
            for (int j = 0; j < Q; j++) {
                a[c][j] = gm(a[c][j], s);
                inv[c][j] = gm(inv[c][j], s);
            }
            for (int r = 0; r < Q; r++) {
                if (r == c || a[r][c] == 0) continue;
                const uint8_t f = a[r][c];
                for (int j = 0; j < Q; j++) {
                    a[r][j] ^= gm(f, a[c][j]);
                    inv[r][j] ^= gm(f, inv[c][j]);
                }
            }
        }
        SmallMat<Q> m{};
        for (int r = 0; r < Q; r++)
            for (int c = 0; c < Q; c++) m.a[r][c] = inv[r][c];
        return m;
    }
    static constexpr SmallMat<Q> HINV = hinv();
    // coefficient of U(node i) in U(Y0, xp): (H_Y0^-1 H_i)[xp]
    static constexpr uint8_t R(int xp, int i) {
        uint8_t v = 0;
        for (int p = 0; p < Q; p++) v ^= gm(HINV.a[xp][p], H(p, i));
        return v;
    }
    static constexpr bool real(int i) { return i < KD || i >= K; }  // not a shortened node
    static constexpr uint32_t wt(int y) {
        uint32_t w = 1;
        for (int i = 0; i < T - 1 - y; i++) w *= Q;
        return w;
    }
    // digit of section y (!= Y0) in plane layer j; j's digits are the non-Y0 digits, MSB first
    static constexpr uint32_t jw(int y) {
        const int k = y < Y0 ? y : y - 1;
        uint32_t w = 1;
        for (int i = 0; i < T - 2 - k; i++) w *= Q;
        return w;
    }
    __device__ static uint32_t layer_of(uint32_t j, uint32_t x0) {
        uint32_t z = x0 * wt(Y0);
#pragma unroll
        for (int y = 0; y < T; y++)
            if (y != Y0) z += ((j / jw(y)) % uint32_t(Q)) * wt(y);
        return z;
    }

    template <int I>
    __device__ static void fold(uint32_t (&u)[8], uint32_t (&acc)[Q * 8]) {
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int xp = decltype(xc)::value;
            constexpr uint8_t c = R(xp, I);
            if constexpr (c != 0) {
                sfor<8>([&](auto bc) BS_INL {
                    constexpr int bo = decltype(bc)::value;
                    acc[xp * 8 + bo] = xor_sel<plane_mask(c, bo, 0), true>(acc[xp * 8 + bo], u);
                });
            }
        });
    }

    // 32 bytes at any alignment (gfx950 global loads run unaligned): two 16-byte loads
    __device__ static void ld32v(uint32_t (&d)[8], const uint8_t *p) {
        const uint4 v0 = *reinterpret_cast<const uint4 *>(p), v1 = *reinterpret_cast<const uint4 *>(p + 16);
        d[0] = v0.x; d[1] = v0.y; d[2] = v0.z; d[3] = v0.w;
        d[4] = v1.x; d[5] = v1.y; d[6] = v1.z; d[7] = v1.w;
    }

    template <bool FULL>
    __device__ static void st32o(uint8_t *p, const uint32_t (&d)[8], int nv) {
        if constexpr (FULL) {
            *reinterpret_cast<uint4 *>(p) = make_uint4(d[0], d[1], d[2], d[3]);
            *reinterpret_cast<uint4 *>(p + 16) = make_uint4(d[4], d[5], d[6], d[7]);
        } else {
            st32<false, true>(p, d, nv);
        }
    }

    template <bool FULL>
    __device__ static void tile(const RepArgs &a, uint32_t j, uint32_t part, uint64_t b0) {
        const uint64_t sc = a.sc;
        const uint64_t pos = b0 + 32u * part;
        const int nv = FULL ? 32 : int(pos >= sc ? 0 : (sc - pos > 32 ? 32 : sc - pos));
        if (!FULL && nv == 0) return;
        const uint32_t x0 = a.x0;
        auto row = [&](int i, uint32_t jj) BS_INL {  // helper of node i at plane layer jj
            const uint64_t l = a.full ? uint64_t(layer_of(jj, x0)) : uint64_t(jj);
            return a.h[i] + l * sc + pos;
        };
        uint32_t acc[Q * 8];
#pragma unroll
        for (int w = 0; w < Q * 8; w++) acc[w] = 0;
        sfor<T>([&](auto yc) BS_INL {
            constexpr int Y = decltype(yc)::value;
            if constexpr (Y != Y0) {
                const uint32_t zy = (j / jw(Y)) % uint32_t(Q);
                // companion node (Y, zy): its helper pointer (per lane), shortened -> none
                const uint8_t *cp = nullptr;
                bool creal = false;
                sfor<Q>([&](auto xc) BS_INL {
                    constexpr int X = decltype(xc)::value;
                    if (zy == uint32_t(X)) {
                        creal = real(Y * Q + X);
                        cp = a.h[Y * Q + X];
                    }
                });
                sfor<Q>([&](auto xc) BS_INL {
                    constexpr int X = decltype(xc)::value;
                    constexpr int I = Y * Q + X;
                    uint32_t o[8], cv[8];
                    const bool keep = creal && zy != uint32_t(X);
                    const uint8_t *op = real(I) ? row(I, j) : nullptr;
                    const uint32_t jc = j + (uint32_t(X) - zy) * jw(Y);
                    const uint64_t l = a.full ? uint64_t(layer_of(jc, x0)) : uint64_t(jc);
                    if constexpr (FULL) {
                        // a masked companion is read from a valid row (its own) and discarded:
                        // no branch around the load, so loads of consecutive nodes overlap
                        const uint8_t *cq = keep ? cp + l * sc + pos : (real(I) ? op : a.out + pos);
                        if constexpr (real(I)) ld32v(o, op);
                        ld32v(cv, cq);
                    } else {
                        if constexpr (real(I)) ld32<false, true>(o, op, nv);
                        if (keep) {
                            ld32<false, true>(cv, cp + l * sc + pos, nv);
                        } else {
#pragma unroll
                            for (int w = 0; w < 8; w++) cv[w] = 0;
                        }
                    }
                    if constexpr (!real(I)) {
#pragma unroll
                        for (int w = 0; w < 8; w++) o[w] = 0;
                    }
                    const uint32_t km = keep ? 0xffffffffu : 0u;
                    uint32_t u[8];
#pragma unroll
                    for (int w = 0; w < 8; w++) u[w] = xor_xtime4(o[w], cv[w] & km);
                    transpose8(u);
                    fold<I>(u, acc);
                });
            }
        });
        // outputs: C(lost, z_j) = U(Y0, x0); C(lost, z_j[Y0 := x]) = gamma^-1 (U(Y0, x) + C(Y0, x))
        const uint32_t zj = layer_of(j, x0);
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int X = decltype(xc)::value;
            constexpr int I = Y0 * Q + X;
            uint32_t v[8];
#pragma unroll
            for (int w = 0; w < 8; w++) v[w] = acc[X * 8 + w];
            transpose8(v);
            if (uint32_t(X) == x0) {
                st32o<FULL>(a.out + uint64_t(zj) * sc + pos, v, nv);
            } else {
                if constexpr (real(I)) {
                    uint32_t c[8];
                    if constexpr (FULL) ld32v(c, row(I, j));
                    else ld32<false, true>(c, row(I, j), nv);
#pragma unroll
                    for (int w = 0; w < 8; w++) v[w] ^= c[w];
                }
                constexpr GfTab tg = gamma_inv_tab();
#pragma unroll
                for (int w = 0; w < 8; w++) v[w] = gf_mul(v[w], tg);
                const uint32_t zo = zj + (uint32_t(X) - x0) * wt(Y0);
                st32o<FULL>(a.out + uint64_t(zo) * sc + pos, v, nv);
            }
        });
    }

    static constexpr GfTab gamma_inv_tab() {
        const uint8_t c = ginv(2);
        uint8_t b[20] = {};
        for (int i = 0; i < 8; i++) b[i] = gm(c, uint8_t(i));
        for (int i = 0; i < 8; i++) b[8 + i] = gm(c, uint8_t(i << 3));
        for (int i = 0; i < 4; i++) b[16 + i] = gm(c, uint8_t(i << 6));
        auto w = [&](int k) {
            return uint32_t(b[4 * k]) | uint32_t(b[4 * k + 1]) << 8 | uint32_t(b[4 * k + 2]) << 16 |
                   uint32_t(b[4 * k + 3]) << 24;
        };
        return GfTab{w(0), w(1), w(2), w(3), w(4)};
    }
};

// grid = 8 * per_xcd blocks: XCD x streams tiles [x * per_xcd, (x + 1) * per_xcd)
template <int KD, int M, int Y0>
__global__ __launch_bounds__(256) void k_bs_repair(RepArgs a) {
    using Kn = BsRepair<KD, M, Y0>;
    if (threadIdx.x >= uint32_t(Kn::LANES)) return;
    const uint32_t tix = (blockIdx.x & 7u) * a.per_xcd + (blockIdx.x >> 3);
    if (tix >= a.ntiles) return;
    const uint32_t j = threadIdx.x / uint32_t(Kn::PARTS), part = threadIdx.x % uint32_t(Kn::PARTS);
    const uint64_t b0 = uint64_t(tix) * Kn::W;
    if (b0 + Kn::W <= a.sc) Kn::template tile<true>(a, j, part, b0);
    else Kn::template tile<false>(a, j, part, b0);
}

}  // namespace bs
}  // namespace clay
