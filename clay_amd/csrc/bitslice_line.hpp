// bitslice_line.hpp -- line-local bit-sliced kernels for small q = m codes without shortened nodes
// (BASELINE config 2: (4,2,5), alpha = 8): a lane owns 32 positions of one "line" of q layers and
// everything a line needs stays in its registers -- no LDS, no barriers.
//
// k_bs_decode1: single-erasure decode, one launch: the whole decode_layered of
// one erasure (decode.rs:167-257) is a fixed GF(2^8)-linear map per byte position, so the erased
// node E is a template parameter and every coefficient is a compile-time XOR network.
//
// Algebra (the syndrome form of stream_decode.hpp, specialised to one erasure e = (ye, xe)).  The
// reference reconstructs each layer from the first K present shards ("used"; reed-solomon-erasure
// 6.0.0 reconstruct, decode.rs:374); with Kset = the M nodes outside them (e + the ignored ones) and
// H = [G | I], U_e(z) = row e of H_Kset^-1 * sum_{i used} H_i U_i(z), so per layer z
//   C_e(z) = sum_{i used} c_i U'_i(z) + Out(e, z) + sum_{s = (ye, x) used, x != xe} gamma c_s C_e(z[ye := x])
// with c_i = (H_Kset^-1)[e] H_i (compile time), U'_i(z) = C_i(z) + gamma C_i*(z*) the PRT value
// (transforms.rs:42-55; the companion term dropped where the companion is e), Out(e, z) = gamma
// C((ye, z_ye), z[ye := xe]) on the layers where e is not red (compute_c_from_u_and_cstar,
// decode.rs:566-576; 0 where red) and the last sum only on the red layers (z_ye = xe: the terms
// dropped from the siblings' U', solved one iscore level earlier -- decode.rs:196-254).
//
// Lane map: a lane owns 32 consecutive positions of one "line" (the q layers that differ only in
// digit ye) and produces those q layers of e: the non-red ones first, the red one last from their
// bit-planes.  PRT in the byte domain (SWAR xtime), one 8x32 transpose per term, compile-time XOR
// folds (bitslice.hpp xor_sel), one transpose back per output layer.  Rows are read with plain
// 8-byte loads (companion rows hit the lines other lanes of the workgroup read: the workgroup
// covers every line of its positions).
#pragma once

#include "bitslice.hpp"
#include "line_args.hpp"

namespace clay {
namespace bs {

template <int KD, int M, int E>
struct Dec1Plan {
    using S = Shape<KD, M>;
    static constexpr int Q = S::Q, T = S::T, N = Q * T, K = S::K;
    static_assert(S::NU == 0 && N <= 8, "small codes without shortened nodes");
    static_assert(E >= 0 && E < N, "erased node");
    static constexpr uint8_t H(int p, int i) { return i < K ? S::RS.g[p][i] : uint8_t(i - K == p ? 1 : 0); }
    struct Coef {
        uint8_t c[N];
        bool used[N];
    };
    static constexpr Coef make() {
        Coef r{};
        int kset[M] = {}, nk = 0, nu = 0;
        for (int i = 0; i < N; i++) {
            if (i != E && nu < K) {  // the first K present nodes (decode.rs:374)
                r.used[i] = true;
                nu++;
            } else {
                kset[nk++] = i;
            }
        }
        // inv = H_Kset^-1 (Gauss-Jordan over GF(2^8))
        uint8_t a[M][M] = {}, inv[M][M] = {};
        for (int p = 0; p < M; p++)
            for (int j = 0; j < M; j++) {
                a[p][j] = H(p, kset[j]);
                inv[p][j] = p == j ? 1 : 0;
            }
        for (int c = 0; c < M; c++) {
            int piv = c;
            while (a[piv][c] == 0) piv++;
            for (int j = 0; j < M; j++) {
                uint8_t t = a[c][j];
                a[c][j] = a[piv][j];
                a[piv][j] = t;
                t = inv[c][j];
                inv[c][j] = inv[piv][j];
                inv[piv][j] = t;
            }
            const uint8_t s = ginv(a[c][c]);
            for (int j = 0; j < M; j++) {
                a[c][j] = gm(a[c][j], s);
                inv[c][j] = gm(inv[c][j], s);
            }
            for (int rr = 0; rr < M; rr++) {
                if (rr == c || a[rr][c] == 0) continue;
                const uint8_t f = a[rr][c];
                for (int j = 0; j < M; j++) {
                    a[rr][j] ^= gm(f, a[c][j]);
                    inv[rr][j] ^= gm(f, inv[c][j]);
                }
            }
        }
        int row = 0;
        for (int j = 0; j < M; j++)
            if (kset[j] == E) row = j;
        for (int i = 0; i < N; i++) {
            uint8_t v = 0;
            if (r.used[i])
                for (int p = 0; p < M; p++) v ^= gm(inv[row][p], H(p, i));
            r.c[i] = v;
        }
        return r;
    }
    static constexpr Coef C = make();
};

template <int KD, int M, int E, int PG>
struct Dec1Kernel {
    using P = Dec1Plan<KD, M, E>;
    static constexpr int Q = P::Q, T = P::T, N = P::N, ALPHA = P::S::ALPHA;
    static constexpr int YE = E / Q, XE = E % Q;
    static constexpr int LINES = ALPHA / Q, UNITS = LINES * PG, BLOCK = UNITS < 1024 ? UNITS : 1024;
    static constexpr int W = 32 * PG;  // positions per tile
    static constexpr int wt(int y) {
        int w = 1;
        for (int i = 0; i < T - 1 - y; i++) w *= Q;
        return w;
    }

    // acc (8 planes) ^= c * v (8 planes), c a compile-time constant
    template <uint8_t CF>
    __device__ __forceinline__ static void fold(uint32_t (&acc)[8], const uint32_t (&v)[8]) {
        if constexpr (CF != 0) {
            sfor<8>([&](auto bc) BS_INL {
                constexpr int bo = decltype(bc)::value;
                acc[bo] = xor_sel<plane_mask(CF, bo, 0), true>(acc[bo], v);
            });
        }
    }

    template <bool FULL, bool BT>
    __device__ static void tile(const Dec1Args &a, uint64_t b0) {
        for (int u = threadIdx.x; u < UNITS; u += BLOCK) {
            const int pg = u % PG, line = u / PG;
            const int hi = line / wt(YE), lo = line % wt(YE);
            const uint32_t z0 = uint32_t(hi * wt(YE) * Q + lo);  // the line's layer with digit ye = 0
            const uint64_t pos = b0 + uint64_t(32 * pg);
            const int nv = FULL ? (BT ? 32 : 4)
                         : BT ? int(pos >= a.sc ? 0 : a.sc - pos > 32 ? 32 : a.sc - pos)                // bytes
                              : int(pos >= a.sc ? 0 : (a.sc - pos) / 8 > 4 ? 4 : (a.sc - pos) / 8);  // pieces
            auto row = [&](int i, uint32_t z) BS_INL { return a.node[i] + uint64_t(z) * a.sc + pos; };
            uint32_t pl[Q][8];  // C_e planes of the line's layers (digit ye = x)
            sfor<Q>([&](auto kc) BS_INL {
                constexpr int x = (XE + 1 + decltype(kc)::value) % Q;  // the red layer (x = xe) last
                const uint32_t z = z0 + uint32_t(x * wt(YE));
                uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                sfor<N>([&](auto ic) BS_INL {
                    constexpr int i = decltype(ic)::value;
                    constexpr int yi = i / Q, xi = i % Q;
                    if constexpr (P::C.used[i]) {
                        uint32_t o[8], cv[8], t[8];
                        ld32<FULL, BT>(o, row(i, z), nv);
                        if constexpr (yi == YE) {
                            // companion (ye, x) at z[ye := xi]: none where red for i (x == xi), dropped
                            // where it is e (x == xe)
                            if constexpr (x != xi && x != XE) {
                                ld32<FULL, BT>(cv, row(YE * Q + x, z + uint32_t((xi - x) * wt(YE))), nv);
#pragma unroll
                                for (int w = 0; w < 8; w++) t[w] = xor_xtime4(o[w], cv[w]);
                            } else {
#pragma unroll
                                for (int w = 0; w < 8; w++) t[w] = o[w];
                            }
                        } else {
                            // companion (yi, d) at z[yi := xi], d = z's digit yi (run time: the line)
                            const int d = int(z / uint32_t(wt(yi))) % Q;
                            const uint8_t *cn = a.node[yi * Q];
#pragma unroll
                            for (int xx = 1; xx < Q; xx++) cn = d == xx ? a.node[yi * Q + xx] : cn;
                            const uint32_t zc = uint32_t(int(z) + (xi - d) * wt(yi));
                            ld32<FULL, BT>(cv, cn + uint64_t(zc) * a.sc + pos, nv);
                            const uint32_t keep = d != xi ? 0xffffffffu : 0u;
                            const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
#pragma unroll
                            for (int w = 0; w < 8; w++) t[w] = xor_xtime4_masked(o[w], cv[w], ks, kr);
                        }
                        transpose8(t);
                        fold<P::C.c[i]>(acc, t);
                    }
                });
                if constexpr (x != XE) {
                    // Out(e, z) = gamma C((ye, x), z[ye := xe])
                    uint32_t cv[8], t[8];
                    ld32<FULL, BT>(cv, row(YE * Q + x, z0 + uint32_t(XE * wt(YE))), nv);
#pragma unroll
                    for (int w = 0; w < 8; w++) t[w] = xor_xtime4(0u, cv[w]);
                    transpose8(t);
#pragma unroll
                    for (int w = 0; w < 8; w++) acc[w] ^= t[w];
                } else {
                    // red: the siblings' dropped terms gamma c_s C_e(z[ye := x'])
                    sfor<Q>([&](auto sc_) BS_INL {
                        constexpr int xs = decltype(sc_)::value;
                        if constexpr (xs != XE) fold<gm(2, P::C.c[YE * Q + xs])>(acc, pl[xs]);
                    });
                }
                uint32_t ob[8];
#pragma unroll
                for (int w = 0; w < 8; w++) {
                    pl[x][w] = acc[w];
                    ob[w] = acc[w];
                }
                transpose8(ob);
                st32<FULL, BT>(a.out + uint64_t(z) * a.sc + pos, ob, nv);
            });
        }
    }
};

template <int KD, int M, int E, int PG, bool BT = false>
__global__ __launch_bounds__((Dec1Kernel<KD, M, E, PG>::BLOCK)) void k_bs_decode1(Dec1Args a) {
    using Kn = Dec1Kernel<KD, M, E, PG>;
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    for (uint32_t tix = slot; tix < a.tiles_per_xcd; tix += a.nslots) {
        const uint32_t tile = xcd * a.tiles_per_xcd + tix;  // each XCD streams a contiguous run
        if (tile >= a.ntiles) break;
        const uint64_t b0 = uint64_t(tile) * Kn::W;
        if (b0 + Kn::W <= a.sc) Kn::template tile<true, BT>(a, b0);
        else Kn::template tile<false, BT>(a, b0);
    }
}

// ---------------- k_bs_encode1: the encode, one line per lane ----------------
// (encode.rs:30-80 -> decode_layered with every parity node erased, decode.rs:167-257: one iscore
// level.)  Lane = 32 positions of the q layers z0 + j (j = the parity section's digit, weight 1):
// per layer, U_i = C_i + gamma C_i* for the data nodes (transforms.rs:42-55; companions of other
// lines read directly), V_p += g_(p,i) U_i (the RS parity rows, compile time), then the parity
// section's PFT pairs (transforms.rs:108-125) -- node (T-1, x) at layer z0 + j pairs with (T-1, j)
// at z0 + x, in the same line -- and the stores.  The same linear map as k_bs_encode (bitslice.hpp),
// whose V accumulators go through LDS because its lanes split a line.
template <int KD, int M, int PG>
struct Enc1Kernel {
    using S = Shape<KD, M>;
    static_assert(S::NU == 0 && S::N <= 8, "small codes without shortened nodes");
    static constexpr int Q = S::Q, T = S::T, ALPHA = S::ALPHA;
    static constexpr int LINES = ALPHA / Q, UNITS = LINES * PG, BLOCK = UNITS < 1024 ? UNITS : 1024;
    static constexpr int W = 32 * PG;  // positions per tile
    static constexpr int wt(int y) {
        int w = 1;
        for (int i = 0; i < T - 1 - y; i++) w *= Q;
        return w;
    }
    template <uint8_t CF>
    __device__ __forceinline__ static void fold(uint32_t (&acc)[8], const uint32_t (&v)[8]) {
        if constexpr (CF != 0) {
            sfor<8>([&](auto bc) BS_INL {
                constexpr int bo = decltype(bc)::value;
                acc[bo] = xor_sel<plane_mask(CF, bo, 0), true>(acc[bo], v);
            });
        }
    }

    template <bool FULL, bool BT>
    __device__ static void tile(const Enc1Args &a, uint64_t b0, int64_t doff, int64_t poff) {
        for (int u = threadIdx.x; u < UNITS; u += BLOCK) {
            const int pg = u % PG, line = u / PG;
            const uint32_t z0 = uint32_t(line * Q);
            const uint64_t pos = b0 + uint64_t(32 * pg);
            const int nv = FULL ? (BT ? 32 : 4)
                         : BT ? int(pos >= a.sc ? 0 : a.sc - pos > 32 ? 32 : a.sc - pos)                // bytes
                              : int(pos >= a.sc ? 0 : (a.sc - pos) / 8 > 4 ? 4 : (a.sc - pos) / 8);  // pieces
            uint32_t V[Q][M][8];  // [layer j of the line][parity node p][plane]: U of the parity nodes
            sfor<Q>([&](auto jc) BS_INL {
                constexpr int j = decltype(jc)::value;
                const uint32_t z = z0 + uint32_t(j);
#pragma unroll
                for (int p = 0; p < M; p++)
#pragma unroll
                    for (int w = 0; w < 8; w++) V[j][p][w] = 0;
                sfor<KD>([&](auto ic) BS_INL {
                    constexpr int i = decltype(ic)::value;
                    constexpr int yi = i / Q, xi = i % Q;
                    uint32_t o[8], cv[8], t[8];
                    ld32<FULL, BT>(o, a.data[i] + doff + uint64_t(z) * a.sc + pos, nv);
                    // companion (yi, d) at z[yi := xi], d = z's digit yi (the line's)
                    const int d = int(z / uint32_t(wt(yi))) % Q;
                    const uint8_t *cn = a.data[yi * Q];
#pragma unroll
                    for (int xx = 1; xx < Q; xx++) cn = d == xx ? a.data[yi * Q + xx] : cn;
                    const uint32_t zc = uint32_t(int(z) + (xi - d) * wt(yi));
                    ld32<FULL, BT>(cv, cn + doff + uint64_t(zc) * a.sc + pos, nv);
                    const uint32_t keep = d != xi ? 0xffffffffu : 0u;
                    const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
#pragma unroll
                    for (int w = 0; w < 8; w++) t[w] = xor_xtime4_masked(o[w], cv[w], ks, kr);
                    transpose8(t);
                    sfor<M>([&](auto pc) BS_INL {
                        constexpr int p = decltype(pc)::value;
                        fold<S::RS.g[p][i]>(V[j][p], t);
                    });
                });
            });
            // PFT: C(x, z0 + j) = det^-1 (V(x, z0 + j) + gamma V(j, z0 + x)); red (x == j): C = V
            sfor<Q>([&](auto jc) BS_INL {
                constexpr int j = decltype(jc)::value;
                sfor<M>([&](auto xc) BS_INL {
                    constexpr int x = decltype(xc)::value;
                    uint32_t c[8];
                    if constexpr (x == j) {
#pragma unroll
                        for (int w = 0; w < 8; w++) c[w] = V[j][x][w];
                    } else {
                        uint32_t in[16];
#pragma unroll
                        for (int w = 0; w < 8; w++) {
                            in[w] = V[j][x][w];
                            in[8 + w] = V[x][j][w];
                        }
                        sfor<8>([&](auto bc) BS_INL {
                            constexpr int bo = decltype(bc)::value;
                            c[bo] = xor_sel<plane_mask(S::DINV, bo, 0) | plane_mask(gm(S::DINV, 2), bo, 8), false>(0u, in);
                        });
                    }
                    transpose8(c);
                    st32<FULL, BT>(a.par[x] + poff + uint64_t(z0 + uint32_t(j)) * a.sc + pos, c, nv);
                });
            });
        }
    }
};

template <int KD, int M, int PG, bool BT = false>
__global__ __launch_bounds__((Enc1Kernel<KD, M, PG>::BLOCK)) void k_bs_encode1(Enc1Args a) {
    using Kn = Enc1Kernel<KD, M, PG>;
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    const uint32_t ns = a.nstripes ? a.nstripes : 1u, total = a.ntiles * ns;
    for (uint32_t tix = slot; tix < a.tiles_per_xcd; tix += a.nslots) {
        // flattened (stripe, tile): each XCD streams a contiguous run of the stripes' tiles
        const uint32_t ft = xcd * a.tiles_per_xcd + tix;
        if (ft >= total) break;
        const uint32_t stripe = ft / a.ntiles, tile = ft - stripe * a.ntiles;
        const uint64_t b0 = uint64_t(tile) * Kn::W;
        const int64_t doff = int64_t(stripe) * a.sdata, poff = int64_t(stripe) * a.spar;
        if (b0 + Kn::W <= a.sc) Kn::template tile<true, BT>(a, b0, doff, poff);
        else Kn::template tile<false, BT>(a, b0, doff, poff);
    }
}

}  // namespace bs
}  // namespace clay
