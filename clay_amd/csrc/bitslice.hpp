// bitslice.hpp -- bit-sliced GF(2^8) fused encode for gfx950 (compile-time code constants).
//
// Representation: one lane owns 32 consecutive byte positions of a sub-chunk.  The
// 32 bytes (8 dwords) are transposed into 8 bit-planes P[b] (bit i of P[b] = bit b of
// byte sigma(i)); in that domain multiplication by a constant c is an 8x8 GF(2)
// matrix, i.e. a fixed XOR network over planes, generated at compile time from the
// Reed-Solomon generator of reed-solomon-erasure 6.0.0 (constexpr restatement of
// vandermonde(total, data) * inv(top), gf256.hpp).  Gamma = 2 (transforms.rs:20) is
// applied in the byte domain (SWAR xtime) before the transpose.
//
// Per y-section line (q nodes x q layers differing in digit y) and per column j,
//   U[x] = C[x][z_j] + g * C[j][z_x]        (PRT, transforms.rs:42-55; x == j: red copy)
//   V[p][z_j] += sum_x M[p][yq+x] * U[x]      (per-layer RS encode, decode.rs:386-404)
// V lives in LDS as bit-planes for the whole tile; the parity y-section then applies
//   C[x][z_j] = det^-1 (V[x][z_j] + g V[j][z_x]) (PFT, transforms.rs:108-125)
// and transposes back to bytes.  Same linear map as the reference, so the bytes are
// identical (GF(2^8) arithmetic is exact).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

namespace clay {
namespace bs {

// ---------------- constexpr GF(2^8), poly 0x11D ----------------
constexpr uint8_t gm(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) r ^= a;
        b >>= 1;
        a = uint8_t((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
    }
    return r;
}
constexpr uint8_t gpw(uint8_t a, int n) {
    uint8_t r = 1;
    for (int i = 0; i < n; i++) r = gm(r, a);
    return r;
}
constexpr uint8_t ginv(uint8_t a) { return gpw(a, 254); }

template <int K, int M>
struct RsRows {
    uint8_t g[M][K];
};

// Parity rows K..K+M-1 of vandermonde(K+M, K) * inv(vandermonde top K x K).
template <int K, int M>
constexpr RsRows<K, M> rs_rows() {
    uint8_t a[K][K] = {}, inv[K][K] = {};
    for (int r = 0; r < K; r++)
        for (int c = 0; c < K; c++) {
            a[r][c] = gpw(uint8_t(r), c);
            inv[r][c] = r == c ? 1 : 0;
        }
    for (int c = 0; c < K; c++) {
        int piv = c;
        while (a[piv][c] == 0) piv++;
        for (int j = 0; j < K; j++) {
            uint8_t t = a[c][j];
            a[c][j] = a[piv][j];
            a[piv][j] = t;
            t = inv[c][j];
            inv[c][j] = inv[piv][j];
            inv[piv][j] = t;
        }
        uint8_t s = ginv(a[c][c]);
        for (int j = 0; j < K; j++) {
            a[c][j] = gm(a[c][j], s);
            inv[c][j] = gm(inv[c][j], s);
        }
        for (int r = 0; r < K; r++) {
            if (r == c || a[r][c] == 0) continue;
            uint8_t f = a[r][c];
            for (int j = 0; j < K; j++) {
                a[r][j] ^= gm(f, a[c][j]);
                inv[r][j] ^= gm(f, inv[c][j]);
            }
        }
    }
    RsRows<K, M> out = {};
    for (int p = 0; p < M; p++)
        for (int c = 0; c < K; c++) {
            uint8_t acc = 0;
            for (int i = 0; i < K; i++) acc ^= gm(gpw(uint8_t(K + p), i), inv[i][c]);
            out.g[p][c] = acc;
        }
    return out;
}

// ---------------- compile-time loops ----------------
// Lambdas passed to sfor must inline completely (arrays captured by reference
// would otherwise be demoted to scratch / LDS).
#define BS_INL __attribute__((always_inline))
template <class F, int... Is>
__device__ __forceinline__ void sfor_impl(F &&f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F &&f) {
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// ---------------- bit-plane kernels ----------------
// v_bitop3_b32 LUTs (inputs a=0xF0, b=0xCC, c=0xAA)
constexpr unsigned kSel = 0xCA;   // a ? b : c
constexpr unsigned kXor3 = 0x96;  // a ^ b ^ c
constexpr unsigned kXorAnd = 0x78;  // a ^ (b & c)

__device__ __forceinline__ uint32_t sel(uint32_t m, uint32_t x, uint32_t y) {
    return __builtin_amdgcn_bitop3_b32(m, x, y, kSel);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, kXor3);
}

// 32 bytes (8 dwords, byte 4w+j at bits 8j..8j+7 of d[w]) <-> 8 bit-planes.
// Three delta swaps exchange the dword-index bits with the bit-in-byte bits; the
// map is an involution, so the same routine transposes back.
template <int S, uint32_t MLO>
__device__ __forceinline__ void swap_bits(uint32_t &a, uint32_t &b) {
    const uint32_t na = sel(MLO, a, b << S);   // keep a's low half, take b's (shifted up)
    const uint32_t nb = sel(MLO, a >> S, b);   // take a's high half (shifted down), keep b's
    a = na;
    b = nb;
}
__device__ __forceinline__ void transpose8(uint32_t (&d)[8]) {
    swap_bits<1, 0x55555555u>(d[0], d[1]);
    swap_bits<1, 0x55555555u>(d[2], d[3]);
    swap_bits<1, 0x55555555u>(d[4], d[5]);
    swap_bits<1, 0x55555555u>(d[6], d[7]);
    swap_bits<2, 0x33333333u>(d[0], d[2]);
    swap_bits<2, 0x33333333u>(d[1], d[3]);
    swap_bits<2, 0x33333333u>(d[4], d[6]);
    swap_bits<2, 0x33333333u>(d[5], d[7]);
    swap_bits<4, 0x0F0F0F0Fu>(d[0], d[4]);
    swap_bits<4, 0x0F0F0F0Fu>(d[1], d[5]);
    swap_bits<4, 0x0F0F0F0Fu>(d[2], d[6]);
    swap_bits<4, 0x0F0F0F0Fu>(d[3], d[7]);
}

// o ^ gamma*c on 4 packed bytes (xtime, poly 0x11D).  Byte-wise "top bit set" masks
// come from v_perm_b32's sign-replicate selectors (8..11), avoiding a multiply.
__device__ __forceinline__ uint32_t xor_xtime4(uint32_t o, uint32_t c) {
    const uint32_t sh = (c << 1) & 0xfefefefeu;
    const uint32_t m = __builtin_amdgcn_perm(c, c << 8, 0x0B090A08u);  // 0xFF where byte MSB set
    return xor3(o, sh, m & 0x1d1d1d1du);
}

// o ^ (gamma*c if keep) with ks = keep & 0xfefefefe, kr = keep & 0x1d1d1d1d
__device__ __forceinline__ uint32_t xor_xtime4_masked(uint32_t o, uint32_t c, uint32_t ks, uint32_t kr) {
    const uint32_t m = __builtin_amdgcn_perm(c, c << 8, 0x0B090A08u);
    const uint32_t t = __builtin_amdgcn_bitop3_b32(o, c << 1, ks, kXorAnd);  // o ^ ((c<<1) & ks)
    return __builtin_amdgcn_bitop3_b32(t, m, kr, kXorAnd);                  // ^ (m & kr)
}

__device__ __forceinline__ void xt_planes(const uint32_t (&in)[8], uint32_t (&out)[8]) {
    out[0] = in[7];
    out[1] = in[0];
    out[2] = in[1] ^ in[7];
    out[3] = in[2] ^ in[7];
    out[4] = in[3] ^ in[7];
    out[5] = in[4];
    out[6] = in[5];
    out[7] = in[6];
}

constexpr int popc(uint64_t v) {
    int n = 0;
    for (; v; v &= v - 1) n++;
    return n;
}

// acc (or 0 if !ACC) ^ XOR of in[i] over the set bits of MASK, as 3-input XOR chains.
template <uint64_t MASK, bool ACC, int N>
__device__ __forceinline__ uint32_t xor_sel(uint32_t acc, const uint32_t (&in)[N]) {
    constexpr int total = popc(MASK);
    if constexpr (total == 0) {
        return ACC ? acc : 0u;
    } else {
        uint32_t pend = 0;
        bool have = ACC;  // compile-time after unrolling
        sfor<N>([&](auto ic) BS_INL {
            constexpr int i = decltype(ic)::value;
            if constexpr ((MASK >> i) & 1) {
                constexpr int rank = popc(MASK & ((uint64_t(1) << i) - 1));
                if constexpr (!ACC && rank == 0) {
                    acc = in[i];
                } else if constexpr ((rank + (ACC ? 1 : 0)) % 2 == 1 && rank != total - 1) {
                    pend = in[i];
                } else if constexpr ((rank + (ACC ? 1 : 0)) % 2 == 1) {
                    acc ^= in[i];
                } else {
                    acc = xor3(acc, pend, in[i]);
                }
            }
        });
        (void)have;
        return acc;
    }
}

// GF(2^8) constant as an 8x8 bit matrix: column bi = C * 2^bi.
constexpr uint64_t plane_mask(uint8_t c, int bo, int shift) {
    uint64_t m = 0;
    for (int bi = 0; bi < 8; bi++)
        if ((gm(c, uint8_t(1u << bi)) >> bo) & 1) m |= uint64_t(1) << (bi + shift);
    return m;
}

}  // namespace bs
}  // namespace clay

namespace clay {
namespace bs {

constexpr int kMaxNodes = 64;

struct BsArgs {
    const uint8_t *data[kMaxNodes];  // internal nodes 0..K-1 (nullptr: shortened, known zero)
    uint8_t *par[8];                 // parity y-section, node x (internal (t-1)q + x)
    uint64_t sc;                     // sub-chunk bytes (v1: any; bs6 / stream: multiple of 8)
    uint32_t ntiles, tiles_per_xcd, nslots;
    // k_bs_encode batches: stripe s's nodes at data[i] + s * sdata, par[x] + s * spar
    // (ntiles tiles per stripe, tiles_per_xcd over all nstripes * ntiles); 0 = one stripe
    uint32_t nstripes;
    int64_t sdata, spar;
};

// Code shape derived at compile time from (k, m) with d = k + m - 1 (q = m).
template <int KD, int M>
struct Shape {
    static constexpr int Q = M;
    static constexpr int N = KD + M;
    static constexpr int NU = (N % Q == 0) ? 0 : Q - N % Q;
    static constexpr int T = (N + NU) / Q;
    static constexpr int K = KD + NU;
    static constexpr int ALPHA = [] { int a = 1; for (int i = 0; i < T; i++) a *= Q; return a; }();
    static constexpr RsRows<K, M> RS = rs_rows<K, M>();
    static constexpr uint8_t DINV = ginv(uint8_t(1 ^ gm(2, 2)));
};

template <int Q>
__device__ __forceinline__ const uint8_t *pick(const uint8_t *const (&p)[Q], int i) {
    const uint8_t *r = p[0];
#pragma unroll
    for (int x = 1; x < Q; x++) r = (i == x) ? p[x] : r;
    return r;
}

// 32-byte lane load/store (four 8-byte pieces; in a partial tile only `nb` bytes exist)
template <bool FULL, bool BT = false>
__device__ __forceinline__ void ld32(uint32_t (&d)[8], const uint8_t *p, int nv) {
    // !BT: nv = valid 8-byte pieces.  BT (byte tails: sc % 8 != 0 or unaligned chunks):
    // nv = valid bytes; gfx950 global loads run unaligned, the partial word is read byte
    // by byte.  Separate instantiations: the byte loop's registers would otherwise cost
    // the aligned kernel occupancy ((4,2,5) 64 MiB 0.030 -> 0.0345 ms measured).
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (FULL || (BT ? 8 * i + 8 <= nv : i < nv)) {
            const uint2 v = *reinterpret_cast<const uint2 *>(p + 8 * i);
            d[2 * i] = v.x;
            d[2 * i + 1] = v.y;
        } else if (BT) {
            uint32_t w[2] = {0u, 0u};
            for (int b = 8 * i; b < nv; b++) w[(b >> 2) & 1] |= uint32_t(p[b]) << (8 * (b & 3));
            d[2 * i] = w[0];
            d[2 * i + 1] = w[1];
        } else {
            d[2 * i] = 0;
            d[2 * i + 1] = 0;
        }
    }
}
template <bool FULL, bool BT = false>
__device__ __forceinline__ void st32(uint8_t *p, const uint32_t (&d)[8], int nv) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (FULL || (BT ? 8 * i + 8 <= nv : i < nv)) {
            *reinterpret_cast<uint2 *>(p + 8 * i) = make_uint2(d[2 * i], d[2 * i + 1]);
        } else if (BT) {
            for (int b = 8 * i; b < nv; b++) p[b] = uint8_t(d[2 * i + ((b >> 2) & 1)] >> (8 * (b & 3)));
        }
    }
}

template <int KD, int M, int PG>
struct BsKernel {
    using S = Shape<KD, M>;
    static constexpr int Q = S::Q, T = S::T, ALPHA = S::ALPHA, UNITS = ALPHA * PG;
    static constexpr int BLOCK = UNITS < 1024 ? UNITS : 1024;
    static constexpr int W = 32 * PG;                          // positions per tile
    static constexpr int LDS_WORDS = Q * ALPHA * PG * 8;       // parity-U planes

    // RS parity row p over the q U-values of y-section Y, output plane bo:
    // XOR of U[x][bi] where bit bo of M[p][Yq+x] * 2^bi is set (flat index x*8+bi).
    template <int Y, int P, int BO>
    static constexpr uint64_t rs_mask() {
        uint64_t m = 0;
        for (int x = 0; x < Q; x++) m |= plane_mask(S::RS.g[P][Y * Q + x], BO, 8 * x);
        return m;
    }
    // PFT output plane bo: det^-1 * a + (det^-1 * gamma) * b over [a planes | b planes]
    template <int BO>
    static constexpr uint64_t pft_mask() {
        return plane_mask(S::DINV, BO, 0) | plane_mask(gm(S::DINV, 2), BO, 8);
    }

    // ---- phase A, one y-section ----
    template <int Y, bool FULL, bool BT>
    __device__ static void section(const BsArgs &a, uint32_t *lds, uint64_t b0, int64_t doff) {
        constexpr int WY = [] { int w = 1; for (int i = 0; i < T - 1 - Y; i++) w *= Q; return w; }();
        for (int u = threadIdx.x; u < UNITS; u += BLOCK) {
            const int pg = u % PG, j = (u / PG) % Q, line = u / (PG * Q);
            const int hi = line / WY, lo = line % WY;
            const int zbase = hi * WY * Q + lo;
            const uint64_t pos = b0 + uint64_t(32 * pg);
            const int nv = FULL ? (BT ? 32 : 4)
                         : BT ? int(pos >= a.sc ? 0 : a.sc - pos > 32 ? 32 : a.sc - pos)                // bytes
                              : int(pos >= a.sc ? 0 : (a.sc - pos) / 8 > 4 ? 4 : (a.sc - pos) / 8);  // pieces
            const uint64_t lane_off = uint64_t(zbase) * a.sc + pos;
            // companion node (Y, j); for j == x or a shortened companion the load is
            // still issued (it hits lines a neighbour lane loads) and masked to zero
            const bool creal = (Y * Q + j) < KD;
            const uint8_t *cnode = a.data[creal ? Y * Q + j : Y * Q] + doff;
            uint32_t U[Q * 8];
            sfor<Q>([&](auto xc) BS_INL {
                constexpr int x = decltype(xc)::value;
                uint32_t o[8], c[8];
                if constexpr (Y * Q + x < KD) {
                    ld32<FULL, BT>(o, a.data[Y * Q + x] + doff + lane_off + uint64_t(j) * WY * a.sc, nv);
                } else {
#pragma unroll
                    for (int w = 0; w < 8; w++) o[w] = 0;
                }
                ld32<FULL, BT>(c, cnode + lane_off + uint64_t(x) * WY * a.sc, nv);
                const uint32_t keep = (creal && x != j) ? 0xffffffffu : 0u;
                const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
                uint32_t t[8];
#pragma unroll
                for (int w = 0; w < 8; w++) t[w] = xor_xtime4_masked(o[w], c[w], ks, kr);
                transpose8(t);
#pragma unroll
                for (int w = 0; w < 8; w++) U[x * 8 + w] = t[w];
            });
            uint32_t *acc = lds + (size_t(zbase + j * WY) * PG + pg) * 8;
            sfor<Q>([&](auto pc) BS_INL {
                constexpr int p = decltype(pc)::value;
                uint4 *l = reinterpret_cast<uint4 *>(acc + size_t(p) * ALPHA * PG * 8);
                uint32_t V[8];
                if constexpr (Y == 0) {
                    sfor<8>([&](auto bc) BS_INL {
                        V[decltype(bc)::value] = xor_sel<rs_mask<Y, p, decltype(bc)::value>(), false>(0u, U);
                    });
                } else {
                    const uint4 v0 = l[0], v1 = l[1];
                    V[0] = v0.x; V[1] = v0.y; V[2] = v0.z; V[3] = v0.w;
                    V[4] = v1.x; V[5] = v1.y; V[6] = v1.z; V[7] = v1.w;
                    sfor<8>([&](auto bc) BS_INL {
                        V[decltype(bc)::value] = xor_sel<rs_mask<Y, p, decltype(bc)::value>(), true>(V[decltype(bc)::value], U);
                    });
                }
                l[0] = make_uint4(V[0], V[1], V[2], V[3]);
                l[1] = make_uint4(V[4], V[5], V[6], V[7]);
            });
        }
    }

    __device__ static void read8(const uint32_t *lds, int p, int z, int pg, uint32_t *v) {
        const uint4 *l = reinterpret_cast<const uint4 *>(lds + ((size_t(p) * ALPHA + z) * PG + pg) * 8);
        const uint4 v0 = l[0], v1 = l[1];
        v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w;
        v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
    }

    // ---- phase B: PFT of the parity y-section (digit t-1, weight 1) + store ----
    template <bool FULL, bool BT>
    __device__ static void finish(const BsArgs &a, const uint32_t *lds, uint64_t b0, int64_t poff) {
        for (int u = threadIdx.x; u < UNITS; u += BLOCK) {
            const int pg = u % PG, j = (u / PG) % Q, g = u / (PG * Q);
            const int z0 = g * Q;
            const uint64_t pos = b0 + uint64_t(32 * pg);
            const int nv = FULL ? (BT ? 32 : 4)
                         : BT ? int(pos >= a.sc ? 0 : a.sc - pos > 32 ? 32 : a.sc - pos)                // bytes
                              : int(pos >= a.sc ? 0 : (a.sc - pos) / 8 > 4 ? 4 : (a.sc - pos) / 8);  // pieces
            const uint64_t off = uint64_t(z0 + j) * a.sc + pos;
            {   // red vertex: C = U
                uint32_t v[8];
                read8(lds, j, z0 + j, pg, v);
                transpose8(v);
                st32<FULL, BT>(a.par[j] + poff + off, v, nv);
            }
#pragma unroll
            for (int k = 1; k < Q; k++) {
                const int x = (j + k) % Q;
                uint32_t in[16], c[8];
                read8(lds, x, z0 + j, pg, in);      // U at (x, z0+j)
                read8(lds, j, z0 + x, pg, in + 8);  // U* at (j, z0+x)
                sfor<8>([&](auto bc) BS_INL {
                    c[decltype(bc)::value] = xor_sel<pft_mask<decltype(bc)::value>(), false>(0u, in);
                });
                transpose8(c);
                st32<FULL, BT>(a.par[x] + poff + off, c, nv);
            }
        }
    }

    template <bool FULL, bool BT>
    __device__ static void tile(const BsArgs &a, uint32_t *lds, uint64_t b0, int64_t doff = 0, int64_t poff = 0) {
        sfor<T - 1>([&](auto yc) BS_INL {
            section<decltype(yc)::value, FULL, BT>(a, lds, b0, doff);
            __syncthreads();
        });
        finish<FULL, BT>(a, lds, b0, poff);
        __syncthreads();
    }
};

template <int KD, int M, int PG, bool BT = false>
__global__ __launch_bounds__((BsKernel<KD, M, PG>::BLOCK)) void k_bs_encode(BsArgs a) {
    using Kn = BsKernel<KD, M, PG>;
    __shared__ __attribute__((aligned(16))) uint32_t lds[Kn::LDS_WORDS];
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    const uint32_t ns = a.nstripes ? a.nstripes : 1u, total = a.ntiles * ns;
    for (uint32_t tix = slot; tix < a.tiles_per_xcd; tix += a.nslots) {
        // flattened (stripe, tile): each XCD streams a contiguous run of stripes' tiles
        const uint32_t ft = xcd * a.tiles_per_xcd + tix;
        if (ft >= total) break;
        const uint32_t stripe = ft / a.ntiles, tile = ft - stripe * a.ntiles;
        const uint64_t b0 = uint64_t(tile) * Kn::W;
        const int64_t doff = int64_t(stripe) * a.sdata, poff = int64_t(stripe) * a.spar;
        if (b0 + Kn::W <= a.sc) Kn::template tile<true, BT>(a, lds, b0, doff, poff);
        else Kn::template tile<false, BT>(a, lds, b0, doff, poff);
    }
}

}  // namespace bs
}  // namespace clay

namespace clay {
namespace bs {

// ---------------- memory helpers shared by the LDS-DMA kernels ----------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// LDS-DMA (global_load_lds_dwordx4) issued from inline asm: 1 KiB per wave instruction,
// LDS dest = M0 + lane*16, global = sbase (SGPR pair) + voff (per-lane 32-bit).  Hidden
// from the compiler's waitcnt pass on purpose (it would otherwise drain vmcnt before
// every LDS access); kernels wait for it with counted s_waitcnt vmcnt.  M0 is
// compiler-reserved: it is saved / restored in the same statement.
__device__ __forceinline__ void dma16(uint32_t lds_addr, const uint8_t *sbase, uint32_t voff) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(lds_addr), "v"(voff), "s"(sbase)
                 : "memory");
}
// Cache-policy variants (bench_tools/stream_probe A/B): CP 1 = nt (streaming), 2 = sc1.
template <int CP>
__device__ __forceinline__ void dma16p(uint32_t lds_addr, const uint8_t *sbase, uint32_t voff) {
    if constexpr (CP == 0) {
        dma16(lds_addr, sbase, voff);
    } else {
        unsigned keep;
        if constexpr (CP == 1)
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3 nt\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(sbase) : "memory");
        else
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3 sc1\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(sbase) : "memory");
    }
}
// 16-byte store, exactly one VMEM instruction.  s_nop 1: hipcc does not pad an asm
// store's data hazard (the next instruction may overwrite the data VGPRs before the
// store has read them).
__device__ __forceinline__ void st16(uint8_t *p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const u32x4 v = {a, b, c, d};
    asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
// same with an SGPR base + per-lane 32-bit offset
__device__ __forceinline__ void st16s(const uint8_t *sbase, uint32_t voff, uint32_t a, uint32_t b, uint32_t c,
                                      uint32_t d) {
    const u32x4 v = {a, b, c, d};
    asm volatile("global_store_dwordx4 %0, %1, %2\n\ts_nop 1" ::"v"(voff), "v"(v), "s"(sbase) : "memory");
}
template <int CP>
__device__ __forceinline__ void st16sp(const uint8_t *sbase, uint32_t voff, uint32_t a, uint32_t b, uint32_t c,
                                       uint32_t d) {
    const u32x4 v = {a, b, c, d};
    if constexpr (CP == 0)
        asm volatile("global_store_dwordx4 %0, %1, %2\n\ts_nop 1" ::"v"(voff), "v"(v), "s"(sbase) : "memory");
    else if constexpr (CP == 1)
        asm volatile("global_store_dwordx4 %0, %1, %2 nt\n\ts_nop 1" ::"v"(voff), "v"(v), "s"(sbase) : "memory");
    else
        asm volatile("global_store_dwordx4 %0, %1, %2 sc1\n\ts_nop 1" ::"v"(voff), "v"(v), "s"(sbase) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr_of(const void *p) {
    return uint32_t(size_t((__attribute__((address_space(3))) const uint8_t *)(p)));
}
template <int N>
__device__ __forceinline__ void wait_vm_n() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// s_waitcnt vmcnt(n) for a wave-uniform run-time n (clamped to the 6-bit field: a
// larger n waits for more than needed, never less)
__device__ __forceinline__ void wait_vm_rt(int n) {
    switch (n < 63 ? n : 63) {
#define CLAY_W1(k) case k: wait_vm_n<k>(); break;
#define CLAY_W8(k) CLAY_W1(k) CLAY_W1(k + 1) CLAY_W1(k + 2) CLAY_W1(k + 3) CLAY_W1(k + 4) CLAY_W1(k + 5) CLAY_W1(k + 6) CLAY_W1(k + 7)
        CLAY_W8(0) CLAY_W8(8) CLAY_W8(16) CLAY_W8(24) CLAY_W8(32) CLAY_W8(40) CLAY_W8(48) CLAY_W8(56)
#undef CLAY_W8
#undef CLAY_W1
        default: wait_vm_n<0>(); break;
    }
}
// workgroup barrier after this wave's LDS reads have returned; VMEM (LDS-DMA) stays in flight
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

}  // namespace bs
}  // namespace clay
