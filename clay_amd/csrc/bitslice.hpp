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
    uint64_t sc;                     // sub-chunk bytes, multiple of 8
    uint32_t ntiles, tiles_per_xcd, nslots;
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

// 32-byte lane load/store (four 8-byte pieces; in a partial tile only `nv` pieces exist)
template <bool FULL>
__device__ __forceinline__ void ld32(uint32_t (&d)[8], const uint8_t *p, int nv) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (FULL || i < nv) {
            const uint2 v = *reinterpret_cast<const uint2 *>(p + 8 * i);
            d[2 * i] = v.x;
            d[2 * i + 1] = v.y;
        } else {
            d[2 * i] = 0;
            d[2 * i + 1] = 0;
        }
    }
}
template <bool FULL>
__device__ __forceinline__ void st32(uint8_t *p, const uint32_t (&d)[8], int nv) {
#pragma unroll
    for (int i = 0; i < 4; i++)
        if (FULL || i < nv) *reinterpret_cast<uint2 *>(p + 8 * i) = make_uint2(d[2 * i], d[2 * i + 1]);
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
    template <int Y, bool FULL>
    __device__ static void section(const BsArgs &a, uint32_t *lds, uint64_t b0) {
        constexpr int WY = [] { int w = 1; for (int i = 0; i < T - 1 - Y; i++) w *= Q; return w; }();
        for (int u = threadIdx.x; u < UNITS; u += BLOCK) {
            const int pg = u % PG, j = (u / PG) % Q, line = u / (PG * Q);
            const int hi = line / WY, lo = line % WY;
            const int zbase = hi * WY * Q + lo;
            const uint64_t pos = b0 + uint64_t(32 * pg);
            const int nv = FULL ? 4 : int(pos >= a.sc ? 0 : (a.sc - pos) / 8 > 4 ? 4 : (a.sc - pos) / 8);
            const uint64_t lane_off = uint64_t(zbase) * a.sc + pos;
            // companion node (Y, j); for j == x or a shortened companion the load is
            // still issued (it hits lines a neighbour lane loads) and masked to zero
            const bool creal = (Y * Q + j) < KD;
            const uint8_t *cnode = a.data[creal ? Y * Q + j : Y * Q];
            uint32_t U[Q * 8];
            sfor<Q>([&](auto xc) BS_INL {
                constexpr int x = decltype(xc)::value;
                uint32_t o[8], c[8];
                if constexpr (Y * Q + x < KD) {
                    ld32<FULL>(o, a.data[Y * Q + x] + lane_off + uint64_t(j) * WY * a.sc, nv);
                } else {
#pragma unroll
                    for (int w = 0; w < 8; w++) o[w] = 0;
                }
                ld32<FULL>(c, cnode + lane_off + uint64_t(x) * WY * a.sc, nv);
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
    template <bool FULL>
    __device__ static void finish(const BsArgs &a, const uint32_t *lds, uint64_t b0) {
        for (int u = threadIdx.x; u < UNITS; u += BLOCK) {
            const int pg = u % PG, j = (u / PG) % Q, g = u / (PG * Q);
            const int z0 = g * Q;
            const uint64_t pos = b0 + uint64_t(32 * pg);
            const int nv = FULL ? 4 : int(pos >= a.sc ? 0 : (a.sc - pos) / 8 > 4 ? 4 : (a.sc - pos) / 8);
            const uint64_t off = uint64_t(z0 + j) * a.sc + pos;
            {   // red vertex: C = U
                uint32_t v[8];
                read8(lds, j, z0 + j, pg, v);
                transpose8(v);
                st32<FULL>(a.par[j] + off, v, nv);
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
                st32<FULL>(a.par[x] + off, c, nv);
            }
        }
    }

    template <bool FULL>
    __device__ static void tile(const BsArgs &a, uint32_t *lds, uint64_t b0) {
        sfor<T - 1>([&](auto yc) BS_INL {
            section<decltype(yc)::value, FULL>(a, lds, b0);
            __syncthreads();
        });
        finish<FULL>(a, lds, b0);
        __syncthreads();
    }
};

template <int KD, int M, int PG>
__global__ __launch_bounds__((BsKernel<KD, M, PG>::BLOCK)) void k_bs_encode(BsArgs a) {
    using Kn = BsKernel<KD, M, PG>;
    __shared__ __attribute__((aligned(16))) uint32_t lds[Kn::LDS_WORDS];
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    for (uint32_t tix = slot; tix < a.tiles_per_xcd; tix += a.nslots) {
        const uint32_t tile = xcd * a.tiles_per_xcd + tix;
        if (tile >= a.ntiles) break;
        const uint64_t b0 = uint64_t(tile) * Kn::W;
        if (b0 + Kn::W <= a.sc) Kn::template tile<true>(a, lds, b0);
        else Kn::template tile<false>(a, lds, b0);
    }
}

}  // namespace bs
}  // namespace clay

namespace clay {
namespace bs {

// ===========================================================================
// v2: wave-private LDS staging with LDS-DMA prefetch.
//
// Wave w owns lines [L*w, L*w + L) of every y-section (L = 64 lanes / (q*PG)).  It
// stages its lines' q*q values (node x, column jj) x W bytes into a private LDS
// region with global_load_lds (coalesced 16-lane x 4 B = 64 B segments; every byte
// read from HBM once; companions come from LDS).  As soon as the wave has pulled a
// stage into registers it issues the DMA for its next section (or the next tile's
// first section), so HBM latency overlaps the XOR networks, the accumulate, the
// section barrier and the PFT.  Barriers are raw s_barrier + lgkmcnt(0) so the DMA
// stays in flight across them.
// ===========================================================================
// LDS-DMA (global_load_lds_dword) issued from inline asm: LDS dest = M0 + lane*4,
// global = sbase (SGPR pair) + voff (per-lane 32-bit).  Hidden from the compiler's
// waitcnt pass on purpose (it would otherwise drain vmcnt before every LDS access);
// the kernel waits for it explicitly with wait_vm0().
__device__ __forceinline__ void dma4(uint32_t lds_addr, const uint8_t *sbase, uint32_t voff) {
    unsigned keep;  // M0 is compiler-reserved: save / restore it in the same statement
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %2, %3\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(lds_addr), "v"(voff), "s"(sbase)
                 : "memory");
}
// 8-byte store issued from asm: exactly one VMEM instruction (never merged or
// split by the compiler), so counted vmcnt waits stay exact.
__device__ __forceinline__ void st8(uint8_t *p, uint32_t lo, uint32_t hi) {
    const uint64_t v = uint64_t(lo) | (uint64_t(hi) << 32);
    asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr_of(const void *p) {
    return uint32_t(size_t((__attribute__((address_space(3))) const uint8_t *)(p)));
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int KD, int M>
struct Bs2Kernel {
    using S = Shape<KD, M>;
    static constexpr int Q = S::Q, T = S::T, ALPHA = S::ALPHA;
    static constexpr int PG = 2;                       // lanes per value (32 positions each)
    static constexpr int W = 32 * PG;                  // 64 positions per tile
    static constexpr int LPW = 64 / (Q * PG);          // lines per wave
    static_assert(Q == 4, "v2 staging assumes q == 4 (uniform node per DMA instruction)");
    static constexpr int LINES = ALPHA / Q;            // lines per section
    static constexpr int WAVES = LINES / LPW;
    static constexpr int BLOCK = 64 * WAVES;
    static_assert(LINES % LPW == 0 && BLOCK <= 1024, "shape");
    static constexpr int ACC_WORDS = Q * ALPHA * PG * 8;
    static constexpr int STAGE_BYTES = LPW * Q * Q * W;      // per wave
    static constexpr int LDS_BYTES = ACC_WORDS * 4 + WAVES * STAGE_BYTES;
    static constexpr int DMA_PER_SECTION = STAGE_BYTES / 256;  // 64 lanes x 4 B per instruction

    template <int Y>
    static constexpr int wy() { int w = 1; for (int i = 0; i < T - 1 - Y; i++) w *= Q; return w; }

    // Issue the wave's DMA for section Y of the tile starting at b0.
    // Value v = (line_local, x, jj) flattened as (line_local*Q + x)*Q + jj; one
    // instruction stages 4 values (16 lanes x 4 B each): with Q == 4 the node x and
    // the line are uniform per instruction (SGPR base), the column jj = lane/16
    // and the byte offset live in a 32-bit per-lane offset computed once.
    template <int Y>
    __device__ static void dma(const BsArgs &a, uint32_t stage_lds, int wave, int lane, uint64_t b0) {
        constexpr int WY = wy<Y>();
        uint64_t pos = b0 + uint64_t(lane & 15) * 4;
        if (pos + 4 > a.sc) pos = 0;  // ragged last tile: any valid bytes (never stored)
        const uint32_t voff = uint32_t(uint64_t(lane >> 4) * WY * a.sc + pos);
#pragma unroll
        for (int i = 0; i < DMA_PER_SECTION; i++) {
            const int x = i % Q, ll = i / Q;
            const int node = Y * Q + x;
            if (node >= KD) continue;  // shortened node: known zero, never read
            const int line = wave * LPW + ll;
            const uint64_t zl = uint64_t((line / WY) * WY * Q + (line % WY));
            dma4(stage_lds + uint32_t(i) * 256u, a.data[node] + zl * a.sc, voff);
        }
    }

    __device__ static void read32(const uint8_t *p, uint32_t (&d)[8]) {
        const uint4 v0 = reinterpret_cast<const uint4 *>(p)[0], v1 = reinterpret_cast<const uint4 *>(p)[1];
        d[0] = v0.x; d[1] = v0.y; d[2] = v0.z; d[3] = v0.w;
        d[4] = v1.x; d[5] = v1.y; d[6] = v1.z; d[7] = v1.w;
    }

    template <int Y, int P, int BO>
    static constexpr uint64_t rs_mask() {
        uint64_t m = 0;
        for (int x = 0; x < Q; x++) m |= plane_mask(S::RS.g[P][Y * Q + x], BO, 8 * x);
        return m;
    }
    template <int BO>
    static constexpr uint64_t pft_mask() {
        return plane_mask(S::DINV, BO, 0) | plane_mask(gm(S::DINV, 2), BO, 8);
    }

    // Section Y: stage -> registers, prefetch the next DMA, XOR networks, accumulate.
    template <int Y>
    __device__ static void section(const BsArgs &a, uint32_t *acc, uint8_t *stage, int wave, int lane,
                                   uint64_t b0, uint64_t next_b0, bool has_next) {
        constexpr int WY = wy<Y>();
        const int pg = lane % PG, j = (lane / PG) % Q, ll = lane / (PG * Q);
        const int line = wave * LPW + ll;
        const int zj = (line / WY) * WY * Q + (line % WY) + j * WY;
        const bool creal = (Y * Q + j) < KD;
        wait_vm0();  // this wave's DMA for section Y has landed
        uint32_t U[Q * 8];
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            uint32_t o[8], c[8];
            if constexpr (Y * Q + x < KD) {
                read32(stage + ((ll * Q + x) * Q + j) * W + pg * 32, o);
            } else {
#pragma unroll
                for (int w = 0; w < 8; w++) o[w] = 0;
            }
            read32(stage + ((ll * Q + j) * Q + x) * W + pg * 32, c);
            const uint32_t keep = (creal && x != j) ? 0xffffffffu : 0u;
            const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
#pragma unroll
            for (int w = 0; w < 8; w++) U[x * 8 + w] = xor_xtime4_masked(o[w], c[w], ks, kr);
        });
        // every lane of the wave has its stage values in registers -> refill the stage
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (Y + 1 < T - 1) {
            dma<Y + 1>(a, lds_addr_of(stage), wave, lane, b0);
        } else {
            if (has_next) dma<0>(a, lds_addr_of(stage), wave, lane, next_b0);
        }
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            uint32_t t[8];
#pragma unroll
            for (int w = 0; w < 8; w++) t[w] = U[x * 8 + w];
            transpose8(t);
#pragma unroll
            for (int w = 0; w < 8; w++) U[x * 8 + w] = t[w];
        });
        uint32_t *accp = acc + (size_t(zj) * PG + pg) * 8;
        sfor<Q>([&](auto pc) BS_INL {
            constexpr int p = decltype(pc)::value;
            uint4 *l = reinterpret_cast<uint4 *>(accp + size_t(p) * ALPHA * PG * 8);
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

    __device__ static void read_acc(const uint32_t *acc, int p, int z, int pg, uint32_t *v) {
        const uint4 *l = reinterpret_cast<const uint4 *>(acc + ((size_t(p) * ALPHA + z) * PG + pg) * 8);
        const uint4 v0 = l[0], v1 = l[1];
        v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w;
        v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
    }

    __device__ static void store32(uint8_t *p, const uint32_t (&d)[8], int nv) {
        if (nv >= 4) {
#pragma unroll
            for (int i = 0; i < 4; i++) *reinterpret_cast<uint2 *>(p + 8 * i) = make_uint2(d[2 * i], d[2 * i + 1]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (i < nv) *reinterpret_cast<uint2 *>(p + 8 * i) = make_uint2(d[2 * i], d[2 * i + 1]);
        }
    }

    // PFT of the parity y-section (digit t-1, weight 1) for this wave's groups + store.
    __device__ static void finish(const BsArgs &a, const uint32_t *acc, int wave, int lane, uint64_t b0) {
        const int pg = lane % PG, j = (lane / PG) % Q, gl = lane / (PG * Q);
        const int z0 = (wave * LPW + gl) * Q;
        const uint64_t pos = b0 + uint64_t(32 * pg);
        const int nv = pos >= a.sc ? 0 : ((a.sc - pos) / 8 > 4 ? 4 : int((a.sc - pos) / 8));
        const uint64_t off = uint64_t(z0 + j) * a.sc + pos;
        {
            uint32_t v[8];
            read_acc(acc, j, z0 + j, pg, v);
            transpose8(v);
            store32(a.par[j] + off, v, nv);
        }
#pragma unroll
        for (int k = 1; k < Q; k++) {
            const int x = (j + k) % Q;
            uint32_t in[16], c[8];
            read_acc(acc, x, z0 + j, pg, in);
            read_acc(acc, j, z0 + x, pg, in + 8);
            sfor<8>([&](auto bc) BS_INL {
                c[decltype(bc)::value] = xor_sel<pft_mask<decltype(bc)::value>(), false>(0u, in);
            });
            transpose8(c);
            store32(a.par[x] + off, c, nv);
        }
    }
};

template <int KD, int M>
__global__ __launch_bounds__((Bs2Kernel<KD, M>::BLOCK)) void k_bs2_encode(BsArgs a) {
    using Kn = Bs2Kernel<KD, M>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *acc = reinterpret_cast<uint32_t *>(smem);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    uint8_t *stage = smem + Kn::ACC_WORDS * 4 + wave * Kn::STAGE_BYTES;
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    uint32_t tix = slot;
    uint32_t tile = xcd * a.tiles_per_xcd + tix;
    if (tix >= a.tiles_per_xcd || tile >= a.ntiles) return;
    Kn::template dma<0>(a, lds_addr_of(stage), wave, lane, uint64_t(tile) * Kn::W);
    while (true) {
        const uint64_t b0 = uint64_t(tile) * Kn::W;
        const uint32_t ntix = tix + a.nslots, ntile = xcd * a.tiles_per_xcd + ntix;
        const bool has_next = ntix < a.tiles_per_xcd && ntile < a.ntiles;
        const uint64_t nb0 = uint64_t(ntile) * Kn::W;
        sfor<Kn::T - 1>([&](auto yc) BS_INL {
            Kn::template section<decltype(yc)::value>(a, acc, stage, wave, lane, b0, nb0, has_next);
            lds_barrier();
        });
        Kn::finish(a, acc, wave, lane, b0);
        lds_barrier();
        if (!has_next) break;
        tix = ntix;
        tile = ntile;
    }
    wait_vm0();
}

}  // namespace bs
}  // namespace clay

namespace clay {
namespace bs {

// ===========================================================================
// v3: layer-per-lane, register accumulators, 2-slot section ring in LDS.
//
// Lane (layer z, half pg) accumulates V[p][z] = sum over the data y-sections of
// M[p][yq+x] * U_y[x][z] in registers: every (line, column) step of the
// reference's per-layer loop is exactly one (layer, section) pair, so nothing is
// recomputed and no accumulator lives in LDS.  A section (q nodes x alpha layers x
// W bytes) is staged by coalesced LDS-DMA two sections ahead in a 2-slot ring
// shared by the workgroup; waits are counted s_waitcnt vmcnt so the next fill stays
// in flight.  The PFT partners of the parity y-section (layers differing in the
// last digit) form a lane quad and exchange through DPP.
// ===========================================================================
template <int N>
__device__ __forceinline__ void wait_vm_n() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wave-uniform run-time count -> immediate
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
#define CLAY_VMW(k) case k: wait_vm_n<k>(); break;
        CLAY_VMW(0) CLAY_VMW(1) CLAY_VMW(2) CLAY_VMW(4) CLAY_VMW(8) CLAY_VMW(12) CLAY_VMW(16)
        CLAY_VMW(20) CLAY_VMW(24) CLAY_VMW(28) CLAY_VMW(32) CLAY_VMW(36) CLAY_VMW(40) CLAY_VMW(44)
        CLAY_VMW(48) CLAY_VMW(52) CLAY_VMW(56) CLAY_VMW(60)
#undef CLAY_VMW
        default: wait_vm_n<0>(); break;  // conservative
    }
}

template <int KD, int M>
struct Bs3Kernel {
    using S = Shape<KD, M>;
    static constexpr int Q = S::Q, T = S::T, ALPHA = S::ALPHA, NSEC = T - 1;
    static_assert(Q == 4, "v3 assumes q == 4 (lane quads, uniform DMA node)");
    static_assert(NSEC >= 2, "2-slot ring needs >= 2 data y-sections");
    static constexpr int PG = 2, W = 64;
    static constexpr int BLOCK = ALPHA * PG;  // one lane per (layer, half)
    static_assert(BLOCK <= 1024 && BLOCK % 64 == 0, "shape");
    static constexpr int WAVES = BLOCK / 64;
    static_assert(WAVES % Q == 0, "each wave fills one node");
    static constexpr int SLOT_BYTES = Q * ALPHA * W;               // one section, all layers
    static constexpr int LDS_BYTES = 2 * SLOT_BYTES;
    static constexpr int INSTR_PER_SLOT = SLOT_BYTES / 256;        // 256 B per DMA instruction
    static constexpr int INSTR_PER_WAVE = INSTR_PER_SLOT / WAVES;
    static constexpr int STORES_PER_TILE = Q * 4;                  // 4 outputs x 4 pieces of 8 B

    template <int Y>
    static constexpr int wy() { int w = 1; for (int i = 0; i < T - 1 - Y; i++) w *= Q; return w; }

    // DMA instructions wave `wave` issues for section y (its node may be shortened)
    __device__ static int n_dma(int y, int wave) { return (y * Q + wave % Q) < KD ? INSTR_PER_WAVE : 0; }

    // Fill a slot with section Y of the tile at b0.  Instruction k covers node
    // x = k % Q, layers [4(k/Q), 4(k/Q)+4); slot layout [x][z][W].  Wave w issues
    // k = w + WAVES*i, so its node x = w % Q is uniform.
    template <int Y>
    __device__ static void dma(const BsArgs &a, uint32_t slot_lds, int wave, int lane, uint64_t b0) {
        const int x = wave % Q;
        if (Y * Q + x >= KD) return;  // shortened node: never staged, never read
        uint64_t pos = b0 + uint64_t(lane & 15) * 4;
        if (pos + 4 > a.sc) pos = 0;  // ragged last tile: any valid bytes (never stored)
        const uint32_t voff = uint32_t(uint64_t(lane >> 4) * a.sc + pos);
        const uint8_t *nb = a.data[Y * Q + x];
#pragma unroll
        for (int i = 0; i < INSTR_PER_WAVE; i++) {
            const int k = wave + WAVES * i;
            const int zb = 4 * (k / Q);
            dma4(slot_lds + uint32_t((x * ALPHA + zb) * W), nb + uint64_t(zb) * a.sc, voff);
        }
    }
    template <int Y>
    __device__ static void dma_sec(int y, const BsArgs &a, uint32_t slot_lds, int wave, int lane, uint64_t b0) {
        if constexpr (Y < NSEC) {
            if (y == Y) dma<Y>(a, slot_lds, wave, lane, b0);
            else dma_sec<Y + 1>(y, a, slot_lds, wave, lane, b0);
        }
    }

    __device__ static void rd32(const uint8_t *p, uint32_t (&d)[8]) {
        const uint4 v0 = reinterpret_cast<const uint4 *>(p)[0], v1 = reinterpret_cast<const uint4 *>(p)[1];
        d[0] = v0.x; d[1] = v0.y; d[2] = v0.z; d[3] = v0.w;
        d[4] = v1.x; d[5] = v1.y; d[6] = v1.z; d[7] = v1.w;
    }

    template <int Y, int P, int BO>
    static constexpr uint64_t rs_mask() {
        uint64_t m = 0;
        for (int x = 0; x < Q; x++) m |= plane_mask(S::RS.g[P][Y * Q + x], BO, 8 * x);
        return m;
    }
    template <int BO>
    static constexpr uint64_t pft_mask() {
        return plane_mask(S::DINV, BO, 0) | plane_mask(gm(S::DINV, 2), BO, 8);
    }

    // Section Y: gather this lane's column (own C[x][z]; companion node (Y,d) at
    // z + (x-d)*WY, d = digit Y of z) and apply the PRT in the byte domain.
    template <int Y>
    __device__ static void gather(const uint8_t *slot, int z, int pg, uint32_t (&U)[Q * 8]) {
        constexpr int WY = wy<Y>();
        const int d = (z / WY) % Q;
        const bool creal = (Y * Q + d) < KD;
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            uint32_t o[8], c[8];
            if constexpr (Y * Q + x < KD) {
                rd32(slot + (x * ALPHA + z) * W + pg * 32, o);
            } else {
#pragma unroll
                for (int w = 0; w < 8; w++) o[w] = 0;
            }
            rd32(slot + (d * ALPHA + z + (x - d) * WY) * W + pg * 32, c);
            const uint32_t keep = (creal && x != d) ? 0xffffffffu : 0u;
            const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
#pragma unroll
            for (int w = 0; w < 8; w++) U[x * 8 + w] = xor_xtime4_masked(o[w], c[w], ks, kr);
        });
    }
    // bit-slice the U column and add the section's RS contribution into V
    template <int Y>
    __device__ static void accumulate(uint32_t (&U)[Q * 8], uint32_t (&V)[Q][8]) {
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            uint32_t t[8];
#pragma unroll
            for (int w = 0; w < 8; w++) t[w] = U[x * 8 + w];
            transpose8(t);
#pragma unroll
            for (int w = 0; w < 8; w++) U[x * 8 + w] = t[w];
        });
        sfor<Q>([&](auto pc) BS_INL {
            constexpr int p = decltype(pc)::value;
            sfor<8>([&](auto bc) BS_INL {
                constexpr int bo = decltype(bc)::value;
                V[p][bo] = xor_sel<rs_mask<Y, p, bo>(), (Y != 0)>(V[p][bo], U);
            });
        });
    }

    template <int CTRL>
    __device__ static uint32_t qperm(uint32_t v) {
        return uint32_t(__builtin_amdgcn_mov_dpp(int(v), CTRL, 0xF, 0xF, false));
    }
    // lane-dependent register / pointer selection through bitop3 masks (a select
    // chain would be folded into a scratch array or a kernarg load by the compiler)
    struct Sel4 {
        uint32_t m1, m2, m3;
        __device__ explicit Sel4(int p)
            : m1(p == 1 ? ~0u : 0u), m2(p == 2 ? ~0u : 0u), m3(p == 3 ? ~0u : 0u) {}
        __device__ uint32_t pick(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) const {
            uint32_t r = sel(m1, a1, a0);
            r = sel(m2, a2, r);
            return sel(m3, a3, r);
        }
    };
    __device__ static uint32_t pick4(const uint32_t (&V)[Q][8], const Sel4 &s, int w) {
        return s.pick(V[0][w], V[1][w], V[2][w], V[3][w]);
    }
    __device__ static uint8_t *par_of(const BsArgs &a, const Sel4 &s) {
        uint64_t p0 = uint64_t(a.par[0]), p1 = uint64_t(a.par[1]), p2 = uint64_t(a.par[2]), p3 = uint64_t(a.par[3]);
        const uint32_t lo = s.pick(uint32_t(p0), uint32_t(p1), uint32_t(p2), uint32_t(p3));
        const uint32_t hi = s.pick(uint32_t(p0 >> 32), uint32_t(p1 >> 32), uint32_t(p2 >> 32), uint32_t(p3 >> 32));
        return reinterpret_cast<uint8_t *>(uint64_t(lo) | (uint64_t(hi) << 32));
    }
    // full tile: exactly 4 asm stores; ragged last tile: masked (that tile is always
    // the workgroup's last, so no counted wait depends on its store count)
    __device__ static void store32(uint8_t *p, const uint32_t (&d)[8], int nv) {
        if (nv >= 4) {
#pragma unroll
            for (int i = 0; i < 4; i++) st8(p + 8 * i, d[2 * i], d[2 * i + 1]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (i < nv) st8(p + 8 * i, d[2 * i], d[2 * i + 1]);
        }
    }
    // PFT (transforms.rs:108-125) for parity node x = j^K at my layer z (last digit j):
    // C[x][z] = det^-1 (V[x][z] + g V[j][z0+x]); lane j^K of the quad holds layer z0+x
    // and sends its V[j] (= V[s^K] for sender s).
    template <int K>
    __device__ static void pft_out(const BsArgs &a, const uint32_t (&V)[Q][8], int j, uint64_t off, int nv) {
        constexpr int CTRL = K == 1 ? 0xB1 : K == 2 ? 0x4E : 0x1B;  // quad lane i reads lane i^K
        const int x = j ^ K;
        const Sel4 sx(x);
        uint32_t in[16], c[8];
#pragma unroll
        for (int w = 0; w < 8; w++) {
            in[w] = pick4(V, sx, w);
            in[8 + w] = qperm<CTRL>(in[w]);  // as sender: my V[me^K]; received: partner's V[j]
        }
        sfor<8>([&](auto bc) BS_INL {
            c[decltype(bc)::value] = xor_sel<pft_mask<decltype(bc)::value>(), false>(0u, in);
        });
        transpose8(c);
        store32(par_of(a, sx) + off, c, nv);
    }
};

template <int KD, int M>
__global__ __launch_bounds__((Bs3Kernel<KD, M>::BLOCK)) void k_bs3_encode(BsArgs a) {
    using Kn = Bs3Kernel<KD, M>;
    constexpr int Q = Kn::Q, NSEC = Kn::NSEC;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int j = lane & 3, pg = (lane >> 2) & 1, gl = lane >> 3;  // quad = one PFT group
    const int z = (wave * 8 + gl) * Q + j;
    const uint32_t lds0 = lds_addr_of(smem), lds1 = lds_addr_of(smem + Kn::SLOT_BYTES);
    const uint32_t xcd = blockIdx.x & 7u, slotid = blockIdx.x >> 3;
    uint32_t tix = slotid;
    if (tix >= a.tiles_per_xcd || xcd * a.tiles_per_xcd + tix >= a.ntiles) return;
    // prologue: sections 0 and 1 of the first tile into slots 0 and 1
    {
        const uint64_t b0 = uint64_t(xcd * a.tiles_per_xcd + tix) * Kn::W;
        Kn::template dma<0>(a, lds0, wave, lane, b0);
        Kn::template dma<1>(a, lds1, wave, lane, b0);
    }
    uint32_t sidx = 0;  // sections consumed so far; slot = sidx & 1
    bool first = true;
    while (true) {
        const uint64_t b0 = uint64_t(xcd * a.tiles_per_xcd + tix) * Kn::W;
        const uint32_t ntix = tix + a.nslots;
        const bool has_next = ntix < a.tiles_per_xcd && xcd * a.tiles_per_xcd + ntix < a.ntiles;
        const uint64_t nb0 = uint64_t(xcd * a.tiles_per_xcd + ntix) * Kn::W;
        uint32_t V[Q][8];
        sfor<NSEC>([&](auto yc) BS_INL {
            constexpr int Y = decltype(yc)::value;
            const int slot = int(sidx & 1);
            // VMEM ops issued after this section's fill may stay in flight: the fill of
            // section Y+1, plus the previous tile's output stores if they came later.
            int younger;
            if constexpr (Y == 0) {
                younger = Kn::n_dma(1, wave) + (first ? 0 : Kn::STORES_PER_TILE);
            } else if constexpr (Y == 1) {
                younger = (first ? 0 : Kn::STORES_PER_TILE) + (NSEC > 2 ? Kn::n_dma(2, wave) : (has_next ? Kn::n_dma(0, wave) : 0));
            } else if constexpr (Y + 1 < NSEC) {
                younger = Kn::n_dma(Y + 1, wave);
            } else {
                younger = has_next ? Kn::n_dma(0, wave) : 0;
            }
            wait_vm(younger);
            lds_barrier();  // every wave's part of the fill has landed
            uint32_t U[Q * 8];
            Kn::template gather<Y>(smem + slot * Kn::SLOT_BYTES, z, pg, U);
            lds_barrier();  // the slot has been read by every wave -> refill it
            const uint32_t sl = slot ? lds1 : lds0;
            if constexpr (Y + 2 < NSEC) {
                Kn::template dma<Y + 2>(a, sl, wave, lane, b0);
            } else {
                if (has_next) Kn::template dma_sec<0>(Y + 2 - NSEC, a, sl, wave, lane, nb0);
            }
            Kn::template accumulate<Y>(U, V);
            sidx++;
        });
        // parity y-section: PFT across the quad, bytes back, store
        const uint64_t pos = b0 + uint64_t(32 * pg);
        const int nv = pos >= a.sc ? 0 : ((a.sc - pos) / 8 > 4 ? 4 : int((a.sc - pos) / 8));
        const uint64_t off = uint64_t(z) * a.sc + pos;
        {
            const typename Kn::Sel4 sj(j);
            uint32_t c[8];
#pragma unroll
            for (int w = 0; w < 8; w++) c[w] = Kn::pick4(V, sj, w);
            transpose8(c);
            Kn::store32(Kn::par_of(a, sj) + off, c, nv);
        }
        Kn::template pft_out<1>(a, V, j, off, nv);
        Kn::template pft_out<2>(a, V, j, off, nv);
        Kn::template pft_out<3>(a, V, j, off, nv);
        first = false;
        if (!has_next) break;
        tix = ntix;
    }
    wait_vm_n<0>();
}

}  // namespace bs
}  // namespace clay

namespace clay {
namespace bs {

// ===========================================================================
// v4: v2's wave-private staging, with 16-byte LDS-DMA and bank-conflict-free LDS.
//
// v2 staged through global_load_lds_dword (4 B/lane): 32 DMA instructions per wave
// and section kept the texture addresser busy ~65 % of the kernel, and its stage /
// accumulator images had 2- to 8-way bank conflicts (75 % of LDS cycles).  v4:
//  * global_load_lds_dwordx4: 1 KiB per instruction, 8 per wave and section.  The
//    destination is lane-linear, so the stage image is permuted through the SOURCE
//    address of each lane (16-B piece granularity).
//  * lane -> (pg, j, line) map chosen against the ds_read_b128 lane groups
//    (group = lane bit 5 and parity of bits 2..4; bits 0,1,3,4 free inside one):
//    b0 = pg, b1 = j0, b3 = j1, b4 = ll0, b5 = ll1, b2 = ll2.
//  * stage piece (line ll, node xn, column jc, piece pc = 2 pg + d) lives at
//    row (xn, ll >> 1, d), slot pg + 2 ((xn + jc) & 3) + 8 (ll & 1): both a lane's own
//    value (ll, x, j) and its companion (ll, j, x) reads hit 16 distinct slots.
//  * accumulator (p, z, pg, h) slot XOR-swizzled by a GF(2)-linear hash of z >> 2
//    (found by tools/acc_swizzle_exhaustive.py): every section's read-modify-write
//    and the PFT reads (partners x = j ^ k) are conflict free.
//  * sub-chunks are only 8-byte aligned; 16-byte DMA from 4/8-byte-aligned
//    addresses is exact (tools/dma_align_test.hip).  The one ragged piece per row
//    of the last tile is DMA'd from a clamped address and patched after landing.
// Parity stores are global_store_dwordx4 from asm, so the next tile's first wait
// can leave exactly those in flight (vmcnt(STORES)).
// ===========================================================================
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void dma16(uint32_t lds_addr, const uint8_t *sbase, uint32_t voff) {
    unsigned keep;  // M0 is compiler-reserved: save / restore it in the same statement
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(lds_addr), "v"(voff), "s"(sbase)
                 : "memory");
}
__device__ __forceinline__ void st16(uint8_t *p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const u32x4 v = {a, b, c, d};
    asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int KD, int M>
struct Bs4Kernel {
    using S = Shape<KD, M>;
    static constexpr int Q = S::Q, T = S::T, ALPHA = S::ALPHA;
    static_assert(Q == 4 && T == 4, "v4 lane map and swizzles are derived for q = 4, t = 4");
    static constexpr int PG = 2, W = 64, LPW = 8;        // 2 lanes x 32 positions; 8 lines per wave
    static constexpr int LINES = ALPHA / Q, WAVES = LINES / LPW, BLOCK = 64 * WAVES;
    static_assert(BLOCK <= 1024 && LINES % LPW == 0, "shape");
    static constexpr int ACC_P = ALPHA * PG * 32;        // bytes per parity row of the accumulator
    static constexpr int ACC_BYTES = Q * ACC_P;
    static constexpr int STAGE_BYTES = LPW * Q * Q * W;  // per wave
    static constexpr int LDS_BYTES = ACC_BYTES + WAVES * STAGE_BYTES;
    static constexpr int NDMA = STAGE_BYTES / 1024;
    static constexpr int STORES = Q * 2;                 // dwordx4 stores per lane per full tile

    template <int Y>
    static constexpr int wy() { int w = 1; for (int i = 0; i < T - 1 - Y; i++) w *= Q; return w; }
    // first layer of line `line` in section Y (digit Y = 0)
    template <int Y>
    __device__ static int zl(int line) { return (line / wy<Y>()) * wy<Y>() * Q + line % wy<Y>(); }

    __device__ static int lane_pg(int lane) { return lane & 1; }
    __device__ static int lane_j(int lane) { return ((lane >> 1) & 1) | ((lane >> 2) & 2); }
    __device__ static int lane_ll(int lane) { return ((lane >> 4) & 3) | (lane & 4); }

    __device__ static uint32_t acc_off(int z, int pg, int h) {
        const int zh = z >> 2;
        const int f = (__builtin_popcount(zh & 0x15) & 1) | ((zh & 1) ? 0xC : 0);
        return uint32_t(zh * 256 + ((((z & 3) << 2) | (pg << 1) | h) ^ f) * 16);
    }

    // Per-lane DMA source for instruction i of section Y.  Returns false when the
    // instruction's node is shortened (never staged).  `pos` is clamped for the
    // ragged last tile; *partial reports a piece with only 8 valid bytes.
    template <int Y>
    __device__ static uint32_t dma_src(int i, int wave, int lane, uint32_t b0, uint32_t sc, uint32_t *ppos) {
        const int s = lane & 15, r = lane >> 4;
        const int pg = s & 1, d = r & 1;
        const int xn = i >> 1;
        const int ll = (s >> 3) | ((((i & 1) << 1) | (r >> 1)) << 1);
        const int jc = (((s >> 1) & 3) - xn) & 3;
        *ppos = b0 + uint32_t(2 * pg + d) * 16u;
        return uint32_t(zl<Y>(wave * LPW + ll) + jc * wy<Y>()) * sc;
    }

    template <int Y>
    __device__ static void dma(const BsArgs &a, uint32_t stage_lds, int wave, int lane, uint32_t b0) {
        const uint32_t sc = uint32_t(a.sc);
#pragma unroll
        for (int i = 0; i < NDMA; i++) {
            const int node = Y * Q + (i >> 1);
            if (node >= KD) continue;  // shortened node: known zero, never read
            uint32_t pos;
            const uint32_t row = dma_src<Y>(i, wave, lane, b0, sc, &pos);
            if (pos + 16u > sc) pos = sc - 16u;  // ragged: any valid bytes, patched after landing
            dma16(stage_lds + uint32_t(i) * 1024u, a.data[node], row + pos);
        }
    }

    // ragged last tile: rewrite the pieces whose DMA source was clamped
    template <int Y>
    __device__ static void patch(const BsArgs &a, uint8_t *stage, int wave, int lane, uint32_t b0) {
        const uint32_t sc = uint32_t(a.sc);
#pragma unroll
        for (int i = 0; i < NDMA; i++) {
            const int node = Y * Q + (i >> 1);
            if (node >= KD) continue;
            uint32_t pos;
            const uint32_t row = dma_src<Y>(i, wave, lane, b0, sc, &pos);
            if (pos < sc && pos + 16u > sc) {  // 8 valid bytes (sc is a multiple of 8)
                const uint2 v = *reinterpret_cast<const uint2 *>(a.data[node] + row + pos);
                *reinterpret_cast<uint4 *>(stage + i * 1024 + lane * 16) = make_uint4(v.x, v.y, 0u, 0u);
            }
        }
    }

    __device__ static void read32(const uint8_t *p, uint32_t (&d)[8]) {
        const uint4 v0 = *reinterpret_cast<const uint4 *>(p), v1 = *reinterpret_cast<const uint4 *>(p + 256);
        d[0] = v0.x; d[1] = v0.y; d[2] = v0.z; d[3] = v0.w;
        d[4] = v1.x; d[5] = v1.y; d[6] = v1.z; d[7] = v1.w;
    }

    template <int Y, int P, int BO>
    static constexpr uint64_t rs_mask() {
        uint64_t m = 0;
        for (int x = 0; x < Q; x++) m |= plane_mask(S::RS.g[P][Y * Q + x], BO, 8 * x);
        return m;
    }
    template <int BO>
    static constexpr uint64_t pft_mask() {
        return plane_mask(S::DINV, BO, 0) | plane_mask(gm(S::DINV, 2), BO, 8);
    }

    template <int Y>
    __device__ static void section(const BsArgs &a, uint8_t *acc, uint8_t *stage, int wave, int lane,
                                   uint32_t b0, uint32_t nb0, bool has_next, bool first, bool ragged) {
        constexpr int WY = wy<Y>();
        const int pg = lane_pg(lane), j = lane_j(lane), ll = lane_ll(lane);
        const int zj = zl<Y>(wave * LPW + ll) + j * WY;
        const bool creal = (Y * Q + j) < KD;
        if constexpr (Y == 0) {
            if (first) wait_vm_n<0>();
            else wait_vm_n<STORES>();  // previous tile's parity stores may stay in flight
        } else {
            wait_vm_n<0>();
        }
        if (ragged) patch<Y>(a, stage, wave, lane, b0);
        const int lbase = (ll >> 1) * 512 + (pg + 8 * (ll & 1)) * 16;
        uint32_t U[Q * 8];
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            const int sw = ((x + j) & 3) * 32;
            uint32_t o[8], c[8];
            if constexpr (Y * Q + x < KD) {
                read32(stage + x * 2048 + lbase + sw, o);
            } else {
#pragma unroll
                for (int w = 0; w < 8; w++) o[w] = 0;
            }
            read32(stage + j * 2048 + lbase + sw, c);
            const uint32_t keep = (creal && x != j) ? 0xffffffffu : 0u;
            const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
#pragma unroll
            for (int w = 0; w < 8; w++) U[x * 8 + w] = xor_xtime4_masked(o[w], c[w], ks, kr);
        });
        // the wave's stage is in registers -> refill it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (Y + 1 < T - 1) {
            dma<Y + 1>(a, lds_addr_of(stage), wave, lane, b0);
        } else {
            if (has_next) dma<0>(a, lds_addr_of(stage), wave, lane, nb0);
        }
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            uint32_t t[8];
#pragma unroll
            for (int w = 0; w < 8; w++) t[w] = U[x * 8 + w];
            transpose8(t);
#pragma unroll
            for (int w = 0; w < 8; w++) U[x * 8 + w] = t[w];
        });
        const uint32_t a0 = acc_off(zj, pg, 0), a1 = acc_off(zj, pg, 1);
        sfor<Q>([&](auto pc) BS_INL {
            constexpr int p = decltype(pc)::value;
            uint4 *l0 = reinterpret_cast<uint4 *>(acc + p * ACC_P + a0);
            uint4 *l1 = reinterpret_cast<uint4 *>(acc + p * ACC_P + a1);
            uint32_t V[8];
            if constexpr (Y == 0) {
                sfor<8>([&](auto bc) BS_INL {
                    V[decltype(bc)::value] = xor_sel<rs_mask<Y, p, decltype(bc)::value>(), false>(0u, U);
                });
            } else {
                const uint4 v0 = *l0, v1 = *l1;
                V[0] = v0.x; V[1] = v0.y; V[2] = v0.z; V[3] = v0.w;
                V[4] = v1.x; V[5] = v1.y; V[6] = v1.z; V[7] = v1.w;
                sfor<8>([&](auto bc) BS_INL {
                    V[decltype(bc)::value] = xor_sel<rs_mask<Y, p, decltype(bc)::value>(), true>(V[decltype(bc)::value], U);
                });
            }
            *l0 = make_uint4(V[0], V[1], V[2], V[3]);
            *l1 = make_uint4(V[4], V[5], V[6], V[7]);
        });
    }

    // lane-dependent parity node: uniform pointer loads + selects (no divergent kernarg load)
    // (each pointer is pinned in SGPRs first; otherwise the compiler folds the selects
    // back into a per-lane global_load whose vmcnt(0) would drain the DMA prefetch)
    __device__ static uint8_t *par_of(const BsArgs &a, int x) {
        uint64_t r = reinterpret_cast<uint64_t>(a.par[0]);
        asm volatile("" : "+s"(r));
#pragma unroll
        for (int i = 1; i < Q; i++) {
            uint64_t pi = reinterpret_cast<uint64_t>(a.par[i]);
            asm volatile("" : "+s"(pi));
            r = (x == i) ? pi : r;
        }
        return reinterpret_cast<uint8_t *>(r);
    }

    __device__ static void read_acc(const uint8_t *acc, int p, int z, int pg, uint32_t *v) {
        const uint4 v0 = *reinterpret_cast<const uint4 *>(acc + p * ACC_P + acc_off(z, pg, 0));
        const uint4 v1 = *reinterpret_cast<const uint4 *>(acc + p * ACC_P + acc_off(z, pg, 1));
        v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w;
        v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
    }

    __device__ static void store32(uint8_t *p, const uint32_t (&d)[8], bool full, int nv) {
        if (full) {
            st16(p, d[0], d[1], d[2], d[3]);
            st16(p + 16, d[4], d[5], d[6], d[7]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (i < nv) *reinterpret_cast<uint2 *>(p + 8 * i) = make_uint2(d[2 * i], d[2 * i + 1]);
        }
    }

    // PFT of the parity y-section (digit t-1, weight 1) for this wave's groups + store.
    __device__ static void finish(const BsArgs &a, const uint8_t *acc, int wave, int lane, uint32_t b0, bool ragged) {
        const int pg = lane_pg(lane), j = lane_j(lane), gl = lane_ll(lane);
        const int z0 = (wave * LPW + gl) * Q;
        const uint32_t sc = uint32_t(a.sc);
        const uint32_t pos = b0 + uint32_t(32 * pg);
        const int nv = pos >= sc ? 0 : ((sc - pos) / 8 > 4 ? 4 : int((sc - pos) / 8));
        const bool full = !ragged;
        const uint32_t off = uint32_t(z0 + j) * sc + pos;
        {
            uint32_t v[8];
            read_acc(acc, j, z0 + j, pg, v);
            transpose8(v);
            store32(par_of(a, j) + off, v, full, nv);
        }
#pragma unroll
        for (int k = 1; k < Q; k++) {
            const int x = j ^ k;
            uint32_t in[16], c[8];
            read_acc(acc, x, z0 + j, pg, in);
            read_acc(acc, j, z0 + x, pg, in + 8);
            sfor<8>([&](auto bc) BS_INL {
                c[decltype(bc)::value] = xor_sel<pft_mask<decltype(bc)::value>(), false>(0u, in);
            });
            transpose8(c);
            store32(par_of(a, x) + off, c, full, nv);
        }
    }
};

template <int KD, int M>
__global__ __launch_bounds__((Bs4Kernel<KD, M>::BLOCK)) void k_bs4_encode(BsArgs a) {
    using Kn = Bs4Kernel<KD, M>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *acc = smem;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    uint8_t *stage = smem + Kn::ACC_BYTES + wave * Kn::STAGE_BYTES;
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    uint32_t tix = slot;
    uint32_t tile = xcd * a.tiles_per_xcd + tix;
    if (tix >= a.tiles_per_xcd || tile >= a.ntiles) return;
    Kn::template dma<0>(a, lds_addr_of(stage), wave, lane, tile * uint32_t(Kn::W));
    bool first = true;
    while (true) {
        const uint32_t b0 = tile * uint32_t(Kn::W);
        const bool ragged = uint64_t(b0) + Kn::W > a.sc;
        const uint32_t ntix = tix + a.nslots, ntile = xcd * a.tiles_per_xcd + ntix;
        const bool has_next = ntix < a.tiles_per_xcd && ntile < a.ntiles;
        const uint32_t nb0 = ntile * uint32_t(Kn::W);
        sfor<Kn::T - 1>([&](auto yc) BS_INL {
            Kn::template section<decltype(yc)::value>(a, acc, stage, wave, lane, b0, nb0, has_next, first, ragged);
            lds_barrier();
        });
        Kn::finish(a, acc, wave, lane, b0, ragged);
        lds_barrier();
        if (!has_next) break;
        first = false;
        tix = ntix;
        tile = ntile;
    }
    wait_vm0();
}

}  // namespace bs
}  // namespace clay

namespace clay {
namespace bs {

// ===========================================================================
// v5: layer-per-lane register accumulators + a ring of node slots (16-byte DMA).
//
// v4 keeps the parity accumulators in LDS (64 KiB) and one 8 KiB stage per wave,
// so only one section (64 KiB per CU) is ever in flight and each section's wait
// is one section of compute after its issue.  v5 frees the LDS for data:
//  * lane (layer z, half pg) owns acc[p][plane] (32 VGPRs) for the whole tile --
//    every (line, column) step of the reference's per-layer loop is one (layer,
//    section) pair of this lane, so no accumulator ever moves;
//  * LDS = 10 node slots of alpha x 64 B = 160 KiB; data node n of a tile always
//    lives in slot n.  A section's slots are refilled with the NEXT tile's
//    section as soon as every wave has read them (right after the next section's
//    barrier), so each section's DMA is issued two sections before it is read;
//  * slot image: 16-byte piece (layer, pg, d) at bank slot B.(layer|pg<<8|d<<9)
//    ^ H.node, rows completing a GF(2) bijection (tools/v5_layout_search.py):
//    own reads (node x, layer z) and companion reads (node z_Y, layer z with
//    digit Y := x) of every section are bank-conflict free on ds_read_b128;
//  * lane bits 0-1 = digit t-1 of z, so the PFT partners of the parity
//    y-section are a lane quad: exchange via DPP quad_perm, no LDS.
// One barrier per section; waits are counted vmcnt (DMA and the asm parity
// stores are the only VMEM ops in flight).
// ===========================================================================
namespace v5 {
constexpr uint32_t BM[4] = {0x297, 0x134, 0x328, 0x62};  // bank bit o = <v, BM[o]> ^ <node, HM[o]>
constexpr uint32_t HM[4] = {0, 0, 2, 0};
constexpr int par10(uint32_t v) { int p = 0; for (; v; v &= v - 1) p ^= 1; return p; }
struct Lin {
    uint16_t fwd[10];  // column i: piece index (row << 4 | bank) of unit vector e_i
    uint16_t inv[10];  // column i: v of piece-index unit vector e_i
};
constexpr Lin make_lin() {
    Lin L{};
    // rows 4..9 of M: unit vectors completing the row space of BM
    uint32_t rows[10] = {BM[0], BM[1], BM[2], BM[3], 0, 0, 0, 0, 0, 0};
    int nr = 4;
    for (int b = 0; b < 10 && nr < 10; b++) {
        // is e_b independent of rows[0..nr)?  reduce by Gaussian elimination
        uint32_t basis[10] = {};
        int piv[10] = {};
        int nb = 0;
        for (int r = 0; r < nr; r++) {
            uint32_t v = rows[r];
            for (int i = 0; i < nb; i++)
                if ((v >> piv[i]) & 1) v ^= basis[i];
            if (v) { int p = 0; while (!((v >> p) & 1)) p++; basis[nb] = v; piv[nb] = p; nb++; }
        }
        uint32_t v = 1u << b;
        for (int i = 0; i < nb; i++)
            if ((v >> piv[i]) & 1) v ^= basis[i];
        if (v) rows[nr++] = 1u << b;
    }
    // piece index bit layout: bank bits 0..3 = rows 0..3, row bits 4..9 = rows 4..9
    for (int i = 0; i < 10; i++) {
        uint16_t p = 0;
        for (int r = 0; r < 10; r++)
            if ((rows[r] >> i) & 1) p |= uint16_t(1u << r);
        L.fwd[i] = p;
    }
    // invert the 10x10 matrix whose column i is fwd[i]
    uint32_t a[10] = {}, inv[10] = {};
    for (int r = 0; r < 10; r++) {
        for (int i = 0; i < 10; i++)
            if ((L.fwd[i] >> r) & 1) a[r] |= 1u << i;
        inv[r] = 1u << r;
    }
    for (int c = 0; c < 10; c++) {
        int p = c;
        while (!((a[p] >> c) & 1)) p++;
        uint32_t t = a[p]; a[p] = a[c]; a[c] = t;
        t = inv[p]; inv[p] = inv[c]; inv[c] = t;
        for (int r = 0; r < 10; r++)
            if (r != c && ((a[r] >> c) & 1)) { a[r] ^= a[c]; inv[r] ^= inv[c]; }
    }
    // inv[r] is row r of M^-1: v bit r = <p, inv[r]>; store columns
    for (int i = 0; i < 10; i++) {
        uint16_t col = 0;
        for (int r = 0; r < 10; r++)
            if ((inv[r] >> i) & 1) col |= uint16_t(1u << r);
        L.inv[i] = col;
    }
    return L;
}
constexpr Lin LIN = make_lin();
constexpr uint32_t fwd_c(uint32_t v) { uint32_t p = 0; for (int i = 0; i < 10; i++) if ((v >> i) & 1) p ^= LIN.fwd[i]; return p; }
constexpr uint32_t inv_c(uint32_t p) { uint32_t v = 0; for (int i = 0; i < 10; i++) if ((p >> i) & 1) v ^= LIN.inv[i]; return v; }
constexpr uint32_t hbank(int node) {
    uint32_t b = 0;
    for (int o = 0; o < 4; o++) b |= uint32_t(par10(uint32_t(node) & HM[o])) << o;
    return b;
}
static_assert(inv_c(fwd_c(0x2A5)) == 0x2A5 && inv_c(fwd_c(0x13F)) == 0x13F, "layout bijection");
__device__ __forceinline__ uint32_t fwd_d(uint32_t v) {
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) p ^= ((v >> i) & 1) ? uint32_t(LIN.fwd[i]) : 0u;
    return p;
}
__device__ __forceinline__ uint32_t inv_d(uint32_t p) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) v ^= ((p >> i) & 1) ? uint32_t(LIN.inv[i]) : 0u;
    return v;
}
}  // namespace v5

template <int KD, int M>
struct Bs5Kernel {
    using S = Shape<KD, M>;
    static constexpr int Q = S::Q, T = S::T, ALPHA = S::ALPHA;
    static_assert(KD == 10 && M == 4 && Q == 4 && T == 4 && ALPHA == 256,
                  "v5 layout and slot ring are derived for (10,4,13)");
    static constexpr int PG = 2, W = 64, BLOCK = ALPHA * PG, WAVES = BLOCK / 64;
    static constexpr int SLOT = ALPHA * W;                 // 16 KiB per data node
    static constexpr int LDS_BYTES = KD * SLOT;            // 160 KiB
    static constexpr int NDMA = SLOT / 1024 / WAVES;       // per wave per node: 2
    static constexpr int STORES = Q * 2;

    template <int Y>
    static constexpr int nreal() { int n = 0; for (int x = 0; x < Q; x++) n += (Y * Q + x < KD); return n; }
    template <int Y>
    static constexpr int ndma() { return nreal<Y>() * NDMA; }
    static constexpr int dshift(int y) { return 2 * (T - 1 - y); }

    // byte offset inside the tile of piece v = layer | pg << 8 | d << 9
    __device__ static uint32_t piece_off(uint32_t v) { return ((v >> 8) & 1u) * 32u + (v >> 9) * 16u; }

    __device__ static int lane_z(int l) { return ((l >> 3) << 2) | (l & 3); }
    __device__ static int lane_pg(int l) { return (l >> 2) & 1; }

    // DMA of data y-section Y of the tile at b0 into the node slots.  Wave w
    // writes pieces [1024 (NDMA w + i), +1024) of each node slot.
    template <int Y>
    __device__ static void dma(const BsArgs &a, uint32_t lds0, int wave, int lane, uint32_t b0) {
        const uint32_t sc = uint32_t(a.sc);
        uint32_t vl = v5::inv_d(uint32_t(lane));
        asm volatile("" : "+v"(vl));  // recompute per call: keeps ~20 offsets out of the live set
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            constexpr int node = Y * Q + x;
            if constexpr (node < KD) {
#pragma unroll
                for (int i = 0; i < NDMA; i++) {
                    const uint32_t blk = uint32_t(wave * NDMA + i);  // 1 KiB block = piece bits 6..9
                    const uint32_t v = vl ^ v5::inv_d((blk << 6) ^ v5::hbank(node));
                    uint32_t pos = b0 + piece_off(v);
                    if (pos + 16u > sc) pos = sc - 16u;  // ragged: patched after landing
                    dma16(lds0 + uint32_t(node * SLOT) + blk * 1024u, a.data[node], (v & 255u) * sc + pos);
                }
            }
        });
    }
    template <int Y>
    __device__ static void patch(const BsArgs &a, uint8_t *lds, int wave, int lane, uint32_t b0) {
        const uint32_t sc = uint32_t(a.sc);
        uint32_t vl = v5::inv_d(uint32_t(lane));
        asm volatile("" : "+v"(vl));  // recompute per call: keeps ~20 offsets out of the live set
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            constexpr int node = Y * Q + x;
            if constexpr (node < KD) {
#pragma unroll
                for (int i = 0; i < NDMA; i++) {
                    const uint32_t blk = uint32_t(wave * NDMA + i);
                    const uint32_t v = vl ^ v5::inv_d((blk << 6) ^ v5::hbank(node));
                    const uint32_t pos = b0 + piece_off(v);
                    if (pos < sc && pos + 16u > sc) {
                        const uint2 g = *reinterpret_cast<const uint2 *>(a.data[node] + (v & 255u) * sc + pos);
                        *reinterpret_cast<uint4 *>(lds + node * SLOT + blk * 1024 + lane * 16) =
                            make_uint4(g.x, g.y, 0u, 0u);
                    }
                }
            }
        });
    }

    __device__ static void read32(const uint8_t *lds, uint32_t off0, uint32_t off1, uint32_t (&d)[8]) {
        const uint4 v0 = *reinterpret_cast<const uint4 *>(lds + off0);
        const uint4 v1 = *reinterpret_cast<const uint4 *>(lds + off1);
        d[0] = v0.x; d[1] = v0.y; d[2] = v0.z; d[3] = v0.w;
        d[4] = v1.x; d[5] = v1.y; d[6] = v1.z; d[7] = v1.w;
    }

    template <int Y, int P, int BO>
    static constexpr uint64_t rs_mask() {
        uint64_t m = 0;
        for (int x = 0; x < Q; x++) m |= plane_mask(S::RS.g[P][Y * Q + x], BO, 8 * x);
        return m;
    }
    template <int BO>
    static constexpr uint64_t pft_mask() {
        return plane_mask(S::DINV, BO, 0) | plane_mask(gm(S::DINV, 2), BO, 8);
    }

    // Section Y: stage -> U (PRT) -> bit planes -> acc += RS.
    template <int Y>
    __device__ static void section(const uint8_t *lds, int z, int pg, uint32_t (&acc)[Q * 8]) {
        constexpr int sh = dshift(Y);
        const int zy = (z >> sh) & 3;
        const bool creal = (Y * Q + zy) < KD;
        // piece index of (layer, pg, d=0) with digit Y cleared, and of the own layer
        const uint32_t fown = v5::fwd_d(uint32_t(z) | uint32_t(pg << 8));
        const uint32_t fcl = v5::fwd_d(uint32_t(z & ~(3 << sh)) | uint32_t(pg << 8));
        const int cnode = Y * Q + (creal ? zy : 0);
        const uint32_t cbase = uint32_t(cnode * SLOT);
        // node-dependent bank XOR of the companion node (lane-dependent node)
        uint32_t hb = 0;
#pragma unroll
        for (int o = 0; o < 4; o++) hb |= uint32_t(v5::par10(uint32_t(cnode) & v5::HM[o]) & 1) << o;
        constexpr uint32_t FD = v5::fwd_c(1u << 9);
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            constexpr int node = Y * Q + x;
            uint32_t o[8], c[8];
            if constexpr (node < KD) {
                constexpr uint32_t hn = v5::hbank(node);
                read32(lds, uint32_t(node * SLOT) + 16u * (fown ^ hn), uint32_t(node * SLOT) + 16u * (fown ^ hn ^ FD), o);
            } else {
#pragma unroll
                for (int w = 0; w < 8; w++) o[w] = 0;
            }
            constexpr uint32_t FX = v5::fwd_c(uint32_t(x) << sh);
            const uint32_t cp = fcl ^ FX ^ hb;
            if (creal) {
                read32(lds, cbase + 16u * cp, cbase + 16u * (cp ^ FD), c);
            } else {
#pragma unroll
                for (int w = 0; w < 8; w++) c[w] = 0;
            }
            const uint32_t keep = (creal && x != zy) ? 0xffffffffu : 0u;
            const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
            uint32_t u[8];
#pragma unroll
            for (int w = 0; w < 8; w++) u[w] = xor_xtime4_masked(o[w], c[w], ks, kr);
            transpose8(u);
            // fold this node's U into every parity accumulator: acc[p] ^= g[p][Yq+x] * U[x]
            sfor<Q>([&](auto pc) BS_INL {
                constexpr int p = decltype(pc)::value;
                sfor<8>([&](auto bc) BS_INL {
                    constexpr int bo = decltype(bc)::value;
                    constexpr uint64_t mk = plane_mask(S::RS.g[p][Y * Q + x], bo, 0);
                    acc[p * 8 + bo] = xor_sel<mk, (Y > 0 || x > 0)>(acc[p * 8 + bo], u);
                });
            });
        });
    }

    __device__ static uint8_t *par_of(const BsArgs &a, int x) {
        uint64_t r = reinterpret_cast<uint64_t>(a.par[0]);
        asm volatile("" : "+s"(r));
#pragma unroll
        for (int i = 1; i < Q; i++) {
            uint64_t pi = reinterpret_cast<uint64_t>(a.par[i]);
            asm volatile("" : "+s"(pi));
            r = (x == i) ? pi : r;
        }
        return reinterpret_cast<uint8_t *>(r);
    }

    template <int K>
    __device__ static uint32_t qxor(uint32_t v) {
        constexpr int ctrl = K == 1 ? 0xB1 : K == 2 ? 0x4E : 0x1B;  // quad_perm lane ^ K
        return uint32_t(__builtin_amdgcn_mov_dpp(int(v), ctrl, 0xF, 0xF, true));
    }

    // PFT of the parity y-section (digit t-1 = lane bits 0-1) and the parity stores.
    __device__ static void finish(const BsArgs &a, const uint32_t (&acc)[Q * 8], int z, int pg, uint32_t b0,
                                  bool ragged) {
        const uint32_t sc = uint32_t(a.sc);
        const int d3 = z & 3;
        const uint32_t m0 = (d3 & 1) ? 0xffffffffu : 0u, m1 = (d3 & 2) ? 0xffffffffu : 0u;
        const uint32_t pos = b0 + uint32_t(32 * pg);
        const int nv = pos >= sc ? 0 : ((sc - pos) / 8 > 4 ? 4 : int((sc - pos) / 8));
        const uint32_t off = uint32_t(z) * sc + pos;
        sfor<Q>([&](auto kc) BS_INL {
            constexpr int k = decltype(kc)::value;
            // s = acc[d3 ^ k] (8 planes): select on the two index bits, flipped by k
            uint32_t s[8];
#pragma unroll
            for (int w = 0; w < 8; w++) {
                const uint32_t a0 = acc[(0 ^ k) * 8 + w], a1 = acc[(1 ^ k) * 8 + w];
                const uint32_t a2 = acc[(2 ^ k) * 8 + w], a3 = acc[(3 ^ k) * 8 + w];
                s[w] = sel(m1, sel(m0, a3, a2), sel(m0, a1, a0));
            }
            uint32_t c[8];
            if constexpr (k == 0) {
#pragma unroll
                for (int w = 0; w < 8; w++) c[w] = s[w];
            } else {
                uint32_t in[16];
#pragma unroll
                for (int w = 0; w < 8; w++) { in[w] = s[w]; in[8 + w] = qxor<k>(s[w]); }
                sfor<8>([&](auto bc) BS_INL {
                    c[decltype(bc)::value] = xor_sel<pft_mask<decltype(bc)::value>(), false>(0u, in);
                });
            }
            transpose8(c);
            uint8_t *p = par_of(a, d3 ^ k) + off;
            if (!ragged) {
                st16(p, c[0], c[1], c[2], c[3]);
                st16(p + 16, c[4], c[5], c[6], c[7]);
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++)
                    if (i < nv) *reinterpret_cast<uint2 *>(p + 8 * i) = make_uint2(c[2 * i], c[2 * i + 1]);
            }
        });
    }
};

template <int KD, int M>
__global__ __launch_bounds__((Bs5Kernel<KD, M>::BLOCK)) void k_bs5_encode(BsArgs a) {
    using Kn = Bs5Kernel<KD, M>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int z = Kn::lane_z(int(threadIdx.x)), pg = Kn::lane_pg(int(threadIdx.x));
    const uint32_t lds0 = lds_addr_of(smem);
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    uint32_t tix = slot;
    uint32_t tile = xcd * a.tiles_per_xcd + tix;
    if (tix >= a.tiles_per_xcd || tile >= a.ntiles) return;
    {
        const uint32_t b0 = tile * uint32_t(Kn::W);
        Kn::template dma<0>(a, lds0, wave, lane, b0);
        Kn::template dma<1>(a, lds0, wave, lane, b0);
        Kn::template dma<2>(a, lds0, wave, lane, b0);
    }
    bool first = true;
    uint32_t acc[Kn::Q * 8];
    while (true) {
        const uint32_t b0 = tile * uint32_t(Kn::W);
        const bool ragged = uint64_t(b0) + Kn::W > a.sc;
        const uint32_t ntix = tix + a.nslots, ntile = xcd * a.tiles_per_xcd + ntix;
        const bool has_next = ntix < a.tiles_per_xcd && ntile < a.ntiles;
        const uint32_t nb0 = ntile * uint32_t(Kn::W);
        // section 0: younger than its DMA: S1 (+ S2 on the first tile) or S1 + last stores
        if (first) wait_vm_n<Kn::template ndma<1>() + Kn::template ndma<2>()>();
        else wait_vm_n<Kn::template ndma<1>() + Kn::STORES>();
        if (ragged) Kn::template patch<0>(a, smem, wave, lane, b0);
        lds_barrier();
        if (!first) Kn::template dma<2>(a, lds0, wave, lane, b0);  // S2 slots <- this tile's S2
        Kn::template section<0>(smem, z, pg, acc);
        // section 1
        if (first) wait_vm_n<Kn::template ndma<2>()>();
        else wait_vm_n<Kn::STORES + Kn::template ndma<2>()>();
        if (ragged) Kn::template patch<1>(a, smem, wave, lane, b0);
        lds_barrier();
        if (has_next) Kn::template dma<0>(a, lds0, wave, lane, nb0);  // S0 slots <- next tile
        Kn::template section<1>(smem, z, pg, acc);
        // section 2
        if (has_next) wait_vm_n<Kn::template ndma<0>()>();
        else wait_vm_n<0>();
        if (ragged) Kn::template patch<2>(a, smem, wave, lane, b0);
        lds_barrier();
        if (has_next) Kn::template dma<1>(a, lds0, wave, lane, nb0);  // S1 slots <- next tile
        Kn::template section<2>(smem, z, pg, acc);
        Kn::finish(a, acc, z, pg, b0, ragged);
        if (!has_next) break;
        first = false;
        tix = ntix;
        tile = ntile;
    }
    wait_vm0();
}

}  // namespace bs
}  // namespace clay
