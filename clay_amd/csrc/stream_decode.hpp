// stream_decode.hpp -- the shared phase A of the streaming decodes for codes with q = 4, t = 4
// (alpha = 256), e.g. the BASELINE (10,4,13): the local decode (stream_local.hpp) and the fused
// decode v2 (stream_fused2.hpp) instantiate StreamDec and add their own iscore solve.
//
// Algebra (syndrome form of decode_layered / decode_uncoupled_layer, decode.rs:260-408).
// Per layer z the RS step sees the 16 uncoupled values U(i, z); H = [G | I] is the 4 x 16
// parity-check matrix of the RS(12,4) generator (G = its parity rows, compile time).  The
// reference reconstructs from the first 12 present shards ("used" set; reed-solomon-erasure
// 6.0.0 reconstruct) -- the unique codeword through them -- so with K = the 4 other nodes
// (erased + ignored) U_K(z) = H_K^-1 * S(z), S(z) = sum_{i used} H_i U(i, z), bit for bit even on
// inputs that are not codewords.  U(i, z) of a used node is its PRT value (transforms.rs:42-55);
// where its companion is erased the term gamma * C(e, z') is unknown until the lower-iscore layer
// z' is solved, so:
//   phase A (streaming): S_known(z) = sum_i H_i U'(i, z) with those terms dropped, and
//            Out(e, z) = gamma * C(companion of e at z) for erased e (compute_c_from_u_and_cstar)
//   phase B (rounds in iscore order): C(e, z) = row e of H_K^-1 S(z)
//            + sum over the dropped terms A_(y,x)[e] C(e_y, z[y:=x])  (A = H_K^-1 gamma H_(y,x)).
// Out needs no storage: S += H_e Out(e, z) in phase A (H_K H_K^-1 = I, so row e of H_K^-1 S
// becomes U_e + Out_e = C_e directly; Out = 0 where e is red).
//
// Phase A tile and lane map.  A workgroup owns W = 64 byte positions of every (node, layer) row.
// Section G (template, 3) is the lane's "slot" digit: lane (column c = the other three digits,
// part p) owns the four layers (c, g = 0..3) x 8 positions = 32 symbols = one bit-sliced dword
// per plane, so section G's PRT pairs stay inside the lane and the other sections' companions
// are read from LDS.  Node buffer (LDS, 16 KiB) = one node x 256 layers x 64 B; row (c, g) at
// c * 256 + (g ^ (c & 3)) * 64 (own and companion ds_read_b64 bank-conflict free; one 1 KiB
// LDS-DMA instruction = 4 columns = 16 whole 64-B row runs).  One step per section: its alive
// nodes stream through a ring of node buffers filled by 4 dedicated loader waves.
//
// Phase B (the iscore rounds, decode.rs:196-254) is kernel specific: in registers and wave
// shuffles in k_stream_local, on dedicated solver waves with LDS atomics in k_stream_fused2.
#pragma once

#include "decode_args.hpp"
#include "kernels.hpp"
#include "stream_encode.hpp"  // uniform_ptr, bit-slice helpers
#include "xor_cse.hpp"

namespace clay {
namespace bs {



// tables read through the constant address space: uniform-address loads become s_load
typedef const __attribute__((address_space(4))) uint32_t *cu32p;
__device__ __forceinline__ GfTab load_tab_c(cu32p t) {
    GfTab r;
    r.w0 = t[0];
    r.w1 = t[1];
    r.w2 = t[2];
    r.w3 = t[3];
    r.w4 = t[4];
    return r;
}

// an opaque copy of a per-lane value: everything derived from it is recomputed where it is
// used instead of being hoisted out of the tile loop into long-lived (spilled) registers
__device__ __forceinline__ uint32_t opq(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}

template <int KD, int G>
struct StreamDec {
    using S = Shape<KD, 4>;
    static_assert(S::Q == 4 && S::T == 4 && S::K == 12, "q = 4, t = 4, 12 RS data rows");
    static constexpr int W = 64, CWAVES = 8, LOADERS = 4, BLOCK = 64 * (CWAVES + LOADERS);
    static constexpr int BUF = 16384;                // one node: 256 layers x 64 B
    static constexpr int LDS_BYTES = 10 * BUF;       // ring + exchange buffers
    static constexpr int BPL = 16 / LOADERS;         // 1 KiB blocks per node buffer per loader wave

    // H = [G | I]: check p, internal node i
    static constexpr uint8_t H(int p, int i) { return i < S::K ? S::RS.g[p][i] : uint8_t(i - S::K == p ? 1 : 0); }
    static constexpr int cd(int k) { return k < G ? k : k + 1; }  // column digit k -> section
    static constexpr int ck(int y) { return y < G ? y : y - 1; }  // section (!= G) -> column digit
    static constexpr int csh(int y) { return 2 * (2 - ck(y)); }   // shift of section y's digit in c
    static constexpr uint32_t wt(int y) { return 1u << (2 * (3 - y)); }  // layer weight 4^(3-y)

    __host__ __device__ static uint32_t layer0(uint32_t c) {
        uint32_t z = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) z += ((c >> (2 * (2 - k))) & 3u) * wt(cd(k));
        return z;
    }
    // the same with the column digits at run-time positions a.csh[y] (k_stream_local)
    __device__ static uint32_t layer0_rt(const DecArgs &a, uint32_t c) {
        uint32_t z = 0;
#pragma unroll
        for (int y = 0; y < 4; y++)
            if (y != G) z += ((c >> a.csh[y]) & 3u) * wt(y);
        return z;
    }
    // byte offset of row (c, g) within a node buffer
    __device__ static uint32_t row(uint32_t c, uint32_t g) { return c * 256u + ((g ^ (c & 3u)) << 6); }

    // 8 dwords = the lane's 4 slots x 8 positions of one node at column cc.  SWZ (k_stream_fused2's
    // lane map, digit 2 of the column wave-uniform): the row swizzle comes from digit 1 instead,
    // row (c, g) at c * 256 + (g ^ ((c >> 2) & 3)) * 64 -- the digit that varies across the lanes of
    // a 32-lane ds_read_b64 group there, so own and companion reads stay conflict free
    template <bool SWZ = false>
    __device__ static void read4(const uint8_t *buf, uint32_t cc, uint32_t poff, uint32_t (&d)[8]) {
        const uint32_t b = cc * 256u + poff, cl = SWZ ? ((cc >> 2) & 3u) : (cc & 3u);
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const uint2 v = *reinterpret_cast<const uint2 *>(buf + (b + ((uint32_t(g) ^ cl) << 6)));
            d[2 * g] = v.x;
            d[2 * g + 1] = v.y;
        }
    }
    __device__ static void write4(uint8_t *buf, uint32_t cc, uint32_t poff, const uint32_t (&d)[8]) {
        const uint32_t b = cc * 256u + poff, cl = cc & 3u;
#pragma unroll
        for (int g = 0; g < 4; g++)
            *reinterpret_cast<uint2 *>(buf + (b + ((uint32_t(g) ^ cl) << 6))) = make_uint2(d[2 * g], d[2 * g + 1]);
    }

    // S[p] (8 planes) ^= f * H(p, I) * u, f = gamma if GAMMA; through compile-time common
    // subexpressions of the 32 rows (xor_cse.hpp)
    template <int I, bool GAMMA>
    struct FoldCse {
        static constexpr XorCse make() {
            uint32_t rows[32] = {};
            for (int p = 0; p < 4; p++) {
                const uint8_t h = GAMMA ? gm(2, H(p, I)) : H(p, I);
                for (int bo = 0; bo < 8; bo++) rows[p * 8 + bo] = uint32_t(plane_mask(h, bo, 0));
            }
            return make_xor_cse(rows);
        }
        static constexpr XorCse C = make();
    };
    template <int I, bool GAMMA>
    __device__ static void fold(const uint32_t (&u)[8], uint32_t (&s)[32]) {
        cse_fold<FoldCse<I, GAMMA>, 32, true>(u, s);
    }

    // ---------------- tile map ----------------
    struct Tile {
        uint32_t b0, vend;
    };
    struct Map {
        uint32_t x0, x1, n;
        __device__ __forceinline__ Map(uint32_t sc, uint32_t region, uint32_t ns, uint32_t xcd, uint32_t slot) {
            x0 = xcd * region;
            x1 = x0 + region < sc ? x0 + region : sc;
            n = 0;
            if (x0 < x1) {
                const uint32_t nt = (x1 - x0 + uint32_t(W) - 1) / uint32_t(W);
                n = nt > slot ? (nt - slot + ns - 1) / ns : 0;
            }
        }
        __device__ __forceinline__ Tile tile(uint32_t k, uint32_t slot, uint32_t ns) const {
            const uint32_t b0 = x0 + (slot + k * ns) * uint32_t(W);
            return {b0, b0 + uint32_t(W) < x1 ? b0 + uint32_t(W) : x1};
        }
    };

    // ---------------- loader ----------------
    struct Loader {
        uint32_t off[BPL];  // layer(c, g) * sc + 16 * piece, per block
        uint32_t pc16;      // 16 * piece
    };
    template <bool SWZ = false>
    __device__ static void loader_init(Loader &L, uint32_t sc, int li, int lane) {
        const uint32_t k = uint32_t(lane);
        L.pc16 = (k & 3u) * 16u;
#pragma unroll
        for (int j = 0; j < BPL; j++) {
            const uint32_t cc = uint32_t(li * BPL + j) * 4u + (k >> 4);
            // the layer whose row lands in 64-byte slot (k >> 2) & 3 of column cc (read4's swizzle)
            const uint32_t g = ((k >> 2) & 3u) ^ (SWZ ? ((cc >> 2) & 3u) : (k >> 4));
            L.off[j] = (layer0(cc) + g * wt(G)) * sc + L.pc16;
        }
    }
    __device__ static void loader_init_rt(Loader &L, const DecArgs &a, int li, int lane) {
        const uint32_t k = uint32_t(lane), sc = uint32_t(a.sc);
        L.pc16 = (k & 3u) * 16u;
#pragma unroll
        for (int j = 0; j < BPL; j++) {
            const uint32_t cc = uint32_t(li * BPL + j) * 4u + (k >> 4);
            const uint32_t g = ((k >> 2) & 3u) ^ (k >> 4);
            L.off[j] = (layer0_rt(a, cc) + g * wt(G)) * sc + L.pc16;
        }
    }
    __device__ static void issue(const DecArgs &a, const Loader &L, uint32_t lds_buf, const uint8_t *node, Tile t,
                                 int li) {
        lds_buf = __builtin_amdgcn_readfirstlane(lds_buf);
        if (t.vend >= t.b0 + uint32_t(W)) {
            const uint8_t *base = uniform_ptr(node + t.b0);
#pragma unroll
            for (int j = 0; j < BPL; j++) dma16(lds_buf + uint32_t(li * BPL + j) * 1024u, base, L.off[j]);
        } else {
            // partial tile: a piece straddling vend is read from vend - 16 (the compute lane
            // of that part reads the slot's upper half), a piece wholly past vend from b0
            const uint8_t *base = uniform_ptr(node);
            uint32_t pos = t.b0 + L.pc16;
            if (pos + 16u > t.vend) pos = t.vend - 16u;  // past vend: unused; vend >= 16 (sc >= 512)
#pragma unroll
            for (int j = 0; j < BPL; j++)
                dma16(lds_buf + uint32_t(li * BPL + j) * 1024u, base, L.off[j] - L.pc16 + pos);
        }
    }

    // ---------------- phase A: one step per section (decode.rs:260-329, transforms.rs:42-89) ----------------
    // S (4 checks x 8 planes, the lane's 4 layers x 8 positions) += sum_i H_i U'(i) + H_e Out(e);
    // section Y's alive nodes are loads qbase + sec_off[Y] .. of the ring (buffer = load % ring).
    // RT (k_stream_local): column digits at a.csh[y], and any number of erased nodes in section G
    // tbar (timing probe of k_stream_fused2 only): cycles spent in the four step barriers
    // SB: a scheduling barrier after every node's fold (one node's values live at a time)
    //
    // k_stream_fused2 (RT = false) dispatches each step on a.scase[Y] (engine.hip dec_setup): the
    // section's erased node XE (4: none) when every other node of the section is used, so the
    // step runs a copy with the section's structure (alive / used / erased) at compile time --
    // straight-line PRT + fold code without the per-node branches, which the scheduler interleaves
    // across nodes; -1 (an ignored node in the section: fewer than 4 erasures) takes the run-time
    // copy.  PROBE 128 (probe library): always the run-time copy.
    // SWZ (k_stream_fused2): read4's digit-1 swizzle, and the light section-2 step below
    template <int PROBE, bool RT = false, bool SB = true, bool MULTI = false, bool SWZ = false>
    __device__ __forceinline__ static void phase_a(const DecArgs &a, uint8_t *smem, uint32_t qbase, uint32_t c0, uint32_t poff0, int xeG,
                                   uint32_t (&S)[32], uint32_t R, uint64_t *tbar = nullptr) {
        sfor<4>([&](auto yc) BS_INL {
            constexpr int Y = decltype(yc)::value;
            if (tbar) {
                const uint64_t t0 = __builtin_amdgcn_s_memtime();
                lds_barrier();
                *tbar += __builtin_amdgcn_s_memtime() - t0;
            } else {
                lds_barrier();  // step (k, Y) landed (the loaders waited before this barrier)
            }
            // k_stream_fused2 split step (the ring held only part of this section's loads during
            // the step before): the loaders issue the rest after the barrier above, wait, and join
            // this second one
            if ((a.split >> Y) & 1u) lds_barrier();
            if constexpr ((PROBE & 2) != 0) return;
            if constexpr (!RT && (PROBE & 128) == 0) {
                switch (a.scase[Y]) {
                case 0: section<Y, 0, false, SB, MULTI, SWZ>(a, smem, qbase, c0, poff0, xeG, S, R); break;
                case 1: section<Y, 1, false, SB, MULTI, SWZ>(a, smem, qbase, c0, poff0, xeG, S, R); break;
                case 2: section<Y, 2, false, SB, MULTI, SWZ>(a, smem, qbase, c0, poff0, xeG, S, R); break;
                case 3: section<Y, 3, false, SB, MULTI, SWZ>(a, smem, qbase, c0, poff0, xeG, S, R); break;
                case 4: section<Y, 4, false, SB, MULTI, SWZ>(a, smem, qbase, c0, poff0, xeG, S, R); break;
                default: section<Y, -1, false, SB, MULTI, SWZ>(a, smem, qbase, c0, poff0, xeG, S, R); break;
                }
            } else {
                section<Y, -1, RT, SB, MULTI, SWZ>(a, smem, qbase, c0, poff0, xeG, S, R);
            }
        });
    }

    // shortened internal nodes of section y (i in [KD, 12): zero data, never loaded, always used)
    static constexpr uint32_t short_nib(int y) {
        uint32_t m = 0;
        for (int x = 0; x < 4; x++)
            if (4 * y + x >= KD && 4 * y + x < S::K) m |= 1u << x;
        return m;
    }

    // one step of phase A.  XE >= 0: the compile-time structure of scase XE (node (Y, XE) erased,
    // XE = 4: none; every other node used); XE = -1: the pattern's masks at run time
    // MULTI (k_stream_fused2<.., TWO>): the run-time copy also takes two erasures in section G
    template <int Y, int XE, bool RT, bool SB, bool MULTI = false, bool SWZ = false>
    __device__ __forceinline__ static void section(const DecArgs &a, uint8_t *smem, uint32_t qbase, uint32_t c0, uint32_t poff0,
                                   int xeG, uint32_t (&S)[32], uint32_t R) {
        constexpr bool CT = XE >= 0;
        constexpr uint32_t kEm = (CT && XE < 4) ? 1u << XE : 0u;
        constexpr uint32_t kAlive = 15u & ~short_nib(Y) & ~kEm;
        const uint32_t c = opq(c0), poff = opq(poff0);
        // the run-time copy's masks, opaque per step: the branch conditions derived from them are
        // not hoisted out of the tile loop into long-lived (spilled) scalar registers
        uint32_t alive_all = __builtin_amdgcn_readfirstlane(a.alive), used_all = __builtin_amdgcn_readfirstlane(a.used),
                 emY = __builtin_amdgcn_readfirstlane(a.emask[Y]);
        if constexpr (!CT && !RT) asm volatile("" : "+s"(alive_all), "+s"(used_all), "+s"(emY));
        const uint32_t aliveY = CT ? kAlive : ((alive_all >> (4 * Y)) & 15u);
        const uint32_t rs = a.sec_off[Y];
        auto buf_of = [&](uint32_t x) BS_INL {  // node (Y, x) buffer (x alive)
            const uint32_t q = rs + uint32_t(__builtin_popcount(aliveY & ((1u << x) - 1u)));
            return smem + ((qbase + q) % R) * BUF;
        };
        if constexpr (Y != G) {
            const uint32_t sh = RT ? a.csh[Y] : uint32_t(csh(Y));
            const uint32_t cy = (c >> sh) & 3u;
            if constexpr (SWZ && Y == 2 && csh(2) == 0) {
                // k_stream_fused2's lane map makes digit 2 wave-uniform: where node (2, cy) is a
                // shortened one (zero data), every PRT companion of the step is zero -- U = C for
                // the alive used nodes, U = 0 for the shortened ones and Out = 0 for an erased one
                // (no term): plain folds, no companion reads.  These light steps fall to waves 4-7,
                // the younger wave of each SIMD (it loses the VALU arbitration; round-6 timing:
                // 47 % slower on the same work)
                const uint32_t cyu = __builtin_amdgcn_readfirstlane(cy);
                if (4u * uint32_t(Y) + cyu >= uint32_t(KD) && 4u * uint32_t(Y) + cyu < uint32_t(S::K)) {
                    sfor<4>([&](auto xc) BS_INL {
                        constexpr int X = decltype(xc)::value;
                        constexpr int I = 4 * Y + X;
                        const bool alive_i = (aliveY >> X) & 1u;
                        const bool used_i = CT ? X != XE : ((used_all >> I) & 1u);
                        if (!(alive_i && used_i)) return;
                        uint32_t u[8];
                        read4<SWZ>(buf_of(X), c, poff, u);
                        transpose8(u);
                        fold<I, false>(u, S);
                        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
                    });
                    asm volatile("; phase A light copy %0" ::"i"(XE + 1));
                    return;
                }
            }
            const bool comp_alive = (aliveY >> cy) & 1u;
            const uint8_t *cbuf = comp_alive ? buf_of(cy) : smem;
            sfor<4>([&](auto xc) BS_INL {
                constexpr int X = decltype(xc)::value;
                constexpr int I = 4 * Y + X;
                const bool alive_i = (aliveY >> X) & 1u;
                const bool used_i = CT ? X != XE : ((used_all >> I) & 1u);
                const bool erased_i = CT ? X == XE : ((emY >> X) & 1u);
                if (!(used_i || erased_i)) return;
                uint32_t o[8], cv[8], u[8];
                if (alive_i) {
                    read4<SWZ>(buf_of(X), c, poff, o);
                } else {
#pragma unroll
                    for (int w = 0; w < 8; w++) o[w] = 0;
                }
                const uint32_t cc = (c & ~(3u << sh)) | (uint32_t(X) << sh);
                read4<SWZ>(cbuf, cc, poff, cv);
                const uint32_t keep = (comp_alive && cy != uint32_t(X)) ? 0xffffffffu : 0u;
                const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
                if (erased_i) {  // S += H_e Out(e, z): Out = gamma * companion (0 where red)
                    uint32_t v[8];
#pragma unroll
                    for (int w = 0; w < 8; w++) v[w] = xor_xtime4_masked(0u, cv[w], ks, kr);
                    transpose8(v);
                    fold<I, false>(v, S);
                }
                if (used_i) {
#pragma unroll
                    for (int w = 0; w < 8; w++) u[w] = xor_xtime4_masked(o[w], cv[w], ks, kr);
                    transpose8(u);
                    fold<I, false>(u, S);
                }
                if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
            });
        } else {
            // section G: all four nodes' slots are in the lane; U(a, g) = C(a, g) + gamma C(g, a)
            uint32_t o[4][8];
            sfor<4>([&](auto xc) BS_INL {
                constexpr int X = decltype(xc)::value;
                if ((aliveY >> X) & 1u) {
                    read4<SWZ>(buf_of(X), c, poff, o[X]);
                } else {
#pragma unroll
                    for (int w = 0; w < 8; w++) o[X][w] = 0;
                }
            });
            if (RT || (MULTI && !CT && __builtin_popcount(emY) > 1)) {
                // every erased node (G, A): Out((G, A), slot g) = gamma * C((G, g), slot A), 0 at
                // slot A and where (G, g) has no data (erased: a both-erased pair, inverted later;
                // k_stream_local, and k_stream_fused2's run-time copy for two erasures in G)
                sfor<4>([&](auto ac) BS_INL {
                    constexpr int A = decltype(ac)::value;
                    if (!((emY >> A) & 1u)) return;
                    uint32_t v[8];
#pragma unroll
                    for (int g = 0; g < 4; g++) {
                        v[2 * g] = g == A ? 0u : gf_xt(o[g][2 * A]);
                        v[2 * g + 1] = g == A ? 0u : gf_xt(o[g][2 * A + 1]);
                    }
                    transpose8(v);
                    fold<4 * G + A, false>(v, S);
                    if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
                });
            } else if ((CT ? (XE < 4 ? XE : -1) : xeG) >= 0) {
                // Out(e_G, slot g) = gamma * C(node (G, g), slot xe), 0 at slot xe
                const int xe = CT ? XE : xeG;
                uint32_t v[8];
                sfor<4>([&](auto gc) BS_INL {
                    constexpr int g = decltype(gc)::value;
                    v[2 * g] = v[2 * g + 1] = 0;
                    sfor<4>([&](auto ac) BS_INL {
                        constexpr int A = decltype(ac)::value;
                        if (A != g && xe == A) {
                            v[2 * g] = gf_xt(o[g][2 * A]);
                            v[2 * g + 1] = gf_xt(o[g][2 * A + 1]);
                        }
                    });
                });
                transpose8(v);
                sfor<4>([&](auto ac) BS_INL {  // S += H_eG Out(e_G, .)
                    constexpr int A = decltype(ac)::value;
                    if (A == xe) fold<4 * G + A, false>(v, S);
                });
            }
            sfor<4>([&](auto ac) BS_INL {
                constexpr int A = decltype(ac)::value;
                constexpr int I = 4 * G + A;
                if (!(CT ? A != XE : ((used_all >> I) & 1u))) return;
                uint32_t u[8];
                sfor<4>([&](auto gc) BS_INL {
                    constexpr int g = decltype(gc)::value;
                    const uint32_t keep = (A != g && ((aliveY >> g) & 1u)) ? 0xffffffffu : 0u;
                    const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
                    u[2 * g] = xor_xtime4_masked(o[A][2 * g], o[g][2 * A], ks, kr);
                    u[2 * g + 1] = xor_xtime4_masked(o[A][2 * g + 1], o[g][2 * A + 1], ks, kr);
                });
                transpose8(u);
                fold<I, false>(u, S);
                if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
            });
        }
        // a distinct marker ends every copy: the copies' common tails are not sunk below phase_a's
        // switch (that merges S's elements behind pointer phis, which then live in scratch)
        asm volatile("; phase A copy %0" ::"i"(XE + 1));
    }

    // v_perm table i of a table block (8 dwords each, 5 used; decode_args.hpp)
    __device__ static GfTab tab_at(const uint8_t *tl, int i) {
        const uint4 v = *reinterpret_cast<const uint4 *>(tl + i * 32);
        return GfTab{v.x, v.y, v.z, v.w, *reinterpret_cast<const uint32_t *>(tl + i * 32 + 16)};
    }
};

}  // namespace bs
}  // namespace clay
