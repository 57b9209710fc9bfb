// stream_decode.hpp -- single-launch decode for codes with q = 4, t = 4 (alpha = 256), e.g. the
// BASELINE (10,4,13) with up to 4 erasures: every survivor byte is read from HBM once, every
// output byte written once, and all iscore rounds of the reference's layered decode
// (decode.rs:196-254) run inside the workgroup.
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
// Phase B: S_known goes to LDS; each round gives every lane ONE item (layer z, part p: 8
// positions) of one iscore level, layers sorted on the host by (level, set of red sections) so a
// wave's corrections are uniform.  A round only reads C of earlier rounds; C overwrites the
// item's own S slots.  The iscore dependency therefore costs a few short rounds instead of
// divergent passes over every lane.
//
// LDS (10 x 16 KiB): a ring of R = 10 node buffers; during phase B the S/C region (4 x 16 KiB,
// [j][z][p] x 8 B) reuses buffers R-4 .. R-1 and the tables buffer R-5, while the loaders
// prefetch the next tile's first five nodes into buffers 0 .. R-6.
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

    // 8 dwords = the lane's 4 slots x 8 positions of one node at column cc
    __device__ static void read4(const uint8_t *buf, uint32_t cc, uint32_t poff, uint32_t (&d)[8]) {
        const uint32_t b = cc * 256u + poff, cl = cc & 3u;
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
        __device__ Map(uint32_t sc, uint32_t region, uint32_t ns, uint32_t xcd, uint32_t slot) {
            x0 = xcd * region;
            x1 = x0 + region < sc ? x0 + region : sc;
            n = 0;
            if (x0 < x1) {
                const uint32_t nt = (x1 - x0 + uint32_t(W) - 1) / uint32_t(W);
                n = nt > slot ? (nt - slot + ns - 1) / ns : 0;
            }
        }
        __device__ Tile tile(uint32_t k, uint32_t slot, uint32_t ns) const {
            const uint32_t b0 = x0 + (slot + k * ns) * uint32_t(W);
            return {b0, b0 + uint32_t(W) < x1 ? b0 + uint32_t(W) : x1};
        }
    };

    // ---------------- loader ----------------
    struct Loader {
        uint32_t off[BPL];  // layer(c, g) * sc + 16 * piece, per block
        uint32_t pc16;      // 16 * piece
    };
    __device__ static void loader_init(Loader &L, uint32_t sc, int li, int lane) {
        const uint32_t k = uint32_t(lane);
        L.pc16 = (k & 3u) * 16u;
#pragma unroll
        for (int j = 0; j < BPL; j++) {
            const uint32_t cc = uint32_t(li * BPL + j) * 4u + (k >> 4);
            const uint32_t g = ((k >> 2) & 3u) ^ (k >> 4);
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
    template <int PROBE, bool RT = false, bool SB = true>
    __device__ static void phase_a(const DecArgs &a, uint8_t *smem, uint32_t qbase, uint32_t c0, uint32_t poff0, int xeG,
                                   uint32_t (&S)[32], uint32_t R, uint64_t *tbar = nullptr) {  // R: ring depth
        sfor<4>([&](auto yc) BS_INL {
            constexpr int Y = decltype(yc)::value;
            if (tbar) {
                const uint64_t t0 = __builtin_amdgcn_s_memtime();
                lds_barrier();
                *tbar += __builtin_amdgcn_s_memtime() - t0;
            } else {
                lds_barrier();  // step (k, Y) landed (the loaders waited before this barrier)
            }
            if constexpr ((PROBE & 2) != 0) return;
            const uint32_t c = opq(c0), poff = opq(poff0);
            const uint32_t aliveY = (a.alive >> (4 * Y)) & 15u;
            const uint32_t rs = a.sec_off[Y];
            auto buf_of = [&](uint32_t x) BS_INL {  // node (Y, x) buffer (x alive)
                const uint32_t q = rs + uint32_t(__builtin_popcount(aliveY & ((1u << x) - 1u)));
                return smem + ((qbase + q) % R) * BUF;
            };
            if constexpr (Y != G) {
                const uint32_t sh = RT ? a.csh[Y] : uint32_t(csh(Y));
                const uint32_t cy = (c >> sh) & 3u;
                const bool comp_alive = (aliveY >> cy) & 1u;
                const uint8_t *cbuf = comp_alive ? buf_of(cy) : smem;
                sfor<4>([&](auto xc) BS_INL {
                    constexpr int X = decltype(xc)::value;
                    constexpr int I = 4 * Y + X;
                    const bool alive_i = (aliveY >> X) & 1u;
                    const bool used_i = (a.used >> I) & 1u;
                    const bool erased_i = (a.emask[Y] >> X) & 1u;
                    if (!(used_i || erased_i)) return;
                    uint32_t o[8], cv[8], u[8];
                    if (alive_i) {
                        read4(buf_of(X), c, poff, o);
                    } else {
#pragma unroll
                        for (int w = 0; w < 8; w++) o[w] = 0;
                    }
                    const uint32_t cc = (c & ~(3u << sh)) | (uint32_t(X) << sh);
                    read4(cbuf, cc, poff, cv);
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
                        read4(buf_of(X), c, poff, o[X]);
                    } else {
#pragma unroll
                        for (int w = 0; w < 8; w++) o[X][w] = 0;
                    }
                });
                if constexpr (RT) {
                    // every erased node (G, A): Out((G, A), slot g) = gamma * C((G, g), slot A), 0 at
                    // slot A and where (G, g) has no data (erased: a both-erased pair, inverted later)
                    const uint32_t emG = a.emask[G];
                    sfor<4>([&](auto ac) BS_INL {
                        constexpr int A = decltype(ac)::value;
                        if (!((emG >> A) & 1u)) return;
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
                } else if (xeG >= 0) {  // Out(e_G, slot g) = gamma * C(node (G, g), slot xeG), 0 at slot xeG
                    uint32_t v[8];
                    sfor<4>([&](auto gc) BS_INL {
                        constexpr int g = decltype(gc)::value;
                        v[2 * g] = v[2 * g + 1] = 0;
                        sfor<4>([&](auto ac) BS_INL {
                            constexpr int A = decltype(ac)::value;
                            if (A != g && xeG == A) {
                                v[2 * g] = gf_xt(o[g][2 * A]);
                                v[2 * g + 1] = gf_xt(o[g][2 * A + 1]);
                            }
                        });
                    });
                    transpose8(v);
                    sfor<4>([&](auto ac) BS_INL {  // S += H_eG Out(e_G, .)
                        constexpr int A = decltype(ac)::value;
                        if (A == xeG) fold<4 * G + A, false>(v, S);
                    });
                }
                sfor<4>([&](auto ac) BS_INL {
                    constexpr int A = decltype(ac)::value;
                    constexpr int I = 4 * G + A;
                    if (!((a.used >> I) & 1u)) return;
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
        });

    }

    // ---------------- phase B: rounds in iscore order (decode.rs:196-254) ----------------
    // S/C region at scb0 ([j][z][p] x 8 B, 4 x 16 KiB), tables + layer order at tl; one
    // workgroup barrier per round (every wave of the block calls this).
    template <bool WORK, bool STORE = true>
    __device__ static void rounds(const DecArgs &a, uint8_t *scb0, const uint8_t *tl, Tile t, uint32_t c0, uint32_t p) {
        const uint32_t sc = uint32_t(a.sc);
        const uint32_t nround = a.nround;
        auto tab = [&](int t) BS_INL {
            const uint4 v = *reinterpret_cast<const uint4 *>(tl + t * 32);
            GfTab r;
            r.w0 = v.x;
            r.w1 = v.y;
            r.w2 = v.z;
            r.w3 = v.w;
            r.w4 = *reinterpret_cast<const uint32_t *>(tl + t * 32 + 16);
            return r;
        };
        for (uint32_t rd = 0; rd < nround; rd++) {
            lds_barrier();  // S of this tile / C of the previous round visible
            if (!WORK) continue;
            // up to two items per lane: layers round_start + lane/8 and + 64 (independent)
            sfor<2>([&](auto hc) BS_INL {
                constexpr int hh = decltype(hc)::value;
                const uint32_t li = a.round_start[rd] + opq(c0) + 64u * hh;
                if (li >= a.round_start[rd + 1]) return;
                const uint32_t z = tl[kDecOrder * 4 + li];
                const uint32_t pp = opq(p);
                const uint8_t *scb = scb0 + z * 64u + 8u * pp;
                // C_r = sum_j Hinv[e_r][j] * S_j (+ the dropped terms below)
                uint32_t U[4][2];
#pragma unroll
                for (int r = 0; r < 4; r++) U[r][0] = U[r][1] = 0;
                // straight-line (no per-row branches: rows r >= ne use zero tables), so the
                // compiler can keep many LDS table reads in flight
                uint2 sv[4];
#pragma unroll
                for (int j = 0; j < 4; j++) sv[j] = *reinterpret_cast<const uint2 *>(scb + j * BUF);
                GfTab tb[2][4];  // tables of check j + 1 are read while check j multiplies
#pragma unroll
                for (int r = 0; r < 4; r++) tb[0][r] = tab(r * 4);
                sfor<4>([&](auto jc) BS_INL {
                    constexpr int j = decltype(jc)::value;
                    if constexpr (j + 1 < 4) {
#pragma unroll
                        for (int r = 0; r < 4; r++) tb[(j + 1) & 1][r] = tab(r * 4 + j + 1);
                    }
                    const GfIdx i0 = gf_idx(sv[j].x), i1 = gf_idx(sv[j].y);
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        U[r][0] ^= gf_mul_idx(i0, tb[j & 1][r]);
                        U[r][1] ^= gf_mul_idx(i1, tb[j & 1][r]);
                    }
                });
                // dropped terms: used nodes whose companion is the red erased node of section y
                sfor<4>([&](auto yc) BS_INL {
                    constexpr int Y = decltype(yc)::value;
                    constexpr uint32_t wy = wt(Y);
                    const uint32_t zy = (z / wy) & 3u;
                    if (!((a.emask[Y] >> zy) & 1u)) return;
                    int ry = a.rix[4 * Y];
#pragma unroll
                    for (int x = 1; x < 4; x++) ry = zy == uint32_t(x) ? a.rix[4 * Y + x] : ry;
                    const uint8_t *cb = scb0 + uint32_t(ry) * BUF + 8u * pp;
                    const uint32_t zb = z - zy * wy;
                    sfor<4>([&](auto xc) BS_INL {
                        constexpr int X = decltype(xc)::value;
                        // masked instead of branched (straight-line code, see above)
                        const uint32_t m = (((a.used >> (4 * Y + X)) & 1u) && uint32_t(X) != zy) ? 0xffffffffu : 0u;
                        uint2 cv = *reinterpret_cast<const uint2 *>(cb + (zb + uint32_t(X) * wy) * 64u);
                        GfTab tc[4];
#pragma unroll
                        for (int r = 0; r < 4; r++) tc[r] = tab(16 + (Y * 4 + X) * 4 + r);
                        cv.x &= m;
                        cv.y &= m;
                        const GfIdx i0 = gf_idx(cv.x), i1 = gf_idx(cv.y);
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            U[r][0] ^= gf_mul_idx(i0, tc[r]);
                            U[r][1] ^= gf_mul_idx(i1, tc[r]);
                        }
                    });
                });
                // C into the item's S slots (for later rounds) and HBM
                const bool pvalid = t.b0 + 8u * pp + 8u <= t.vend;
                sfor<4>([&](auto rc) BS_INL {
                    constexpr int r = decltype(rc)::value;
                    if (uint32_t(r) >= a.ne) return;
                    *reinterpret_cast<uint2 *>(scb0 + r * BUF + z * 64u + 8u * pp) = make_uint2(U[r][0], U[r][1]);
                    uint8_t *dst = a.out[r];
                    if (STORE && dst && pvalid)
                        *reinterpret_cast<uint2 *>(dst + (uint64_t(z) * sc + t.b0 + 8u * pp)) = make_uint2(U[r][0], U[r][1]);
                });
            });
        }
    }

    // ---------------- phase B, split form (k_stream_solve) ----------------
    // Tile of the solve kernel: 128 byte positions (two phase-A tiles), so every output row run is
    // a whole 128-byte line.  S/C region [j][z][128 B] (4 x 32 KiB); item = (layer, part): 16
    // bytes, lane (c0 = 0..127, p = 0..7) of a 1024-thread workgroup.
    static constexpr uint32_t SW = 128, SBUF = 256 * SW;
    __device__ static GfTab tab_at(const uint8_t *tl, int i) {
        const uint4 v = *reinterpret_cast<const uint4 *>(tl + i * 32);
        return GfTab{v.x, v.y, v.z, v.w, *reinterpret_cast<const uint32_t *>(tl + i * 32 + 16)};
    }
    __device__ static uint4 mul4(const GfIdx (&ix)[4], const GfTab &t) {
        return make_uint4(gf_mul_idx(ix[0], t), gf_mul_idx(ix[1], t), gf_mul_idx(ix[2], t), gf_mul_idx(ix[3], t));
    }
    __device__ static void idx4(const uint4 v, GfIdx (&ix)[4]) {
        ix[0] = gf_idx(v.x);
        ix[1] = gf_idx(v.y);
        ix[2] = gf_idx(v.z);
        ix[3] = gf_idx(v.w);
    }
    __device__ static void xor4(uint4 &a, const uint4 b) {
        a.x ^= b.x;
        a.y ^= b.y;
        a.z ^= b.z;
        a.w ^= b.w;
    }
    // presolve: S'(z) = H_K^-1 S(z) for every layer, in place (no dependencies between layers: one
    // parallel pass, 2 items per lane).  Rows r >= ne have zero tables.
    __device__ static void presolve(uint8_t *scb0, const uint8_t *tl0, uint32_t c0, uint32_t p) {
        // 4 passes of 8 bytes (layer c0 + 128 k, half h of the lane's 16 bytes): bounded registers
#pragma unroll 1
        for (uint32_t kh = 0; kh < 4; kh++) {
            const uint8_t *tl = tl0 + opq(0u);  // table reads stay in the loop (not hoisted into VGPRs)
            uint8_t *scb = scb0 + (opq(c0) + 128u * (kh >> 1)) * SW + 16u * opq(p) + 8u * (kh & 1u);
            uint32_t U[4][2] = {};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint2 v = *reinterpret_cast<const uint2 *>(scb + j * SBUF);
                const GfIdx i0 = gf_idx(v.x), i1 = gf_idx(v.y);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const GfTab t = tab_at(tl, r * 4 + j);
                    U[r][0] ^= gf_mul_idx(i0, t);
                    U[r][1] ^= gf_mul_idx(i1, t);
                }
                __builtin_amdgcn_sched_barrier(0);  // one check's tables live at a time
            }
#pragma unroll
            for (int r = 0; r < 4; r++) *reinterpret_cast<uint2 *>(scb + r * SBUF) = make_uint2(U[r][0], U[r][1]);
        }
    }
    // rounds over the iscore levels >= 1 (level 0 has no dropped terms: C = S'): C_e(z) = S'_e(z)
    // + sum over red sections Y and used X != x_e(Y) of A_(Y,X)[e] C(e_Y, z[Y:=X]), in place.
    // x_e(Y) and "used" are uniform, so the X loop branches instead of masking.
    __device__ static void rounds2(const DecArgs &a, uint8_t *scb0, const uint8_t *tl0, uint32_t c0, uint32_t p) {
        const uint32_t nround = a.nround;
        for (uint32_t rd = a.round1; rd < nround; rd++) {
            lds_barrier();  // S' / C of the previous round visible
            const uint8_t *tl = tl0 + opq(0u);  // table reads stay in the loop
            const uint32_t li = a.round_start[rd] + opq(c0);
            if (li >= a.round_start[rd + 1]) continue;
            const uint32_t z = tl[kDecOrder * 4 + li];
            uint8_t *scb = scb0 + z * SW + 16u * opq(p);
            uint4 U[4];
#pragma unroll
            for (int r = 0; r < 4; r++) U[r] = *reinterpret_cast<const uint4 *>(scb + r * SBUF);
            sfor<4>([&](auto yc) BS_INL {
                constexpr int Y = decltype(yc)::value;
                constexpr uint32_t wy = wt(Y);
                const uint32_t em = a.emask[Y];
                const uint32_t zy = (z / wy) & 3u;
                if (!((em >> zy) & 1u)) return;
                const uint32_t xe = uint32_t(__builtin_ctz(em));  // = zy (one erasure per section)
                const int ry = a.rix[4 * Y + xe];
                const uint8_t *cb = scb0 + uint32_t(ry) * SBUF + 16u * p + (z - zy * wy) * SW;
                sfor<4>([&](auto xc) BS_INL {
                    constexpr int X = decltype(xc)::value;
                    if (uint32_t(X) == xe || !((a.used >> (4 * Y + X)) & 1u)) return;
                    GfIdx ix[4];
                    idx4(*reinterpret_cast<const uint4 *>(cb + uint32_t(X) * wy * SW), ix);
#pragma unroll
                    for (int r = 0; r < 4; r++) xor4(U[r], mul4(ix, tab_at(tl, 16 + (Y * 4 + X) * 4 + r)));
                    __builtin_amdgcn_sched_barrier(0);  // one term's tables live at a time
                });
            });
#pragma unroll
            for (int r = 0; r < 4; r++) *reinterpret_cast<uint4 *>(scb + r * SBUF) = U[r];
        }
        lds_barrier();  // every C of the tile in LDS
    }
    // rounds3: the same corrections, one work item per (pair, 8 bytes): the pair's term
    // A_(Y,X)[r] C(e_Y, z[Y:=X]) of 8 positions for every r, XORed into C_r(z) with 64-bit LDS
    // atomics (ds_xor_b64).  Rounds of the 4-erasure 1 GiB decode: 0.087 ms (4-byte items 0.124,
    // 16-byte items 0.097).
    // A round's latency is then its item count / 1024 instead of its layers' term count.
    __device__ static void rounds3(const DecArgs &a, uint8_t *scb0, const uint8_t *tl, uint32_t tid) {
        const uint32_t nround = a.nround;
        const uint16_t *pairs = reinterpret_cast<const uint16_t *>(tl + kDecPairs * 4);
        for (uint32_t rd = a.round1; rd < nround; rd++) {
            lds_barrier();  // C of the previous round visible
            // items of 8 bytes: 16 per pair (one 128-byte row)
            const uint32_t i0 = a.pstart[rd] * 16u, i1 = a.pstart[rd + 1] * 16u;
            for (uint32_t i = i0 + tid; i < i1; i += 1024u) {
                const uint32_t pr = pairs[i >> 4], d8 = (i & 15u) * 8u;
                const uint32_t z = pr & 255u, Y = (pr >> 8) & 3u, X = pr >> 10;
                const uint32_t sh = 2u * (3u - Y), zy = (z >> sh) & 3u;
                const uint32_t zs = z + ((X - zy) << sh);  // z[Y := X]
                const int ry = a.rix[4 * Y + zy];           // the erased node of section Y (red in z)
                const uint2 cv = *reinterpret_cast<const uint2 *>(scb0 + uint32_t(ry) * SBUF + zs * SW + d8);
                const GfIdx ix0 = gf_idx(cv.x), ix1 = gf_idx(cv.y);
                const uint8_t *tb = tl + (16u + (Y * 4u + X) * 4u) * 32u;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    if (uint32_t(r) >= a.ne) break;
                    const GfTab t = tab_at(tb, r);
                    const uint64_t v = uint64_t(gf_mul_idx(ix0, t)) | (uint64_t(gf_mul_idx(ix1, t)) << 32);
                    __hip_atomic_fetch_xor(reinterpret_cast<uint64_t *>(scb0 + r * SBUF + z * SW + d8), v, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        }
        lds_barrier();  // every C of the tile in LDS
    }
    // C of the tile to the output chunks: 8 lanes x 16 bytes per 128-byte row
    template <bool STORE>
    __device__ static void store_out(const DecArgs &a, const uint8_t *scb0, int r, uint32_t b0, uint32_t vend, uint32_t tid) {
        const uint32_t sc = uint32_t(a.sc);
        const uint32_t q16 = (tid & 7u) * 16u;
        const bool full = b0 + q16 + 16u <= vend;
        const bool half = !full && b0 + q16 + 8u <= vend;  // sc % 8 == 0: valid length is a multiple of 8
        uint8_t *dst = a.out[r];
        if (!STORE || uint32_t(r) >= a.ne || !dst) return;
#pragma unroll
        for (uint32_t zz = 0; zz < 2; zz++) {
            const uint32_t z = (tid >> 3) + 128u * zz;
            const uint8_t *src = scb0 + r * SBUF + z * SW + q16;
            uint8_t *o = dst + uint64_t(z) * sc + b0 + q16;
            if (full) *reinterpret_cast<uint4 *>(o) = *reinterpret_cast<const uint4 *>(src);
            else if (half) *reinterpret_cast<uint2 *>(o) = *reinterpret_cast<const uint2 *>(src);
        }
    }
};

// PROBE (bench_tools / CLAY_DECODE_PROBE only; the product runs PROBE = 0): bit 1 = no phase-B
// work (rounds keep their barriers), 2 = no phase-A math, 4 = loaders issue no DMA.
template <int KD, int G, int PROBE = 0>
__global__ __launch_bounds__((StreamDec<KD, G>::BLOCK)) void k_stream_decode(DecArgs a) {
    using Kn = StreamDec<KD, G>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t xcd = blockIdx.x & 7u, wslot = blockIdx.x >> 3, ns = a.nslots;
    const uint32_t sc = uint32_t(a.sc);
    const typename Kn::Map tm(sc, a.region, ns, xcd, wslot);
    const uint32_t ntile = tm.n;
    if (ntile == 0) return;  // uniform per workgroup
    const uint32_t R = a.ring, NT = a.nt, nround = a.nround;
    constexpr uint32_t BUF = uint32_t(Kn::BUF);

    if (wave >= Kn::CWAVES) {
        // ---------------- loader waves ----------------
        // Tile-relative ring: load q of a tile goes to buffer q % R.  Within a tile a load is
        // issued once the step that last used its buffer is done; the next tile's first R - 4
        // loads are issued during phase B (buffers outside the S/C region), the rest after it.
        __builtin_amdgcn_s_setprio(3);
        const int li = wave - Kn::CWAVES;
        typename Kn::Loader L;
        Kn::loader_init(L, sc, li, lane);
        const uint32_t lds0 = lds_addr_of(smem);
        uint32_t issued = 0;  // loads issued in total (all tiles)
        auto issue_upto = [&](uint32_t k, uint32_t lim) {  // tile k, tile-relative limit
            if (k >= ntile) return;
            if (lim > NT) lim = NT;
            const typename Kn::Tile t = tm.tile(k, wslot, ns);
            for (uint32_t q = issued - k * NT; q < lim; q++, issued++) {
                const uint32_t nd = a.load_node[q];
                if constexpr (!(PROBE & 4)) Kn::issue(a, L, lds0 + (q % R) * BUF, a.node[nd], t, li);
            }
        };
        issue_upto(0, R);
        for (uint32_t k = 0; k < ntile; k++) {
            for (int y = 0; y < 4; y++) {
                // loads of step (k, y) landed: everything issued after them may stay in flight
                const uint32_t qend = k * NT + a.sec_off[y + 1];
                wait_vm_rt(int((issued - qend) * uint32_t(Kn::BPL)));
                lds_barrier();
                issue_upto(k, a.sec_off[y] + R);  // steps before (k, y) are done
            }
            lds_barrier();  // B0: every step of tile k done -> S/C region written
            {   // phase-B tables into buffer R - 5 (3 KiB: one 1 KiB block per loader wave 0..2)
                if (li < 3) dma16(lds0 + (R - 5u) * BUF + uint32_t(li) * 1024u, uniform_ptr(reinterpret_cast<const uint8_t *>(a.tabs)),
                                  uint32_t(li) * 1024u + uint32_t(lane) * 16u);
                issue_upto(k + 1, R - 5);
                // the tables landed (the prefetch issued after them may stay in flight)
                wait_vm_rt(int((issued - (k + 1 < ntile ? (k + 1) * NT : issued)) * uint32_t(Kn::BPL)));
            }
            for (uint32_t rd = 0; rd < nround; rd++) lds_barrier();
            lds_barrier();  // B_end: phase B done, the S/C region is free
            issue_upto(k + 1, R);
        }
        wait_vm0();
        return;
    }

    // ---------------- compute waves ----------------
    const uint32_t c0 = uint32_t(threadIdx.x) >> 3, p = uint32_t(threadIdx.x) & 7u;
    const uint32_t emG = a.emask[G];
    const int xeG = emG ? __builtin_ctz(emG) : -1;
    const uint32_t scbase = (R - 4u) * BUF;

    for (uint32_t k = 0; k < ntile; k++) {
        const typename Kn::Tile t = tm.tile(k, wslot, ns);
        const bool straddle = t.vend < t.b0 + uint32_t(Kn::W) && ((t.vend - t.b0) & 15u) == 8u;
        const uint32_t pcs = (t.vend - t.b0) >> 4;
        const uint32_t poff0 = 8u * p + ((straddle && p == 2u * pcs) ? 8u : 0u);

        uint32_t S[32];
#pragma unroll
        for (int w = 0; w < 32; w++) S[w] = 0;

        // ---------------- phase A: one step per section ----------------
        Kn::template phase_a<PROBE>(a, smem, 0u, c0, poff0, xeG, S, R);

        // ---------------- S_known -> LDS (S/C region, [j][z][p]) ----------------
        lds_barrier();  // B0: every wave is done with the ring buffers of tile k
        {
            const uint32_t c = opq(c0);
            const uint32_t z0 = Kn::layer0(c);
            sfor<4>([&](auto jc) BS_INL {
                constexpr int j = decltype(jc)::value;
                uint32_t v[8];
#pragma unroll
                for (int w = 0; w < 8; w++) v[w] = S[j * 8 + w];
                transpose8(v);
                uint8_t *sb = smem + scbase + uint32_t(j) * BUF + 8u * p;
#pragma unroll
                for (int g = 0; g < 4; g++)
                    *reinterpret_cast<uint2 *>(sb + (z0 + uint32_t(g) * Kn::wt(G)) * 64u) = make_uint2(v[2 * g], v[2 * g + 1]);
            });
        }

        // ---------------- phase B: rounds in iscore order ----------------
        // tables (v_perm, 8-dword stride) and the layer order in LDS buffer R - 5 (the loaders
        // copied them after B0; visible after the first round's barrier)
        Kn::template rounds<!(PROBE & 1)>(a, smem + scbase, smem + (R - 5u) * BUF, t, c0, p);
        lds_barrier();  // B_end
    }
}


// ---------------------------------------------------------------------------------------------
// Split decode: the same two phases in two launches, so that phase B (latency-bound rounds behind
// workgroup barriers, no memory traffic of its own) no longer stalls the streaming of phase A.
//  k_stream_syn   phase A of every tile with the ring streaming continuously across tiles (global
//                 load index -> buffer), then the presolve S' = H_K^-1 S; S' of tile b0 written to
//                 ws + b0 * 1024 (64 KiB per 64-byte tile, [r][z][64 B] as the fused kernel's S/C
//                 region)
//  k_stream_solve phase B: one 1024-thread workgroup per CU (a 128-byte tile: 4 x 256 x 128 B of
//                 S' + 5 KiB of tables, ~133 KiB of LDS), one tile at a time: LDS-DMA of the S'
//                 tile, the term-parallel rounds (LDS atomics), C to HBM in 128-byte row runs,
//                 with the next tile's S' DMA issued before the output stores.
// Extra HBM traffic: S written and read once (2 x 4 x 256 x sc bytes).
// ---------------------------------------------------------------------------------------------
template <int KD, int G, int PROBE = 0>
__global__ __launch_bounds__((StreamDec<KD, G>::BLOCK)) void k_stream_syn(DecArgs a) {
    using Kn = StreamDec<KD, G>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t xcd = blockIdx.x & 7u, wslot = blockIdx.x >> 3, ns = a.nslots;
    const uint32_t sc = uint32_t(a.sc);
    const typename Kn::Map tm(sc, a.region, ns, xcd, wslot);
    const uint32_t ntile = tm.n;
    if (ntile == 0) return;  // uniform per workgroup
    // ring of a.ring - 1 node buffers; the last buffer holds the presolve tables (H_K^-1 rows)
    const uint32_t R = a.ring - 1u, NT = a.nt;
    constexpr uint32_t BUF = uint32_t(Kn::BUF);

    if (wave >= Kn::CWAVES) {
        // ---------------- loader waves: global ring, load g -> buffer g % R ----------------
        __builtin_amdgcn_s_setprio(3);
        const int li = wave - Kn::CWAVES;
        typename Kn::Loader L;
        Kn::loader_init(L, sc, li, lane);
        const uint32_t lds0 = lds_addr_of(smem);
        if (li < 3)  // tables, before any ring load: the first step's counted wait covers them
            dma16(lds0 + R * BUF + uint32_t(li) * 1024u, uniform_ptr(reinterpret_cast<const uint8_t *>(a.tabs)),
                  uint32_t(li) * 1024u + uint32_t(lane) * 16u);
        const uint32_t nloads = ntile * NT;
        uint32_t issued = 0;
        auto issue_upto = [&](uint32_t lim) {
            if (lim > nloads) lim = nloads;
            for (; issued < lim; issued++) {
                const uint32_t k = issued / NT, q = issued % NT;
                if constexpr (!(PROBE & 4))
                    Kn::issue(a, L, lds0 + (issued % R) * BUF, a.node[a.load_node[q]], tm.tile(k, wslot, ns), li);
            }
        };
        issue_upto(R);
        for (uint32_t k = 0; k < ntile; k++) {
            for (int y = 0; y < 4; y++) {
                // loads of step (k, y) landed: everything issued after them may stay in flight
                const uint32_t qend = k * NT + a.sec_off[y + 1];
                wait_vm_rt(int((issued - qend) * uint32_t(Kn::BPL)));
                lds_barrier();
                issue_upto(k * NT + a.sec_off[y] + R);  // steps before (k, y) are done
            }
        }
        wait_vm0();
        return;
    }

    // ---------------- compute waves ----------------
    const uint32_t c0 = uint32_t(threadIdx.x) >> 3, p = uint32_t(threadIdx.x) & 7u;
    const uint32_t emG = a.emask[G];
    const int xeG = emG ? __builtin_ctz(emG) : -1;
    for (uint32_t k = 0; k < ntile; k++) {
        const typename Kn::Tile t = tm.tile(k, wslot, ns);
        const bool straddle = t.vend < t.b0 + uint32_t(Kn::W) && ((t.vend - t.b0) & 15u) == 8u;
        const uint32_t pcs = (t.vend - t.b0) >> 4;
        const uint32_t poff0 = 8u * p + ((straddle && p == 2u * pcs) ? 8u : 0u);
        uint32_t S[32];
#pragma unroll
        for (int w = 0; w < 32; w++) S[w] = 0;
        Kn::template phase_a<PROBE>(a, smem, k * NT, c0, poff0, xeG, S, R);
        // S back to bytes, then the presolve S' = H_K^-1 S (run-time v_perm tables from LDS; the
        // kernel is memory-bound, so this VALU work hides under the streaming), S' -> the
        // workspace tile ([r][z][p] x 8 B)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t v[8];
#pragma unroll
            for (int w = 0; w < 8; w++) v[w] = S[j * 8 + w];
            transpose8(v);
#pragma unroll
            for (int w = 0; w < 8; w++) S[j * 8 + w] = v[w];
        }
        const uint32_t c = opq(c0);
        const uint32_t z0 = Kn::layer0(c);
        uint8_t *wtile = a.ws + uint64_t(t.b0) * 1024u + 8u * p;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            uint32_t U[4][2] = {};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                // tables re-read per (g, j) through an opaque address: 4 live at a time instead of
                // all 16 hoisted into registers
                const uint8_t *tl = smem + R * BUF + opq(0u);
                const GfIdx i0 = gf_idx(S[j * 8 + 2 * g]), i1 = gf_idx(S[j * 8 + 2 * g + 1]);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    if (uint32_t(r) < a.ne) {  // the erased rows only (uniform)
                        const GfTab tb = Kn::tab_at(tl, r * 4 + j);
                        U[r][0] ^= gf_mul_idx(i0, tb);
                        U[r][1] ^= gf_mul_idx(i1, tb);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int r = 0; r < 4; r++)
                if (uint32_t(r) < a.ne)  // S' rows of the erased nodes only: ne x 16 KiB of the tile's 64 KiB
                    *reinterpret_cast<uint2 *>(wtile + uint32_t(r) * BUF + (z0 + uint32_t(g) * Kn::wt(G)) * 64u) =
                        make_uint2(U[r][0], U[r][1]);
        }
    }
}

constexpr int kSolveLds = 4 * 256 * 128 + kDecTabWords * 4;  // S/C tile (128 positions) + tables, order, pairs

// PROBE (CLAY_DECODE_PROBE, probe library only): bit 1 = no presolve / rounds, 2 = no HBM
// stores, 4 = no S DMA, 8 = no presolve, 16 = no rounds, 32 = non-temporal output stores.  grid = 8 * ns (one 1024-thread workgroup per CU); XCD x owns 128-byte
// tiles [x * per, (x + 1) * per) (a.region = per * 128), its ns workgroups take them round robin.
template <int KD, int G, int PROBE = 0>
__global__ __launch_bounds__(1024) void k_stream_solve(DecArgs a) {
    using Kn = StreamDec<KD, G>;
    constexpr uint32_t SW = Kn::SW;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t xcd = blockIdx.x & 7u, wslot = blockIdx.x >> 3, ns = a.nslots;
    const uint32_t sc = uint32_t(a.sc);
    const uint32_t nst = (sc + SW - 1) / SW, per = a.region / SW;
    const uint32_t t0 = xcd * per, t1 = t0 + per < nst ? t0 + per : nst;
    const uint32_t ntile = t0 + wslot < t1 ? (t1 - t0 - wslot + ns - 1) / ns : 0u;
    if (ntile == 0) return;  // uniform per workgroup
    const uint32_t lds0 = lds_addr_of(smem);
    uint8_t *const tl = smem + 4 * Kn::SBUF;
    if (wave < kDecTabWords / 256)  // tables, layer order, correction pairs: once per workgroup
        dma16(lds0 + 4u * Kn::SBUF + uint32_t(wave) * 1024u, uniform_ptr(reinterpret_cast<const uint8_t *>(a.tabs)),
              uint32_t(wave) * 1024u + uint32_t(lane) * 16u);
    // S of phase-A tiles b0 and b0 + 64 (ws + b * 1024, [j][z][64 B]) into buffer j of the
    // [j][z][128 B] region: LDS block (j, 8 rows) <- 8 x 2 pieces of 64 B; 32 blocks, 2 per wave
    const uint32_t zl = uint32_t(lane) >> 3, q = (uint32_t(lane) & 7u) * 16u;
    auto dma_check = [&](uint32_t b0, uint32_t j) {
        if constexpr (!(PROBE & 4)) {
            const uint32_t h2 = b0 + 64u < sc ? 65536u : 0u;  // no second phase-A tile: any valid one
            const uint8_t *src = uniform_ptr(a.ws + uint64_t(b0) * 1024u);
            const uint32_t hoff = (q >= 64u ? h2 : 0u) + (q & 63u);
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const uint32_t zb = uint32_t(wave) * 2u + uint32_t(i);  // 8-row block within the check
                dma16(lds0 + j * Kn::SBUF + zb * 1024u, src, hoff + j * 16384u + (zb * 8u + zl) * 64u);
            }
        }
    };
    auto tile_b0 = [&](uint32_t k) { return (t0 + wslot + k * ns) * SW; };
#pragma unroll
    for (uint32_t j = 0; j < 4; j++)
        if (j < a.ne) dma_check(tile_b0(0), j);  // S' rows of the erased nodes only
    // output stores of a full tile per lane (issued after the next tile's DMA, so the wait for
    // that DMA lets them stay in flight): 2 per erased index with an output
    uint32_t nstores = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) nstores += (uint32_t(r) < a.ne && a.out[r]) ? 2u : 0u;
    for (uint32_t k = 0; k < ntile; k++) {
        const uint32_t b0 = tile_b0(k);
        const uint32_t vend = b0 + SW < sc ? b0 + SW : sc;
        if (k == 0) wait_vm0();                 // S of tile 0 and the tables
        else wait_vm_rt(PROBE & 2 ? 0 : int(nstores));  // S of tile k (tile k-1's stores may stay in flight)
        lds_barrier();  // S (and, first time, the tables) landed
        if constexpr (!(PROBE & 1)) {
            // S' arrives presolved (k_stream_syn): only the rounds
            if constexpr (!(PROBE & 16)) Kn::rounds3(a, smem, tl, threadIdx.x);  // ends with a barrier
            else lds_barrier();
        } else {
            lds_barrier();
        }
        // C of the tile into registers (32 VGPRs: the rounds' registers are free by now), the
        // next tile's S DMA into the freed region, then the output stores from registers
        uint4 cv[4][2];
        const uint32_t q16 = (threadIdx.x & 7u) * 16u;
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (uint32_t zz = 0; zz < 2; zz++)
                cv[r][zz] = *reinterpret_cast<const uint4 *>(smem + r * Kn::SBUF + ((threadIdx.x >> 3) + 128u * zz) * SW + q16);
        lds_barrier();  // the region is free
        if (k + 1 < ntile)
#pragma unroll
            for (uint32_t j = 0; j < 4; j++)
                if (j < a.ne) dma_check(tile_b0(k + 1), j);
        if constexpr (!(PROBE & 2)) {
            const bool full = b0 + q16 + 16u <= vend;
            const bool half = !full && b0 + q16 + 8u <= vend;  // sc % 8 == 0: valid length is a multiple of 8
#pragma unroll
            for (int r = 0; r < 4; r++) {
                uint8_t *dst = a.out[r];
                if (uint32_t(r) >= a.ne || !dst) continue;
#pragma unroll
                for (uint32_t zz = 0; zz < 2; zz++) {
                    uint8_t *o = dst + uint64_t((threadIdx.x >> 3) + 128u * zz) * sc + b0 + q16;
                    if (full) {
                        if constexpr ((PROBE & 32) != 0) {  // probe: non-temporal output stores
                            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                            const v4u v = {cv[r][zz].x, cv[r][zz].y, cv[r][zz].z, cv[r][zz].w};
                            __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(o));
                        } else {
                            *reinterpret_cast<uint4 *>(o) = cv[r][zz];
                        }
                    }
                    else if (half) *reinterpret_cast<uint2 *>(o) = make_uint2(cv[r][zz].x, cv[r][zz].y);
                }
            }
        }
    }
}

}  // namespace bs
}  // namespace clay
