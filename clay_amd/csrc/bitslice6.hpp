// bitslice6.hpp -- v6 bit-sliced encode for (10,4,13): 128-byte runs per sub-chunk row.
//
// Why: the v4 kernel (64-byte tiles) runs at the ceiling of its own access pattern --
// bench_tools/run_width_probe shows 64-byte runs per sub-chunk row cap the LDS-DMA sweep at ~3.8 TB/s
// and 128-byte runs reach ~4.6 TB/s (reads + parity stores, no math).  v4's accumulators
// (64 KiB LDS per 64-byte tile) leave no room to double the tile, so v6 re-partitions:
//
//  * lane = (column c = (d0,d1,d2) of the layer digits, part = 32-byte quarter of the
//    128-byte tile); it owns the four layers z = 4c + g, g = d3 = the digit of the
//    parity y-section.  Every PFT partner pair (x, z) <-> (d3(z), z with d3 := x) then
//    lives in ONE lane: the PFT needs no exchange at all.
//  * the lines of the data y-sections 0..2 never change d3, so a tile is processed as
//    12 steps (group g, section Y), each reading one "slot": 4 nodes x 64 layers x 128 B
//    = 32 KiB.  Slots stream through a 5-deep LDS ring (160 KiB) by 16-byte LDS-DMA,
//    issued 4 steps ahead; one barrier per step; counted vmcnt waits.
//  * accumulators: the current group's 4 parity x 8 planes (32 VGPRs) plus the U values
//    later groups' PFT pairs need (at most 6 x 8 VGPRs), all in registers.  When group g
//    finishes, its red vertex and its PFT pairs with groups h < g are written out.
//  * slot image: 16-byte piece (c, part, d) of node x at bank slot B.(c|part<<6|d<<8)
//    ^ H.x (tools/v6_layout_search.py): own and companion ds_read_b128 of every section
//    are bank-conflict free.
#pragma once

#include "bitslice.hpp"
#include "xor_cse.hpp"

namespace clay {
namespace bs {

// GF(2)-linear piece map: NB input bits v -> piece index p = (row << 4) | bank, with
// bank bit o = <v, BM[o]> and rows completing the bijection with unit vectors.
template <int NB>
struct GfLin {
    uint16_t fwd[NB];  // column i: p of unit vector e_i
    uint16_t inv[NB];  // column i: v of unit vector e_i in piece-index space
};
template <int NB>
constexpr GfLin<NB> make_gflin(const uint32_t (&bm)[4]) {
    GfLin<NB> L{};
    uint32_t rows[NB] = {};
    int nr = 0;
    for (int o = 0; o < 4; o++) rows[nr++] = bm[o];
    for (int b = 0; b < NB && nr < NB; b++) {
        uint32_t basis[NB] = {};
        int piv[NB] = {};
        int nb = 0;
        for (int r = 0; r < nr; r++) {
            uint32_t v = rows[r];
            for (int i = 0; i < nb; i++)
                if ((v >> piv[i]) & 1) v ^= basis[i];
            if (v) {
                int p = 0;
                while (!((v >> p) & 1)) p++;
                basis[nb] = v;
                piv[nb] = p;
                nb++;
            }
        }
        uint32_t v = 1u << b;
        for (int i = 0; i < nb; i++)
            if ((v >> piv[i]) & 1) v ^= basis[i];
        if (v) rows[nr++] = 1u << b;
    }
    for (int i = 0; i < NB; i++) {
        uint16_t p = 0;
        for (int r = 0; r < NB; r++)
            if ((rows[r] >> i) & 1) p |= uint16_t(1u << r);
        L.fwd[i] = p;
    }
    uint32_t a[NB] = {}, inv[NB] = {};
    for (int r = 0; r < NB; r++) {
        for (int i = 0; i < NB; i++)
            if ((L.fwd[i] >> r) & 1) a[r] |= 1u << i;
        inv[r] = 1u << r;
    }
    for (int c = 0; c < NB; c++) {
        int p = c;
        while (!((a[p] >> c) & 1)) p++;
        uint32_t t = a[p];
        a[p] = a[c];
        a[c] = t;
        t = inv[p];
        inv[p] = inv[c];
        inv[c] = t;
        for (int r = 0; r < NB; r++)
            if (r != c && ((a[r] >> c) & 1)) {
                a[r] ^= a[c];
                inv[r] ^= inv[c];
            }
    }
    for (int i = 0; i < NB; i++) {
        uint16_t col = 0;
        for (int r = 0; r < NB; r++)
            if ((inv[r] >> i) & 1) col |= uint16_t(1u << r);
        L.inv[i] = col;
    }
    return L;
}

namespace v6 {
constexpr int par32(uint32_t v) {
    int p = 0;
    for (; v; v &= v - 1) p ^= 1;
    return p;
}
// Slot image per tile width: piece v = c | part << 6 | d << (6 + log2 PARTS);
// BM over v, HM over the slot-local node x (tools/v6_layout_search.py, v7_layout_search.py)
template <int PARTS>
struct Layout;
template <>
struct Layout<4> {
    static constexpr int PB = 2, NB = 9;
    static constexpr uint32_t BM[4] = {0xf3, 0x85, 0x17a, 0x1e5};
    static constexpr uint32_t HM[4] = {0, 0, 3, 2};
};
template <>
struct Layout<8> {
    static constexpr int PB = 3, NB = 10;
    static constexpr uint32_t BM[4] = {0x269, 0x6, 0x2b4, 0x87};
    static constexpr uint32_t HM[4] = {2, 2, 2, 3};
};
template <int PARTS>
struct Map {
    using L = Layout<PARTS>;
    static constexpr int NB = L::NB;
    static constexpr GfLin<NB> LIN = make_gflin<NB>(L::BM);
    static constexpr uint32_t fwd_c(uint32_t v) {
        uint32_t p = 0;
        for (int i = 0; i < NB; i++)
            if ((v >> i) & 1) p ^= LIN.fwd[i];
        return p;
    }
    static constexpr uint32_t inv_c(uint32_t p) {
        uint32_t v = 0;
        for (int i = 0; i < NB; i++)
            if ((p >> i) & 1) v ^= LIN.inv[i];
        return v;
    }
    static constexpr uint32_t hbank(int x) {
        uint32_t b = 0;
        for (int o = 0; o < 4; o++) b |= uint32_t(par32(uint32_t(x) & L::HM[o])) << o;
        return b;
    }
    static_assert(inv_c(fwd_c(0x1A5)) == 0x1A5 && inv_c(fwd_c(0x0FF)) == 0x0FF, "v6 layout bijection");
    static_assert((fwd_c(0x1FF) & 15) == uint32_t(par32(0x1FF & L::BM[0]) | (par32(0x1FF & L::BM[1]) << 1) |
                                                  (par32(0x1FF & L::BM[2]) << 2) | (par32(0x1FF & L::BM[3]) << 3)),
                  "bank bits of the piece index");
    __device__ static __forceinline__ uint32_t fwd_d(uint32_t v) {
        uint32_t p = 0;
#pragma unroll
        for (int i = 0; i < NB; i++) p ^= ((v >> i) & 1) ? uint32_t(LIN.fwd[i]) : 0u;
        return p;
    }
    __device__ static __forceinline__ uint32_t inv_d(uint32_t p) {
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < NB; i++) v ^= ((p >> i) & 1) ? uint32_t(LIN.inv[i]) : 0u;
        return v;
    }
    __device__ static __forceinline__ uint32_t hbank_d(uint32_t x) {
        uint32_t b = 0;
#pragma unroll
        for (int o = 0; o < 4; o++) b |= uint32_t(__builtin_popcount(x & L::HM[o]) & 1) << o;
        return b;
    }
};
}  // namespace v6

template <int KD, int M, int PARTS>
struct Bs6Kernel {
    using S = Shape<KD, M>;
    using MP = v6::Map<PARTS>;
    static constexpr int PB = v6::Layout<PARTS>::PB;
    static constexpr int Q = S::Q, T = S::T, ALPHA = S::ALPHA;
    static_assert(M == 4 && Q == 4 && T == 4 && ALPHA == 256 && KD <= 12,
                  "v6 slot layout is derived for q = 4, t = 4 (alpha 256)");
    static constexpr int W = 32 * PARTS, COLS = ALPHA / Q, BLOCK = COLS * PARTS, WAVES = BLOCK / 64;
    static constexpr int NODE_BYTES = COLS * W;            // one node of one (Y, g) slot
    static constexpr int SLOT = Q * NODE_BYTES;            // 32 KiB (W 128) / 64 KiB (W 256)
    static constexpr int RING = (160 * 1024) / SLOT;       // 5 / 2
    static constexpr int LDS_BYTES = RING * SLOT;
    // slots in flight ahead of the one being read (the slot just read is refilled next step)
    static constexpr int AHEAD = RING - 1;
    static constexpr int STEPS = (T - 1) * Q;              // (section, group) steps per tile
    static constexpr int DMA_PER_NODE = NODE_BYTES / 1024 / WAVES;  // per wave: 2

    static constexpr int nreal(int y) { int n = 0; for (int x = 0; x < Q; x++) n += (y * Q + x < KD); return n; }
    static constexpr int ndma(int y) { return nreal(y) * DMA_PER_NODE; }
    static constexpr int stores(int g) { return (1 + 2 * g) * 2; }  // dwordx4 per lane at group end
    static constexpr int dshift(int y) { return 2 * (T - 2 - y); }   // digit y of the column c

    __device__ static uint32_t piece_off(uint32_t v) {
        return ((v >> 6) & uint32_t(PARTS - 1)) * 32u + (v >> (6 + PB)) * 16u;
    }

    // DMA of slot (section Y, group g) of the tile at b0: wave w fills 1 KiB blocks
    // [2w, 2w+2) of every real node region.  Returns the instructions issued.
    template <int Y>
    __device__ static void dma(const BsArgs &a, uint32_t slot_lds, int wave, int lane, uint32_t b0, int g) {
        const uint32_t sc = uint32_t(a.sc);
        uint32_t vl = MP::inv_d(uint32_t(lane));
        asm volatile("" : "+v"(vl));
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            constexpr int node = Y * Q + x;
            if constexpr (node < KD) {
#pragma unroll
                for (int i = 0; i < DMA_PER_NODE; i++) {
                    const uint32_t blk = uint32_t(wave * DMA_PER_NODE + i);
                    const uint32_t v = vl ^ MP::inv_d((blk << 6) ^ MP::hbank(x));
                    uint32_t pos = b0 + piece_off(v);
                    if (pos + 16u > sc) pos = sc - 16u;  // ragged: patched after landing
                    const uint32_t layer = (v & 63u) * 4u + uint32_t(g);
                    dma16(slot_lds + uint32_t(x * NODE_BYTES) + blk * 1024u, a.data[node], layer * sc + pos);
                }
            }
        });
    }
    template <int Y>
    __device__ static void patch(const BsArgs &a, uint8_t *slot, int wave, int lane, uint32_t b0, int g) {
        const uint32_t sc = uint32_t(a.sc);
        const uint32_t vl = MP::inv_d(uint32_t(lane));
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            constexpr int node = Y * Q + x;
            if constexpr (node < KD) {
#pragma unroll
                for (int i = 0; i < DMA_PER_NODE; i++) {
                    const uint32_t blk = uint32_t(wave * DMA_PER_NODE + i);
                    const uint32_t v = vl ^ MP::inv_d((blk << 6) ^ MP::hbank(x));
                    const uint32_t pos = b0 + piece_off(v);
                    if (pos < sc && pos + 16u > sc) {  // 8 valid bytes (sc is a multiple of 8)
                        const uint32_t layer = (v & 63u) * 4u + uint32_t(g);
                        const uint2 gv = *reinterpret_cast<const uint2 *>(a.data[node] + layer * sc + pos);
                        *reinterpret_cast<uint4 *>(slot + x * NODE_BYTES + blk * 1024 + lane * 16) =
                            make_uint4(gv.x, gv.y, 0u, 0u);
                    }
                }
            }
        });
    }
    // DMA of node x of slot (section Y, group g) only (DMA_PER_NODE instructions if real)
    template <int Y, int X>
    __device__ static void dma_node(const BsArgs &a, uint32_t slot_lds, int wave, uint32_t vl, uint32_t b0, int g) {
        constexpr int node = Y * Q + X;
        if constexpr (node < KD) {
            const uint32_t sc = uint32_t(a.sc);
#pragma unroll
            for (int i = 0; i < DMA_PER_NODE; i++) {
                const uint32_t blk = uint32_t(wave * DMA_PER_NODE + i);
                const uint32_t v = vl ^ MP::inv_d((blk << 6) ^ MP::hbank(X));
                uint32_t pos = b0 + piece_off(v);
                if (pos + 16u > sc) pos = sc - 16u;  // ragged: patched after landing
                const uint32_t layer = (v & 63u) * 4u + uint32_t(g);
                dma16(slot_lds + uint32_t(X * NODE_BYTES) + blk * 1024u, a.data[node], layer * sc + pos);
            }
        }
    }
    template <int X>
    __device__ static void dma_node_any(int y, const BsArgs &a, uint32_t slot_lds, int wave, uint32_t vl, uint32_t b0,
                                        int g) {
        if (y == 0) dma_node<0, X>(a, slot_lds, wave, vl, b0, g);
        else if (y == 1) dma_node<1, X>(a, slot_lds, wave, vl, b0, g);
        else dma_node<2, X>(a, slot_lds, wave, vl, b0, g);
    }
    __device__ static void dma_any(int y, const BsArgs &a, uint32_t slot_lds, int wave, int lane, uint32_t b0, int g) {
        if (y == 0) dma<0>(a, slot_lds, wave, lane, b0, g);
        else if (y == 1) dma<1>(a, slot_lds, wave, lane, b0, g);
        else dma<2>(a, slot_lds, wave, lane, b0, g);
    }
    __device__ static void patch_any(int y, const BsArgs &a, uint8_t *slot, int wave, int lane, uint32_t b0, int g) {
        if (y == 0) patch<0>(a, slot, wave, lane, b0, g);
        else if (y == 1) patch<1>(a, slot, wave, lane, b0, g);
        else patch<2>(a, slot, wave, lane, b0, g);
    }

    __device__ static void read32(const uint8_t *p0, const uint8_t *p1, uint32_t (&d)[8]) {
        const uint4 v0 = *reinterpret_cast<const uint4 *>(p0), v1 = *reinterpret_cast<const uint4 *>(p1);
        d[0] = v0.x; d[1] = v0.y; d[2] = v0.z; d[3] = v0.w;
        d[4] = v1.x; d[5] = v1.y; d[6] = v1.z; d[7] = v1.w;
    }

    template <int BO>
    static constexpr uint64_t pft_mask() {
        return plane_mask(S::DINV, BO, 0) | plane_mask(gm(S::DINV, 2), BO, 8);
    }

    // Per-lane piece indices (loop invariant): own piece, and per data section Y the
    // companion base (digit Y of c cleared, bank XOR of the companion node folded in).
    struct LaneC {
        uint32_t fown;
        uint32_t fcl[T - 1];
        int cy[T - 1];
    };
    __device__ static LaneC lane_consts(int c, int part) {
        LaneC L;
        L.fown = MP::fwd_d(uint32_t(c) | uint32_t(part << 6));
#pragma unroll
        for (int y = 0; y < T - 1; y++) {
            const int sh = dshift(y);
            L.cy[y] = (c >> sh) & 3;
            L.fcl[y] = MP::fwd_d(uint32_t(c & ~(3 << sh)) | uint32_t(part << 6)) ^ MP::hbank_d(uint32_t(L.cy[y]));
        }
        return L;
    }

    // Stage reads of section Y for the lane's layer: own value and companion per node x.
    template <int Y, int X>
    __device__ static void load_x(const uint8_t *slot, const LaneC &L, uint32_t (&o)[8], uint32_t (&cv)[8]) {
        constexpr int sh = dshift(Y);
        constexpr uint32_t FD = MP::fwd_c(1u << (6 + PB));
        const int cy = L.cy[Y];
        if constexpr (Y * Q + X < KD) {
            const uint32_t po = L.fown ^ MP::hbank(X);
            read32(slot + X * NODE_BYTES + 16u * po, slot + X * NODE_BYTES + 16u * (po ^ FD), o);
        } else {
#pragma unroll
            for (int w = 0; w < 8; w++) o[w] = 0;
        }
        const uint32_t pc = L.fcl[Y] ^ MP::fwd_c(uint32_t(X) << sh);
        if ((Y * Q + cy) < KD) {
            const uint8_t *cbase = slot + cy * NODE_BYTES;
            read32(cbase + 16u * pc, cbase + 16u * (pc ^ FD), cv);
        } else {
#pragma unroll
            for (int w = 0; w < 8; w++) cv[w] = 0;
        }
    }
    // PRT of node x in the byte domain: U = O + gamma * C* (C* masked off for the red
    // vertex and for shortened companions).
    template <int Y, int X>
    __device__ static void prt_x(const uint32_t (&o)[8], const uint32_t (&cv)[8], const LaneC &L, uint32_t (&u)[8]) {
        const int cy = L.cy[Y];
        const bool creal = (Y * Q + cy) < KD;
        const uint32_t keep = (creal && X != cy) ? 0xffffffffu : 0u;
        const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
#pragma unroll
        for (int w = 0; w < 8; w++) u[w] = xor_xtime4_masked(o[w], cv[w], ks, kr);
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
    // One step, reads interleaved with compute (the slot stays busy until the next step).
    // pre(x) runs before node x: the caller issues that node's part of the next slot's
    // DMA there, so the DMA queue drains while the XOR networks run instead of stalling
    // every wave in issue right after the barrier.
    template <int Y, class Pre>
    __device__ static void section(const uint8_t *slot, const LaneC &L, uint32_t (&acc)[Q * 8], Pre &&pre) {
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            pre(xc);
            uint32_t o[8], cv[8], u[8];
            load_x<Y, x>(slot, L, o, cv);
            prt_x<Y, x>(o, cv, L, u);
            fold_x<Y, x>(u, acc);
        });
    }
    // Parity output C (8 planes) -> bytes -> HBM at parity node x, layer z.  Stores use
    // the SGPR-base + 32-bit offset form; the offset is formed here and kept opaque,
    // otherwise LICM hoists all 16 (node, layer) 64-bit addresses out of the tile loop.
    template <int X>
    __device__ static void put(const BsArgs &a, uint32_t (&cv)[8], uint32_t z, uint32_t pos, bool ragged, int nv) {
        transpose8(cv);
        uint32_t off = z * uint32_t(a.sc);
        asm volatile("" : "+v"(off));
        off += pos;
        if (!ragged) {
            st16s(a.par[X], off, cv[0], cv[1], cv[2], cv[3]);
            st16s(a.par[X], off + 16u, cv[4], cv[5], cv[6], cv[7]);
        } else {
            uint8_t *p = a.par[X] + off;
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (i < nv) *reinterpret_cast<uint2 *>(p + 8 * i) = make_uint2(cv[2 * i], cv[2 * i + 1]);
        }
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

    // Group g finished: red vertex C[g][z_g] = U, and the PFT pairs with groups h < g.
    template <int G>
    __device__ static void end_group(const BsArgs &a, const uint32_t (&acc)[Q * 8], Hold &H, int c, uint32_t pos,
                                     bool ragged, int nv) {
        const uint32_t zg = uint32_t(c * 4 + G);
        uint32_t cv[8];
#pragma unroll
        for (int w = 0; w < 8; w++) cv[w] = acc[G * 8 + w];
        put<G>(a, cv, zg, pos, ragged, nv);
        auto pair = [&](const uint32_t *uh_at_g, const uint32_t *ug_at_h, auto hc) BS_INL {
            constexpr int h = decltype(hc)::value;
            const uint32_t zh = uint32_t(c * 4 + h);
            uint32_t c1[8], c2[8];
            pft(uh_at_g, ug_at_h, c1);  // C[h][z_g]
            put<h>(a, c1, zg, pos, ragged, nv);
            pft(ug_at_h, uh_at_g, c2);  // C[g][z_h]
            put<G>(a, c2, zh, pos, ragged, nv);
        };
        auto keep = [&](int ri, int p) BS_INL {
#pragma unroll
            for (int w = 0; w < 8; w++) H.r[ri][w] = acc[p * 8 + w];
        };
        if constexpr (G == 0) {
            keep(0, 1);
            keep(1, 2);
            keep(2, 3);
        } else if constexpr (G == 1) {
            pair(acc + 0, H.r[0], std::integral_constant<int, 0>{});  // U[1][z0]
            keep(0, 2);
            keep(3, 3);
        } else if constexpr (G == 2) {
            pair(acc + 0, H.r[1], std::integral_constant<int, 0>{});  // U[2][z0]
            pair(acc + 8, H.r[0], std::integral_constant<int, 1>{});  // U[2][z1]
            keep(1, 3);
        } else {
            pair(acc + 0, H.r[2], std::integral_constant<int, 0>{});   // U[3][z0]
            pair(acc + 8, H.r[3], std::integral_constant<int, 1>{});   // U[3][z1]
            pair(acc + 16, H.r[1], std::integral_constant<int, 2>{});  // U[3][z2]
        }
    }
};

template <int KD, int M, int PARTS>
__global__ __launch_bounds__((Bs6Kernel<KD, M, PARTS>::BLOCK)) void k_bs6_encode(BsArgs a) {
    using Kn = Bs6Kernel<KD, M, PARTS>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int c = int(threadIdx.x) >> Kn::PB, part = int(threadIdx.x) & (PARTS - 1);
    const uint32_t lds0 = lds_addr_of(smem);
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    // tiles of this workgroup: xcd * tpx + slot + k * nslots
    int ntile = 0;
    for (uint32_t tix = slot; tix < a.tiles_per_xcd && xcd * a.tiles_per_xcd + tix < a.ntiles; tix += a.nslots) ntile++;
    if (ntile == 0) return;
    const int nsteps = ntile * Kn::STEPS;
    auto tile_b0 = [&](int k) { return (xcd * a.tiles_per_xcd + slot + uint32_t(k) * a.nslots) * uint32_t(Kn::W); };
    // counted waits: T = VMEM instructions issued so far by this wave; mk[j] = T right
    // after the DMA of slot (s + j) was issued (j = 0 .. AHEAD-1)
    int Tn = 0, mk[5] = {0, 0, 0, 0, 0};
    static_assert(Kn::AHEAD >= 1 && Kn::AHEAD <= 5, "mark shift register has 5 entries");
    auto issue = [&](int s) {
        if (s < nsteps) {
            const int k = s / Kn::STEPS, r = s % Kn::STEPS, g = r / 3, y = r % 3;
            Kn::dma_any(y, a, lds0 + uint32_t((s % Kn::RING) * Kn::SLOT), wave, lane, tile_b0(k), g);
            Tn += Kn::ndma(y);
        }
#pragma unroll
        for (int j = 0; j + 1 < Kn::AHEAD; j++) mk[j] = mk[j + 1];
        mk[Kn::AHEAD - 1] = Tn;
    };
    for (int s = 0; s < Kn::AHEAD; s++) issue(s);
    uint32_t acc[Kn::Q * 8];
    typename Kn::Hold H;
    const typename Kn::LaneC L = Kn::lane_consts(c, part);
    const uint32_t sc = uint32_t(a.sc);
    for (int s = 0; s < nsteps; s++) {
        const int k = s / Kn::STEPS, r = s % Kn::STEPS, g = r / 3, y = r % 3;
        const uint32_t b0 = tile_b0(k);
        const bool ragged = uint64_t(b0) + Kn::W > a.sc;
        uint8_t *slotp = smem + (s % Kn::RING) * Kn::SLOT;
        if (ragged) {  // plain (uncounted) stores may be in flight: wait for everything
            wait_vm_n<0>();
            Kn::patch_any(y, a, slotp, wave, lane, b0, g);
        } else {
            wait_vm_rt(Tn - mk[0]);
        }
        lds_barrier();
        {
            // refill the slot every wave finished reading last step, one node per x below
            const int s2 = s + Kn::AHEAD;
            const bool more = s2 < nsteps;
            const int k2 = s2 / Kn::STEPS, r2 = s2 % Kn::STEPS, g2 = r2 / 3, y2 = r2 % 3;
            const uint32_t nb0 = tile_b0(k2), slot2 = lds0 + uint32_t((s2 % Kn::RING) * Kn::SLOT);
            uint32_t vl = Kn::MP::inv_d(uint32_t(lane));
            asm volatile("" : "+v"(vl));
            auto pre = [&](auto xc) BS_INL {
                constexpr int x = decltype(xc)::value;
                if (more) Kn::template dma_node_any<x>(y2, a, slot2, wave, vl, nb0, g2);
            };
            if (y == 0) Kn::template section<0>(slotp, L, acc, pre);
            else if (y == 1) Kn::template section<1>(slotp, L, acc, pre);
            else Kn::template section<2>(slotp, L, acc, pre);
            if (more) Tn += Kn::ndma(y2);
#pragma unroll
            for (int j = 0; j + 1 < Kn::AHEAD; j++) mk[j] = mk[j + 1];
            mk[Kn::AHEAD - 1] = Tn;
        }
        if (y == 2) {
            const uint32_t pos = b0 + uint32_t(32 * part);
            const int nv = pos >= sc ? 0 : ((sc - pos) / 8 > 4 ? 4 : int((sc - pos) / 8));
            if (g == 0) Kn::template end_group<0>(a, acc, H, c, pos, ragged, nv);
            else if (g == 1) Kn::template end_group<1>(a, acc, H, c, pos, ragged, nv);
            else if (g == 2) Kn::template end_group<2>(a, acc, H, c, pos, ragged, nv);
            else Kn::template end_group<3>(a, acc, H, c, pos, ragged, nv);
            Tn += Kn::stores(g);
        }
    }
    wait_vm0();
}

}  // namespace bs
}  // namespace clay
