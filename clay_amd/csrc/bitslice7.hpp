// bitslice7.hpp -- v7 bit-sliced encode for (10,4,13): v6's compute on a per-section LDS
// map that keeps two steps of DMA in flight, and a balanced tail.
//
// v6 (256-byte tiles) streams (section Y, group g) slots through a 2-slot ring of 64 KiB:
// while a step computes, only the next step's slot is in flight, and it must land in
// full before the next barrier -- a sawtooth that leaves the memory pipe idle at every
// step boundary.  v7 keys the LDS by node instead: node i of the current group lives at
// node-slot i (10 x 16 KiB = 160 KiB, the whole CU), so step s = (g, Y) reads region Y
// while region Y+1 (step s+1) and region Y-1 (step s+2, refilled as soon as the barrier
// of step s proves step s-1's reads are done) are in flight: two steps ahead, 6 of 10
// node-slots (96 KiB) loading during a 4-node step, 8 during a 2-node step.
//
// Tail: v6 deals 256-byte tiles round-robin, so 1,639 tiles over 256 workgroups take 7
// rounds where 6.4 carry data.  v7 gives every XCD a contiguous byte region, deals full
// tiles to its workgroups in rounds (adjacent workgroups read adjacent 256-byte runs, so
// the 128-byte lines they share are fetched once into the XCD's L2), and cuts the
// remainder into one partial tile per workgroup (a multiple of 32 bytes), so the last
// round costs about the fraction of a round it carries.
//
// Bytes are identical to v6 (same XOR networks, same slot image per node).
#pragma once

#include "bitslice6.hpp"

namespace clay {
namespace bs {

template <bool NT>
__device__ __forceinline__ void dma16p(uint32_t lds_addr, const uint8_t *sbase, uint32_t voff) {
    unsigned keep;  // M0 is compiler-reserved: save / restore it in the same statement
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3 nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "s"(lds_addr), "v"(voff), "s"(sbase)
                     : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "s"(lds_addr), "v"(voff), "s"(sbase)
                     : "memory");
}

// A tile: positions [b0, b0 + 256) of every sub-chunk row, valid below vend.
struct Tile7 {
    uint32_t b0, vend;
};

// Tile k of a workgroup.  XCD x owns bytes [x * region, min((x + 1) * region, sc));
// full tiles go round-robin over the XCD's ns workgroups, the remainder is cut into
// one partial tile per workgroup (width a multiple of 32 bytes), always its last.
struct TileMap7 {
    uint32_t x0, x1, nfull, p0, p1;
    __device__ TileMap7(uint32_t sc, uint32_t region, uint32_t ns, uint32_t xcd, uint32_t slot) {
        x0 = xcd * region;
        x1 = x0 + region < sc ? x0 + region : sc;
        nfull = p0 = p1 = 0;
        if (x0 >= x1) return;
        const uint32_t len = x1 - x0, round = ns * 256u;
        nfull = len / round;
        const uint32_t left = len - nfull * round;
        const uint32_t wp = ((left + ns - 1) / ns + 31u) & ~31u;
        const uint32_t q0 = x0 + nfull * round + slot * wp;
        if (left && q0 < x1) {
            p0 = q0;
            p1 = q0 + wp < x1 ? q0 + wp : x1;
        }
    }
    __device__ int ntile() const { return int(nfull) + (p0 < p1 ? 1 : 0); }
    __device__ Tile7 tile(int k, uint32_t slot, uint32_t ns) const {
        if (uint32_t(k) < nfull) {
            const uint32_t b0 = x0 + (uint32_t(k) * ns + slot) * 256u;
            return {b0, b0 + 256u};
        }
        return {p0, p1};
    }
};

template <bool NT>
struct Bs7Kernel {
    using K6 = Bs6Kernel<10, 4, 8, false>;
    using MP = typename K6::MP;
    static constexpr int Q = K6::Q, T = K6::T, KD = 10;
    static constexpr int W = K6::W, BLOCK = K6::BLOCK, WAVES = K6::WAVES;
    static constexpr int NODE_BYTES = K6::NODE_BYTES;  // 64 layers x 256 B = 16 KiB
    static constexpr int REGION = Q * NODE_BYTES;      // section Y's nodes: node-slots 4Y..4Y+3
    static constexpr int LDS_BYTES = KD * NODE_BYTES;  // 160 KiB
    static constexpr int STEPS = K6::STEPS;            // 12 (group, section) steps per tile
    static constexpr int AHEAD = 2;
    static constexpr int DMA_PER_NODE = K6::DMA_PER_NODE;
    static_assert(W == 256 && NODE_BYTES == 16384 && LDS_BYTES == 163840, "v7 geometry");

    // DMA of node X of step (section Y, group g), pieces past vend clamped: a straddling
    // piece (8 valid bytes) to vend - 16 (patched after landing), a piece wholly past
    // vend to b0 (a line this tile reads anyway; the bytes are never used).
    template <int Y, int X>
    __device__ static void dma_node(const BsArgs &a, uint32_t lds0, int wave, uint32_t vl, Tile7 t, int g) {
        constexpr int node = Y * Q + X;
        if constexpr (node < KD) {
            const uint32_t sc = uint32_t(a.sc);
#pragma unroll
            for (int i = 0; i < DMA_PER_NODE; i++) {
                const uint32_t blk = uint32_t(wave * DMA_PER_NODE + i);
                const uint32_t v = vl ^ MP::inv_d((blk << 6) ^ MP::hbank(X));
                uint32_t pos = t.b0 + K6::piece_off(v);
                if (pos + 16u > t.vend) pos = pos >= t.vend ? t.b0 : t.vend - 16u;
                const uint32_t layer = (v & 63u) * 4u + uint32_t(g);
                dma16p<NT>(lds0 + uint32_t(node * NODE_BYTES) + blk * 1024u, a.data[node], layer * sc + pos);
            }
        }
    }
    template <int X>
    __device__ static void dma_node_any(int y, const BsArgs &a, uint32_t lds0, int wave, uint32_t vl, Tile7 t,
                                        int g) {
        if (y == 0) dma_node<0, X>(a, lds0, wave, vl, t, g);
        else if (y == 1) dma_node<1, X>(a, lds0, wave, vl, t, g);
        else dma_node<2, X>(a, lds0, wave, vl, t, g);
    }
    __device__ static void dma_step(int y, const BsArgs &a, uint32_t lds0, int wave, uint32_t vl, Tile7 t, int g) {
        sfor<Q>([&](auto xc) BS_INL { dma_node_any<decltype(xc)::value>(y, a, lds0, wave, vl, t, g); });
    }
    static constexpr int ndma(int y) { return K6::ndma(y); }

    // The straddling piece of each row (vend - b0 not a multiple of 16): 8 valid bytes.
    template <int Y>
    __device__ static void patch(const BsArgs &a, uint8_t *smem, int wave, int lane, Tile7 t, int g) {
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
                    const uint32_t pos = t.b0 + K6::piece_off(v);
                    if (pos < t.vend && pos + 16u > t.vend) {
                        const uint32_t layer = (v & 63u) * 4u + uint32_t(g);
                        const uint2 gv = *reinterpret_cast<const uint2 *>(a.data[node] + layer * sc + pos);
                        *reinterpret_cast<uint4 *>(smem + node * NODE_BYTES + blk * 1024 + lane * 16) =
                            make_uint4(gv.x, gv.y, 0u, 0u);
                    }
                }
            }
        });
    }
    __device__ static void patch_any(int y, const BsArgs &a, uint8_t *smem, int wave, int lane, Tile7 t, int g) {
        if (y == 0) patch<0>(a, smem, wave, lane, t, g);
        else if (y == 1) patch<1>(a, smem, wave, lane, t, g);
        else patch<2>(a, smem, wave, lane, t, g);
    }
};

// a.tiles_per_xcd carries the XCD region length in bytes (multiple of 32), a.nslots the
// workgroups per XCD; grid = 8 * nslots, one 512-lane workgroup per CU (160 KiB LDS).
// PROBE (measurement only, wrong bytes), bits: 1 = no compute, 2 = no DMA, 4 = no parity
// stores, 8 = no workgroup barriers
template <bool NT, int PROBE = 0>
__global__ __launch_bounds__(512) void k_bs7_encode(BsArgs a) {
    using Kn = Bs7Kernel<NT>;
    using K6 = typename Kn::K6;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int c = int(threadIdx.x) >> K6::PB, part = int(threadIdx.x) & 7;
    const uint32_t lds0 = lds_addr_of(smem);
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3, ns = a.nslots;
    const TileMap7 tm(uint32_t(a.sc), a.tiles_per_xcd, ns, xcd, slot);
    const int ntile = tm.ntile();
    if (ntile == 0) return;
    const int nsteps = ntile * Kn::STEPS;
    const uint32_t vl0 = Kn::MP::inv_d(uint32_t(lane));
    // counted waits: Tn = VMEM instructions issued so far by this wave; mk[j] = Tn right
    // after the DMA of step s + j was issued
    int Tn = 0, mk[Kn::AHEAD] = {};
    auto push = [&]() {
#pragma unroll
        for (int j = 0; j + 1 < Kn::AHEAD; j++) mk[j] = mk[j + 1];
        mk[Kn::AHEAD - 1] = Tn;
    };
    for (int s = 0; s < Kn::AHEAD; s++) {  // nsteps >= 12
        if (PROBE & 2) break;
        Kn::dma_step(s % 3, a, lds0, wave, vl0, tm.tile(0, slot, ns), s / 3);
        Tn += Kn::ndma(s % 3);
        push();
    }
    uint32_t acc[Kn::Q * 8];
    typename K6::Hold H;
    const typename K6::LaneC L = K6::lane_consts(c, part);
    for (int s = 0; s < nsteps; s++) {
        const int k = s / Kn::STEPS, r = s % Kn::STEPS, g = r / 3, y = r % 3;
        const Tile7 t = tm.tile(k, slot, ns);
        const bool ragged = t.vend < t.b0 + uint32_t(Kn::W);
        if (PROBE & 2) {
        } else if (ragged) {  // partial tile (a workgroup's last): drain, patch the straddlers
            wait_vm_n<0>();
            if ((t.vend - t.b0) & 15u) Kn::patch_any(y, a, smem, wave, lane, t, g);
        } else {
            wait_vm_rt(Tn - mk[0]);
        }
        if constexpr ((PROBE & 8) == 0) lds_barrier();
        // refill region y - 1 (read by step s - 1; the barrier proved every wave is done)
        // with step s + 2, one node ahead of each node's compute below
        const int s2 = s + Kn::AHEAD;
        const bool more = s2 < nsteps && !(PROBE & 2);
        const int k2 = s2 / Kn::STEPS, r2 = s2 % Kn::STEPS, g2 = r2 / 3, y2 = r2 % 3;
        const Tile7 t2 = tm.tile(k2, slot, ns);
        uint32_t vl = vl0;
        asm volatile("" : "+v"(vl));
        auto pre = [&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            if (more) Kn::template dma_node_any<x>(y2, a, lds0, wave, vl, t2, g2);
        };
        if constexpr ((PROBE & 1) != 0) {
            sfor<Kn::Q>([&](auto xc) BS_INL { pre(xc); });
            if (y == 0 && g == 0)
#pragma unroll
                for (int w = 0; w < Kn::Q * 8; w++) acc[w] = (threadIdx.x * 0x9E3779B9u) ^ uint32_t(w) ^ uint32_t(s);
        } else {
            if (y == 0) K6::template section<0>(smem, L, acc, pre);
            else if (y == 1) K6::template section<1>(smem + Kn::REGION, L, acc, pre);
            else K6::template section<2>(smem + 2 * Kn::REGION, L, acc, pre);
        }
        if (more) Tn += Kn::ndma(y2);
        push();
        if (y == 2 && !(PROBE & 4)) {
            const uint32_t pos = t.b0 + uint32_t(32 * part);
            const int nv = pos >= t.vend ? 0 : ((t.vend - pos) / 8 > 4 ? 4 : int((t.vend - pos) / 8));
            if (g == 0) K6::template end_group<0>(a, acc, H, c, pos, ragged, nv);
            else if (g == 1) K6::template end_group<1>(a, acc, H, c, pos, ragged, nv);
            else if (g == 2) K6::template end_group<2>(a, acc, H, c, pos, ragged, nv);
            else K6::template end_group<3>(a, acc, H, c, pos, ragged, nv);
            if (!ragged) Tn += K6::stores(g);  // a ragged tile's plain stores stay uncounted
        }
    }
    wait_vm0();
}

}  // namespace bs
}  // namespace clay
