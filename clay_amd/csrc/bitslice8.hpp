// bitslice8.hpp -- v8 bit-sliced encode for (10,4,13): register-staged loads three steps
// deep, bit-planes exchanged through LDS, PRT in the plane domain.
//
// What the v7 probes measured (1 GiB stripe): memory-only 0.355 ms, compute-only 0.28 ms,
// both 0.41 ms; the same access pattern from registers with 4x the bytes in flight per CU
// reads at 5.3 TB/s (bench_tools/page_probe.hip).  v7 keeps at most ~2 steps (96-128 KiB)
// in flight because its LDS ring is the landing buffer.  v8 lands a lane's OWN bytes in
// VGPRs instead (global_load_dwordx4, no LDS-DMA):
//
//  * one VGPR buffer per section Y (step s = (g, Y) uses buffer Y; 32 / 32 / 16 VGPRs),
//    refilled with step s + 3 as soon as step s has been transposed and written to LDS:
//    three steps of loads in flight;
//  * each lane transposes its own 32 bytes per node to 8 bit-planes ONCE and writes the
//    planes to an LDS exchange image (v6's conflict-free piece map); after a barrier it
//    reads back its own planes and its companion's planes;
//  * PRT U = C + gamma C* is then 8 plane XORs (gamma = x: plane rename + 3 XORs) instead
//    of the byte-domain xtime; RS fold and PFT as in v6;
//  * the U values held for later PFT pairs live in lane-private LDS sets (64 KiB), so the
//    three register buffers fit in 256 VGPRs without spilling.
//
// Tiles and the balanced tail as in v7 (TileMap7).  Bytes are identical to v6/v7.
#pragma once

#include "bitslice7.hpp"

namespace clay {
namespace bs {

struct Bs8Kernel {
    using K6 = Bs6Kernel<10, 4, 8, false>;
    using MP = typename K6::MP;
    using S = typename K6::S;
    static constexpr int Q = 4, T = 4, KD = 10, W = 256, BLOCK = 512;
    static constexpr int NODE_BYTES = K6::NODE_BYTES;  // 64 columns x 256 B = 16 KiB
    static constexpr int REGION = Q * NODE_BYTES;      // one step's exchange image (64 KiB)
    static constexpr int HOLD_SET = BLOCK * 32;        // one lane-private 8-plane set per lane
    static constexpr int LDS_BYTES = REGION + 4 * HOLD_SET;  // image + 4 hold sets: 128 KiB
    static constexpr int STEPS = 12;
    static constexpr uint32_t FD = MP::fwd_c(1u << (6 + K6::PB));  // piece-index bit of the second 16 bytes
    static_assert(NODE_BYTES == 16384, "v8 geometry");

    // own bytes of node X: two 16-byte pieces at chunk offsets o0, o1; lanes whose first
    // piece straddles the end of a partial tile (8 valid bytes) loaded it from vend - 16
    // and take its upper half (m0)
    template <int Y, int X>
    __device__ static void load_own(const BsArgs &a, uint32_t o0, uint32_t o1, uint32_t m0, uint32_t m1,
                                    uint32_t (&d)[8]) {
        constexpr int node = Y * Q + X;
        const uint4 v0 = *reinterpret_cast<const uint4 *>(a.data[node] + o0);
        const uint4 v1 = *reinterpret_cast<const uint4 *>(a.data[node] + o1);
        d[0] = sel(m0, v0.z, v0.x); d[1] = sel(m0, v0.w, v0.y); d[2] = v0.z; d[3] = v0.w;
        d[4] = sel(m1, v1.z, v1.x); d[5] = sel(m1, v1.w, v1.y); d[6] = v1.z; d[7] = v1.w;
    }
    // One code path for full and partial tiles (no per-piece branches: they doubled the
    // buffers' live copies and spilled).  In a partial tile a piece wholly past vend reads
    // the tile's first piece instead (its bytes are never stored), a straddling piece reads
    // [vend - 16, vend) (tile ends are 8-byte aligned, so 8 bytes are valid).
    template <int Y>
    __device__ static void load_step(const BsArgs &a, uint32_t lane_off, uint32_t g, Tile7 t, uint32_t pos_part,
                                     uint32_t (&buf)[Q][8]) {
        uint32_t q0 = t.b0 + pos_part, q1 = q0 + 16u, m0 = 0u, m1 = 0u;
        if (t.vend < t.b0 + uint32_t(W)) {
            auto fix = [&](uint32_t &q, uint32_t &m) BS_INL {
                if (q + 16u > t.vend) {
                    m = q + 8u <= t.vend ? 0xffffffffu : 0u;
                    q = q + 8u <= t.vend ? t.vend - 16u : t.b0;
                }
            };
            fix(q0, m0);
            fix(q1, m1);
        }
        const uint32_t row = g * uint32_t(a.sc) + lane_off - pos_part;  // layer 4c + g, position 0
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            if constexpr (Y * Q + x < KD) load_own<Y, x>(a, row + q0, row + q1, m0, m1, buf[x]);
        });
    }

    // transpose own bytes to planes and write them to the exchange image of node x
    template <int Y>
    __device__ static void put_planes(uint8_t *img, uint32_t fown, uint32_t (&buf)[Q][8]) {
        asm volatile("" : "+v"(fown));
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            if constexpr (Y * Q + x < KD) {
                transpose8(buf[x]);
                const uint32_t po = fown ^ MP::hbank(x);
                uint8_t *b = img + x * NODE_BYTES;
                *reinterpret_cast<uint4 *>(b + 16u * po) = make_uint4(buf[x][0], buf[x][1], buf[x][2], buf[x][3]);
                *reinterpret_cast<uint4 *>(b + 16u * (po ^ FD)) =
                    make_uint4(buf[x][4], buf[x][5], buf[x][6], buf[x][7]);
            }
        });
    }

    // plane-domain PRT of node x + RS fold (section Y): U = own ^ gamma * comp (comp masked
    // for the red vertex and for shortened companions; a shortened node's own C is zero)
    template <int Y>
    __device__ static void section(const uint8_t *img, const typename K6::LaneC &L, uint32_t (&acc)[Q * 8]) {
        constexpr int sh = K6::dshift(Y);
        // lane constants made opaque here: otherwise LICM hoists every derived LDS address
        // and mask (~60 values) out of the tile loop and the kernel spills
        uint32_t fown = L.fown, fcl = L.fcl[Y];
        int cy = L.cy[Y];
        asm volatile("" : "+v"(fown), "+v"(fcl), "+v"(cy));
        const bool creal = (Y * Q + cy) < KD;
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            {  // shortened nodes (C = 0) still have U = gamma * C* != 0 (decode.rs:290-298)
                uint32_t o[8], cv[8], u[8];
                uint32_t po = fown ^ MP::hbank(x);
                asm volatile("" : "+v"(po));
                if constexpr (Y * Q + x < KD) {
                    K6::read32(img + x * NODE_BYTES + 16u * po, img + x * NODE_BYTES + 16u * (po ^ FD), o);
                } else {
#pragma unroll
                    for (int w = 0; w < 8; w++) o[w] = 0;
                }
                uint32_t pc = fcl ^ MP::fwd_c(uint32_t(x) << sh);
                asm volatile("" : "+v"(pc));
                if (creal) {
                    const uint8_t *cb = img + cy * NODE_BYTES;
                    K6::read32(cb + 16u * pc, cb + 16u * (pc ^ FD), cv);
                } else {
#pragma unroll
                    for (int w = 0; w < 8; w++) cv[w] = 0;
                }
                const uint32_t keep = (creal && x != cy) ? 0xffffffffu : 0u;
                // gamma * comp on planes: [c7, c0, c1^c7, c2^c7, c3^c7, c4, c5, c6] (poly 0x11D)
                u[0] = __builtin_amdgcn_bitop3_b32(o[0], cv[7], keep, kXorAnd);
                u[1] = __builtin_amdgcn_bitop3_b32(o[1], cv[0], keep, kXorAnd);
                u[2] = __builtin_amdgcn_bitop3_b32(o[2], cv[1] ^ cv[7], keep, kXorAnd);
                u[3] = __builtin_amdgcn_bitop3_b32(o[3], cv[2] ^ cv[7], keep, kXorAnd);
                u[4] = __builtin_amdgcn_bitop3_b32(o[4], cv[3] ^ cv[7], keep, kXorAnd);
                u[5] = __builtin_amdgcn_bitop3_b32(o[5], cv[4], keep, kXorAnd);
                u[6] = __builtin_amdgcn_bitop3_b32(o[6], cv[5], keep, kXorAnd);
                u[7] = __builtin_amdgcn_bitop3_b32(o[7], cv[6], keep, kXorAnd);
                sfor<Q>([&](auto pc_) BS_INL {
                    constexpr int p = decltype(pc_)::value;
                    sfor<8>([&](auto bc) BS_INL {
                        constexpr int bo = decltype(bc)::value;
                        constexpr uint64_t mk = plane_mask(S::RS.g[p][Y * Q + x], bo, 0);
                        acc[p * 8 + bo] = xor_sel<mk, (Y > 0 || x > 0)>(acc[p * 8 + bo], u);
                    });
                });
            }
            // one node's reads + XOR network at a time: hoisting every node's LDS reads
            // ahead (64 VGPRs) spills the kernel
            __builtin_amdgcn_sched_barrier(0);
        });
    }

    // one step: planes of step s out to LDS, refill the section's buffer with step s + 3,
    // barrier, PRT + fold from LDS
    template <int Y>
    __device__ static void step(const BsArgs &a, uint8_t *smem, int s, uint32_t (&buf)[Q][8],
                                const typename K6::LaneC &L, uint32_t (&acc)[Q * 8], uint32_t lane_off,
                                uint32_t pos_part, const TileMap7 &tm, uint32_t slot, uint32_t ns, int nsteps) {
        uint8_t *img = smem;
        lds_barrier();  // every wave has finished reading the previous step's image
        put_planes<Y>(img, L.fown, buf);
        __builtin_amdgcn_sched_barrier(0);
        const int s3 = s + 3;
        if (s3 < nsteps) {
            const int k3 = s3 / STEPS, g3 = (s3 % STEPS) / 3;
            load_step<Y>(a, lane_off, uint32_t(g3), tm.tile(k3, slot, ns), pos_part, buf);
        }
        lds_barrier();
        section<Y>(img, L, acc);
    }
};

// Group g finished (as Bs6Kernel::end_group): red vertex C[g][z_g] = U, and the PFT pairs
// with groups h < g.  The U values later groups' pairs need stay in four lane-private LDS
// sets instead of 32 VGPRs (with three steps of loads in registers the kernel would spill):
// after group 0 set 0 = U[1][z0], 1 = U[2][z0], 2 = U[3][z0]; after group 1 set 0 =
// U[2][z1], 3 = U[3][z1]; after group 2 set 1 = U[3][z2].
template <int G>
__device__ __forceinline__ void bs8_end_group(const BsArgs &a, const uint32_t (&acc)[32], uint8_t *hold, int c,
                                              uint32_t pos, bool ragged, int nv) {
    using K6 = typename Bs8Kernel::K6;
    uint8_t *const hp = hold + threadIdx.x * 32u;
    auto ldh = [&](int r, uint32_t (&d)[8]) BS_INL {
        K6::read32(hp + r * Bs8Kernel::HOLD_SET, hp + r * Bs8Kernel::HOLD_SET + 16, d);
    };
    auto sth = [&](int r, int p) BS_INL {
        *reinterpret_cast<uint4 *>(hp + r * Bs8Kernel::HOLD_SET) =
            make_uint4(acc[p * 8 + 0], acc[p * 8 + 1], acc[p * 8 + 2], acc[p * 8 + 3]);
        *reinterpret_cast<uint4 *>(hp + r * Bs8Kernel::HOLD_SET + 16) =
            make_uint4(acc[p * 8 + 4], acc[p * 8 + 5], acc[p * 8 + 6], acc[p * 8 + 7]);
    };
    const uint32_t zg = uint32_t(c * 4 + G);
    {
        uint32_t cv[8];
#pragma unroll
        for (int w = 0; w < 8; w++) cv[w] = acc[G * 8 + w];
        K6::template put<G>(a, cv, zg, pos, ragged, nv);
    }
    auto pair = [&](const uint32_t *uh_at_g, int r, auto hc) BS_INL {
        constexpr int h = decltype(hc)::value;
        uint32_t ug_at_h[8];
        ldh(r, ug_at_h);
        const uint32_t zh = uint32_t(c * 4 + h);
        uint32_t c1[8], c2[8];
        K6::pft(uh_at_g, ug_at_h, c1);  // C[h][z_g]
        K6::template put<h>(a, c1, zg, pos, ragged, nv);
        K6::pft(ug_at_h, uh_at_g, c2);  // C[g][z_h]
        K6::template put<G>(a, c2, zh, pos, ragged, nv);
        __builtin_amdgcn_sched_barrier(0);
    };
    if constexpr (G == 0) {
        sth(0, 1);
        sth(1, 2);
        sth(2, 3);
    } else if constexpr (G == 1) {
        pair(acc + 0, 0, std::integral_constant<int, 0>{});  // U[1][z0]
        sth(0, 2);
        sth(3, 3);
    } else if constexpr (G == 2) {
        pair(acc + 0, 1, std::integral_constant<int, 0>{});  // U[2][z0]
        pair(acc + 8, 0, std::integral_constant<int, 1>{});  // U[2][z1]
        sth(1, 3);
    } else {
        pair(acc + 0, 2, std::integral_constant<int, 0>{});   // U[3][z0]
        pair(acc + 8, 3, std::integral_constant<int, 1>{});   // U[3][z1]
        pair(acc + 16, 1, std::integral_constant<int, 2>{});  // U[3][z2]
    }
}

// a.tiles_per_xcd = XCD region bytes, a.nslots = workgroups per XCD (as v7); 128 KiB LDS
__global__ __launch_bounds__(512) void k_bs8_encode(BsArgs a) {
    using Kn = Bs8Kernel;
    using K6 = typename Kn::K6;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int c = int(threadIdx.x) >> K6::PB, part = int(threadIdx.x) & 7;
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3, ns = a.nslots;
    const TileMap7 tm(uint32_t(a.sc), a.tiles_per_xcd, ns, xcd, slot);
    const int ntile = tm.ntile();
    if (ntile == 0) return;
    const int nsteps = ntile * Kn::STEPS;
    const uint32_t pos_part = uint32_t(32 * part);
    const uint32_t lane_off = uint32_t(c) * 4u * uint32_t(a.sc) + pos_part;  // row 4c of the group
    const typename K6::LaneC L = K6::lane_consts(c, part);
    uint32_t buf0[4][8], buf1[4][8], buf2[4][8];
    {
        const Tile7 t0 = tm.tile(0, slot, ns);
        Kn::load_step<0>(a, lane_off, 0u, t0, pos_part, buf0);
        Kn::load_step<1>(a, lane_off, 0u, t0, pos_part, buf1);
        Kn::load_step<2>(a, lane_off, 0u, t0, pos_part, buf2);
    }
    uint32_t acc[32];
    uint8_t *const hold = smem + Kn::REGION;
    for (int s = 0; s < nsteps; s += 3) {
        const int k = s / Kn::STEPS, g = (s % Kn::STEPS) / 3;
        const Tile7 t = tm.tile(k, slot, ns);
        Kn::step<0>(a, smem, s, buf0, L, acc, lane_off, pos_part, tm, slot, ns, nsteps);
        Kn::step<1>(a, smem, s + 1, buf1, L, acc, lane_off, pos_part, tm, slot, ns, nsteps);
        Kn::step<2>(a, smem, s + 2, buf2, L, acc, lane_off, pos_part, tm, slot, ns, nsteps);
        const bool ragged = t.vend < t.b0 + uint32_t(Kn::W);
        const uint32_t pos = t.b0 + pos_part;
        const int nv = pos >= t.vend ? 0 : ((t.vend - pos) / 8 > 4 ? 4 : int((t.vend - pos) / 8));
        if (g == 0) bs8_end_group<0>(a, acc, hold, c, pos, ragged, nv);
        else if (g == 1) bs8_end_group<1>(a, acc, hold, c, pos, ragged, nv);
        else if (g == 2) bs8_end_group<2>(a, acc, hold, c, pos, ragged, nv);
        else bs8_end_group<3>(a, acc, hold, c, pos, ragged, nv);
    }
}

}  // namespace bs
}  // namespace clay
