// stream_encode3.hpp -- the streaming encode for q = m = 3, t = 4 codes whose data nodes fill
// y-sections 0-2 and whose parity nodes are section 3: (9,3,11) (alpha 81).  The (10,4) kernel's
// memory structure (stream_encode.hpp) with the streaming repair kernel's tile (repair_kernel.hpp):
//
//  * group g = layer digit 3 (the parity section's digit); a group's 27 layers z = 3c + g are the
//    "plane" of column c = (d0, d1, d2).  Encode = decode with every parity node erased
//    (encode.rs:57-68, decode.rs:167-257): all layers have iscore 1, so one pass fuses
//    PRT -> RS fold -> PFT, the PRT companions of data section Y vary digit Y (same group), the
//    PFT pairs of section 3 vary digit 3 (the lane's other groups: held in registers).
//  * tile = W = 512 byte positions of every row; lane = (column c, part), 27 x 16 = 432 lanes
//    (7 compute waves), 32 positions per lane = pieces part and part + 16 of its row; a 16-lane
//    group reads one row's 256 contiguous bytes, so LDS reads need no swizzle.
//  * step (g, Y): section Y's three data nodes at group g's 27 rows, one LDS node buffer each
//    (27 x 512 B = 13.5 KiB in 14 KiB); 9 steps per tile; a ring of 11 node buffers filled by
//    LOADERS dedicated waves (LDS-DMA takes any byte alignment: the 2 mod 8 rows of the 256 MiB
//    BASELINE chunk stream like aligned ones; the partial last tile is patched byte by byte).
//  * end of group g: red vertex C[g][z_g] = U, PFT pairs with the earlier groups, 16-byte stores
//    at any alignment (each 16-lane group writes two 256-byte runs of one parity row).
#pragma once

#include "bitslice.hpp"
#include "encode3_args.hpp"
#include "stream_encode.hpp"  // uniform_ptr
#include "xor_cse.hpp"

namespace clay {
namespace bs {

template <int KD, int M, int LOADERS>
struct StreamEnc3 {
    using S = Shape<KD, M>;
    static constexpr int Q = S::Q, T = S::T, ALPHA = S::ALPHA;
    static_assert(KD == 9 && M == 3 && Q == 3 && T == 4 && S::NU == 0, "data sections 0-2, parity section 3");
    static constexpr int COLS = ALPHA / Q;                     // 27 rows per group
    static constexpr int PARTS = 16, W = 32 * PARTS, LANES = COLS * PARTS;
    static constexpr int CWAVES = (LANES + 63) / 64;            // 7
    static constexpr int BLOCK = 64 * (CWAVES + LOADERS);
    static constexpr int NBLK = (COLS * W + 1023) / 1024;       // 14 DMA instructions per node buffer
    static constexpr int NODE = NBLK * 1024;
    static constexpr int NB = (160 * 1024) / NODE;              // 11 buffers
    static constexpr int LDS_BYTES = NB * NODE;
    static constexpr int BPL = NBLK / LOADERS;
    static_assert(NBLK % LOADERS == 0, "node blocks split evenly over the loader waves");
    static constexpr int RPB = 1024 / W;                        // rows per DMA block (2)
    static constexpr int STEPS = Q * (T - 1);                   // 9 (group, section) steps
    static constexpr int NT = STEPS * Q;                        // 27 loads per tile
    static_assert(NB >= 2 * Q, "ring: two steps' loads in flight");
    static constexpr uint32_t jw(int y) { return y == 0 ? 9u : y == 1 ? 3u : 1u; }  // digit y's weight in c

    // ---------------- loader ----------------
    struct Loader {
        uint32_t roff[BPL];  // (3 row) * sc + 16 * piece: row r of a group buffer is layer 3 r + g
        uint32_t k16[BPL];
    };
    __device__ static void loader_init(Loader &L, uint32_t sc, int li, int lane) {
#pragma unroll
        for (int j = 0; j < BPL; j++) {
            const uint32_t blk = uint32_t(li * BPL + j);
            uint32_t r = blk * uint32_t(RPB) + uint32_t(lane) * 16u / uint32_t(W);
            if (r >= uint32_t(COLS)) r = 0;  // padding of the last block: any valid row
            L.roff[j] = 3u * r * sc;
            L.k16[j] = (uint32_t(lane) * 16u) % uint32_t(W);
        }
    }
    // node row base = data[node] + g * sc (the group's first layer)
    __device__ static void issue(const Loader &L, uint32_t lds_buf, const uint8_t *nbase, uint32_t b0, uint32_t vend,
                                 int li) {
        lds_buf = __builtin_amdgcn_readfirstlane(lds_buf);
        if (vend >= b0 + uint32_t(W)) {
            const uint8_t *base = uniform_ptr(nbase + b0);
#pragma unroll
            for (int j = 0; j < BPL; j++) dma16(lds_buf + uint32_t(li * BPL + j) * 1024u, base, L.roff[j] + L.k16[j]);
        } else {
            // partial tile: a piece straddling vend (or past it) is read from vend - 16 and the
            // straddling one rewritten by patch() (vend = sc >= 16)
            const uint8_t *base = uniform_ptr(nbase);
#pragma unroll
            for (int j = 0; j < BPL; j++) {
                uint32_t pos = b0 + L.k16[j];
                if (pos + 16u > vend) pos = vend - 16u;
                dma16(lds_buf + uint32_t(li * BPL + j) * 1024u, base, L.roff[j] + pos);
            }
        }
    }
    __device__ static void patch(const Loader &L, uint8_t *buf, const uint8_t *nbase, uint32_t b0, uint32_t vend, int li,
                                 int lane) {
#pragma unroll
        for (int j = 0; j < BPL; j++) {
            const uint32_t pos = b0 + L.k16[j];
            if (pos < vend && pos + 16u > vend) {
                uint32_t w[4] = {0u, 0u, 0u, 0u};
                const uint8_t *src = nbase + L.roff[j] + pos;
                for (uint32_t b = 0; b < vend - pos; b++) w[b >> 2] |= uint32_t(src[b]) << (8u * (b & 3u));
                *reinterpret_cast<uint4 *>(buf + (li * BPL + j) * 1024 + lane * 16) = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
    }

    // ---------------- compute ----------------
    __device__ static void read32(const uint8_t *buf, uint32_t r, uint32_t part, uint32_t (&d)[8]) {
        const uint8_t *row = buf + r * uint32_t(W);
        const uint4 v0 = *reinterpret_cast<const uint4 *>(row + (part << 4));
        const uint4 v1 = *reinterpret_cast<const uint4 *>(row + ((part + uint32_t(PARTS)) << 4));
        d[0] = v0.x; d[1] = v0.y; d[2] = v0.z; d[3] = v0.w;
        d[4] = v1.x; d[5] = v1.y; d[6] = v1.z; d[7] = v1.w;
    }
    // the fold of data node (Y, X) into the Q parity accumulators: 24 output rows over 8 input
    // planes, CSE-factored at compile time (xor_cse.hpp)
    template <int I>
    struct FoldCse {
        static constexpr XorCse make() {
            uint32_t rows[Q * 8] = {};
            for (int p = 0; p < Q; p++)
                for (int bo = 0; bo < 8; bo++) rows[p * 8 + bo] = uint32_t(plane_mask(S::RS.g[p][I], bo, 0));
            return make_xor_cse<Q * 8>(rows);
        }
        static constexpr XorCse C = make();
    };
    // both PFT outputs of a pair (transforms.rs:108-125), through shared subexpressions
    struct PftCse {
        static constexpr uint64_t mask(int bo, int base) {
            return base == 0 ? (plane_mask(S::DINV, bo, 0) | plane_mask(gm(S::DINV, 2), bo, 8))
                             : (plane_mask(S::DINV, bo, 8) | plane_mask(gm(S::DINV, 2), bo, 0));
        }
        static constexpr XorCse make() {
            uint32_t rows[16] = {};
            for (int bo = 0; bo < 8; bo++) {
                rows[bo] = uint32_t(mask(bo, 0));
                rows[8 + bo] = uint32_t(mask(bo, 8));
            }
            return make_xor_cse<16, 16>(rows);
        }
        static constexpr XorCse C = make();
    };
    __device__ static void pft_pair(const uint32_t *u, const uint32_t *us, uint32_t (&c)[16]) {
        uint32_t in[16];
#pragma unroll
        for (int w = 0; w < 8; w++) {
            in[w] = u[w];
            in[8 + w] = us[w];
        }
        cse_fold<PftCse, 16, false, 16>(in, c);
    }
    // 16 bytes v[w0 .. w0+3] at p, of which the first nv are inside the sub-chunk
    __device__ static void store_part(uint8_t *p, const uint32_t (&v)[8], int w0, int nv) {
        if (nv >= 16) {
            *reinterpret_cast<uint4 *>(p) = make_uint4(v[w0], v[w0 + 1], v[w0 + 2], v[w0 + 3]);
        } else {
            for (int b = 0; b < nv; b++) p[b] = uint8_t(v[w0 + (b >> 2)] >> (8 * (b & 3)));
        }
    }
    // step (group, section Y): PRT of section Y's nodes with their companions (digit Y of the
    // column), transpose, RS fold into the parity accumulators (the first fold of a group sets them)
    template <int Y>
    __device__ static void section(const uint8_t *smem, uint32_t gq0, uint32_t c, uint32_t part, uint32_t (&acc)[Q * 8]) {
        const uint32_t cy = (c / jw(Y)) % uint32_t(Q);
        const uint8_t *cbuf = smem + ((gq0 + cy) % uint32_t(NB)) * uint32_t(NODE);
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int X = decltype(xc)::value;
            uint32_t o[8], cv[8], u[8];
            read32(smem + ((gq0 + uint32_t(X)) % uint32_t(NB)) * uint32_t(NODE), c, part, o);
            read32(cbuf, c + (uint32_t(X) - cy) * jw(Y), part, cv);
            const uint32_t km = cy != uint32_t(X) ? 0xffffffffu : 0u;
#pragma unroll
            for (int w = 0; w < 8; w++) u[w] = xor_xtime4(o[w], cv[w] & km);
            transpose8(u);
            cse_fold<FoldCse<Y * Q + X>, Q * 8, (Y > 0 || X > 0)>(u, acc);
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    // group G done: red vertex C[G][z_G] = U[G][z_G]; PFT pairs with the groups h < G
    template <int G>
    __device__ static void end_group(const Enc3Args &a, const uint32_t (&acc)[Q * 8], uint32_t (&H)[2][8], uint32_t c,
                                     uint32_t part, uint32_t b0, uint32_t vend, bool active) {
        const uint32_t zg = 3u * c + uint32_t(G);
        uint32_t cv[8];
#pragma unroll
        for (int w = 0; w < 8; w++) cv[w] = acc[G * 8 + w];
        put(a.par[G], cv, zg, a.sc, b0, vend, part, active);
        auto pair = [&](const uint32_t *uh_at_g, const uint32_t *ug_at_h, auto hc) BS_INL {
            constexpr int h = decltype(hc)::value;
            uint32_t c12[16], c1[8], c2[8];
            pft_pair(uh_at_g, ug_at_h, c12);
#pragma unroll
            for (int w = 0; w < 8; w++) {
                c1[w] = c12[w];
                c2[w] = c12[8 + w];
            }
            put(a.par[h], c1, zg, a.sc, b0, vend, part, active);                    // C[h][z_G]
            put(a.par[G], c2, 3u * c + uint32_t(h), a.sc, b0, vend, part, active);  // C[G][z_h]
        };
        if constexpr (G == 0) {
#pragma unroll
            for (int w = 0; w < 8; w++) {
                H[0][w] = acc[8 + w];   // U[1][z0]
                H[1][w] = acc[16 + w];  // U[2][z0]
            }
        } else if constexpr (G == 1) {
            pair(acc + 0, H[0], std::integral_constant<int, 0>{});  // U[0][z1], U[1][z0]
#pragma unroll
            for (int w = 0; w < 8; w++) H[0][w] = acc[16 + w];      // U[2][z1]
        } else {
            pair(acc + 0, H[1], std::integral_constant<int, 0>{});  // U[0][z2], U[2][z0]
            pair(acc + 8, H[0], std::integral_constant<int, 1>{});  // U[1][z2], U[2][z1]
        }
    }
    // parity C (8 planes) -> bytes -> parity node X, layer z
    __device__ static void put(uint8_t *parx, uint32_t (&cv)[8], uint32_t z, uint64_t sc, uint32_t b0, uint32_t vend,
                               uint32_t part, bool active) {
        transpose8(cv);
        if (!active) return;
        uint8_t *dst = parx + uint64_t(z) * sc + b0;
        if (vend == b0 + uint32_t(W)) {
            *reinterpret_cast<uint4 *>(dst + 16u * part) = make_uint4(cv[0], cv[1], cv[2], cv[3]);
            *reinterpret_cast<uint4 *>(dst + 16u * (part + uint32_t(PARTS))) = make_uint4(cv[4], cv[5], cv[6], cv[7]);
        } else {
            store_part(dst + 16u * part, cv, 0, int(vend - b0) - int(16u * part));
            store_part(dst + 16u * (part + uint32_t(PARTS)), cv, 4, int(vend - b0) - int(16u * (part + uint32_t(PARTS))));
        }
    }
};

// grid = 8 * ns (one workgroup per CU); XCD x owns bytes [x * region, (x + 1) * region): full
// tiles round robin over its ns workgroups, the remainder one partial tile each (StreamMap).  PROBE (bench_tools only): 1 = no math, 2 = no DMA, 4 = no stores.
template <int KD, int M, int LOADERS, int PROBE = 0>
__global__ __launch_bounds__((StreamEnc3<KD, M, LOADERS>::BLOCK)) void k_stream_encode3(Enc3Args a) {
    using Kn = StreamEnc3<KD, M, LOADERS>;
    constexpr int Q = Kn::Q, NT = Kn::NT, STEPS = Kn::STEPS;
    constexpr uint32_t NB = uint32_t(Kn::NB), NODE = uint32_t(Kn::NODE);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3, ns = a.ns;
    const uint32_t sc32 = uint32_t(a.sc);
    const StreamMap tm(sc32, a.region, ns, xcd, slot, uint32_t(Kn::W));
    const uint32_t ntile = uint32_t(tm.ntile());
    if (ntile == 0) return;  // uniform per workgroup
    const uint32_t nsteps = ntile * uint32_t(STEPS);

    if (wave >= Kn::CWAVES) {
        // ---------------- loader waves: load q of a tile = step q / 3 (group, section), node q % 3 ----------------
        __builtin_amdgcn_s_setprio(3);
        const int li = wave - Kn::CWAVES;
        typename Kn::Loader L;
        Kn::loader_init(L, sc32, li, lane);
        const uint32_t lds0 = lds_addr_of(smem);
        const uint32_t nloads = ntile * uint32_t(NT);
        auto nbase_of = [&](uint32_t q) {  // node row base of tile-relative load q
            const uint32_t st = q / uint32_t(Q), g = st / 3u, y = st % 3u;
            return a.data[y * uint32_t(Q) + q % uint32_t(Q)] + uint64_t(g) * a.sc;
        };
        uint32_t issued = 0;
        auto issue_upto = [&](uint32_t lim) {
            if (lim > nloads) lim = nloads;
            for (; issued < lim; issued++) {
                const uint32_t k = issued / uint32_t(NT), q = issued % uint32_t(NT);
                const StreamTile t = tm.tile(int(k), slot, ns);
                if constexpr (!(PROBE & 2)) Kn::issue(L, lds0 + (issued % NB) * NODE, nbase_of(q), t.b0, t.vend, li);
            }
        };
        issue_upto(NB);
        for (uint32_t s = 0; s < nsteps; s++) {
            const uint32_t k = s / uint32_t(STEPS), st = s % uint32_t(STEPS);
            const uint32_t qs = k * uint32_t(NT) + st * uint32_t(Q), qend = qs + uint32_t(Q);
            const StreamTile t = tm.tile(int(k), slot, ns);
            const uint32_t b0 = t.b0, vend = t.vend;
            if (vend < b0 + uint32_t(Kn::W)) {
                wait_vm0();  // partial tile: everything landed, then this step's straddling pieces
                if constexpr (!(PROBE & 2))
                    for (uint32_t g = qs; g < qend; g++)
                        Kn::patch(L, smem + (g % NB) * NODE, nbase_of(g % uint32_t(NT)), b0, vend, li, lane);
            } else {
                wait_vm_rt(int((issued - qend) * uint32_t(Kn::BPL)));
            }
            lds_barrier();
            issue_upto(qs + NB);  // steps before s are done: their buffers take the loads NB ahead
        }
        wait_vm0();
        return;
    }

    // ---------------- compute waves ----------------
    // one step per loop iteration (run-time dispatch to the templated section / group end, as
    // k_stream_encode): only one step's registers are live at a time
    const uint32_t j = uint32_t(threadIdx.x) / uint32_t(Kn::PARTS), part = uint32_t(threadIdx.x) % uint32_t(Kn::PARTS);
    const bool active = j < uint32_t(Kn::COLS);
    const uint32_t c = active ? j : 0u;  // idle lanes of the last wave compute column 0, store nothing
    uint32_t acc[Q * 8];
    uint32_t H[2][8];  // U values later PFT pairs need (see the group ends)
    for (uint32_t s = 0; s < nsteps; s++) {
        const uint32_t k = s / uint32_t(STEPS), st = s % uint32_t(STEPS), G = st / 3u, Y = st % 3u;
        const StreamTile t = tm.tile(int(k), slot, ns);
        const uint32_t b0 = t.b0, vend = t.vend;
        lds_barrier();  // step s landed
        const uint32_t gq0 = k * uint32_t(NT) + st * uint32_t(Q);
        uint32_t co = c;
        asm volatile("" : "+v"(co));  // per-step copy: derived addresses are not hoisted
        if constexpr (PROBE & 1) {
            if (s == 0)
#pragma unroll
                for (int w = 0; w < Q * 8; w++) acc[w] = (threadIdx.x * 0x9E3779B9u) ^ uint32_t(w);
        } else {
            if (Y == 0) Kn::template section<0>(smem, gq0, co, part, acc);
            else if (Y == 1) Kn::template section<1>(smem, gq0, co, part, acc);
            else Kn::template section<2>(smem, gq0, co, part, acc);
        }
        if (Y == 2 && !(PROBE & 4)) {
            if (G == 0) Kn::template end_group<0>(a, acc, H, co, part, b0, vend, active);
            else if (G == 1) Kn::template end_group<1>(a, acc, H, co, part, b0, vend, active);
            else Kn::template end_group<2>(a, acc, H, co, part, b0, vend, active);
        }
    }
}

}  // namespace bs
}  // namespace clay
