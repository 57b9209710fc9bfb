// stream_local256.hpp -- the local decode on 256-byte row runs, for q = 4, t = 4 codes
// ((10,4,13), (9,4,12)) with one erasure e_G = (G, xg) in a y-section G plus at most one
// erasure e2 = (g2, x2) in one other section ({0}, {12}, {0,4}, ...), or two erasures in one
// section and none elsewhere ({0,1}, {12,13}, ...).  The same algebra as
// k_stream_local (stream_local.hpp: syndrome form, decode.rs:260-408, iscore order of
// decode.rs:196-254), on the encode's LDS image (stream_encode.hpp) instead of 64-byte tiles.
//
// Why the encode's image fits.  A tile is W = 256 byte positions of every (node, layer) row and is
// processed as 4 groups b (layer digit G = b) x 4 section steps; step (b, Y) streams the alive
// nodes of section Y at the 64 layers with digit G = b (one 16 KiB node buffer each: 64 columns c
// x 256 B, every LDS-DMA instruction 4 whole 256-byte row runs).  Lane = (column c, part p), 32
// positions ([16p, 16p + 16) and [128 + 16p, +16) of the tile), the same column in every group.
//   * Sections Y != G couple layers that differ in digit Y only, inside the group: phase A of
//     k_stream_local (PRT, transpose, RS check fold into the group's syndromes S_b), with the
//     companion read from the same step's buffers.
//   * Section G couples group b with the other groups: U((G, X), z) = C((G, X), z) + gamma
//     C((G, b), z[G := X]).  Its own term folds into S_b; the coupled term is collected by its
//     SOURCE: node (G, X) streamed at group b != X is the companion of node (G, b) at group X, so
//     it adds A_(G,b)[r] C((G, X) @ b) to the presolved row r of group X (A_i = H_K^-1 gamma H_i,
//     the tables the rounds use) -- for (G, b) used, or erased (its Out term).  Nothing of
//     section G crosses groups in the bit-sliced domain, so a lane carries only S_b (32 registers)
//     and the presolved rows C_r(group) (8 registers per erased row and group).
//   * End of group b: C_r(b) += row e_r of H_K^-1 S_b (the presolve, byte domain).
//   * After the four groups, the solve of k_stream_local with "slot" = group: (i) g2-lines of the
//     groups outside E_G (lanes l ^ 8, l ^ 16: section g2's digit is at bits 0-1 of c), (ii) the
//     groups in E_G: the dropped terms A_(G,A) C_(G,g)(group A) of the used (G, A), in-lane,
//     (iii) g2-lines of the groups in E_G, (iv) a both-erased pair of section G, in-lane.  Each
//     step reads only values the previous steps finished.
// The loader waves, the ring (a.ring - 1 node buffers streaming continuously across groups and
// tiles; the tables in the last buffer) and the counted waits follow k_stream_local; the tile map
// and the partial-tile handling (the piece straddling the end of a row rewritten in LDS after
// landing) follow k_stream_encode; any sub-chunk >= 512 (rows at any byte alignment: LDS-DMA and
// the 16-byte stores take any alignment, the partial pieces are patched and stored byte by byte).
#pragma once

#include "stream_decode.hpp"

namespace clay {
namespace bs {

// ANY: sub-chunks that are not multiples of 8 (rows at any byte alignment): the partial pieces
// are shifted into place in LDS and stored byte by byte; the ANY = false instantiation keeps the
// 8-byte tail handling (a separate kernel: the byte paths, though cold, slowed the 8-byte-row
// kernel by 28 % when compiled into it)
template <int KD, int G, int NE, bool ANY = false>
struct Local256 {
    using D = StreamDec<KD, G>;
    static_assert(NE == 1 || NE == 2, "one or two erased rows");
    static constexpr int W = 256, CWAVES = 8, LOADERS = 4, BLOCK = 64 * (CWAVES + LOADERS);
    static constexpr int BUF = 16384;  // 64 columns x 256 B
    static constexpr int BPL = 16 / LOADERS;
    static constexpr int LDS_BYTES = 10 * BUF;

    // node-buffer image of the encode (stream_encode.hpp sw()): row c at [256 c, 256 c + 256),
    // its 16-byte piece k at slot k ^ sw(c)
    __host__ __device__ static constexpr uint32_t sw(uint32_t c) { return ((c >> 1) & 1u) * 8u; }
    __device__ static uint32_t piece0(uint32_t c, uint32_t p) { return c * 256u + ((p ^ sw(c)) << 4); }
    // the lane's 32 bytes (pieces p and 8 + p) of a node buffer
    __device__ static void read32(const uint8_t *buf, uint32_t o0, uint32_t (&d)[8]) {
        const uint4 v0 = *reinterpret_cast<const uint4 *>(buf + o0);
        const uint4 v1 = *reinterpret_cast<const uint4 *>(buf + (o0 ^ 128u));
        d[0] = v0.x; d[1] = v0.y; d[2] = v0.z; d[3] = v0.w;
        d[4] = v1.x; d[5] = v1.y; d[6] = v1.z; d[7] = v1.w;
    }

    // ---------------- loader ----------------
    struct Loader {
        uint32_t off[BPL];  // layer0(column) * sc + 16 * piece, per block
        uint32_t k16, rl;
        int li;
    };
    __device__ static void loader_init(Loader &L, const DecArgs &a, int li, int lane) {
        const uint32_t sc = uint32_t(a.sc);
        L.li = li;
        L.rl = uint32_t(lane) >> 4;
        L.k16 = ((uint32_t(lane) & 15u) ^ sw(L.rl)) * 16u;
#pragma unroll
        for (int j = 0; j < BPL; j++) {
            const uint32_t c = uint32_t(li * BPL + j) * 4u + L.rl;
            L.off[j] = D::layer0_rt(a, c) * sc + L.k16;
        }
    }
    // node buffer at LDS address lds_buf <- 64 layers (digit G = b) x the tile of node
    __device__ static void issue(const DecArgs &a, const Loader &L, uint32_t lds_buf, const uint8_t *node, StreamTile t,
                                 uint32_t b) {
        const uint32_t sc = uint32_t(a.sc);
        lds_buf = __builtin_amdgcn_readfirstlane(lds_buf) + uint32_t(L.li * BPL) * 1024u;
        const uint64_t gofs = uint64_t(b * D::wt(G)) * sc;
        if (t.vend >= t.b0 + uint32_t(W)) {
            const uint8_t *base = uniform_ptr(node + gofs + t.b0);
#pragma unroll
            for (int j = 0; j < BPL; j++) dma16(lds_buf + uint32_t(j) * 1024u, base, L.off[j]);
        } else {
            // partial tile: a piece straddling vend is read from vend - 16 (patched after
            // landing), a piece wholly past vend from there too (never used)
            const uint8_t *base = uniform_ptr(node + gofs);
            uint32_t pos = t.b0 + L.k16;
            if (pos + 16u > t.vend) pos = t.vend - 16u;  // vend >= 16 (sc >= 512)
#pragma unroll
            for (int j = 0; j < BPL; j++) dma16(lds_buf + uint32_t(j) * 1024u, base, L.off[j] - L.k16 + pos);
        }
    }
    // a tile end inside a 16-byte piece: the DMA read the straddling piece of every row from
    // vend - 16 (issue()); once it has landed, rewrite it with its nv = vend - pos valid bytes at
    // the piece's start: ANY = false (nv = 8, sc % 16 == 8) from global memory; ANY = true (any nv)
    // by a funnel shift of the landed bytes by 16 - nv in LDS
    __device__ static void patch(const DecArgs &a, const Loader &L, uint8_t *buf, const uint8_t *node, StreamTile t,
                                 uint32_t b, int lane) {
        const uint32_t sc = uint32_t(a.sc), pos = t.b0 + L.k16;
        if (!(pos < t.vend && pos + 16u > t.vend)) return;
        if constexpr (!ANY) {
#pragma unroll
            for (int j = 0; j < BPL; j++) {
                const int blk = L.li * BPL + j;
                const uint64_t o = uint64_t(L.off[j] - L.k16) + uint64_t(b * D::wt(G)) * sc + pos;
                const uint2 gv = *reinterpret_cast<const uint2 *>(node + o);
                *reinterpret_cast<uint4 *>(buf + blk * 1024 + lane * 16) = make_uint4(gv.x, gv.y, 0u, 0u);
            }
        } else {
            const uint32_t sh = 16u - (t.vend - pos);  // bytes to drop at the front: 1..15
            const uint32_t ws = sh >> 2, bs = (sh & 3u) * 8u;
#pragma unroll
            for (int j = 0; j < BPL; j++) {
                uint4 *q = reinterpret_cast<uint4 *>(buf + (L.li * BPL + j) * 1024 + lane * 16);
                const uint4 v = *q;
                const uint32_t d[5] = {v.x, v.y, v.z, v.w, 0u};
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    // words k + ws and k + ws + 1 of d (0 past the end), selected without indexing d
                    uint32_t lo = 0u, hi = 0u;
#pragma unroll
                    for (int m = 0; m < 4; m++) {
                        lo = (k + m < 5 && ws == uint32_t(m)) ? d[k + m < 5 ? k + m : 4] : lo;
                        hi = (k + m + 1 < 5 && ws == uint32_t(m)) ? d[k + m + 1 < 5 ? k + m + 1 : 4] : hi;
                    }
                    o[k] = bs ? ((lo >> bs) | (hi << (32u - bs))) : lo;
                }
                *q = make_uint4(o[0], o[1], o[2], o[3]);
            }
        }
    }

    // ---------------- compute helpers ----------------
    // C_r rows of the lane: R_[r][group][8 dwords] (byte domain)
    using Rows = uint32_t[NE][4][8];
    // row r (uniform at run time) of group gi: opaque masks, not selects (a select between
    // register arrays becomes a dynamic index and moves them to scratch)
    __device__ static void get(const Rows &C, uint32_t r, int gi, uint32_t (&v)[8]) {
#pragma unroll
        for (int w = 0; w < 8; w++) v[w] = 0;
#pragma unroll
        for (int k = 0; k < NE; k++) {
            const uint32_t m = opq(r == uint32_t(k) ? 0xffffffffu : 0u);
#pragma unroll
            for (int w = 0; w < 8; w++) v[w] |= C[k][gi][w] & m;
        }
    }
    __device__ static void put(Rows &C, uint32_t r, int gi, const uint32_t (&v)[8]) {
#pragma unroll
        for (int k = 0; k < NE; k++) {
            const uint32_t m = opq(r == uint32_t(k) ? 0xffffffffu : 0u);
#pragma unroll
            for (int w = 0; w < 8; w++) C[k][gi][w] = (C[k][gi][w] & ~m) | (v[w] & m);
        }
    }
    // C_r(group gi) ^= T_r * v for every erased row r
    __device__ static void add_mul(Rows &C, const uint8_t *tl, int tab0, const uint32_t (&v)[8], int gi) {
        GfTab tb[NE];
#pragma unroll
        for (int r = 0; r < NE; r++) tb[r] = D::tab_at(tl, tab0 + r);
#pragma unroll
        for (int w = 0; w < 8; w++) {
            const GfIdx ix = gf_idx(v[w]);
#pragma unroll
            for (int r = 0; r < NE; r++) C[r][gi][w] ^= gf_mul_idx(ix, tb[r]);
        }
    }
    // steps (i) / (iii): group gi, terms of the g2-line (lanes differing in bits 3-4)
    __device__ static void line_g2(const DecArgs &a, Rows &C, const uint8_t *tl, uint32_t c, int gi) {
        const uint32_t g2 = uint32_t(a.g2), x2 = a.x2;
        const uint32_t d2 = c & 3u;  // this lane's digit of section g2
        const uint32_t r2 = uint32_t(a.rix[4 * g2 + x2]);
        const bool red = d2 == x2;
        const bool src = !red && ((a.used >> (4u * g2 + d2)) & 1u);
        const int ti = int(16u + (4u * g2 + d2) * 4u);  // per-lane table row (d2 varies over the line)
        uint32_t v[8];
        get(C, r2, gi, v);
        GfTab tb[NE];
#pragma unroll
        for (int r = 0; r < NE; r++) tb[r] = D::tab_at(tl, ti + r);
#pragma unroll
        for (int w = 0; w < 8; w++) {
            const GfIdx ix = gf_idx(src ? v[w] : 0u);
#pragma unroll
            for (int r = 0; r < NE; r++) {
                uint32_t t = gf_mul_idx(ix, tb[r]);
                t ^= uint32_t(__shfl_xor(int(t), 8));
                t ^= uint32_t(__shfl_xor(int(t), 16));
                if (red) C[r][gi][w] ^= t;
            }
        }
    }

    // one step (group b, section Y): S_b += the section's terms; section G's coupled terms into C.
    // SC >= 0 (NE = 1): the section's structure at compile time (DecArgs::scase: node (Y, SC)
    // erased and every other node used for SC < 4; none erased, all alive and all / only node 0 /
    // nodes 0-1 used for SC = 4 / 5 / 6); SC = -1: the run-time masks
    template <int Y, int SC = -1>
    __device__ __forceinline__ static void step(const DecArgs &a, uint8_t *smem, uint32_t gbase, uint32_t R, uint32_t c,
                                                uint32_t p, uint32_t b, uint32_t eG, uint32_t (&S)[32], Rows &C,
                                                const uint8_t *tl) {
        constexpr bool CT = SC >= 0;
        if constexpr (CT) {
            // a distinct marker opens and closes every copy, and the lane constants are opaque per
            // copy: no code is hoisted above or sunk below the caller's switch
            asm volatile("; local256 step copy %0 begin" ::"i"(SC));
            c = opq(c);
            p = opq(p);
        }
        constexpr uint32_t kEm = (CT && SC < 4) ? 1u << SC : 0u;
        constexpr uint32_t kUsed = !CT ? 0u : SC <= 4 ? (~kEm & 15u) : SC == 5 ? 1u : 3u;
        constexpr uint32_t kAlive = 15u & ~D::short_nib(Y) & ~kEm;
        uint32_t alive_all = __builtin_amdgcn_readfirstlane(a.alive), used_all = __builtin_amdgcn_readfirstlane(a.used),
                 emY = __builtin_amdgcn_readfirstlane(a.emask[Y]);
        asm volatile("" : "+s"(alive_all), "+s"(used_all), "+s"(emY));
        if constexpr (CT) {
            alive_all = kAlive << (4 * Y);
            used_all = kUsed << (4 * Y);
            emY = kEm;
        }
        const uint32_t aliveY = (alive_all >> (4 * Y)) & 15u;
        const uint32_t rs = a.sec_off[Y];
        auto buf_of = [&](uint32_t x) BS_INL {  // node (Y, x) buffer (x alive)
            const uint32_t q = rs + uint32_t(__builtin_popcount(aliveY & ((1u << x) - 1u)));
            return smem + ((gbase + q) % R) * BUF;
        };
        const uint32_t own0 = piece0(c, p);
        if constexpr (Y != G) {
            const uint32_t sh = a.csh[Y];
            const uint32_t cy = (c >> sh) & 3u;
            const bool comp_alive = (aliveY >> cy) & 1u;
            const uint8_t *cbuf = comp_alive ? buf_of(cy) : smem;
            sfor<4>([&](auto xc) BS_INL {
                constexpr int X = decltype(xc)::value;
                constexpr int I = 4 * Y + X;
                const bool alive_i = (aliveY >> X) & 1u;
                const bool used_i = (used_all >> I) & 1u;
                const bool erased_i = (emY >> X) & 1u;
                if (!(used_i || erased_i)) return;
                uint32_t o[8], cv[8], u[8];
                if (alive_i) {
                    read32(buf_of(X), own0, o);
                } else {
#pragma unroll
                    for (int w = 0; w < 8; w++) o[w] = 0;
                }
                const uint32_t cc = (c & ~(3u << sh)) | (uint32_t(X) << sh);
                read32(cbuf, piece0(cc, p), cv);
                const uint32_t keep = (comp_alive && cy != uint32_t(X)) ? 0xffffffffu : 0u;
                const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
                if (erased_i) {  // S += H_e Out(e, z): Out = gamma * companion (0 where red)
                    uint32_t v[8];
#pragma unroll
                    for (int w = 0; w < 8; w++) v[w] = xor_xtime4_masked(0u, cv[w], ks, kr);
                    transpose8(v);
                    D::template fold<I, false>(v, S);
                }
                if (used_i) {
#pragma unroll
                    for (int w = 0; w < 8; w++) u[w] = xor_xtime4_masked(o[w], cv[w], ks, kr);
                    transpose8(u);
                    D::template fold<I, false>(u, S);
                }
                __builtin_amdgcn_sched_barrier(0);
            });
        } else {
            // the coupled terms of group b's sources go to group X: coefficient A_(G,b)[r] when
            // (G, b) is used, or is e_G (its Out term); none from the red node (G, b) itself
            const bool cross = (((used_all >> (4 * G)) | eG) >> b) & 1u;
            sfor<4>([&](auto xc) BS_INL {
                constexpr int X = decltype(xc)::value;
                constexpr int I = 4 * G + X;
                if (!((aliveY >> X) & 1u)) return;
                uint32_t o[8];
                read32(buf_of(X), own0, o);
                if (cross && uint32_t(X) != b) add_mul(C, tl, int(16u + (4u * G + b) * 4u), o, X);
                if ((used_all >> I) & 1u) {
                    transpose8(o);
                    D::template fold<I, false>(o, S);
                }
                __builtin_amdgcn_sched_barrier(0);
            });
        }
        if constexpr (CT) asm volatile("; local256 step copy %0 end" ::"i"(SC));
    }
    // the step's copy for a.scase[Y] (one erased row only: with two the copies' registers spill)
    template <int Y>
    __device__ __forceinline__ static void step_any(const DecArgs &a, uint8_t *smem, uint32_t gbase, uint32_t R,
                                                    uint32_t c, uint32_t p, uint32_t b, uint32_t eG, uint32_t (&S)[32],
                                                    Rows &C, const uint8_t *tl) {
        if constexpr (NE != 1) {
            step<Y>(a, smem, gbase, R, c, p, b, eG, S, C, tl);
        } else if constexpr (Y == G) {
            switch (a.scase[Y]) {
            case 0: step<Y, 0>(a, smem, gbase, R, c, p, b, eG, S, C, tl); break;
            case 1: step<Y, 1>(a, smem, gbase, R, c, p, b, eG, S, C, tl); break;
            case 2: step<Y, 2>(a, smem, gbase, R, c, p, b, eG, S, C, tl); break;
            case 3: step<Y, 3>(a, smem, gbase, R, c, p, b, eG, S, C, tl); break;
            default: step<Y>(a, smem, gbase, R, c, p, b, eG, S, C, tl); break;
            }
        } else {
            switch (a.scase[Y]) {
            case 4: step<Y, 4>(a, smem, gbase, R, c, p, b, eG, S, C, tl); break;
            case 5: step<Y, 5>(a, smem, gbase, R, c, p, b, eG, S, C, tl); break;
            case 6: step<Y, 6>(a, smem, gbase, R, c, p, b, eG, S, C, tl); break;
            default: step<Y>(a, smem, gbase, R, c, p, b, eG, S, C, tl); break;
            }
        }
    }
};

// grid = 8 * nslots (one workgroup per CU); LDS = 10 x 16 KiB: a ring of a.ring - 1 node
// buffers and the tables (presolve, A_i) in the last.  a.region: XCD region bytes (multiple of 32).
template <int KD, int G, int NE, bool ANY = false>
__global__ __launch_bounds__((Local256<KD, G, NE, ANY>::BLOCK)) void k_stream_local256(DecArgs a) {
    using Kn = Local256<KD, G, NE, ANY>;
    using D = typename Kn::D;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t xcd = blockIdx.x & 7u, wslot = blockIdx.x >> 3, ns = a.nslots;
    const uint32_t sc = uint32_t(a.sc);
    const StreamMap tm(sc, a.region, ns, xcd, wslot);
    const uint32_t ntile = uint32_t(tm.ntile());
    if (ntile == 0) return;  // uniform per workgroup
    const uint32_t R = a.ring - 1u, NT = a.nt;
    constexpr uint32_t BUF = uint32_t(Kn::BUF);

    if (wave >= Kn::CWAVES) {
        // ---------------- loader waves: load l -> buffer l % R, 4 groups x NT loads per tile ----------------
        __builtin_amdgcn_s_setprio(3);
        typename Kn::Loader L;
        Kn::loader_init(L, a, wave - Kn::CWAVES, lane);
        const uint32_t lds0 = lds_addr_of(smem);
        if (L.li < 3)  // tables, before any ring load: the first step's counted wait covers them
            dma16(lds0 + R * BUF + uint32_t(L.li) * 1024u, uniform_ptr(reinterpret_cast<const uint8_t *>(a.tabs)),
                  uint32_t(L.li) * 1024u + uint32_t(lane) * 16u);
        const uint32_t NG = 4u * NT;  // loads per tile
        const uint32_t nloads = ntile * NG;
        uint32_t issued = 0;
        auto issue_upto = [&](uint32_t lim) {
            if (lim > nloads) lim = nloads;
            for (; issued < lim; issued++) {
                const uint32_t k = issued / NG, rem = issued % NG, b = rem / NT, q = rem % NT;
                Kn::issue(a, L, lds0 + (issued % R) * BUF, a.node[a.load_node[q]], tm.tile(int(k), wslot, ns), b);
            }
        };
        issue_upto(R);
        for (uint32_t k = 0; k < ntile; k++) {
            const StreamTile t = tm.tile(int(k), wslot, ns);
            const bool straddle = t.vend < t.b0 + uint32_t(Kn::W) && ((t.vend - t.b0) & 15u);
            for (uint32_t b = 0; b < 4; b++) {
                const uint32_t gb = (k * 4u + b) * NT;
                for (int y = 0; y < 4; y++) {
                    const uint32_t q0 = gb + a.sec_off[y], qend = gb + a.sec_off[y + 1];
                    if (straddle) {
                        wait_vm0();
                        for (uint32_t l = q0; l < qend; l++)
                            Kn::patch(a, L, smem + (l % R) * BUF, a.node[a.load_node[l % NT]], t, b, lane);
                    } else {
                        wait_vm_rt(int((issued - qend) * uint32_t(Kn::BPL)));
                    }
                    lds_barrier();
                    issue_upto(q0 + R);
                }
            }
        }
        wait_vm0();
        return;
    }

    // ---------------- compute waves ----------------
    const uint32_t c0 = uint32_t(threadIdx.x) >> 3, p0 = uint32_t(threadIdx.x) & 7u;
    const uint32_t eG = a.emask[G];
    const bool has2 = a.g2 >= 0;
    for (uint32_t k = 0; k < ntile; k++) {
        const StreamTile t = tm.tile(int(k), wslot, ns);
        uint32_t C[NE][4][8];
#pragma unroll
        for (int r = 0; r < NE; r++)
#pragma unroll
            for (int g = 0; g < 4; g++)
#pragma unroll
                for (int w = 0; w < 8; w++) C[r][g][w] = 0;
#pragma unroll 1
        for (uint32_t b = 0; b < 4; b++) {
            uint32_t S[32];
#pragma unroll
            for (int w = 0; w < 32; w++) S[w] = 0;
            const uint32_t gb = (k * 4u + b) * a.nt;
            sfor<4>([&](auto yc) BS_INL {
                constexpr int Y = decltype(yc)::value;
                lds_barrier();  // step (k, b, Y) landed
                const uint8_t *tl = smem + R * BUF + opq(0u);
                Kn::template step_any<Y>(a, smem, gb, R, opq(c0), opq(p0), b, eG, S, C, tl);
            });
            // end of group b: C_r(b) += row e_r of H_K^-1 S_b (bit planes -> bytes, then v_perm)
            const uint8_t *tl = smem + R * BUF + opq(0u);
            uint32_t T[NE][8];
#pragma unroll
            for (int r = 0; r < NE; r++)
#pragma unroll
                for (int w = 0; w < 8; w++) T[r][w] = 0;
            sfor<4>([&](auto jc) BS_INL {
                constexpr int j = decltype(jc)::value;
                uint32_t v[8];
#pragma unroll
                for (int w = 0; w < 8; w++) v[w] = S[j * 8 + w];
                transpose8(v);
                GfTab tb[NE];
#pragma unroll
                for (int r = 0; r < NE; r++) tb[r] = D::tab_at(tl, r * 4 + j);
#pragma unroll
                for (int w = 0; w < 8; w++) {
                    const GfIdx ix = gf_idx(v[w]);
#pragma unroll
                    for (int r = 0; r < NE; r++) T[r][w] ^= gf_mul_idx(ix, tb[r]);
                }
                __builtin_amdgcn_sched_barrier(0);
            });
            sfor<4>([&](auto gc) BS_INL {
                constexpr int g = decltype(gc)::value;
                if (b != uint32_t(g)) return;
#pragma unroll
                for (int r = 0; r < NE; r++)
#pragma unroll
                    for (int w = 0; w < 8; w++) C[r][g][w] ^= T[r][w];
            });
        }
        const uint8_t *tl = smem + R * BUF + opq(0u);
        const uint32_t c = opq(c0), p = opq(p0);
        // (i) g2-lines of the groups outside E_G (sources: level-0 values)
        if (has2) {
            sfor<4>([&](auto gc) BS_INL {
                constexpr int g = decltype(gc)::value;
                if (!((eG >> g) & 1u)) Kn::line_g2(a, C, tl, c, g);
            });
        }
        // (ii) groups g in E_G: the in-lane terms of the used nodes (G, A), A not in E_G
        {
            const uint32_t used_all = a.used;
            sfor<4>([&](auto gc) BS_INL {
                constexpr int g = decltype(gc)::value;
                if (!((eG >> g) & 1u)) return;
                const uint32_t rg = uint32_t(a.rix[4 * G + g]);
                sfor<4>([&](auto ac) BS_INL {
                    constexpr int A = decltype(ac)::value;
                    if (((eG >> A) & 1u) || !((used_all >> (4 * G + A)) & 1u)) return;
                    uint32_t v[8];
                    Kn::get(C, rg, A, v);
                    Kn::add_mul(C, tl, 16 + (4 * G + A) * 4, v, g);
                });
            });
        }
        // (iii) red lanes of the g2-lines of the groups in E_G (sources final after (ii))
        if (has2) {
            sfor<4>([&](auto gc) BS_INL {
                constexpr int g = decltype(gc)::value;
                if ((eG >> g) & 1u) Kn::line_g2(a, C, tl, c, g);
            });
        }
        // (iv) a both-erased pair of section G (two erasures there, none elsewhere): (G, x) at
        // group g <-> (G, g) at group x, C = det^-1 (U + gamma U*) (transforms.rs:108-125)
        if constexpr (NE == 2) {
            if (__builtin_popcount(eG) == 2) {
                const uint32_t gl = uint32_t(__builtin_ctz(eG)), xh = 31u - uint32_t(__builtin_clz(eG));
                const uint32_t rx = uint32_t(a.rix[4 * G + xh]), rg = uint32_t(a.rix[4 * G + gl]);
                const GfTab dinv = D::tab_at(tl, kDecDetInv);
                sfor<4>([&](auto gc) BS_INL {
                    constexpr int g = decltype(gc)::value;
                    if (uint32_t(g) != gl) return;
                    sfor<4>([&](auto xc) BS_INL {
                        constexpr int x = decltype(xc)::value;
                        if (x <= g || uint32_t(x) != xh) return;
                        uint32_t u1[8], u2[8], c1[8], c2[8];
                        Kn::get(C, rx, g, u1);  // (G, x) at group g
                        Kn::get(C, rg, x, u2);  // (G, g) at group x
#pragma unroll
                        for (int w = 0; w < 8; w++) {
                            c1[w] = gf_mul(u1[w] ^ gf_xt(u2[w]), dinv);
                            c2[w] = gf_mul(u2[w] ^ gf_xt(u1[w]), dinv);
                        }
                        Kn::put(C, rx, g, c1);
                        Kn::put(C, rg, x, c2);
                    });
                });
            }
        }
        // outputs: pieces p and 8 + p of row (layer z) per erased row and group
        const bool full = t.vend >= t.b0 + uint32_t(Kn::W);
        if (full) {
            // lanes c and c ^ 1 (lane ^ 8) swap halves by DPP (as the encode's parity stores), so
            // each 16-byte store instruction of a wave writes 4 whole 256-byte row runs
            const bool odd = c & 1u;
            const uint32_t ze = D::layer0_rt(a, c & ~1u), zo = D::layer0_rt(a, c | 1u);
            const uint32_t prel = t.b0 + 16u * p + (odd ? 128u : 0u);
#pragma unroll
            for (int r = 0; r < NE; r++) {
                const uint8_t *base = uniform_ptr(a.out[r]);
                if (!base) continue;
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    uint32_t lo[4], hi[4];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const uint32_t send = odd ? C[r][g][i] : C[r][g][4 + i];
                        const uint32_t rv = uint32_t(__builtin_amdgcn_update_dpp(0, int(send), 0x128, 0xf, 0xf, false));  // row_ror:8
                        lo[i] = odd ? rv : C[r][g][i];      // row of the even column
                        hi[i] = odd ? C[r][g][4 + i] : rv;  // row of the odd column
                    }
                    const uint32_t zg = uint32_t(g) * D::wt(G);
                    st16sp<0>(base, (ze + zg) * sc + prel, lo[0], lo[1], lo[2], lo[3]);
                    st16sp<0>(base, (zo + zg) * sc + prel, hi[0], hi[1], hi[2], hi[3]);
                }
            }
        } else {
            const uint32_t z0 = D::layer0_rt(a, c);
#pragma unroll
            for (int r = 0; r < NE; r++) {
                uint8_t *dst = a.out[r];
                if (!dst) continue;
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    uint8_t *row = dst + uint64_t(z0 + uint32_t(g) * D::wt(G)) * sc + t.b0 + 16u * p;
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint32_t pos = t.b0 + 16u * p + 128u * uint32_t(h);
                        const uint32_t nv = pos >= t.vend ? 0u : (t.vend - pos >= 16u ? 16u : t.vend - pos);
                        const uint32_t w0 = C[r][g][4 * h], w1 = C[r][g][4 * h + 1], w2 = C[r][g][4 * h + 2],
                                       w3 = C[r][g][4 * h + 3];
                        if (nv == 16u) {
                            *reinterpret_cast<uint4 *>(row + 128 * h) = make_uint4(w0, w1, w2, w3);
                        } else if constexpr (ANY) {
                            // the row's last bytes (any count: sub-chunks need not be multiples of 8)
#pragma unroll 1
                            for (uint32_t i = 0; i < nv; i++) {
                                const uint32_t q = i >> 2;
                                const uint32_t wv = q == 0u ? w0 : q == 1u ? w1 : q == 2u ? w2 : w3;
                                row[128 * h + int(i)] = uint8_t(wv >> (8u * (i & 3u)));
                            }
                        } else if (nv >= 8u) {
                            *reinterpret_cast<uint2 *>(row + 128 * h) = make_uint2(w0, w1);
                        }
                    }
                }
            }
        }
    }
}

}  // namespace bs
}  // namespace clay
