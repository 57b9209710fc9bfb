// stream_encode.hpp -- the encode kernel for codes with q = 4, t = 4 (alpha = 256), e.g. the
// BASELINE (10,4,13): loader waves stream the data through per-node LDS buffers while
// compute waves run the bit-sliced GF(2^8) math of encode_math.hpp.
//
// Data flow per workgroup (one per CU, 160 KiB LDS):
//  * A tile is W = 256 byte positions of every (node, layer) sub-chunk row.  It is
//    processed as 12 steps (group g = layer digit d3, data section Y = 0..2); step (g, Y)
//    reads the real nodes of section Y at the 64 layers with d3 = g (16 KiB per node).
//  * LDS holds one 16 KiB buffer per real data node.  Step s reads section Y's buffers;
//    sections Y+1 and Y+2 hold steps s+1 and s+2 (landed or in flight), so 6-8 node
//    buffers (96-128 KiB) stream while a step computes.
//  * Dedicated loader waves (LOADERS of them) issue every LDS-DMA (16-byte
//    global_load_lds_dwordx4, 1 KiB per instruction) and do every vmcnt wait: after the
//    barrier of step s they refill the buffers step s-1 read with step s+2, then wait
//    (counted) for step s+1 and join the next barrier.  Compute waves never wait on
//    memory -- their only synchronisation is the one barrier per step -- and never
//    issue DMA, so their issue slots go to the XOR networks.
//  * Every DMA instruction reads 4 whole 256-byte row runs (4 layers of one node), so the
//    reads are as coalesced as a plain streaming copy; the LDS image is XOR-swizzled
//    through the choice of piece per lane (see sw() below) so the compute reads stay
//    bank-conflict free (bench_tools/stream_probe: coalesced DMA 0.345 vs 0.375 ms
//    memory-only for the scattered piece map of the v6 image).
//  * Compute (8 waves, 512 lanes): lane = (column c, part).  The math is encode_math.hpp's
//    v6 kernel: PRT in the byte domain, 8x8 bit transpose, the RS generator as
//    compile-time XOR networks into 4 x 8 plane accumulators, PFT in registers at the end
//    of each group, transposed back and stored.
//  * A lane's 32 positions are bytes [16p, 16p+16) and [128+16p, 128+16p+16) of the tile
//    (p = part); at the parity stores neighbouring columns swap halves (DPP), so each
//    16-byte store instruction of a wave writes 4 whole 256-byte row runs.
//  * Tiles: every XCD owns a contiguous byte region of the sub-chunks; its workgroups
//    take full tiles round robin (adjacent workgroups stream adjacent 256-byte runs of the
//    same rows), and the remainder is cut into one partial tile per workgroup, always its
//    last (bench_tools/ring_probe: XCD-blocked order streams 17 % faster than a global
//    round robin and 25 % faster than one contiguous range per workgroup).
//
// Same linear map as the reference (decode_layered with erased = parity, decode.rs:167-257),
// so the bytes are identical to the oracle's.
#pragma once

#include "encode_math.hpp"

namespace clay {
namespace bs {

// a wave-uniform pointer the compiler cannot prove uniform -> SGPRs (for the asm "s" operand)
__device__ __forceinline__ const uint8_t *uniform_ptr(const uint8_t *p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(v)), hi = __builtin_amdgcn_readfirstlane(uint32_t(v >> 32));
    return reinterpret_cast<const uint8_t *>((uint64_t(hi) << 32) | lo);
}

struct StreamTile {
    uint32_t b0, vend;  // positions [b0, b0 + 256) of every row, valid below vend
};

// XCD x owns bytes [x * region, min((x + 1) * region, sc)); full W-byte tiles round robin over
// the XCD's ns workgroups, the remainder one partial tile per workgroup (its last), so every
// workgroup of an XCD streams the same number of bytes to within 32.
struct StreamMap {
    uint32_t x0, x1, nfull, p0, p1, w;
    __device__ StreamMap(uint32_t sc, uint32_t region, uint32_t ns, uint32_t xcd, uint32_t slot, uint32_t W = 256u) {
        w = W;
        x0 = xcd * region;
        x1 = x0 + region < sc ? x0 + region : sc;
        nfull = p0 = p1 = 0;
        if (x0 >= x1) return;
        const uint32_t len = x1 - x0, round = ns * W;
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
    __device__ StreamTile tile(int k, uint32_t slot, uint32_t ns) const {
        if (uint32_t(k) < nfull) {
            const uint32_t b0 = x0 + (uint32_t(k) * ns + slot) * w;
            return {b0, b0 + w};
        }
        return {p0, p1};
    }
};

// Chip round robin (probe): full tile t -> workgroup t % G (the whole chip covers G adjacent
// tiles at a time), the partial last tile to workgroup nfull % G.
struct ChipMap {
    uint32_t b, G, nfull, pend, sc;
    __device__ ChipMap(uint32_t sc_, uint32_t b_, uint32_t G_) : b(b_), G(G_), nfull(sc_ / 256u), sc(sc_) {
        pend = (sc_ % 256u) && (nfull % G_) == b_ ? 1u : 0u;
    }
    __device__ int ntile() const { return int((nfull > b ? (nfull - b + G - 1) / G : 0u) + pend); }
    __device__ StreamTile tile(int k, uint32_t, uint32_t) const {
        const uint32_t t = b + uint32_t(k) * G;
        if (t < nfull) return {t * 256u, t * 256u + 256u};
        return {nfull * 256u, sc};
    }
};

// CPL / CPS: cache policy of the LDS-DMA loads / parity stores (0 default, 1 nt, 2 sc1);
// CSE: RS folds through compile-time common subexpressions (xor_cse.hpp);
// SINK (probe builds only): every parity store is replaced by an XOR of its data into a per-lane
// sink, so the math stays live without the stores (bench_tools/stream_probe "live" variants)
// MAP: compute-lane map (0: column c = 8 * wave + (lane >> 3), round 5; 1: the round-6 map below,
// digit 2 of c per wave so that section 2's work is wave-uniform, the light waves 4-7; 2: the same
// with the light waves 0-3, for A/B)
template <int KD, int LOADERS, int CPL = 0, int CPS = 0, bool CSE = true, bool SINK = false, bool CHECK = false,
          int MAP = 0>
struct StreamEnc {
    using K6 = EncMath<KD>;
    using S = typename K6::S;
    static constexpr int Q = 4, T = 4, W = 256, CWAVES = 8;
    static constexpr int BLOCK = 64 * (CWAVES + LOADERS);
    static constexpr int NODE_BYTES = 64 * W;      // 64 layers (columns c) x 256 B = 16 KiB
    static constexpr int REGION = Q * NODE_BYTES;  // section Y's nodes: buffers 4Y .. 4Y+3
    static constexpr int LDS_BYTES = KD * NODE_BYTES;
    static constexpr int STEPS = 12;
    // DMA issuers: the LOADERS dedicated waves, or (LOADERS == 0) the 8 compute waves
    static constexpr int DMA_WAVES = LOADERS ? LOADERS : CWAVES;
    static constexpr int BPL = 16 / DMA_WAVES;  // 1 KiB blocks of every node buffer per issuing wave
    static_assert(LOADERS == 0 || LOADERS == 1 || LOADERS == 2 || LOADERS == 4, "loader waves");
    static_assert(KD >= 9 && KD <= 10 && LDS_BYTES <= 160 * 1024, "one 16 KiB buffer per data node");

    static constexpr int nreal(int y) {
        int n = 0;
        for (int x = 0; x < Q; x++) n += (y * Q + x < KD);
        return n;
    }
    // instructions one loader wave issues for a step of section y
    static constexpr int ninstr(int y) { return nreal(y) * BPL; }
    // parity stores (16-byte instructions) a lane issues at the end of group g (full tile)
    static constexpr int nstores(int g) { return 2 * (1 + 2 * g); }
    static constexpr int dshift(int y) { return 2 * (T - 2 - y); }  // digit y of the column c

    // ---- node-buffer image ----
    // Row r (= column c, layer 4c + g) occupies bytes [256 r, 256 r + 256); its 16-byte
    // piece k sits at 16-byte slot k ^ sw(r), sw(r) = 8 * bit 1 of r.  1 KiB block j holds
    // rows 4j .. 4j+3, so ONE LDS-DMA instruction fills a block from 4 whole 256-byte row
    // runs in HBM (coalesced); the swizzle only permutes which lane fetches which piece.
    // Reads (lane = column c, part p; pieces p and 8 + p of a row): within every 16-lane
    // group of ds_read_b128 the columns c, c+3 and c+1, c+2 share parts, and sw separates
    // exactly those pairs, so own and companion reads are bank-conflict free (companions of
    // sections 0/1 keep c mod 4; section 2's companion row is shared = broadcast).
    __host__ __device__ static constexpr uint32_t sw(uint32_t r) { return ((r >> 1) & 1u) * 8u; }
    // Round-6 maps (MAP >= 1).  Compute lane (wave w, lane l): part p = l & 7, in-lane column index
    // k = l >> 3 (its three bits are column bits kb0, kb1, kb2 of c), the wave supplies digit 2
    // (column bits 0-1) and column bit wb.  Digit 2 per wave makes section 2 wave-uniform: for
    // d2 in {2, 3} the PRT companions of nodes 8, 9 are the shortened nodes 10, 11 (zero), so U = C
    // for 8 and 9 and U = 0 for 10 and 11 -- a light section-2 step of two plain node folds
    // (section2_u<2>).  The light waves are 4-7 (the younger wave of each SIMD, the one that loses
    // the VALU arbitration; MAP 2: waves 0-3).  The LDS image is swizzled per node and row, piece k
    // of row r of node (Y, x) at slot k ^ swn(x, r), swn = 8 (bit swb of r ^ bit 1 of x): own and
    // companion reads of every section step stay bank-conflict free for the maps below
    // (bench_tools/lds_conflicts.py: 0 extra cycles).  The store pair is lane ^ 8 (DPP; columns c,
    // c ^ 2^kb0: rows z, z + 4 * 2^kb0) or, MAP 3, lane ^ 16 through v_permlane16_swap (c ^ 2^kb1).
    // The maps differ in which parity rows one store instruction writes (memory-only A/B).
    // redskip: the heavy waves' section-2 red vertex (x = d2) without companion read and PRT
    struct MapSpec {
        int kb0, kb1, kb2, wb, swb;
        bool light_old, pswap, redskip;
    };
    static constexpr MapSpec spec() {
        switch (MAP) {
            case 1: return {2, 3, 4, 5, 3, false, false, true};
            case 2: return {2, 3, 4, 5, 3, true, false, true};
            case 3: return {2, 3, 4, 5, 3, false, true, true};
            case 4: return {3, 2, 4, 5, 3, false, false, true};
            case 5: return {4, 3, 2, 5, 3, false, false, true};
            case 6: return {5, 4, 3, 2, 5, false, false, true};
            case 7: return {2, 5, 4, 3, 5, false, false, true};
            case 8: return {4, 5, 3, 2, 5, false, false, true};
            case 9: return {4, 5, 3, 2, 5, false, false, false};
            default: return {0, 1, 2, 3, 1, false, false, false};  // MAP 0: unused
        }
    }
    static constexpr MapSpec MS = spec();
    static constexpr bool PSWAP = MS.pswap;
    static constexpr uint32_t PAIR = MAP == 0 ? 4u : (4u << (PSWAP ? MS.kb1 : MS.kb0));  // row distance of the store pair
    __device__ static int colmap(int w, int k) {
        if constexpr (MAP == 0) return 8 * w + k;
        const int hi = MS.light_old ? (((w >> 2) & 1) ^ 1) : ((w >> 2) & 1);
        return (w & 1) | (hi << 1) | ((k & 1) << MS.kb0) | (((k >> 1) & 1) << MS.kb1) | (((k >> 2) & 1) << MS.kb2) |
               (((w >> 1) & 1) << MS.wb);
    }
    __host__ __device__ static constexpr uint32_t swn(uint32_t x, uint32_t r) {
        return MAP == 0 ? sw(r) : ((((r >> MS.swb) & 1u) ^ ((x >> 1) & 1u))) * 8u;
    }
    // does the swizzle's row bit lie in digit y (then a companion row's bit comes from x)?
    static constexpr bool sw_in_digit(int y) { return MS.swb == dshift(y) || MS.swb == dshift(y) + 1; }
    // piece-pair swap of the companion read of node x in section y (the x part of its swizzle)
    static constexpr int comp_swap(int y, int x) { return sw_in_digit(y) ? ((x >> (MS.swb - dshift(y))) & 1) : 0; }

    // ---------------- loader ----------------
    struct Loader {
        // per block and node class b = bit 1 of the section-local node index (MAP 1 / 2 swizzle;
        // MAP 0: both the same): lane offset in its node chunk for g = 0, b0 = 0
        uint32_t off[2][BPL];
        uint32_t rl;        // row-in-block of this lane
        uint32_t slot;      // 16-byte LDS slot this lane fills in every block
        int li;
    };
    // 16 x the piece lane L fetches in block j of a node of class b
    __device__ static uint32_t k16_of(const Loader &L, int j, uint32_t b) {
        const uint32_t r = uint32_t(L.li * BPL + j) * 4u + L.rl;
        return (L.slot ^ swn(b * 2u, r)) * 16u;
    }
    __device__ static void loader_init(Loader &L, uint32_t sc, int li, int lane) {
        L.li = li;
        L.rl = uint32_t(lane) >> 4;
        L.slot = uint32_t(lane) & 15u;
#pragma unroll
        for (int j = 0; j < BPL; j++) {
            const uint32_t r = uint32_t(li * BPL + j) * 4u + L.rl;
            L.off[0][j] = r * 4u * sc + k16_of(L, j, 0u);
            L.off[1][j] = r * 4u * sc + k16_of(L, j, 1u);
        }
    }
    // DMA of step (section Y, group g) of tile t into section Y's node buffers
    template <int Y>
    __device__ static void issue(const BsArgs &a, const Loader &L, uint32_t lds0, StreamTile t, int g) {
        const uint32_t sc = uint32_t(a.sc);
        const bool full = t.vend >= t.b0 + uint32_t(W);
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            constexpr int node = Y * Q + x;
            if constexpr (node < KD) {
                constexpr uint32_t b = (uint32_t(x) >> 1) & 1u;
                const uint32_t dst = lds0 + uint32_t(node * NODE_BYTES) + uint32_t(L.li * BPL) * 1024u;
                if (full) {
                    const uint8_t *base = uniform_ptr(a.data[node] + (uint64_t(g) * sc + t.b0));
#pragma unroll
                    for (int j = 0; j < BPL; j++) dma16p<CPL>(dst + uint32_t(j) * 1024u, base, L.off[b][j]);
                } else {
                    // partial tile: a piece straddling vend is read from vend - 16 (patched
                    // after landing), a piece wholly past vend from b0 (never used)
                    const uint8_t *base = uniform_ptr(a.data[node] + uint64_t(g) * sc);
#pragma unroll
                    for (int j = 0; j < BPL; j++) {
                        const uint32_t k16 = k16_of(L, j, b);
                        uint32_t pos = t.b0 + k16;
                        if (pos + 16u > t.vend) pos = t.vend - 16u;  // past vend: unused; vend = sc >= 16
                        dma16p<CPL>(dst + uint32_t(j) * 1024u, base, L.off[b][j] - k16 + pos);
                    }
                }
            }
        });
    }
    __device__ static void issue_any(int y, const BsArgs &a, const Loader &L, uint32_t lds0, StreamTile t, int g) {
        if (y == 0) issue<0>(a, L, lds0, t, g);
        else if (y == 1) issue<1>(a, L, lds0, t, g);
        else issue<2>(a, L, lds0, t, g);
    }
    // A partial tile whose end is not 16-byte aligned (sc % 16 == 8): the straddling piece
    // of every row holds 8 valid bytes; rewrite it in LDS from global memory (after the
    // DMA of the step has landed).
    template <int Y>
    __device__ static void patch(const BsArgs &a, const Loader &L, uint8_t *smem, StreamTile t, int g, int lane) {
        const uint32_t sc = uint32_t(a.sc);
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            constexpr int node = Y * Q + x;
            if constexpr (node < KD) {
#pragma unroll
                for (int j = 0; j < BPL; j++) {
                    const uint32_t pos = t.b0 + k16_of(L, j, (uint32_t(x) >> 1) & 1u);
                    if (!(pos < t.vend && pos + 16u > t.vend)) continue;
                    const int blk = L.li * BPL + j;
                    const uint32_t layer = (uint32_t(blk) * 4u + L.rl) * 4u + uint32_t(g);
                    const uint2 gv = *reinterpret_cast<const uint2 *>(a.data[node] + uint64_t(layer) * sc + pos);
                    *reinterpret_cast<uint4 *>(smem + node * NODE_BYTES + blk * 1024 + lane * 16) =
                        make_uint4(gv.x, gv.y, 0u, 0u);
                }
            }
        });
    }
    __device__ static void patch_any(int y, const BsArgs &a, const Loader &L, uint8_t *smem, StreamTile t, int g,
                                     int lane) {
        if (y == 0) patch<0>(a, L, smem, t, g, lane);
        else if (y == 1) patch<1>(a, L, smem, t, g, lane);
        else patch<2>(a, L, smem, t, g, lane);
    }

    // ---------------- compute ----------------
    // Per-lane LDS offsets (loop invariant).  Own value of node x: x * 16 KiB + own[h] for
    // piece h * 8 + p.  Companion in section Y (node cy[Y] of the section, column c with
    // digit Y := x): cb[Y][h] + x * 4^(2-Y) * 256, plus for Y = 2 the swizzle of row x.
    struct LaneS {
        uint32_t own[2], cb[3][2];
        int cy[3];
    };
    __device__ static LaneS lane_consts(int c, int part) {
        LaneS L;
        if constexpr (MAP != 0) {
            // own: row c, slot p ^ swn(x, c); the node's bit-1 term swaps the two pieces (load_x)
            const uint32_t uc = uint32_t(c), up = uint32_t(part);
            L.own[0] = uc * 256u + ((up ^ (((uc >> MS.swb) & 1u) * 8u)) * 16u);
            L.own[1] = L.own[0] ^ 128u;
#pragma unroll
            for (int y = 0; y < 3; y++) {
                const int sh = dshift(y);
                L.cy[y] = (c >> sh) & 3;
                const uint32_t cy = uint32_t(L.cy[y]);
                const uint32_t row0 = (uc & ~(3u << sh)) * 256u + cy * uint32_t(NODE_BYTES);
                // companion row c' = c[y := x]: its swizzle bit is c's unless that bit lies in digit
                // y, then x's (the x term swaps the pieces, load_x)
                const uint32_t rb = sw_in_digit(y) ? 0u : ((uc >> MS.swb) & 1u);
                L.cb[y][0] = row0 + ((up ^ ((rb ^ ((cy >> 1) & 1u)) * 8u)) * 16u);
                L.cb[y][1] = L.cb[y][0] ^ 128u;
            }
            return L;
        }
        const uint32_t pk = (uint32_t(part) ^ sw(uint32_t(c))) * 16u;
        L.own[0] = uint32_t(c) * 256u + pk;
        L.own[1] = L.own[0] ^ 128u;
#pragma unroll
        for (int y = 0; y < 3; y++) {
            const int sh = dshift(y);
            L.cy[y] = (c >> sh) & 3;
            const uint32_t row0 = uint32_t(c & ~(3 << sh)) * 256u + uint32_t(L.cy[y]) * uint32_t(NODE_BYTES);
            if (y < 2) {
                L.cb[y][0] = row0 + pk;
                L.cb[y][1] = L.cb[y][0] ^ 128u;
            } else {
                L.cb[y][0] = L.cb[y][1] = row0 + uint32_t(part) * 16u;
            }
        }
        return L;
    }
    __device__ static void read32(const uint8_t *p0, const uint8_t *p1, uint32_t (&d)[8]) {
        const uint4 v0 = *reinterpret_cast<const uint4 *>(p0), v1 = *reinterpret_cast<const uint4 *>(p1);
        d[0] = v0.x; d[1] = v0.y; d[2] = v0.z; d[3] = v0.w;
        d[4] = v1.x; d[5] = v1.y; d[6] = v1.z; d[7] = v1.w;
    }
    // own value and companion of node x of section Y (zero for shortened nodes)
    template <int Y, int X>
    __device__ static void load_x(const uint8_t *slot, const LaneS &L, uint32_t (&o)[8], uint32_t (&cv)[8]) {
        if constexpr (MAP != 0) {
            constexpr int bx = (X >> 1) & 1;
            if constexpr (Y * Q + X < KD) {
                read32(slot + X * NODE_BYTES + L.own[bx], slot + X * NODE_BYTES + L.own[bx ^ 1], o);
            } else {
#pragma unroll
                for (int w = 0; w < 8; w++) o[w] = 0;
            }
            // (section 2: digit 2 is wave-uniform, so the red vertex's companion read is skipped)
            if ((Y * Q + L.cy[Y]) < KD && (Y != 2 || !MS.redskip || X != L.cy[Y])) {
                constexpr uint32_t step = uint32_t(256) << dshift(Y);
                constexpr int hb = comp_swap(Y, X);
                read32(slot + L.cb[Y][hb] + X * step, slot + L.cb[Y][hb ^ 1] + X * step, cv);
            } else {
#pragma unroll
                for (int w = 0; w < 8; w++) cv[w] = 0;
            }
            return;
        }
        if constexpr (Y * Q + X < KD) {
            read32(slot + X * NODE_BYTES + L.own[0], slot + X * NODE_BYTES + L.own[1], o);
        } else {
#pragma unroll
            for (int w = 0; w < 8; w++) o[w] = 0;
        }
        if ((Y * Q + L.cy[Y]) < KD) {
            constexpr uint32_t step = uint32_t(256) << dshift(Y);
            if constexpr (Y < 2) {
                read32(slot + L.cb[Y][0] + X * step, slot + L.cb[Y][1] + X * step, cv);
            } else {
                constexpr uint32_t s0 = sw(uint32_t(X)) * 16u;
                read32(slot + L.cb[Y][0] + (X * step + s0), slot + L.cb[Y][0] + (X * step + (s0 ^ 128u)), cv);
            }
        } else {
#pragma unroll
            for (int w = 0; w < 8; w++) cv[w] = 0;
        }
    }
    // PRT of node x in the byte domain: U = O + gamma * C* (C* masked off for the red
    // vertex and for shortened companions), transforms.rs:42-55
    template <int Y, int X>
    __device__ static void prt_x(const uint32_t (&o)[8], const uint32_t (&cv)[8], const LaneS &L, uint32_t (&u)[8]) {
        const int cy = L.cy[Y];
        if constexpr (MAP != 0 && Y == 2 && MS.redskip) {
            if (X == cy) {  // wave-uniform red vertex: U = C, no PRT
#pragma unroll
                for (int w = 0; w < 8; w++) u[w] = o[w];
                return;
            }
        }
        const bool creal = (Y * Q + cy) < KD;
        const uint32_t keep = (creal && X != cy) ? 0xffffffffu : 0u;
        const uint32_t ks = keep & 0xfefefefeu, kr = keep & 0x1d1d1d1du;
#pragma unroll
        for (int w = 0; w < 8; w++) u[w] = xor_xtime4_masked(o[w], cv[w], ks, kr);
    }
    // One step: the 4 nodes of section Y (own + companion reads, PRT, transpose, RS fold),
    // each node's LDS reads issued one node ahead; the scheduling barrier after every node
    // keeps the compiler from hoisting more reads (register pressure: 3 waves per SIMD).
    // SBN (probe builds): a scheduling barrier after every SBN nodes (0: none); BAL (probe
    // builds): issue priority 1 for the first half of the section and 0 for the second, so the
    // older of two compute waves on a SIMD yields to the younger once it is ahead
    template <int Y, int SBN = 1, bool BAL = false>
    __device__ __forceinline__ static void section(const uint8_t *slot, const LaneS &L, uint32_t (&acc)[Q * 8]) {
        uint32_t o[2][8], cv[2][8];
        if constexpr (BAL) __builtin_amdgcn_s_setprio(1);
        load_x<Y, 0>(slot, L, o[0], cv[0]);
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            if constexpr (BAL && x == 2) __builtin_amdgcn_s_setprio(0);
            if constexpr (x + 1 < Q) load_x<Y, x + 1>(slot, L, o[(x + 1) & 1], cv[(x + 1) & 1]);
            uint32_t u[8];
            prt_x<Y, x>(o[x & 1], cv[x & 1], L, u);
            if constexpr (CSE) K6::template fold_x_cse<Y, x>(u, acc);
            else K6::template fold_x<Y, x>(u, acc);
            if constexpr (SBN > 0 && (x + 1) % SBN == 0) __builtin_amdgcn_sched_barrier(0);
        });
    }

    // Section 2 with a wave-uniform digit 2 (MAP >= 1): D2 = the wave's d2 (2 stands for 2 and 3).
    // Node x of the section: own value real iff 8 + x < KD; PRT companion (node (2, D2) at layer
    // z[2 := x], transforms.rs:42-55) real iff x != D2 (else the red vertex: U = C) and 8 + D2 < KD.
    // So for KD = 10: D2 in {2, 3} (the light waves) U = C for nodes 8, 9 and U = 0 for 10, 11 (no
    // fold); D2 in {0, 1}: the red node without companion read or PRT, the shortened nodes U = gamma
    // C*.  Everything is compile-time: no masks, no per-lane branches.
    template <int D2, int SBN = 1>
    __device__ __forceinline__ static void section2_u(const uint8_t *slot, const LaneS &L, uint32_t (&acc)[Q * 8]) {
        static_assert(MAP != 0, "wave-uniform digit 2");
        constexpr int Y = 2;
        auto load = [&](auto xc, uint32_t (&o)[8], uint32_t (&cv)[8]) BS_INL {
            constexpr int x = decltype(xc)::value;
            constexpr bool own_real = Y * Q + x < KD;
            constexpr bool comp_real = x != D2 && Y * Q + D2 < KD;
            constexpr int bx = (x >> 1) & 1;
            if constexpr (own_real) read32(slot + x * NODE_BYTES + L.own[bx], slot + x * NODE_BYTES + L.own[bx ^ 1], o);
            constexpr int hb = comp_swap(Y, x);
            if constexpr (comp_real) read32(slot + L.cb[Y][hb] + x * 256, slot + L.cb[Y][hb ^ 1] + x * 256, cv);
        };
        uint32_t o[2][8], cv[2][8];
        load(std::integral_constant<int, 0>{}, o[0], cv[0]);
        sfor<Q>([&](auto xc) BS_INL {
            constexpr int x = decltype(xc)::value;
            constexpr bool own_real = Y * Q + x < KD;
            constexpr bool comp_real = x != D2 && Y * Q + D2 < KD;
            if constexpr (x + 1 < Q) load(std::integral_constant<int, x + 1>{}, o[(x + 1) & 1], cv[(x + 1) & 1]);
            if constexpr (own_real || comp_real) {
                uint32_t u[8];
#pragma unroll
                for (int w = 0; w < 8; w++) {
                    if constexpr (own_real && comp_real) u[w] = xor_xtime4_masked(o[x & 1][w], cv[x & 1][w], 0xfefefefeu, 0x1d1d1d1du);
                    else if constexpr (comp_real) u[w] = xor_xtime4_masked(0u, cv[x & 1][w], 0xfefefefeu, 0x1d1d1d1du);
                    else u[w] = o[x & 1][w];
                }
                if constexpr (CSE) K6::template fold_x_cse<Y, x>(u, acc);
                else K6::template fold_x<Y, x>(u, acc);
                if constexpr (SBN > 0) __builtin_amdgcn_sched_barrier(0);
            }
        });
        // a distinct marker ends every copy: otherwise SimplifyCFG sinks the copies' common tail
        // (the last fold) below the switch and the accumulators meet in phis (spilled)
        asm volatile("; section2_u end %0" ::"n"(D2));
    }

    // ---------------- compute: outputs ----------------
    // Parity C (8 planes) -> bytes -> HBM at parity node X, layer z = 4c + G.  A lane holds
    // pieces p and 8 + p of its row; lanes c and c ^ 1 (lane ^ 8, same row of 16 lanes) swap
    // halves by DPP so that each 16-byte store instruction of a wave writes 4 whole
    // 256-byte row runs (even columns, then odd columns) instead of 8 rows x 128 B.
    // The store pair's halves: lanes of a column and of its partner (lane ^ 8 in the same DPP row,
    // or MAP 3: lane ^ 16, the other row of a row pair) exchange halves so that lo holds the even
    // column's row (the even lane piece p, the odd lane piece 8 + p) and hi the odd column's.
    __device__ __forceinline__ static void pair_halves(const uint32_t (&cv)[8], uint32_t (&lo)[4], uint32_t (&hi)[4]) {
        if constexpr (PSWAP) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const auto r = __builtin_amdgcn_permlane16_swap(cv[i], cv[4 + i], false, false);
                lo[i] = r[0];
                hi[i] = r[1];
            }
        } else {
            const bool odd = (threadIdx.x >> 3) & 1u;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t send = odd ? cv[i] : cv[4 + i];
                const uint32_t r = uint32_t(__builtin_amdgcn_update_dpp(0, int(send), 0x128, 0xf, 0xf, false));  // row_ror:8
                lo[i] = odd ? r : cv[i];      // row of the even column, piece (odd ? 8 : 0) + p
                hi[i] = odd ? cv[4 + i] : r;  // row of the odd column
            }
        }
    }
    template <int X>
    __device__ __forceinline__ static void put(const BsArgs &a, uint32_t (&cv)[8], uint32_t z, StreamTile t, uint32_t prel,
                               bool ragged, uint32_t &sink) {
        transpose8(cv);
        if (SINK && !ragged) {
            uint32_t lo[4], hi[4];
            pair_halves(cv, lo, hi);
            sink ^= xor3(xor3(lo[0], lo[1], lo[2]), xor3(lo[3], hi[0], hi[1]), hi[2] ^ hi[3]);
            sink += X;  // keeps the per-output order visible (no cancellation across outputs)
            return;
        }
        if (SINK) {
            sink ^= xor3(xor3(cv[0], cv[1], cv[2]), xor3(cv[3], cv[4], cv[5]), cv[6] ^ cv[7]);
            return;
        }
        (void)sink;
        if (!ragged) {
            const bool odd = PSWAP ? ((threadIdx.x >> 4) & 1u) : ((threadIdx.x >> 3) & 1u);
            uint32_t lo[4], hi[4];
            pair_halves(cv, lo, hi);
            uint32_t off = (z - (odd ? PAIR : 0u)) * uint32_t(a.sc);
            asm volatile("" : "+v"(off));  // keep the 16 (node, layer) offsets out of LICM
            off += t.b0 + prel + (odd ? 128u : 0u);
            const uint8_t *base = uniform_ptr(a.par[X]);  // SGPR base (also under the probes' deferred flow)
            if constexpr (CHECK) {
                // probe bounds check (stream_probe "f"): flag and skip a store outside par[X]
                const uint64_t lim = uint64_t(a.sc) * 256u;
                if (uint64_t(off) + 16u > lim || uint64_t(off) + PAIR * a.sc + 16u > lim) {
                    atomicOr(reinterpret_cast<unsigned int *>(a.par[5]), 1u << X);
                    return;
                }
            }
            st16sp<CPS>(base, off, lo[0], lo[1], lo[2], lo[3]);
            st16sp<CPS>(base, off + PAIR * uint32_t(a.sc), hi[0], hi[1], hi[2], hi[3]);
        } else {
            uint8_t *p = a.par[X] + uint64_t(z) * a.sc + t.b0 + prel;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t pos = t.b0 + prel + 128u * uint32_t(h);
                const uint32_t nv = pos >= t.vend ? 0u : (t.vend - pos >= 16u ? 16u : t.vend - pos);
                if constexpr (CHECK) {
                    if (nv && (z >= 256u || pos + nv > a.sc)) {
                        atomicOr(reinterpret_cast<unsigned int *>(a.par[5]), 16u << X);
                        continue;
                    }
                }
                if (nv == 16u)
                    *reinterpret_cast<uint4 *>(p + 128 * h) = make_uint4(cv[4 * h], cv[4 * h + 1], cv[4 * h + 2], cv[4 * h + 3]);
                else if (nv >= 8u)
                    *reinterpret_cast<uint2 *>(p + 128 * h) = make_uint2(cv[4 * h], cv[4 * h + 1]);
            }
        }
    }
    // Group G finished: red vertex C[G][z_G] = U, and the PFT pairs with groups h < G
    // (transforms.rs:108-125) (Hold: encode_math.hpp).  Force-inlined: called out of line
    // (several instantiations in one translation unit), acc and Hold would go through scratch.
    template <int G>
    __device__ __forceinline__ static void end_group(const BsArgs &a, const uint32_t (&acc)[Q * 8], typename K6::Hold &H, int c,
                                     StreamTile t, uint32_t prel, bool ragged, uint32_t &sink) {
        const uint32_t zg = uint32_t(c * 4 + G);
        uint32_t cv[8];
#pragma unroll
        for (int w = 0; w < 8; w++) cv[w] = acc[G * 8 + w];
        put<G>(a, cv, zg, t, prel, ragged, sink);
        auto pair = [&](const uint32_t *uh_at_g, const uint32_t *ug_at_h, auto hc) BS_INL {
            constexpr int h = decltype(hc)::value;
            const uint32_t zh = uint32_t(c * 4 + h);
            uint32_t c12[16];
            if constexpr (CSE) {
                K6::pft_pair(uh_at_g, ug_at_h, c12);  // both outputs through shared subexpressions
            } else {
                uint32_t c1[8], c2[8];
                K6::pft(uh_at_g, ug_at_h, c1);
                K6::pft(ug_at_h, uh_at_g, c2);
#pragma unroll
                for (int w = 0; w < 8; w++) {
                    c12[w] = c1[w];
                    c12[8 + w] = c2[w];
                }
            }
            uint32_t c1[8], c2[8];
#pragma unroll
            for (int w = 0; w < 8; w++) {
                c1[w] = c12[w];
                c2[w] = c12[8 + w];
            }
            put<h>(a, c1, zg, t, prel, ragged, sink);  // C[h][z_G]
            put<G>(a, c2, zh, t, prel, ragged, sink);  // C[G][z_h]
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

// a.tiles_per_xcd = XCD region length in bytes (multiple of 32), a.nslots = workgroups per
// XCD; grid = 8 * nslots; LDS = KD x 16 KiB (one workgroup per CU).
// PROBE is for bench_tools/stream_probe.hip only (the library instantiates PROBE = 0):
// bit 1 = compute waves skip the math, 2 = loaders skip the DMA, 4 = no parity stores,
// 64/128 = LDS-DMA loads nt / sc1, 256/512 = parity stores nt / sc1, 1024 = row-by-row folds
// (no CSE: bench_tools/stream_probe x, 0.350 vs 0.353 ms full, 0.257 vs 0.281 math + stores),
// 8 = loaders at default priority, 16 = compute waves 4-7 at priority 1, 32 = the group whose
// outputs are stored at the end of group g is (g + slot) % 4 (store bursts desynchronised
// across workgroups; only meaningful with bit 1), 2048 = chip round-robin tile map (ChipMap),
// 4096 = s_memtime segment timing (TimeAcc), 8192 = a group's end work after the next barrier,
// 16384 / 32768 = no scheduling barrier between nodes / one after every two nodes,
// 262144 = SINK (StreamEnc): the end-of-group work runs in full but every parity store becomes an
// XOR into a per-lane sink, stored once at the end under a run-time predicate the compiler cannot
// fold -- the live-math "no stores" variants (262144: reads + math; 262146: math only);
// 524288 = CHECK (probe): every parity store and timing record is bounds-checked, a violation is
// flagged in a.par[5] (atomicOr of a bit per kind) and the access skipped.  Bit 4
// (no end-of-group work at all) lets the compiler delete the math and is kept only as a record
// of that (PROBE 4 / 6 compiled to 4 / 3 v_bitop3).
// Segment timing of the probe instantiations (PROBE bit 4096): s_memtime cycles summed per
// kind (compute wave: 0 barrier wait, 1 section math; loader wave: 0 vmcnt wait, 1 barrier,
// 2 DMA issue) and per section y, plus the end-of-group work (outputs) per group g; written by
// lane 0 of every wave to a.par[4] (a record of 17 uint64 at (workgroup * 12 + wave) * 24).
struct TimeAcc {
    uint64_t v[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, gend[4] = {0, 0, 0, 0};
    uint64_t t_start = 0, t_first = 0, t_end = 0;
    __device__ __forceinline__ void add(int kind, int y, uint64_t &t0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        const uint64_t d = t1 - t0;
        t0 = t1;
        // uniform branches: the sums stay in SGPRs
        if (y == 0) v[kind][0] += d;
        else if (y == 1) v[kind][1] += d;
        else v[kind][2] += d;
    }
    __device__ __forceinline__ void addg(int g, uint64_t &t0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        const uint64_t d = t1 - t0;
        t0 = t1;
        if (g == 0) gend[0] += d;
        else if (g == 1) gend[1] += d;
        else if (g == 2) gend[2] += d;
        else gend[3] += d;
    }
    __device__ void put(uint64_t *p, int ntile) const {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) p[i * 3 + j] = v[i][j];
        for (int g = 0; g < 4; g++) p[9 + g] = gend[g];
        p[13] = t_start;
        p[14] = t_first;
        p[15] = t_end;
        p[16] = uint64_t(ntile);
    }
};

// The lane map the library launches (round 6: map 8, light section-2 waves 4-7; same-box A/B on
// the BASELINE stripe, profiles/r06/encode/: 0.3311-0.3317 ms vs 0.3349-0.3355 for map 0 and
// 0.3484-0.3489 for the round-5 kernel)
constexpr int kStreamEncMap = 8;

template <int KD, int LOADERS, int PROBE = 0, int MAP = 0>
__global__ __launch_bounds__((StreamEnc<KD, LOADERS>::BLOCK)) void k_stream_encode(BsArgs a) {
    using Kn = StreamEnc<KD, LOADERS, (PROBE >> 6) & 3, (PROBE >> 8) & 3, ((PROBE >> 10) & 1) == 0, (PROBE & 262144) != 0,
                         (PROBE & 524288) != 0, MAP>;
    uint32_t sink = 0;  // SINK probes only
    constexpr bool TM = (PROBE & 4096) != 0;
    using K6 = typename Kn::K6;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3, ns = a.nslots;
    const auto tm = [&] {
        if constexpr ((PROBE & 2048) != 0) return ChipMap(uint32_t(a.sc), blockIdx.x, gridDim.x);
        else return StreamMap(uint32_t(a.sc), a.tiles_per_xcd, ns, xcd, slot);
    }();
    const int ntile = tm.ntile();
    if (ntile == 0) return;  // uniform per workgroup
    const int nsteps = ntile * Kn::STEPS;
    if (LOADERS > 0 && wave >= Kn::CWAVES) {
        // ---- loader wave ----
        // top issue priority: a loader issues a few instructions per step and otherwise
        // waits, but as the youngest wave on its SIMD it would lose every arbitration to the
        // compute waves and delay the whole pipeline (measured: 1 loader 0.46 ms, 4 loaders
        // 0.39 ms per 1 GiB stripe without this)
        if constexpr (!(PROBE & 8)) __builtin_amdgcn_s_setprio(3);
        typename Kn::Loader L;
        Kn::loader_init(L, uint32_t(a.sc), wave - Kn::CWAVES, lane);
        const uint32_t lds0 = lds_addr_of(smem);
        TimeAcc T;
        T.t_start = TM ? __builtin_amdgcn_s_memtime() : 0;
        if constexpr (!(PROBE & 2))
            for (int s = 0; s < 3 && s < nsteps; s++) Kn::issue_any(s % 3, a, L, lds0, tm.tile(0, slot, ns), s / 3);
        uint64_t t0 = TM ? __builtin_amdgcn_s_memtime() : 0;  // chained: every cycle lands in one sum
        if constexpr (TM) T.t_first = t0;
        for (int s = 0; s < nsteps; s++) {
            const int k = s / Kn::STEPS, r = s % Kn::STEPS, g = r / 3, y = r % 3;
            const StreamTile t = tm.tile(k, slot, ns);
            // step s landed: everything issued after it may stay in flight
            int after = 0;
            if (s == 0) {
                after = (nsteps > 1 ? Kn::ninstr(1) : 0) + (nsteps > 2 ? Kn::ninstr(2) : 0);
            } else if (s + 1 < nsteps) {
                after = Kn::ninstr((y + 1) % 3);
            }
            const bool straddle = t.vend < t.b0 + uint32_t(Kn::W) && ((t.vend - t.b0) & 15u);
            if (PROBE & 2) {
            } else if (straddle) {
                wait_vm_n<0>();
                Kn::patch_any(y, a, L, smem, t, g, lane);
            } else {
                wait_vm_rt(after);
            }
            if constexpr (TM) T.add(0, y, t0);
            if constexpr (!(PROBE & 65536)) lds_barrier();
            if constexpr (TM) T.add(1, y, t0);
            // step s-1's buffers are free: refill them with step s+2
            const int s2 = s + 2;
            if (!(PROBE & 2) && s >= 1 && s2 < nsteps) {
                const int k2 = s2 / Kn::STEPS, r2 = s2 % Kn::STEPS;
                Kn::issue_any(r2 % 3, a, L, lds0, tm.tile(k2, slot, ns), r2 / 3);
            }
            if constexpr (TM) T.add(2, y, t0);
        }
        if constexpr (TM) {
            T.t_end = __builtin_amdgcn_s_memtime();
            const uint32_t rec = blockIdx.x * 12u + uint32_t(wave);
            if ((PROBE & 524288) != 0 && (rec >= gridDim.x * 12u || wave >= 12)) {
                if (lane == 0) atomicOr(reinterpret_cast<unsigned int *>(a.par[5]), 512u);
            } else if (lane == 0) {
                T.put(reinterpret_cast<uint64_t *>(a.par[4]) + rec * 24u, ntile);
            }
        }
        return;
    }
    // ---- compute waves ----
    if constexpr ((PROBE & 16) != 0) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    const int c = Kn::colmap(wave, (int(threadIdx.x) >> 3) & 7), part = int(threadIdx.x) & 7;
    // PROBE 1048576 (probe builds): section 2 of the heavy waves as compile-time copies per d2 too
    constexpr bool SEC2U = (PROBE & 1048576) != 0;
    const uint32_t prel = uint32_t(part) * 16u;
    uint32_t acc[Kn::Q * 8];
    typename K6::Hold H;
    const typename Kn::LaneS LC = Kn::lane_consts(c, part);
    // LOADERS == 0: every compute wave issues its share of the DMA right after each barrier
    // and does the counted wait itself (VMEM ops after step s's DMA: the next step's DMA
    // and the parity stores of the two steps in between)
    typename Kn::Loader LD;
    const uint32_t lds0 = lds_addr_of(smem);
    if constexpr (LOADERS == 0) {
        Kn::loader_init(LD, uint32_t(a.sc), wave, lane);
        if constexpr (!(PROBE & 2))
            for (int s = 0; s < 3 && s < nsteps; s++) Kn::issue_any(s % 3, a, LD, lds0, tm.tile(0, slot, ns), s / 3);
    }
    int st1 = 0, st2 = 0;  // counted stores issued in steps s-1 and s-2
    // PROBE 8192 (probe builds only): group g's end work deferred to after the next step's barrier
    constexpr bool DEFER = (PROBE & 8192) != 0 && LOADERS > 0;
    int pend = -1;
    StreamTile pt{0, 0};
    auto end_any = [&](int ge, StreamTile t) BS_INL {
        const bool ragged = t.vend < t.b0 + uint32_t(Kn::W);
        // opaque per-call copy of the column: the store rows derived from it are computed here,
        // not hoisted out of the tile loop into long-lived (spilled) registers
        int cc = c;
        asm volatile("" : "+v"(cc));
        if (ge == 0) Kn::template end_group<0>(a, acc, H, cc, t, prel, ragged, sink);
        else if (ge == 1) Kn::template end_group<1>(a, acc, H, cc, t, prel, ragged, sink);
        else if (ge == 2) Kn::template end_group<2>(a, acc, H, cc, t, prel, ragged, sink);
        else Kn::template end_group<3>(a, acc, H, cc, t, prel, ragged, sink);
    };
    TimeAcc T;
    T.t_start = TM ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t t0 = TM ? __builtin_amdgcn_s_memtime() : 0;  // chained: every cycle lands in one sum
    if constexpr (TM) T.t_first = t0;
    for (int s = 0; s < nsteps; s++) {
        const int k = s / Kn::STEPS, r = s % Kn::STEPS, g = r / 3, y = r % 3;
        if constexpr (LOADERS == 0 && !(PROBE & 2)) {
            const StreamTile t = tm.tile(k, slot, ns);
            int after;
            if (s == 0) after = (nsteps > 1 ? Kn::ninstr(1) : 0) + (nsteps > 2 ? Kn::ninstr(2) : 0);
            else if (s == 1) after = (nsteps > 2 ? Kn::ninstr(2) : 0) + st1;
            else after = st2 + (s + 1 < nsteps ? Kn::ninstr((y + 1) % 3) : 0) + st1;
            if (t.vend < t.b0 + uint32_t(Kn::W) && ((t.vend - t.b0) & 15u)) {
                wait_vm_n<0>();
                Kn::patch_any(y, a, LD, smem, t, g, lane);
            } else {
                wait_vm_rt(after);
            }
        }
        if constexpr (!(PROBE & 65536)) lds_barrier();  // 65536 (probe, with 2 only): no step barriers
        if constexpr (TM) T.add(0, y, t0);
        if constexpr (DEFER) {
            // the previous group's outputs (PFT, transposes, stores) after this step's barrier:
            // the barrier, and with it the loaders' next DMA, no longer waits for them
            if (pend >= 0) {
                end_any(pend, pt);
                if constexpr (TM) T.addg(pend, t0);
                pend = -1;
            }
        }
        if constexpr (LOADERS == 0 && !(PROBE & 2)) {
            const int s2 = s + 2;
            if (s >= 1 && s2 < nsteps) {
                const int k2 = s2 / Kn::STEPS, r2 = s2 % Kn::STEPS;
                Kn::issue_any(r2 % 3, a, LD, lds0, tm.tile(k2, slot, ns), r2 / 3);
            }
        }
        // opaque per-step copy of the lane constants: everything derived from them (read
        // addresses, PRT masks) is recomputed per step instead of hoisted out of the tile
        // loop into ~30 long-lived registers (which spilled at the 168-VGPR budget)
        typename Kn::LaneS L = LC;
        asm volatile("" : "+v"(L.own[0]), "+v"(L.own[1]), "+v"(L.cb[0][0]), "+v"(L.cb[0][1]));
        asm volatile("" : "+v"(L.cb[1][0]), "+v"(L.cb[1][1]), "+v"(L.cb[2][0]));
        if constexpr (MAP != 0) {
            // digit 2 is wave-uniform: cy[2] lives in an SGPR (the VGPR goes to cb[2][1])
            asm volatile("" : "+v"(L.cb[2][1]));
            asm volatile("" : "+v"(L.cy[0]), "+v"(L.cy[1]));
            L.cy[2] = __builtin_amdgcn_readfirstlane(L.cy[2]);
        } else {
            asm volatile("" : "+v"(L.cy[0]), "+v"(L.cy[1]), "+v"(L.cy[2]));
        }
        if constexpr ((PROBE & 1) != 0) {
            if (s == 0)
#pragma unroll
                for (int w = 0; w < Kn::Q * 8; w++) acc[w] = (threadIdx.x * 0x9E3779B9u) ^ uint32_t(w) ^ L.own[0];
        } else {
            constexpr int SBN = (PROBE & 16384) ? 0 : (PROBE & 32768) ? 2 : 1;
            constexpr bool BAL = (PROBE & 131072) != 0;
            if (y == 0) Kn::template section<0, SBN, BAL>(smem, L, acc);
            else if (y == 1) Kn::template section<1, SBN, BAL>(smem + Kn::REGION, L, acc);
            else if constexpr (MAP != 0) {
                // wave-uniform digit 2 (an SGPR): compile-time section-2 copies
                const int d2 = L.cy[2];
                if constexpr (SEC2U) {
                    if (d2 == 0) Kn::template section2_u<0, SBN>(smem + 2 * Kn::REGION, L, acc);
                    else if (d2 == 1) Kn::template section2_u<1, SBN>(smem + 2 * Kn::REGION, L, acc);
                    else Kn::template section2_u<2, SBN>(smem + 2 * Kn::REGION, L, acc);
                } else {
                    // light waves (d2 in {2, 3}): the compile-time copy; d2 in {0, 1}: the generic step
                    if (d2 >= 2) Kn::template section2_u<2, SBN>(smem + 2 * Kn::REGION, L, acc);
                    else Kn::template section<2, SBN, BAL>(smem + 2 * Kn::REGION, L, acc);
                }
            } else Kn::template section<2, SBN, BAL>(smem + 2 * Kn::REGION, L, acc);
        }
        if constexpr (TM) T.add(1, y, t0);
        if (y == 2 && !(PROBE & 4)) {
            const StreamTile t = tm.tile(k, slot, ns);
            const bool ragged = t.vend < t.b0 + uint32_t(Kn::W);
            const int ge = (PROBE & 32) ? ((g + int(slot)) & 3) : g;
            if constexpr (DEFER) {
                pend = ge;
                pt = t;
            } else {
                end_any(ge, t);
            }
            st2 = st1;
            st1 = ragged ? 0 : Kn::nstores(ge);  // a ragged tile's plain stores are not counted:
                                                 // the waits then cover more than needed
        } else {
            st2 = st1;
            st1 = 0;
        }
        if constexpr (TM) T.addg(g, t0);
    }
    if constexpr (DEFER) {
        if (pend >= 0) end_any(pend, pt);
    }
    if constexpr ((PROBE & 262144) != 0) {
        // a.sdata is 0 in the probe: the predicate is (almost) never true, but not foldable
        if (sink == uint32_t(a.sdata) + 0x9E3779B9u) a.par[0][threadIdx.x] = uint8_t(sink);
    }
    if constexpr (TM) {
        T.t_end = __builtin_amdgcn_s_memtime();
        const uint32_t rec = blockIdx.x * 12u + uint32_t(wave);
        if ((PROBE & 524288) != 0 && (rec >= gridDim.x * 12u || wave >= 12)) {
            if (lane == 0) atomicOr(reinterpret_cast<unsigned int *>(a.par[5]), 256u);
        } else if (lane == 0) {
            T.put(reinterpret_cast<uint64_t *>(a.par[4]) + rec * 24u, ntile);
        }
    }
}

}  // namespace bs
}  // namespace clay
