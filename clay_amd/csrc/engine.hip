// engine.hip -- MI355X (gfx950) kernels, per-device runtime and the C ABI of include/clay.h.
//
// Two device paths:
//   * fused encode (k_fused_encode): the north-star path.  One workgroup owns a
//     tile of W byte positions across ALL alpha layers of a stripe; it streams the
//     data y-section by y-section (PRT on q x q (node, digit) blocks, then the
//     per-layer RS parity contraction accumulated in LDS) and finishes with the
//     PFT of the parity y-section.  Data bytes are read from HBM once, parity
//     bytes written once, shortened (zero) nodes never touched.  Valid when the
//     parity nodes form exactly the last y-section (q == m, i.e. d = k+m-1).
//   * staged engine (k_exec): executes a Plan (plan.hpp) -- the reference's
//     decode_layered / repair replayed into GF region ops -- one launch per
//     dependency level, U-plane in an HBM workspace.  Used for decode, repair and
//     encode shapes the fused kernel does not cover.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/clay.h"
#include "code.hpp"
#include "gf256.hpp"
#include "bitslice.hpp"
#include "stream_encode.hpp"
#include "repair_args.hpp"  // bit-sliced repair kernel: repair_kernel.hpp, instantiated in repair_stream.hip
#include "decode_args.hpp"  // streaming-decode kernel: stream_decode.hpp, instantiated in decode_stream.hip
#include "line_args.hpp"  // line-local bit-sliced (4,2,5) encode / single-erasure decode: bitslice_line.hpp, in line_kernels.hip
#include "kernels.hpp"
#include "plan.hpp"
#include "tuning.hpp"
#include "encode3_args.hpp"

namespace clay {

constexpr int kMaxTn = 64;                 // internal nodes supported on device
constexpr int kMaxBases = 2 * kMaxTn + 2;  // C[tn], H[tn], U, OUT
constexpr int kExecBlock = 256;
constexpr int kGxBatch = 4;  // 8 measured slower (decode 4 erasures 0.87 -> 0.97 ms)
constexpr int kFusedBlock = 512;
constexpr size_t kFusedLdsBudget = 128 * 1024;

struct ExecPtrs {
    uint8_t *p[kMaxBases];
};
// Affine batches: region base b of stripe s is p[b] + s * stride[b] (bytes).
struct ExecStride {
    int64_t s[kMaxBases];
};
// k_gexec operand addressing: one stripe (kernarg pointers), a batch through a device
// pointer table, or an affine batch (kernarg base + stripe * stride).
enum : int { kBatchNone = 0, kBatchTable = 1, kBatchAffine = 2 };

// Grouped staged executor: one workgroup = one source-sharing op group x one tile.
// Each source tile is loaded once, split into its perm-table indices once, and
// multiplied into up to MAXD destination accumulators (dst_d = XOR_s coef[d][s] * src_s).
template <int VW, int MAXD, int BATCH = kBatchNone, bool PIPE = false>
__global__ __launch_bounds__(kExecBlock) void k_gexec(ExecPtrs P, const DevGroup *__restrict__ groups,
                                                      const DevSrc *__restrict__ gsrcs,
                                                      const DevSrc *__restrict__ gdsts,
                                                      const uint32_t *__restrict__ gcoef,
                                                      const uint32_t *__restrict__ tabs, uint32_t g0,
                                                      uint32_t tiles, uint64_t sc, uint64_t r0, uint64_t r1,
                                                      uint32_t ngroups, uint32_t order, uint32_t bx,
                                                      uint8_t *const *__restrict__ ptab, uint32_t lps,
                                                      uint32_t nstripes, const ExecStride S, uint32_t tpw) {
    constexpr int NW = (VW + 3) / 4;
    // perm tables of all 256 constants in LDS: a multiply's table is a broadcast LDS read,
    // not a scalar-cache load whose address waits on the loaded coefficient
    __shared__ __attribute__((aligned(16))) uint32_t ltab[256 * 8];
    for (uint32_t i = threadIdx.x; i < 256u * 8u / 4u; i += kExecBlock)
        reinterpret_cast<uint4 *>(ltab)[i] = reinterpret_cast<const uint4 *>(tabs)[i];
    __syncthreads();
    // Block -> (group, tile).  order 0: group-major.  1: tile-major -- all groups of a
    // tile run back to back, so an input sub-chunk tile read by several groups is
    // re-read while still in L2 / MALL.  2: tile-major within contiguous per-XCD
    // block ranges (blocks round-robin over the 8 XCDs: xcd = blockIdx % 8).
    uint32_t gi, tile;
    if (order == 0) {
        gi = blockIdx.x / tiles;
        tile = blockIdx.x - gi * tiles;
    } else {
        uint32_t v = blockIdx.x;
        if (order == 2) {
            v = (blockIdx.x & 7u) * bx + (blockIdx.x >> 3);
            if (v >= ngroups * tiles) return;
        }
        tile = v / ngroups;
        gi = v - tile * ngroups;
    }
    // BATCH: lps lanes per stripe; a block runs kExecBlock / lps stripes (small sub-chunks
    // fill the block with stripes instead of idle lanes)
    uint32_t lane = threadIdx.x, stripe = 0;
    if constexpr (BATCH != kBatchNone) {
        const uint32_t spb = kExecBlock / lps;
        stripe = blockIdx.y * spb + threadIdx.x / lps;
        lane = threadIdx.x % lps;
        if (threadIdx.x >= spb * lps || stripe >= nstripes) return;
    }
    const DevGroup g = groups[g0 + gi];
    // tpw consecutive tiles per block (one group's scalar work amortised over tpw tiles)
    for (uint32_t tk = 0; tk < tpw; tk++) {
    const uint64_t pos = r0 + ((uint64_t(tile) * tpw + tk) * lps + lane) * VW;
    if (pos >= r1) return;
    // Regions start at slot*sc, which is only 2-byte aligned for e.g. the (9,3,11)
    // chunk of 268,435,458 B; gfx950 global loads/stores run in unaligned mode, so
    // full lanes use 16-byte accesses at any address and only the last lane of a
    // region (pos + VW > sc) falls back to bytes.
    const bool full = pos + VW <= r1;
    const uint32_t nb = full ? uint32_t(VW) : uint32_t(r1 - pos);
    uint32_t acc[MAXD][NW];
#pragma unroll
    for (int d = 0; d < MAXD; d++)
#pragma unroll
        for (int w = 0; w < NW; w++) acc[d][w] = 0;
    // kGxBatch source loads in flight before the first multiply (memory-level parallelism)
    auto load_batch = [&](uint32_t s0, Words<NW>(&v)[kGxBatch]) __attribute__((always_inline)) {
#pragma unroll
        for (int b = 0; b < kGxBatch; b++) {
            const uint32_t s = s0 + b;
#pragma unroll
            for (int w = 0; w < NW; w++) v[b].w[w] = 0;
            if (s < g.nsrc) {
                const DevSrc src = gsrcs[g.src_begin + s];
                // BATCH (template, so the single-stripe kernel keeps its kernarg pointer table)
                const uint8_t *sp;
                if constexpr (BATCH == kBatchTable)
                    sp = ptab[stripe * kMaxBases + src.base] + uint64_t(src.slot) * sc + pos;
                else if constexpr (BATCH == kBatchAffine)
                    sp = P.p[src.base] + int64_t(stripe) * S.s[src.base] + uint64_t(src.slot) * sc + pos;
                else
                    sp = P.p[src.base] + uint64_t(src.slot) * sc + pos;
                if (full) {
                    __builtin_memcpy(&v[b], sp, sizeof(v[b]));
                } else {
                    uint8_t tb[NW * 4] = {};
                    for (uint32_t i = 0; i < nb; i++) tb[i] = sp[i];
                    __builtin_memcpy(&v[b], tb, sizeof(v[b]));
                }
            }
        }
    };
    auto mac_batch = [&](uint32_t s0, const Words<NW>(&v)[kGxBatch]) __attribute__((always_inline)) {
#pragma unroll
        for (int b = 0; b < kGxBatch; b++) {
            const uint32_t s = s0 + b;
            if (s >= g.nsrc) break;
            GfIdx ix[NW];
#pragma unroll
            for (int w = 0; w < NW; w++) ix[w] = gf_idx(v[b].w[w]);
#pragma unroll
            for (int d = 0; d < MAXD; d++) {
                if (d >= int(g.ndst)) break;
                const uint32_t c = gcoef[g.coef_begin + d * g.nsrc + s];
                if (c == 0) continue;  // merged groups: source absent from this row
                if (c == 1) {
#pragma unroll
                    for (int w = 0; w < NW; w++) acc[d][w] ^= v[b].w[w];
                } else {
                    const uint4 t4 = *reinterpret_cast<const uint4 *>(ltab + c * 8u);
                    const GfTab t{t4.x, t4.y, t4.z, t4.w, ltab[c * 8u + 4u]};
#pragma unroll
                    for (int w = 0; w < NW; w++) acc[d][w] ^= gf_mul_idx(ix[w], t);
                }
            }
        }
    };
    if constexpr (PIPE) {
        // software pipeline: the next batch's loads are in flight while this one multiplies
        Words<NW> va[kGxBatch], vb[kGxBatch];
        load_batch(0, va);
        for (uint32_t s0 = 0; s0 < g.nsrc; s0 += 2 * kGxBatch) {
            const bool more = s0 + kGxBatch < g.nsrc;
            if (more) load_batch(s0 + kGxBatch, vb);
            mac_batch(s0, va);
            if (!more) break;
            if (s0 + 2 * kGxBatch < g.nsrc) load_batch(s0 + 2 * kGxBatch, va);
            mac_batch(s0 + kGxBatch, vb);
        }
    } else {
        for (uint32_t s0 = 0; s0 < g.nsrc; s0 += kGxBatch) {
            Words<NW> v[kGxBatch];
            load_batch(s0, v);
            mac_batch(s0, v);
        }
    }
#pragma unroll
    for (int d = 0; d < MAXD; d++) {
        if (d >= int(g.ndst)) break;
        const DevSrc dst = gdsts[g.dst_begin + d];
        uint8_t *dp;
        if constexpr (BATCH == kBatchTable)
            dp = ptab[stripe * kMaxBases + dst.base] + uint64_t(dst.slot) * sc + pos;
        else if constexpr (BATCH == kBatchAffine)
            dp = P.p[dst.base] + int64_t(stripe) * S.s[dst.base] + uint64_t(dst.slot) * sc + pos;
        else
            dp = P.p[dst.base] + uint64_t(dst.slot) * sc + pos;
        if (full) {
            __builtin_memcpy(dp, acc[d], sizeof(acc[d]));
        } else {
            uint8_t tb[NW * 4];
            __builtin_memcpy(tb, acc[d], sizeof(tb));
            for (uint32_t i = 0; i < nb; i++) dp[i] = tb[i];
        }
    }
    }  // tiles of the block
}


// ---------------------------------------------------------------------------
// Tile-fused executor (k_texec): ONE launch runs every level of a plan.  A workgroup owns
// the byte tile [64*VW*blockIdx.x, +64*VW) of every sub-chunk and keeps the plan's U
// workspace slots for that tile in LDS (dense slot u at u * 64 * VW), so U values never
// round-trip through HBM and the chip never idles at level boundaries (a level boundary
// is a workgroup barrier, not a kernel boundary).  Each wave walks its share of a level's
// groups as a flat stream of (group, source) terms, TEX_BATCH loads in flight at a time
// across group boundaries -- so 1-2 source groups (repair's C outputs, decode's PFT ops)
// are not latency-bound -- multiplies every loaded source into up to MAXD destination
// accumulators, and writes a group's destinations (LDS slot or HBM) after its last term.
// Eligible when the plan's dense U slot count fits the LDS budget (host: texec_vw).
// ---------------------------------------------------------------------------
constexpr int kTexMaxStages = 64;
constexpr int kTexBatch = 8;
constexpr size_t kTexLdsMax = 160 * 1024;
constexpr size_t kTexTabBytes = 256 * 8 * 4;  // perm tables of all GF(2^8) constants
constexpr size_t kTexAutoGroups = 32;

// Host-flattened term stream (texec_flatten): per level and wave, the terms of the wave's
// groups back to back, so a batch of term records is one run of independent scalar
// loads (no group-header -> source-descriptor -> address chain).
//   x: source base << 24 | slot (U sources: LDS slot)
//   y, w: the coefficients of destinations 0-3 (y) and 4-7 (w), one byte each
//   z: ndst << 24, | bit 31 + first destination index on the last term of a group
// The perm tables of all 256 GF(2^8) constants sit in LDS (8 KiB, behind the U slots), so a
// multiply's table is a broadcast LDS read instead of a dependent scalar-cache load.
template <int VW, int MAXD, int NWV>
__global__ __launch_bounds__(64 * NWV) void k_texec(ExecPtrs P, const uint4 *__restrict__ terms,
                                                    const uint32_t *__restrict__ wbeg,
                                                    const uint32_t *__restrict__ tabs,
                                                    const DevSrc *__restrict__ tdsts, uint32_t nstages, uint64_t sc,
                                                    uint32_t ubase, uint32_t nu) {
    constexpr int NW = VW / 4;
    constexpr uint32_t W = 64u * VW;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint64_t pos = uint64_t(blockIdx.x) * W + lane * VW;
    const bool full = pos + VW <= sc;
    const uint32_t nb = pos >= sc ? 0u : (full ? uint32_t(VW) : uint32_t(sc - pos));
    uint8_t *const lds_lane = smem + lane * VW;
    uint32_t *const ltab = reinterpret_cast<uint32_t *>(smem + size_t(nu) * W);
    for (uint32_t i = threadIdx.x; i < 256u * 8u; i += 64u * NWV) ltab[i] = tabs[i];
    __syncthreads();
    for (uint32_t L = 0; L < nstages; L++) {
        const uint32_t te = wbeg[L * NWV + wave + 1];
        uint32_t acc[MAXD][NW];
#pragma unroll
        for (int d = 0; d < MAXD; d++)
#pragma unroll
            for (int w = 0; w < NW; w++) acc[d][w] = 0;
        for (uint32_t t = wbeg[L * NWV + wave]; t < te; t += kTexBatch) {
            uint4 rec[kTexBatch];
            Words<NW> v[kTexBatch];
#pragma unroll
            for (int b = 0; b < kTexBatch; b++) rec[b] = t + b < te ? terms[t + b] : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int b = 0; b < kTexBatch; b++) {
#pragma unroll
                for (int w = 0; w < NW; w++) v[b].w[w] = 0;
                if (t + b >= te) continue;
                const uint32_t base = rec[b].x >> 24, slot = rec[b].x & 0xFFFFFFu;
                if (base == ubase) {
                    __builtin_memcpy(&v[b], lds_lane + slot * W, sizeof(v[b]));
                } else {
                    const uint8_t *sp = P.p[base] + uint64_t(slot) * sc + pos;
                    if (full) {
                        __builtin_memcpy(&v[b], sp, sizeof(v[b]));
                    } else {
                        uint8_t tb[VW] = {};
                        for (uint32_t i = 0; i < nb; i++) tb[i] = sp[i];
                        __builtin_memcpy(&v[b], tb, sizeof(v[b]));
                    }
                }
            }
#pragma unroll
            for (int b = 0; b < kTexBatch; b++) {
                if (t + b >= te) break;
                const uint32_t nd = (rec[b].z >> 24) & 15u;
                GfIdx ix[NW];
#pragma unroll
                for (int w = 0; w < NW; w++) ix[w] = gf_idx(v[b].w[w]);
#pragma unroll
                for (int d = 0; d < MAXD; d++) {
                    if (d >= int(nd)) break;
                    const uint32_t c = ((d < 4 ? rec[b].y : rec[b].w) >> (8 * (d & 3))) & 0xFFu;
                    if (c == 0u) continue;
                    if (c == 1u) {
#pragma unroll
                        for (int w = 0; w < NW; w++) acc[d][w] ^= v[b].w[w];
                    } else {
                        const uint4 t4 = *reinterpret_cast<const uint4 *>(ltab + c * 8u);
                        const GfTab tab{t4.x, t4.y, t4.z, t4.w, ltab[c * 8u + 4u]};
#pragma unroll
                        for (int w = 0; w < NW; w++) acc[d][w] ^= gf_mul_idx(ix[w], tab);
                    }
                }
                if (rec[b].z >> 31) {
                    const uint32_t db = rec[b].z & 0xFFFFFFu;
#pragma unroll
                    for (int d = 0; d < MAXD; d++) {
                        if (d >= int(nd)) break;
                        const DevSrc dst = tdsts[db + d];
                        if (dst.base == ubase) {
                            __builtin_memcpy(lds_lane + dst.slot * W, acc[d], sizeof(acc[d]));
                        } else if (nb) {
                            uint8_t *dp = P.p[dst.base] + uint64_t(dst.slot) * sc + pos;
                            if (full) {
                                __builtin_memcpy(dp, acc[d], sizeof(acc[d]));
                            } else {
                                uint8_t tb[VW];
                                __builtin_memcpy(tb, acc[d], sizeof(tb));
                                for (uint32_t i = 0; i < nb; i++) dp[i] = tb[i];
                            }
                        }
#pragma unroll
                        for (int w = 0; w < NW; w++) acc[d][w] = 0;
                    }
                }
            }
        }
        // level boundary: U slots written above are read by the next level; outputs
        // written to HBM by this workgroup are visible to it (workgroup-scope fence)
        if (L + 1 < nstages) __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Y-grouped chunk layout (docs/clay-practical-implementation.md
// "Option C", written there with least-significant-digit-first layer digits; here the
// crate's most-significant-digit-first convention, coords.rs:30-40).  For y-section y the
// chunk's alpha sub-chunks are reordered as q blocks x = 0..q-1 of beta sub-chunks, block x
// holding the layers z with digit_y(z) == x in ascending z -- exactly the sub-chunks
// repair of node (y, x) reads from every helper (repair.rs:22-49), so a helper's repair
// payload is one contiguous range: group + x * beta * sc.
// ---------------------------------------------------------------------------
// Layer of position i of group y: insert digit x = i / beta at digit y of p = i % beta.
__device__ __forceinline__ uint32_t ygroup_layer(uint32_t i, uint32_t beta, uint32_t q, uint32_t pw) {
    const uint32_t x = i / beta, p = i - x * beta;  // pw = q^(t-1-y)
    return ((p / pw) * q + x) * pw + p % pw;
}
// TO_GROUP: dst position i <- src layer z(i); else dst layer z(i) <- src position i.
// One block per (sub-chunk, 4 KiB piece); 16-byte lanes at any alignment.
template <bool TO_GROUP>
__global__ __launch_bounds__(256) void k_ygroup(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, uint64_t sc,
                                                uint32_t beta, uint32_t q, uint32_t pw, uint32_t pieces) {
    const uint32_t i = blockIdx.x / pieces, piece = blockIdx.x - i * pieces;
    const uint64_t z = ygroup_layer(i, beta, q, pw);
    const uint64_t so = (TO_GROUP ? z : i) * sc, dofs = (TO_GROUP ? i : z) * sc;
    const uint64_t b = (uint64_t(piece) * 256 + threadIdx.x) * 16;
    if (b + 16 <= sc) {
        uint4 v;
        __builtin_memcpy(&v, src + so + b, 16);
        __builtin_memcpy(dst + dofs + b, &v, 16);
    } else {
        for (uint64_t j = b; j < sc; j++) dst[dofs + j] = src[so + j];
    }
}

// ---------------------------------------------------------------------------
// Fused encode (parity = last y-section).  See file header and DESIGN.md.
// LDS: acc[p][z][W] bytes (p < Q parity rows, z < alpha layers, W positions).
// ---------------------------------------------------------------------------
constexpr int kFusedMaxK = 64;
struct FusedArgs {
    const uint8_t *data[kFusedMaxK];  // internal nodes 0..K-1, nullptr = shortened (zero)
    uint8_t *par[8];                  // parity y-section, node x
    uint64_t sc;                      // sub-chunk size (bytes)
    uint32_t alpha, t, K, W;          // layers, y-sections, K = k+nu, tile positions
    uint32_t ntiles, tiles_per_xcd, nslots;
    uint32_t dinv[5];                 // perm table of det^-1 (PFT, transforms.rs:307-308)
};

template <int Q, int PPT>
__global__ __launch_bounds__(kFusedBlock) void k_fused_encode(FusedArgs a, const uint32_t *__restrict__ mtab) {
    constexpr int NW = PPT / 4;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t W = a.W, PG = W / PPT, alpha = a.alpha;
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    GfTab dinv;
    dinv.w0 = a.dinv[0]; dinv.w1 = a.dinv[1]; dinv.w2 = a.dinv[2]; dinv.w3 = a.dinv[3]; dinv.w4 = a.dinv[4];

    for (uint32_t tix = slot; tix < a.tiles_per_xcd; tix += a.nslots) {
        const uint32_t tile = xcd * a.tiles_per_xcd + tix;
        if (tile >= a.ntiles) break;  // uniform per workgroup
        const uint64_t b0 = uint64_t(tile) * W;

        // ---- phase A: y-sections 0..t-2 -> parity-U accumulators in LDS ----
        uint32_t wy = alpha / Q;  // q^(t-1-y), starting at y = 0
        for (uint32_t y = 0; y + 1 < a.t; ++y, wy /= Q) {
            const uint32_t nlines = alpha / Q, units = nlines * PG;
            for (uint32_t u = threadIdx.x; u < units; u += kFusedBlock) {
                const uint32_t line = u / PG, pg = u - line * PG;
                const uint64_t pos = b0 + uint64_t(pg) * PPT;
                const bool ok = pos < a.sc;
                const uint32_t hi = line / wy, lo = line - hi * wy;
                const uint32_t z0 = hi * wy * Q + lo;
                uint32_t B[Q][Q][NW];
#pragma unroll
                for (int x = 0; x < Q; x++) {
                    const uint8_t *nd = a.data[y * Q + x];
#pragma unroll
                    for (int j = 0; j < Q; j++) {
                        if (nd != nullptr && ok) {
                            Words<NW> v = vload<PPT>(nd + uint64_t(z0 + j * wy) * a.sc + pos);
#pragma unroll
                            for (int w = 0; w < NW; w++) B[x][j][w] = v.w[w];
                        } else {
#pragma unroll
                            for (int w = 0; w < NW; w++) B[x][j][w] = 0;
                        }
                    }
                }
                // PRT on every off-diagonal pair: U[x][j] = C[x][j] + g*C[j][x]  (transforms.rs:42-55)
#pragma unroll
                for (int x = 0; x < Q; x++)
#pragma unroll
                    for (int j = x + 1; j < Q; j++)
#pragma unroll
                        for (int w = 0; w < NW; w++) {
                            const uint32_t bxj = B[x][j][w], bjx = B[j][x][w];
                            B[x][j][w] = bxj ^ gf_xt(bjx);
                            B[j][x][w] = bjx ^ gf_xt(bxj);
                        }
                // RS parity rows: V[p][z_j] += M[p][yQ+x] * U[x][j]  (decode.rs:386-404)
#pragma unroll
                for (int j = 0; j < Q; j++) {
                    uint32_t V[Q][NW];
#pragma unroll
                    for (int p = 0; p < Q; p++)
#pragma unroll
                        for (int w = 0; w < NW; w++) V[p][w] = 0;
#pragma unroll
                    for (int x = 0; x < Q; x++) {
#pragma unroll
                        for (int w = 0; w < NW; w++) {
                            const GfIdx ix = gf_idx(B[x][j][w]);
#pragma unroll
                            for (int p = 0; p < Q; p++) {
                                const GfTab tb = load_tab(mtab + (uint32_t(p) * a.K + y * Q + x) * 8);
                                V[p][w] ^= gf_mul_idx(ix, tb);
                            }
                        }
                    }
                    const uint32_t z = z0 + j * wy;
#pragma unroll
                    for (int p = 0; p < Q; p++) {
                        uint8_t *l = lds + (size_t(p) * alpha + z) * W + size_t(pg) * PPT;
                        Words<NW> v;
                        if (y == 0) {
#pragma unroll
                            for (int w = 0; w < NW; w++) v.w[w] = V[p][w];
                        } else {
                            v = vload<PPT>(l);
#pragma unroll
                            for (int w = 0; w < NW; w++) v.w[w] ^= V[p][w];
                        }
                        vstore<PPT>(l, v);
                    }
                }
            }
            __syncthreads();
        }

        // ---- phase B: PFT of the parity y-section (digit t-1, weight 1) ----
        {
            const uint32_t ngroups = alpha / Q, units = ngroups * PG;
            for (uint32_t u = threadIdx.x; u < units; u += kFusedBlock) {
                const uint32_t g = u / PG, pg = u - g * PG;
                const uint64_t pos = b0 + uint64_t(pg) * PPT;
                const uint32_t z0 = g * Q;
                uint32_t A[Q][Q][NW];
#pragma unroll
                for (int x = 0; x < Q; x++)
#pragma unroll
                    for (int j = 0; j < Q; j++) {
                        Words<NW> v = vload<PPT>(lds + (size_t(x) * alpha + z0 + j) * W + size_t(pg) * PPT);
#pragma unroll
                        for (int w = 0; w < NW; w++) A[x][j][w] = v.w[w];
                    }
#pragma unroll
                for (int x = 0; x < Q; x++)
#pragma unroll
                    for (int j = x + 1; j < Q; j++)
#pragma unroll
                        for (int w = 0; w < NW; w++) {  // C = det^-1 (U + g U*)  (transforms.rs:108-125)
                            const uint32_t axj = A[x][j][w], ajx = A[j][x][w];
                            A[x][j][w] = gf_mul(axj ^ gf_xt(ajx), dinv);
                            A[j][x][w] = gf_mul(ajx ^ gf_xt(axj), dinv);
                        }
                if (pos < a.sc) {
#pragma unroll
                    for (int x = 0; x < Q; x++)
#pragma unroll
                        for (int j = 0; j < Q; j++) {
                            Words<NW> v;
#pragma unroll
                            for (int w = 0; w < NW; w++) v.w[w] = A[x][j][w];
                            vstore<PPT>(a.par[x] + uint64_t(z0 + j) * a.sc + pos, v);
                        }
                }
            }
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------
// Runtime
// ---------------------------------------------------------------------------
#define CLAY_HIP(expr)                                                                                  \
    do {                                                                                                \
        hipError_t _e = (expr);                                                                         \
        if (_e != hipSuccess)                                                                           \
            return make_error(CLAY_ERR_DEVICE, size_t(_e), 0, 0, "HIP error: %s (%s)", hipGetErrorString(_e), \
                              #expr);                                                                   \
    } while (0)

// Thread safety (include/clay.h): like the reference's immutable ClayCode (lib.rs:58),
// every entry point may be called concurrently from any thread on any stream.  There
// is no process-wide lock: the code/plan caches and the per-device pools each have
// their own mutex, held only for lookups and bookkeeping, never across a launch or a
// synchronisation of a caller's stream.
static thread_local std::string t_last_path = "none";
static thread_local size_t t_last_launches = 0;
static thread_local const char *t_last_exec = "none";  // plan executor of the last run_plan
// Encode path selection (clay_set_encode_path): process-wide, read without locks (4 was the
// retired v6 kernel, now unused).
enum : int { kModeAuto = 0, kModeStaged = 1, kModeFused = 2, kModeBs = 3, kModeStream = 5 };
static std::atomic<int> g_encode_mode{kModeAuto};
static std::atomic<int> g_encode_tile{0};  // per-mode variant (see clay_set_encode_path)

// Device properties the launchers need, queried once per device.
struct DevProps {
    int dev = 0;
    int cus = 256;
    hipDeviceProp_t raw{};
};
static DevProps g_props[64];
static std::once_flag g_props_once[64];
static const DevProps &dev_props(int dev) {
    std::call_once(g_props_once[dev], [dev] {
        DevProps &p = g_props[dev];
        p.dev = dev;
        if (hipGetDeviceProperties(&p.raw, dev) == hipSuccess) p.cus = p.raw.multiProcessorCount;
    });
    return g_props[dev];
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device)
static Error lds_attr_once(const void *fn, int bytes, int dev) {
    static std::mutex mu;
    static std::set<std::pair<const void *, int>> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done.count({fn, dev})) return Error{};
    CLAY_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    done.insert({fn, dev});
    return Error{};
}

static bool capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}
// id of the capture `st` is in (0: none)
static unsigned long long capture_id(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    if (hipStreamGetCaptureInfo(st, &cs, &id) != hipSuccess || cs != hipStreamCaptureStatusActive) return 0;
    return id;
}

// A pooled device buffer (U workspaces, host-API staging).  A lease is handed to one
// call at a time; on release an event is recorded on the caller's stream, and the
// buffer is handed out again only once that event has completed -- so streams that
// come and go reuse the same few buffers instead of growing HBM per stream.  A lease
// used inside a stream capture belongs to the captured graph for good (pinned).
struct Lease {
    void *d = nullptr;
    size_t bytes = 0;
    hipEvent_t ev = nullptr;
    hipStream_t last = nullptr;  // stream of the last use (reuse there needs no event query)
    bool used = false, busy = false, pinned = false;
    // taken by a call inside a stream capture: the capturing stream and its capture id, so
    // clay_release_captured can refuse while that capture is still open
    bool captured = false;
    hipStream_t cap_st = nullptr;
    unsigned long long cap_id = 0;
};
// A batched launch's device pointer table, cached by content (immutable once
// uploaded, so concurrent users may share it); freed LRU after its users' events.
struct PtrTable {
    void *d = nullptr;
    void *h = nullptr;  // pinned source of the upload, kept: a captured copy node reads it
    hipEvent_t up = nullptr;  // recorded after the (eager) upload: other streams wait on it
    std::map<hipStream_t, hipEvent_t> evs;
    uint64_t last = 0;
    int users = 0;  // calls between ptr_table() and ptr_table_done(): never freed meanwhile
    bool pinned = false;
    hipStream_t cap_st = nullptr;  // captured tables: the capturing stream and its capture id
    unsigned long long cap_id = 0;
};
constexpr size_t kMaxPtrTables = 64;
constexpr size_t kCapArena = size_t(4) << 20;  // pointer tables created inside stream captures

struct DevState {
    std::mutex mu;  // everything below
    bool init = false;
    uint32_t *d_tabs = nullptr;                  // perm tables of all 256 constants
    std::vector<std::unique_ptr<Lease>> pool;    // workspaces and staging buffers
    std::map<std::vector<uint8_t *>, PtrTable> tables;       // eager uploads, shared by content
    // tables of calls inside a stream capture: bump-allocated from this arena (no hipMalloc
    // while capturing), owned by the captured graphs for good
    uint8_t *cap_d = nullptr, *cap_h = nullptr;
    size_t cap_used = 0;
    std::vector<std::unique_ptr<PtrTable>> captured;
    uint64_t tick = 0;
    std::vector<hipStream_t> host_streams;       // idle streams of the host-streaming pipeline
};
static DevState g_dev[64];

struct CodeState {
    clay_code_t code{};
    RsCtx rs;
    std::mutex mu;  // the plan maps, device uploads and mtab (plans are immutable once built)
    std::unique_ptr<Plan> enc;
    std::map<std::vector<uint8_t>, std::unique_ptr<Plan>> dec, rep;
    struct DevGrouped {
        const DevGroup *groups;
        const DevSrc *srcs, *dsts;
        const uint32_t *coef;
        // k_texec form: U slots register-allocated to nu LDS slots; the term streams
        const DevSrc *tsrcs, *tdsts;
        uint32_t nu;
        const uint4 *terms;
        const uint32_t *wbeg;         // term ranges per (level, wave)
        uint32_t nwv;                 // waves per workgroup the streams were cut for
    };
    std::map<std::pair<const Plan *, int>, DevGrouped> gplan;
    std::map<int, uint32_t *> mtab;
    std::map<std::pair<std::vector<uint32_t>, int>, const uint32_t *> dtabs;  // stream-decode tables
    explicit CodeState(const clay_code_t &c) : code(c), rs(c) {}
};
static std::mutex g_codes_mu;
static std::map<std::tuple<size_t, size_t, size_t>, std::unique_ptr<CodeState>> g_codes;

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

static Error check_code(const clay_code_t *c) {
    if (!c) return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null code");
    clay_code_t chk{};
    Error e = code_new(c->k, c->m, c->d, &chk);
    if (e) return e;
    if (std::memcmp(&chk, c, sizeof(chk)) != 0)
        return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: code struct not produced by clay_new");
    return Error{};
}

static Error dev_state(int dev, DevState **out) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "HIP error: no GPU device available (no CPU fallback)");
    if (dev < 0 || dev >= ndev || dev >= 64)
        return make_error(CLAY_ERR_DEVICE, size_t(dev), 0, 0, "HIP error: invalid device ordinal %d", dev);
    DevState &s = g_dev[dev];
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.init) {
        DeviceGuard g(dev);
        std::vector<uint32_t> tabs(256 * 8);
        for (int c = 0; c < 256; c++) perm_table(uint8_t(c), &tabs[c * 8]);
        CLAY_HIP(hipMalloc(&s.d_tabs, tabs.size() * 4));
        CLAY_HIP(hipMemcpy(s.d_tabs, tabs.data(), tabs.size() * 4, hipMemcpyHostToDevice));
        CLAY_HIP(hipMalloc(&s.cap_d, kCapArena));
        CLAY_HIP(hipHostMalloc(&s.cap_h, kCapArena, hipHostMallocDefault));
        s.init = true;
    }
    *out = &s;
    return Error{};
}

static CodeState *code_state(const clay_code_t &c) {
    std::lock_guard<std::mutex> lk(g_codes_mu);
    auto key = std::make_tuple(c.k, c.m, c.d);
    auto it = g_codes.find(key);
    if (it != g_codes.end()) return it->second.get();
    auto cs = std::make_unique<CodeState>(c);
    CodeState *p = cs.get();
    g_codes[key] = std::move(cs);
    return p;
}

// Idle pooled buffers beyond this many are freed when a new one is allocated.
constexpr size_t kMaxIdleLeases = 4;

static bool event_done(hipEvent_t ev) { return hipEventQuery(ev) == hipSuccess; }

// Lease a device buffer of at least `bytes` for work on stream `st` (best fit among idle
// buffers whose last use is complete or was on `st` itself; while `st` is capturing no
// event is queried and nothing is freed).
static Error lease_acquire(DevState &ds, size_t bytes, hipStream_t st, Lease **out) {
    std::lock_guard<std::mutex> lk(ds.mu);
    const bool cap = capturing(st);
    Lease *best = nullptr;
    if (!cap)  // idle buffers whose last use has completed are free for any stream (and for a
               // later stream capture, which may not query events or allocate)
        for (auto &l : ds.pool)
            if (!l->busy && !l->pinned && l->used && event_done(l->ev)) l->used = false;
    for (auto &l : ds.pool) {
        if (l->busy || l->pinned || l->bytes < bytes || (best && l->bytes >= best->bytes)) continue;
        if (!l->used || l->last == st || (!cap && event_done(l->ev))) best = l.get();
    }
    if (!best && !cap) {
        // free idle leases too small for this request, keeping the pool bounded
        size_t idle = 0;
        for (auto &l : ds.pool) idle += (!l->busy && !l->pinned);
        for (auto it = ds.pool.begin(); it != ds.pool.end() && idle >= kMaxIdleLeases;) {
            Lease &l = **it;
            if (!l.busy && !l.pinned && l.bytes < bytes && hipEventSynchronize(l.ev) == hipSuccess) {
                (void)hipFree(l.d);
                (void)hipEventDestroy(l.ev);
                it = ds.pool.erase(it);
                idle--;
            } else {
                ++it;
            }
        }
    }
    if (!best && cap)  // no allocation while capturing (it would invalidate the capture)
        return make_error(CLAY_ERR_DEVICE, bytes, 0, 0,
                          "no idle workspace of %zu bytes for a stream capture: call clay_reserve_workspace before "
                          "capturing (a captured call keeps its workspace until clay_release_captured)",
                          bytes);
    if (!best) {
        auto l = std::make_unique<Lease>();
        CLAY_HIP(hipMalloc(&l->d, std::max<size_t>(bytes, 256)));
        l->bytes = std::max<size_t>(bytes, 256);
        CLAY_HIP(hipEventCreateWithFlags(&l->ev, hipEventDisableTiming));
        best = l.get();
        ds.pool.push_back(std::move(l));
    }
    // order after the previous user even if `st` is a recycled handle of a destroyed
    // stream whose work is still running (free when that work is complete)
    if (best->used && !cap) CLAY_HIP(hipStreamWaitEvent(st, best->ev, 0));
    best->busy = true;
    if (cap) {
        best->captured = true;
        best->cap_st = st;
        best->cap_id = capture_id(st);
    }
    *out = best;
    return Error{};
}
// Hand a lease back after its last use was enqueued on `st`.
static void lease_release(DevState &ds, Lease *l, hipStream_t st) {
    if (!l) return;
    std::lock_guard<std::mutex> lk(ds.mu);
    if (capturing(st)) {
        l->pinned = true;
    } else {
        (void)hipEventRecord(l->ev, st);
        l->last = st;
        l->used = true;
    }
    l->busy = false;
}
struct LeaseGuard {
    DevState &ds;
    Lease *l = nullptr;
    hipStream_t st;
    LeaseGuard(DevState &d, hipStream_t s) : ds(d), st(s) {}
    ~LeaseGuard() { lease_release(ds, l, st); }
    uint8_t *ptr() const { return static_cast<uint8_t *>(l->d); }
};

// Device copy of a batched launch's pointer table: uploaded once per distinct table
// (hipMemcpyAsync from pinned memory), then reused by every call with the same buffers --
// no per-call synchronisation or blocking copy.
//  * An eager upload records `up` on its stream; every later user waits on it
//    (hipStreamWaitEvent), so a table first uploaded on stream A is never read on stream B
//    before the copy has landed.
//  * An upload inside a stream capture is only a graph node (it runs at replay), so it is
//    never shared: each capture gets its own table, owned by the graph for good.
//  * `users` counts calls between ptr_table() and ptr_table_done(); eviction and
//    clay_release_workspace skip such tables, so a table is never freed between the lookup
//    and the event that guards its last launch.
static void free_table(PtrTable &t) {
    for (auto &se : t.evs) {
        (void)hipEventSynchronize(se.second);
        (void)hipEventDestroy(se.second);
    }
    if (t.up) {
        (void)hipEventSynchronize(t.up);
        (void)hipEventDestroy(t.up);
    }
    (void)hipFree(t.d);
    (void)hipHostFree(t.h);
}
static Error upload_table(PtrTable &t, const std::vector<uint8_t *> &tab, hipStream_t st, bool cap) {
    const size_t bytes = tab.size() * sizeof(uint8_t *);
    CLAY_HIP(hipMalloc(&t.d, bytes));
    CLAY_HIP(hipHostMalloc(&t.h, bytes, hipHostMallocDefault));
    std::memcpy(t.h, tab.data(), bytes);
    CLAY_HIP(hipMemcpyAsync(t.d, t.h, bytes, hipMemcpyHostToDevice, st));
    if (!cap) {
        CLAY_HIP(hipEventCreateWithFlags(&t.up, hipEventDisableTiming));
        CLAY_HIP(hipEventRecord(t.up, st));
    }
    return Error{};
}
static Error ptr_table(DevState &ds, const std::vector<uint8_t *> &tab, hipStream_t st, PtrTable **out) {
    std::lock_guard<std::mutex> lk(ds.mu);
    if (capturing(st)) {
        // no allocation and no cross-capture event while capturing: a private copy from the
        // arena, uploaded by the graph's own copy node at every replay
        const size_t bytes = (tab.size() * sizeof(uint8_t *) + 255) / 256 * 256;
        if (ds.cap_used + bytes > kCapArena)
            return make_error(CLAY_ERR_DEVICE, ds.cap_used, bytes, 0, "pointer-table arena for captured calls exhausted");
        auto t = std::make_unique<PtrTable>();
        t->pinned = true;
        t->cap_st = st;
        t->cap_id = capture_id(st);
        t->d = ds.cap_d + ds.cap_used;
        t->h = ds.cap_h + ds.cap_used;
        ds.cap_used += bytes;
        std::memcpy(t->h, tab.data(), tab.size() * sizeof(uint8_t *));
        CLAY_HIP(hipMemcpyAsync(t->d, t->h, tab.size() * sizeof(uint8_t *), hipMemcpyHostToDevice, st));
        t->users = 1;
        *out = t.get();
        ds.captured.push_back(std::move(t));
        return Error{};
    }
    auto it = ds.tables.find(tab);
    if (it == ds.tables.end()) {
        if (ds.tables.size() >= kMaxPtrTables) {  // evict the least recently used idle table
            auto victim = ds.tables.end();
            for (auto j = ds.tables.begin(); j != ds.tables.end(); ++j)
                if (j->second.users == 0 && (victim == ds.tables.end() || j->second.last < victim->second.last))
                    victim = j;
            if (victim != ds.tables.end()) {
                free_table(victim->second);
                ds.tables.erase(victim);
            }
        }
        PtrTable t;
        Error e = upload_table(t, tab, st, false);
        if (e) {
            free_table(t);
            return e;
        }
        it = ds.tables.emplace(tab, t).first;
    } else if (it->second.up) {
        CLAY_HIP(hipStreamWaitEvent(st, it->second.up, 0));  // the upload may be on another stream
    }
    it->second.last = ++ds.tick;
    it->second.users++;
    *out = &it->second;
    return Error{};
}
// After the launches that read the table were enqueued on `st` (or failed to be):
// record the guard event and drop the caller's use.
static Error ptr_table_done(DevState &ds, PtrTable *t, hipStream_t st, bool launched) {
    std::lock_guard<std::mutex> lk(ds.mu);
    t->users--;
    if (t->pinned || !launched) return Error{};
    auto it = t->evs.find(st);
    if (it == t->evs.end()) {
        hipEvent_t ev;
        CLAY_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        it = t->evs.emplace(st, ev).first;
    }
    CLAY_HIP(hipEventRecord(it->second, st));
    return Error{};
}
struct PtrTableUse {
    DevState &ds;
    hipStream_t st;
    PtrTable *t = nullptr;
    bool launched = false;
    PtrTableUse(DevState &d, hipStream_t s) : ds(d), st(s) {}
    Error done() {
        PtrTable *x = t;
        t = nullptr;
        return x ? ptr_table_done(ds, x, st, launched) : Error{};
    }
    ~PtrTableUse() {
        if (t) (void)ptr_table_done(ds, t, st, true);  // error path: guard whatever was enqueued
    }
};

template <typename T>
static Error upload_vec(const std::vector<T> &v, const T **out) {
    void *p = nullptr;
    CLAY_HIP(hipMalloc(&p, std::max<size_t>(1, v.size()) * sizeof(T)));
    if (!v.empty()) CLAY_HIP(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    *out = static_cast<const T *>(p);
    return Error{};
}

// Device copy of a plan's groups (once per plan and device; plans are never freed).
// Waves per workgroup of the tile-fused executor: enough for the widest level's groups
// (4 / 8 / 16), or CLAY_TEXEC_WAVES.
static uint32_t texec_waves(const Plan &pl) {
    const int forced = tuning().texec_waves;
    if (forced) return uint32_t(forced);
    uint32_t mx = 0;
    for (size_t L = 0; L + 1 < pl.gstage_begin.size(); L++)
        mx = std::max(mx, pl.gstage_begin[L + 1] - pl.gstage_begin[L]);
    return mx <= 8 ? 4u : mx <= 16 ? 8u : 16u;
}

// A plan or table first needed inside a stream capture cannot be uploaded there (hipMalloc +
// a blocking copy would invalidate the capture): the call fails instead, and the caller runs one
// call of that shape (erasure pattern, lost node) outside the capture first.
static Error not_prepared(const char *what) {
    return make_error(CLAY_ERR_DEVICE, 0, 0, 0,
                      "%s not prepared before stream capture: run one call of this shape outside the capture "
                      "first (clay_reserve_workspace prepares the encode plan)", what);
}

static Error upload_groups(CodeState &cs, const Plan &pl, int dev, CodeState::DevGrouped *out,
                           hipStream_t st = nullptr) {
    std::lock_guard<std::mutex> lk(cs.mu);
    auto key = std::make_pair(&pl, dev);
    auto it = cs.gplan.find(key);
    if (it == cs.gplan.end()) {
        if (st && capturing(st)) return not_prepared("plan");
        CodeState::DevGrouped g{};
        Error e = upload_vec(pl.groups, &g.groups);
        if (!e) e = upload_vec(pl.gsrcs, &g.srcs);
        if (!e) e = upload_vec(pl.gdsts, &g.dsts);
        if (!e) e = upload_vec(pl.gcoef, &g.coef);
        if (e) return e;
        // U slots of the tile-fused executor: register-allocated by level.  A slot is live
        // from the level that writes it through the last level that reads it; an LDS slot
        // is reused only by a later level than every reader of its previous value (a level
        // runs on all waves at once, so same-level reuse would race).
        std::vector<DevSrc> ts(pl.gsrcs), td(pl.gdsts);
        const uint32_t ub = 2 * pl.tn;
        const size_t nst = pl.gstage_begin.size() - 1;
        std::map<uint32_t, size_t> last_read;
        for (size_t L = 0; L < nst; L++)
            for (uint32_t gi = pl.gstage_begin[L]; gi < pl.gstage_begin[L + 1]; gi++) {
                const DevGroup &dg = pl.groups[gi];
                for (uint32_t j = 0; j < dg.nsrc; j++)
                    if (pl.gsrcs[dg.src_begin + j].base == ub) last_read[pl.gsrcs[dg.src_begin + j].slot] = L;
            }
        std::map<uint32_t, uint32_t> phys;  // plan slot -> LDS slot
        std::vector<uint32_t> free_slots;
        std::vector<std::pair<size_t, uint32_t>> busy;  // (last read level, LDS slot)
        uint32_t nphys = 0;
        for (size_t L = 0; L < nst; L++) {
            for (size_t i = 0; i < busy.size();) {  // values no level >= L reads
                if (busy[i].first < L) {
                    free_slots.push_back(busy[i].second);
                    busy[i] = busy.back();
                    busy.pop_back();
                } else {
                    i++;
                }
            }
            for (uint32_t gi = pl.gstage_begin[L]; gi < pl.gstage_begin[L + 1]; gi++) {
                const DevGroup &dg = pl.groups[gi];
                for (uint32_t j = 0; j < dg.ndst; j++) {
                    const DevSrc &d = pl.gdsts[dg.dst_begin + j];
                    if (d.base != ub || phys.count(d.slot)) continue;
                    uint32_t p;
                    if (!free_slots.empty()) {
                        p = free_slots.back();
                        free_slots.pop_back();
                    } else {
                        p = nphys++;
                    }
                    phys[d.slot] = p;
                    auto lr = last_read.find(d.slot);
                    busy.emplace_back(lr == last_read.end() ? L : lr->second, p);
                }
            }
        }
        g.nu = nphys;
        for (auto *v : {&td, &ts})
            for (auto &x : *v)
                if (x.base == ub) {
                    auto it = phys.find(x.slot);
                    if (it == phys.end()) g.nu = UINT32_MAX;  // read before any write: never tile-run
                    else x.slot = it->second;
                }
        // term streams (k_texec): level L, wave w runs groups gstage_begin[L] + w + i * nwv
        const uint32_t nwv = texec_waves(pl);
        std::vector<uint4> terms;
        std::vector<uint32_t> wbeg;
        for (size_t L = 0; L < nst; L++)
            for (uint32_t w = 0; w < nwv; w++) {
                wbeg.push_back(uint32_t(terms.size()));
                for (uint32_t gi = pl.gstage_begin[L] + w; gi < pl.gstage_begin[L + 1]; gi += nwv) {
                    const DevGroup &dg = pl.groups[gi];
                    // a group without sources emits no term records, so k_texec would never
                    // write its (zero) destinations: such plans run on k_gexec only
                    if (dg.nsrc == 0 && dg.ndst > 0) g.nu = UINT32_MAX;
                    for (uint32_t j = 0; j < dg.nsrc; j++) {
                        const DevSrc &x = ts[dg.src_begin + j];
                        if (x.base > 255 || x.slot > 0xFFFFFFu || dg.dst_begin > 0xFFFFFFu || dg.ndst > 8)
                            g.nu = UINT32_MAX;  // not encodable: never tile-run
                        uint4 r;
                        r.x = x.base << 24 | (x.slot & 0xFFFFFFu);
                        r.y = r.w = 0;
                        r.z = dg.ndst << 24 | (j + 1 == dg.nsrc ? (1u << 31) | (dg.dst_begin & 0xFFFFFFu) : 0u);
                        for (uint32_t d = 0; d < dg.ndst && d < 8; d++) {
                            const uint32_t c = pl.gcoef[dg.coef_begin + d * dg.nsrc + j] & 0xFFu;
                            (d < 4 ? r.y : r.w) |= c << (8 * (d & 3));
                        }
                        terms.push_back(r);
                    }
                }
            }
        wbeg.push_back(uint32_t(terms.size()));
        g.nwv = nwv;
        e = upload_vec(ts, &g.tsrcs);
        if (!e) e = upload_vec(td, &g.tdsts);
        if (!e) e = upload_vec(terms, &g.terms);
        if (!e) e = upload_vec(wbeg, &g.wbeg);
        if (e) return e;
        it = cs.gplan.emplace(key, g).first;
    }
    *out = it->second;
    return Error{};
}

// Cached plan lookup / build (plans are immutable once built).
template <class Build>
static Error cached_plan(CodeState &cs, std::map<std::vector<uint8_t>, std::unique_ptr<Plan>> &m,
                         const std::vector<uint8_t> &key, Build &&build, const Plan **out) {
    std::lock_guard<std::mutex> lk(cs.mu);
    auto it = m.find(key);
    if (it == m.end()) {
        std::unique_ptr<Plan> p;
        Error e = build(p);
        if (e) return e;
        it = m.emplace(key, std::move(p)).first;
    }
    *out = it->second.get();
    return Error{};
}
static Error encode_plan(CodeState &cs, const Plan **out) {
    std::lock_guard<std::mutex> lk(cs.mu);
    if (!cs.enc) {
        Error e = plan_encode(cs.code, cs.rs, cs.enc);
        if (e) return e;
    }
    *out = cs.enc.get();
    return Error{};
}

template <int VW, int MAXD>
static void launch_gexec1(int mode, dim3 grid, dim3 block, hipStream_t stream, const ExecPtrs &ptrs,
                          const CodeState::DevGrouped &g, const uint32_t *tabs, uint32_t b, uint32_t tiles,
                          uint64_t sc, uint64_t r0, uint64_t r1, uint32_t n, uint32_t order, uint32_t bx,
                          uint8_t *const *ptab, uint32_t lps, uint32_t nstripes, const ExecStride &S,
                          uint32_t tpw) {
    // software-pipelined source loads (default; CLAY_GEXEC_PIPE=0 disables): repair (9,3,11)
    // 0.330 -> 0.323 ms, decode 4 erasures 0.863 -> 0.855 ms (profiles/r02/gexec_pipe.txt)
    const bool pipe = tuning().gexec_pipe;
    auto k = mode == kBatchTable ? k_gexec<VW, MAXD, kBatchTable>
           : mode == kBatchAffine ? k_gexec<VW, MAXD, kBatchAffine>
           : pipe ? k_gexec<VW, MAXD, kBatchNone, true> : k_gexec<VW, MAXD, kBatchNone>;
    k<<<grid, block, 0, stream>>>(ptrs, g.groups, g.srcs, g.dsts, g.coef, tabs, b, tiles, sc, r0, r1, n, order, bx,
                                  ptab, lps, nstripes, S, tpw);
}
template <int VW>
static void launch_gexec(uint32_t maxd, dim3 grid, hipStream_t stream, const ExecPtrs &ptrs,
                         const CodeState::DevGrouped &g, const uint32_t *tabs, uint32_t b, uint32_t tiles,
                         uint64_t sc, uint64_t r0, uint64_t r1, uint32_t n, int mode = kBatchNone,
                         uint8_t *const *ptab = nullptr, const ExecStride *stride = nullptr, uint32_t nstripes = 1,
                         uint32_t lps = kExecBlock, uint32_t tpw = 1) {
    dim3 block(kExecBlock);
    const uint32_t order = tuning().gexec_order;
    static const ExecStride zero{};
    const ExecStride &S = stride ? *stride : zero;
    const uint32_t nb = n * tiles, bx = (nb + 7) / 8;
    if (order == 2) grid = dim3(8 * bx);
    const uint32_t spb = kExecBlock / lps;
    grid.y = (nstripes + spb - 1) / spb;
    if (maxd <= 1) launch_gexec1<VW, 1>(mode, grid, block, stream, ptrs, g, tabs, b, tiles, sc, r0, r1, n, order, bx, ptab, lps, nstripes, S, tpw);
    else if (maxd <= 2) launch_gexec1<VW, 2>(mode, grid, block, stream, ptrs, g, tabs, b, tiles, sc, r0, r1, n, order, bx, ptab, lps, nstripes, S, tpw);
    else if (maxd <= 4) launch_gexec1<VW, 4>(mode, grid, block, stream, ptrs, g, tabs, b, tiles, sc, r0, r1, n, order, bx, ptab, lps, nstripes, S, tpw);
    else launch_gexec1<VW, 8>(mode, grid, block, stream, ptrs, g, tabs, b, tiles, sc, r0, r1, n, order, bx, ptab, lps, nstripes, S, tpw);
}

static int align_of(uintptr_t p) {
    for (int a = 16; a > 1; a >>= 1)
        if ((p % a) == 0) return a;
    return 1;
}

// Executor selection (clay_set_exec_mode): process-wide, read without locks.
// Modes only choose kernels: every mode returns the reference's bytes on any input (4, the
// retired single-launch decode, and 7, now the per-call clay_decode_device_codeword, are unused).
enum : int { kExecAuto = 0, kExecGrouped = 1, kExecTile = 2, kExecStream = 3, kExecStreamLocal = 5,
              kExecStreamFused2 = 6 };  // see clay_set_exec_mode
static std::atomic<int> g_exec_mode{kExecAuto};
static size_t tex_lds_budget() { return tuning().texec_lds; }
// Lane width of the tile-fused executor for a plan (0 = not eligible): the widest of
// 16 / 8 / 4 bytes whose tile of U slots (nu x 64 x VW) fits the LDS budget (default
// 80 KiB: two workgroups per CU); failing that, 4-byte lanes with up to 160 KiB (one
// workgroup per CU) when CLAY_TEXEC_BIG=1.
static int texec_vw(const Plan &pl, uint32_t nu, uint32_t maxd) {
    const size_t stages = pl.gstage_begin.size() - 1;
    if (stages == 0 || stages > size_t(kTexMaxStages) || maxd > 8 || nu == UINT32_MAX) return 0;
    for (int vw = 16; vw >= 4; vw >>= 1)
        if (uint64_t(nu) * 64 * vw + kTexTabBytes <= tex_lds_budget()) return vw;
    const bool big = tuning().texec_big;
    if (big && uint64_t(nu) * 64 * 4 + kTexTabBytes <= kTexLdsMax) return 4;
    return 0;
}
template <int VW, int MAXD, int NWV>
static Error launch_texec2(const ExecPtrs &ptrs, const CodeState::DevGrouped &g, const uint32_t *tabs,
                           uint32_t nstages, uint64_t sc, uint32_t ubase, hipStream_t stream, int dev) {
    const size_t lds = size_t(g.nu) * 64 * VW + kTexTabBytes;
    Error e = lds_attr_once(reinterpret_cast<const void *>(&k_texec<VW, MAXD, NWV>), int(kTexLdsMax), dev);
    if (e) return e;
    const uint64_t tiles = (sc + 64 * VW - 1) / (64 * VW);
    k_texec<VW, MAXD, NWV><<<dim3(uint32_t(tiles)), dim3(64 * NWV), lds, stream>>>(ptrs, g.terms, g.wbeg, tabs,
                                                                                  g.tdsts, nstages, sc, ubase, g.nu);
    CLAY_HIP(hipGetLastError());
    return Error{};
}
template <int VW, int MAXD>
static Error launch_texec1(const ExecPtrs &ptrs, const CodeState::DevGrouped &g, const uint32_t *tabs,
                           uint32_t nstages, uint64_t sc, uint32_t ubase, hipStream_t stream, int dev) {
    if (g.nwv == 4) return launch_texec2<VW, MAXD, 4>(ptrs, g, tabs, nstages, sc, ubase, stream, dev);
    if (g.nwv == 8) return launch_texec2<VW, MAXD, 8>(ptrs, g, tabs, nstages, sc, ubase, stream, dev);
    return launch_texec2<VW, MAXD, 16>(ptrs, g, tabs, nstages, sc, ubase, stream, dev);
}
template <int VW>
static Error launch_texec(uint32_t maxd, const ExecPtrs &ptrs, const CodeState::DevGrouped &g, const uint32_t *tabs,
                          uint32_t nstages, uint64_t sc, uint32_t ubase, hipStream_t stream, int dev) {
    if (maxd <= 1) return launch_texec1<VW, 1>(ptrs, g, tabs, nstages, sc, ubase, stream, dev);
    if (maxd <= 2) return launch_texec1<VW, 2>(ptrs, g, tabs, nstages, sc, ubase, stream, dev);
    if (maxd <= 4) return launch_texec1<VW, 4>(ptrs, g, tabs, nstages, sc, ubase, stream, dev);
    return launch_texec1<VW, 8>(ptrs, g, tabs, nstages, sc, ubase, stream, dev);
}

// Execute a plan: C/H/OUT pointer bindings given, U workspace bound here.  The
// tile-fused executor (one launch, U in LDS) where the plan's U slots fit, else one
// k_gexec launch per dependency level; 16 bytes per lane regardless of sc / pointer
// alignment.
static Error run_plan(CodeState &cs, const Plan &pl, int dev, DevState &ds, hipStream_t stream,
                      ExecPtrs ptrs, size_t sc, size_t chunk_for_ws) {
    CodeState::DevGrouped g{};
    Error e = upload_groups(cs, pl, dev, &g, stream);
    if (e) return e;
    const int xm = g_exec_mode.load(std::memory_order_relaxed);
    // auto: the tile executor only for small plans (at most kTexAutoGroups groups), where
    // the grouped executor's launches are latency-bound -- (4,2,5) decode 64 MiB: 0.043 ->
    // 0.038 ms.  On the big plans it measured slower than the grouped executor ((9,3,11)
    // repair 0.53 vs 0.43 ms, (10,4,13) 1-erasure decode 0.72 vs 0.41 ms),
    // so "tile" mode runs it wherever eligible but auto does not.
    const bool tex_ok = xm == kExecTile || (xm != kExecGrouped && pl.groups.size() <= kTexAutoGroups &&
                                             pl.gstage_begin.size() > 2);  // one level: nothing to fuse
    if (tex_ok && sc > 0 && sc / (64 * 4) < 0x7fffffffu) {
        uint32_t maxd = 1;
        for (uint32_t m : pl.gstage_maxd) maxd = std::max(maxd, m);
        const int vw = texec_vw(pl, g.nu, maxd);
        if (tuning().plan_debug) fprintf(stderr, "run_plan: %zu levels, %u LDS U slots, maxd %u -> tile executor vw %d\n",
                         pl.gstage_begin.size() - 1, g.nu, maxd, vw);
        if (vw) {
            const uint32_t nst = uint32_t(pl.gstage_begin.size() - 1), ub = 2 * pl.tn;
            t_last_exec = "tile";
            e = vw == 16 ? launch_texec<16>(maxd, ptrs, g, ds.d_tabs, nst, sc, ub, stream, dev)
              : vw == 8  ? launch_texec<8>(maxd, ptrs, g, ds.d_tabs, nst, sc, ub, stream, dev)
                         : launch_texec<4>(maxd, ptrs, g, ds.d_tabs, nst, sc, ub, stream, dev);
            if (!e) t_last_launches += 1;
            return e;
        }
    }
    LeaseGuard ws(ds, stream);
    if (pl.uses_u) {
        e = lease_acquire(ds, size_t(pl.tn) * chunk_for_ws, stream, &ws.l);
        if (e) return e;
        ptrs.p[2 * pl.tn] = ws.ptr();
    }
    size_t launches = 0;
    t_last_exec = "grouped";
    // Per-level block shape, from the level's block count at 4 KiB tiles (nwg = groups x
    // tiles): tiny levels (nwg < CLAY_GEXEC_SMALL, default 2048 -- e.g. the 13-group tail
    // level of a 4-erasure decode, latency-bound on ~1,300 blocks) run 1 KiB tiles (4-byte
    // lanes) for 4x the blocks; large levels (nwg >= CLAY_GEXEC_BIG, default 32768: many
    // small groups) give each block 2 consecutive tiles so a group's scalar work is
    // amortised.  (10,4,13) 4-erasure decode 1.045 -> 0.968 ms same box; 1 KiB tiles on
    // mid-size levels of wide groups cost 2x ((10,4,13) repair, 64 groups: 0.21 -> 0.40 ms),
    // hence the low threshold (profiles/r02/gexec_block_shape.txt).  CLAY_GEXEC_TPW fixes
    // the tiles per block for every level.
    const int tpw_env = tuning().gexec_tpw;
    const uint64_t small_wg = tuning().gexec_small, big_wg = tuning().gexec_big;
    const uint32_t tiles16 = uint32_t((sc / 16 + 1 + kExecBlock - 1) / kExecBlock);
    const uint32_t tiles4 = uint32_t((sc / 4 + 1 + kExecBlock - 1) / kExecBlock);
    for (size_t s = 0; s + 1 < pl.gstage_begin.size(); s++) {
        uint32_t b = pl.gstage_begin[s], end = pl.gstage_begin[s + 1];
        const uint32_t maxd = pl.gstage_maxd[s];
        const uint64_t nwg = uint64_t(end - b) * tiles16;
        const bool narrow = !tpw_env && nwg < small_wg;
        const uint32_t tpw = tpw_env ? uint32_t(tpw_env) : (nwg >= big_wg ? 2u : 1u);
        const uint32_t tiles = narrow ? tiles4 : (tiles16 + tpw - 1) / tpw;
        while (b < end) {
            uint32_t n = std::min<uint32_t>(end - b, uint32_t(0x7fffffffu / tiles));
            if (narrow)
                launch_gexec<4>(maxd, dim3(n * tiles), stream, ptrs, g, ds.d_tabs, b, tiles, sc, 0, sc, n, kBatchNone,
                                nullptr, nullptr, 1, kExecBlock, 1);
            else
                launch_gexec<16>(maxd, dim3(n * tiles), stream, ptrs, g, ds.d_tabs, b, tiles, sc, 0, sc, n,
                                 kBatchNone, nullptr, nullptr, 1, kExecBlock, tpw);
            CLAY_HIP(hipGetLastError());
            launches++;
            b += n;
        }
    }
    t_last_launches += launches;
    return Error{};
}

// ---------------------------------------------------------------------------
// Encode paths
// ---------------------------------------------------------------------------
static bool fused_shape_ok(const clay_code_t &c) {
    return c.q == c.m && c.k + c.nu == (c.t - 1) * c.q && c.q >= 2 && c.q <= 4 && c.original_count <= kFusedMaxK;
}

template <int Q, int PPT>
static Error launch_fused(const FusedArgs &a, const uint32_t *mtab, size_t lds, hipStream_t stream, int grid) {
    int dev = 0;
    CLAY_HIP(hipGetDevice(&dev));
    Error e = lds_attr_once(reinterpret_cast<const void *>(&k_fused_encode<Q, PPT>), int(kFusedLdsBudget), dev);
    if (e) return e;
    k_fused_encode<Q, PPT><<<dim3(grid), dim3(kFusedBlock), lds, stream>>>(a, mtab);
    CLAY_HIP(hipGetLastError());
    return Error{};
}

static Error encode_fused(CodeState &cs, DevState &ds, int dev, const uint8_t *const *data, uint8_t *const *par,
                          size_t n_stripes, size_t chunk, hipStream_t stream, bool *done) {
    *done = false;
    const clay_code_t &c = cs.code;
    if (!fused_shape_ok(c)) return Error{};
    const size_t alpha = c.sub_chunk_no, sc = chunk / alpha, K = c.original_count, Q = c.q;
    int ppt = 16;
    while (ppt >= 4 && (sc % ppt) != 0) ppt >>= 1;
    if (ppt < 4) return Error{};
    for (size_t s = 0; s < n_stripes; s++) {
        for (size_t i = 0; i < c.k; i++) ppt = std::min(ppt, align_of(reinterpret_cast<uintptr_t>(data[s * c.k + i])));
        for (size_t i = 0; i < c.m; i++) ppt = std::min(ppt, align_of(reinterpret_cast<uintptr_t>(par[s * c.m + i])));
    }
    if (ppt < 4) return Error{};
    size_t W = (kFusedLdsBudget / (Q * alpha)) / size_t(ppt) * size_t(ppt);
    W = std::min<size_t>(W, 2048);
    if (W < size_t(ppt)) return Error{};
    // device RS parity rows as perm tables [p][i][8]
    const uint32_t *mt = nullptr;
    {
        std::lock_guard<std::mutex> lk(cs.mu);
        auto it = cs.mtab.find(dev);
        if (it == cs.mtab.end()) {
            std::vector<uint32_t> t(Q * K * 8);
            for (size_t p = 0; p < Q; p++)
                for (size_t i = 0; i < K; i++) perm_table(cs.rs.gen[(K + p) * K + i], &t[(p * K + i) * 8]);
            uint32_t *d = nullptr;
            CLAY_HIP(hipMalloc(&d, t.size() * 4));
            CLAY_HIP(hipMemcpy(d, t.data(), t.size() * 4, hipMemcpyHostToDevice));
            it = cs.mtab.emplace(dev, d).first;
        }
        mt = it->second;
    }
    const hipDeviceProp_t &prop = dev_props(dev).raw;
    const size_t lds = Q * alpha * W;
    const int per_cu = std::max<int>(1, int((160 * 1024) / lds));
    for (size_t s = 0; s < n_stripes; s++) {
        FusedArgs a{};
        for (size_t i = 0; i < K; i++) a.data[i] = i < c.k ? data[s * c.k + i] : nullptr;
        for (size_t x = 0; x < Q; x++) a.par[x] = par[s * c.m + x];
        a.sc = sc;
        a.alpha = uint32_t(alpha);
        a.t = uint32_t(c.t);
        a.K = uint32_t(K);
        a.W = uint32_t(W);
        a.ntiles = uint32_t((sc + W - 1) / W);
        a.tiles_per_xcd = (a.ntiles + 7) / 8;
        const uint32_t max_slots = uint32_t(std::max(1, prop.multiProcessorCount / 8) * per_cu);
        a.nslots = std::min(max_slots, a.tiles_per_xcd);
        uint32_t w[8];
        perm_table(gamma_det_inv(), w);
        for (int i = 0; i < 5; i++) a.dinv[i] = w[i];
        const int grid = int(a.nslots * 8);
        Error e;
        switch (Q * 100 + ppt) {
        case 216: e = launch_fused<2, 16>(a, mt, lds, stream, grid); break;
        case 208: e = launch_fused<2, 8>(a, mt, lds, stream, grid); break;
        case 204: e = launch_fused<2, 4>(a, mt, lds, stream, grid); break;
        case 316: e = launch_fused<3, 16>(a, mt, lds, stream, grid); break;
        case 308: e = launch_fused<3, 8>(a, mt, lds, stream, grid); break;
        case 304: e = launch_fused<3, 4>(a, mt, lds, stream, grid); break;
        case 416: e = launch_fused<4, 16>(a, mt, lds, stream, grid); break;
        case 408: e = launch_fused<4, 8>(a, mt, lds, stream, grid); break;
        case 404: e = launch_fused<4, 4>(a, mt, lds, stream, grid); break;
        default: return Error{};
        }
        if (e) return e;
        t_last_launches++;
    }
    char buf[64];
    std::snprintf(buf, sizeof(buf), "fused-q%zuw%zup%d", Q, W, ppt);
    t_last_path = buf;
    *done = true;
    return Error{};
}

// ---------------------------------------------------------------------------
// Bit-sliced fused encode (bitslice.hpp): compile-time instantiations per code.
// ---------------------------------------------------------------------------
template <int KD, int M, int PG>
static Error launch_bs(CodeState &cs, const hipDeviceProp_t &prop, const uint8_t *const *data, uint8_t *const *par,
                       size_t n_stripes, size_t sc, hipStream_t stream, bool *done) {
    using Kn = bs::BsKernel<KD, M, PG>;
    using S = typename Kn::S;
    const clay_code_t &c = cs.code;
    if (int(c.k) != KD || int(c.m) != M || int(c.d) != KD + M - 1) return Error{};
    // the compile-time generator must equal the run-time one (same construction)
    for (int p = 0; p < M; p++)
        for (int i = 0; i < S::K; i++)
            if (S::RS.g[p][i] != cs.rs.gen[(S::K + p) * S::K + i])
                return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "bit-sliced RS table mismatch");
    const int per_cu = std::max(1, int((160 * 1024) / (Kn::LDS_WORDS * 4)));
    for (size_t s = 0; s < n_stripes; s++) {
        bs::BsArgs a{};
        for (int i = 0; i < S::K; i++) a.data[i] = i < KD ? data[s * KD + i] : nullptr;
        for (int x = 0; x < M; x++) a.par[x] = par[s * M + x];
        a.sc = sc;
        a.ntiles = uint32_t((sc + Kn::W - 1) / Kn::W);
        a.tiles_per_xcd = (a.ntiles + 7) / 8;
        const uint32_t max_slots = uint32_t(std::max(1, prop.multiProcessorCount / 8) * per_cu);
        a.nslots = std::min(max_slots, a.tiles_per_xcd);
        bool bt = sc % 8 != 0;  // byte tails: unaligned rows or chunks
        for (int i = 0; i < KD; i++) bt |= (reinterpret_cast<uintptr_t>(a.data[i]) & 7u) != 0;
        for (int x = 0; x < M; x++) bt |= (reinterpret_cast<uintptr_t>(a.par[x]) & 7u) != 0;
        if (bt) bs::k_bs_encode<KD, M, PG, true><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), 0, stream>>>(a);
        else bs::k_bs_encode<KD, M, PG><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), 0, stream>>>(a);
        CLAY_HIP(hipGetLastError());
        t_last_launches++;
    }
    char buf[64];
    std::snprintf(buf, sizeof(buf), "bitsliced-k%dm%d-w%d", KD, M, Kn::W);
    t_last_path = buf;
    *done = true;
    return Error{};
}

// The streaming encode (stream_encode.hpp) for q = 4, t = 4 codes with k = 9 or 10.
template <int KD, int LOADERS>
static Error launch_stream(CodeState &cs, const DevProps &prop, const uint8_t *const *data, uint8_t *const *par,
                           size_t n_stripes, size_t sc, hipStream_t stream, bool *done) {
    using Kn = bs::StreamEnc<KD, LOADERS>;
    using S = typename Kn::S;
    const clay_code_t &c = cs.code;
    if (int(c.k) != KD || c.m != 4 || c.d != c.k + 3) return Error{};
    // per-lane DMA offsets are 32-bit chunk offsets; a clamped 16-byte piece needs sc >= 16
    if (double(S::ALPHA) * double(sc) >= 4294967296.0 || sc < 16) return Error{};
    for (int p = 0; p < 4; p++)
        for (int i = 0; i < S::K; i++)
            if (S::RS.g[p][i] != cs.rs.gen[(S::K + p) * S::K + i])
                return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "bit-sliced RS table mismatch");
    Error ae = lds_attr_once(reinterpret_cast<const void *>(&bs::k_stream_encode<KD, LOADERS, 0, bs::kStreamEncMap>),
                             Kn::LDS_BYTES, prop.dev);
    if (ae) return ae;
    // XCD region: sc / 8 rounded up to 32 bytes; one workgroup per CU
    const uint32_t region = uint32_t(((sc + 7) / 8 + 31) / 32 * 32);
    const uint32_t per_xcd = uint32_t(std::max(1, prop.cus / 8));
    const uint32_t nslots = std::min(per_xcd, std::max(1u, (region + 255u) / 256u));
    for (size_t s = 0; s < n_stripes; s++) {
        bs::BsArgs a{};
        for (int i = 0; i < S::K; i++) a.data[i] = i < KD ? data[s * KD + i] : nullptr;
        for (int x = 0; x < 4; x++) a.par[x] = par[s * 4 + x];
        a.sc = sc;
        a.tiles_per_xcd = region;
        a.nslots = nslots;
        a.ntiles = 0;
        bs::k_stream_encode<KD, LOADERS, 0, bs::kStreamEncMap><<<dim3(nslots * 8), dim3(Kn::BLOCK), Kn::LDS_BYTES, stream>>>(a);
        CLAY_HIP(hipGetLastError());
        t_last_launches++;
    }
    char buf[64];
    std::snprintf(buf, sizeof(buf), "stream-k%dm4-w256-l%d", KD, LOADERS);
    t_last_path = buf;
    *done = true;
    return Error{};
}

hipError_t launch_stream_encode3_kernel(int loaders, const bs::Enc3Args &a, hipStream_t stream, int dev);  // encode_stream3.hip

// The streaming encode for (9,3,11) (stream_encode3.hpp): any sub-chunk size >= 16 and any row
// alignment (LDS-DMA reads, unaligned 16-byte stores, byte-exact partial tiles).
static Error launch_stream3(CodeState &cs, const DevProps &prop, const uint8_t *const *data, uint8_t *const *par,
                            size_t n_stripes, size_t sc, hipStream_t stream, int loaders, bool *done) {
    using S = bs::Shape<9, 3>;
    const clay_code_t &c = cs.code;
    if (c.k != 9 || c.m != 3 || c.d != 11 || sc < 16 || double(S::ALPHA) * double(sc) >= 4294967296.0) return Error{};
    for (int p = 0; p < 3; p++)
        for (int i = 0; i < S::K; i++)
            if (S::RS.g[p][i] != cs.rs.gen[(S::K + p) * S::K + i])
                return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "bit-sliced RS table mismatch");
    const uint32_t W = 512;
    bs::Enc3Args a{};
    a.sc = sc;
    a.region = uint32_t(((sc + 7) / 8 + 31) / 32 * 32);
    a.ns = std::min(uint32_t(std::max(1, prop.cus / 8)), std::max(1u, (a.region + W - 1) / W));
    for (size_t s = 0; s < n_stripes; s++) {
        for (int i = 0; i < 9; i++) a.data[i] = data[s * 9 + i];
        for (int x = 0; x < 3; x++) a.par[x] = par[s * 3 + x];
        CLAY_HIP(launch_stream_encode3_kernel(loaders, a, stream, prop.dev));
        t_last_launches++;
    }
    char buf[64];
    std::snprintf(buf, sizeof(buf), "stream3-k9m3-w512-l%d", loaders == 7 ? 7 : 2);
    t_last_path = buf;
    *done = true;
    return Error{};
}

// (4,2,5) on the line-local bit-sliced encode (bitslice_line.hpp: no LDS, one launch per stripe)
static Error launch_bs_encode1(CodeState &cs, const DevProps &prop, const uint8_t *const *data, uint8_t *const *par,
                               size_t n_stripes, size_t sc, hipStream_t stream, bool *done) {
    *done = false;
    const clay_code_t &c = cs.code;
    const int W = bs_decode1_tile(int(c.k), int(c.m));  // the line kernels' tile (same lane map)
    if (!W || c.d != c.k + c.m - 1 || c.nu != 0 || sc == 0) return Error{};
    using S = bs::Shape<4, 2>;
    for (int p = 0; p < 2; p++)
        for (int i = 0; i < S::K; i++)
            if (S::RS.g[p][i] != cs.rs.gen[(S::K + p) * S::K + i])
                return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "bit-sliced RS table mismatch");
    for (size_t s = 0; s < n_stripes; s++) {
        bs::Enc1Args a{};
        bool bt = sc % 8 != 0;
        for (size_t i = 0; i < c.k; i++) {
            a.data[i] = data[s * c.k + i];
            bt |= (reinterpret_cast<uintptr_t>(a.data[i]) & 7u) != 0;
        }
        for (size_t x = 0; x < c.m; x++) {
            a.par[x] = par[s * c.m + x];
            bt |= (reinterpret_cast<uintptr_t>(a.par[x]) & 7u) != 0;
        }
        a.sc = sc;
        a.ntiles = uint32_t((sc + size_t(W) - 1) / size_t(W));
        a.tiles_per_xcd = (a.ntiles + 7) / 8;
        a.nslots = std::min(a.tiles_per_xcd, uint32_t(std::max(1, prop.cus / 8) * 8));
        CLAY_HIP(launch_bs_encode1_kernel(int(c.k), int(c.m), bt, a, stream));
        t_last_launches++;
    }
    char buf[64];
    std::snprintf(buf, sizeof(buf), "bitsliced-line-k%zum%zu-w%d", c.k, c.m, W);
    t_last_path = buf;
    *done = true;
    return Error{};
}

static Error encode_bitsliced(CodeState &cs, int dev, const uint8_t *const *data, uint8_t *const *par,
                              size_t n_stripes, size_t chunk, hipStream_t stream, int mode, int tile, bool *done) {
    *done = false;
    const clay_code_t &c = cs.code;
    const size_t sc = chunk / c.sub_chunk_no;
    if (c.d != c.k + c.m - 1) return Error{};
    // the LDS-DMA kernel (stream) needs 8-byte rows: sc % 8 == 0, 8-byte aligned chunks;
    // the v1 kernel takes any sub-chunk size and alignment (byte-granular partial words)
    bool rows8 = sc % 8 == 0;
    for (size_t s = 0; s < n_stripes && rows8; s++) {
        for (size_t i = 0; i < c.k; i++)
            if (reinterpret_cast<uintptr_t>(data[s * c.k + i]) % 8) rows8 = false;
        for (size_t i = 0; i < c.m; i++)
            if (reinterpret_cast<uintptr_t>(par[s * c.m + i]) % 8) rows8 = false;
    }
    const DevProps &prop = dev_props(dev);
    Error e;
    const int key = int(c.k * 100 + c.m);
    // streaming kernel (q = 4, t = 4, k 9 / 10): auto's first choice; tile = loader waves
    // (9,3) streaming kernel: any row alignment; tile = loader waves (2, or 7)
    if (key == 903 && (mode == kModeStream || mode == kModeAuto)) {
        e = launch_stream3(cs, prop, data, par, n_stripes, sc, stream, tile == 7 ? 7 : 2, done);
        if (e || *done || mode == kModeStream) return e;
    }
    if (rows8 && (mode == kModeStream || mode == kModeAuto)) {
        if (key == 1004 || key == 904) {
            const int l = tile ? tile : 4;
            if (key == 1004)
                e = l == 1 ? launch_stream<10, 1>(cs, prop, data, par, n_stripes, sc, stream, done)
                  : l == 4 ? launch_stream<10, 4>(cs, prop, data, par, n_stripes, sc, stream, done)
                           : launch_stream<10, 2>(cs, prop, data, par, n_stripes, sc, stream, done);
            else
                e = launch_stream<9, 4>(cs, prop, data, par, n_stripes, sc, stream, done);
        }
        if (e || *done || mode == kModeStream) return e;
    }
    // (4,2,5): the line-local kernel (auto and "stream"; "bitsliced" keeps the v1 kernel for A/B)
    if (key == 402 && (mode == kModeStream || mode == kModeAuto)) {
        e = launch_bs_encode1(cs, prop, data, par, n_stripes, sc, stream, done);
        if (e || *done) return e;
    }
    if (mode == kModeStream) return e;
    // v1 (register loads, PG x 32 positions per lane): every q = m code it is instantiated for
    switch (key) {
    case 1004:
        if (tile == 1) e = launch_bs<10, 4, 1>(cs, prop.raw, data, par, n_stripes, sc, stream, done);
        else if (tile == 4) e = launch_bs<10, 4, 4>(cs, prop.raw, data, par, n_stripes, sc, stream, done);
        else e = launch_bs<10, 4, 2>(cs, prop.raw, data, par, n_stripes, sc, stream, done);
        break;
    case 402: e = launch_bs<4, 2, 64>(cs, prop.raw, data, par, n_stripes, sc, stream, done); break;
    case 804: e = launch_bs<8, 4, 8>(cs, prop.raw, data, par, n_stripes, sc, stream, done); break;
    case 903: e = launch_bs<9, 3, 6>(cs, prop.raw, data, par, n_stripes, sc, stream, done); break;
    case 603: e = launch_bs<6, 3, 16>(cs, prop.raw, data, par, n_stripes, sc, stream, done); break;
    default: break;
    }
    return e;
}

static Error encode_staged(CodeState &cs, DevState &ds, int dev, const uint8_t *const *data, uint8_t *const *par,
                           size_t n_stripes, size_t chunk, hipStream_t stream) {
    const clay_code_t &c = cs.code;
    if (c.q * c.t > size_t(kMaxTn))
        return make_error(CLAY_ERR_DEVICE, c.q * c.t, 0, 0, "device engine supports at most %d internal nodes", kMaxTn);
    const Plan *pl = nullptr;
    Error pe = encode_plan(cs, &pl);
    if (pe) return pe;
    const size_t sc = chunk / c.sub_chunk_no;
    for (size_t s = 0; s < n_stripes; s++) {
        ExecPtrs P{};
        for (size_t i = 0; i < c.k; i++) P.p[i] = const_cast<uint8_t *>(data[s * c.k + i]);
        for (size_t i = 0; i < c.m; i++) P.p[c.k + c.nu + i] = par[s * c.m + i];
        Error e = run_plan(cs, *pl, dev, ds, stream, P, sc, chunk);
        if (e) return e;
    }
    t_last_path = "staged";
    return Error{};
}

// Batched small stripes: every level of the staged encode plan
// runs for ALL stripes in one k_gexec launch (grid.y = stripe), pointers from a
// cached device table of kMaxBases entries per stripe; U workspace per stripe.
// Sub-chunks under 4 KiB put several stripes in one block (lps lanes of 16 B per
// stripe); at most 65,535 blocks of stripes per launch group (grid.y limit).
// Stripes laid out at fixed strides (clay_encode_device_strided): node i of stripe s at
// data + s * dstripe + i * dnode, parity j at par + s * pstripe + j * pnode.
struct Strided {
    const uint8_t *data;
    int64_t dnode, dstripe;
    uint8_t *par;
    int64_t pnode, pstripe;
};

static Error encode_staged_batch(CodeState &cs, DevState &ds, int dev, const uint8_t *const *data,
                                 uint8_t *const *par, size_t n_stripes, size_t chunk, hipStream_t stream,
                                 const Strided *sd) {
    const clay_code_t &c = cs.code;
    const uint32_t tn = uint32_t(c.q * c.t);
    const Plan *plp = nullptr;
    Error e = encode_plan(cs, &plp);
    if (e) return e;
    const Plan &pl = *plp;
    CodeState::DevGrouped g{};
    e = upload_groups(cs, pl, dev, &g, stream);
    if (e) return e;
    const uint64_t sc = chunk / c.sub_chunk_no;
    const uint32_t lanes = uint32_t(sc / 16 + 1);  // 16-byte lanes incl. the byte tail
    const uint32_t lps = std::min<uint32_t>(kExecBlock, lanes);
    const uint32_t tiles = (lanes + lps - 1) / lps;
    const size_t max_group = size_t(65535) * (kExecBlock / lps);
    size_t launches = 0;
    for (size_t s0 = 0; s0 < n_stripes; s0 += max_group) {
        const size_t ns = std::min(max_group, n_stripes - s0);
        LeaseGuard ws(ds, stream);
        if (pl.uses_u) {
            e = lease_acquire(ds, ns * tn * chunk, stream, &ws.l);
            if (e) return e;
        }
        // operand of base b for stripe s: affine in s (rows of one buffer, the common
        // case) -> kernarg base + stride, no table; otherwise a cached device table
        ExecPtrs P{};
        ExecStride S{};
        bool affine = true;
        auto affine_of = [&](size_t base, auto ptr_of) {
            if (sd) {  // strided layout: affine by construction
                P.p[base] = ptr_of(0);
                S.s[base] = int64_t(ptr_of(1) - ptr_of(0));
                return;
            }
            uint8_t *p0 = ptr_of(0);
            const int64_t st = ns > 1 ? int64_t(ptr_of(1) - p0) : 0;
            for (size_t s = 2; s < ns && affine; s++) affine = ptr_of(s) == p0 + int64_t(s) * st;
            P.p[base] = p0;
            S.s[base] = st;
        };
        for (size_t i = 0; i < c.k && affine; i++)
            affine_of(i, [&](size_t s) {
                return sd ? const_cast<uint8_t *>(sd->data) + int64_t(s0 + s) * sd->dstripe + int64_t(i) * sd->dnode
                          : const_cast<uint8_t *>(data[(s0 + s) * c.k + i]);
            });
        for (size_t i = 0; i < c.m && affine; i++)
            affine_of(c.k + c.nu + i, [&](size_t s) {
                return sd ? sd->par + int64_t(s0 + s) * sd->pstripe + int64_t(i) * sd->pnode : par[(s0 + s) * c.m + i];
            });
        if (ws.l) {
            P.p[2 * tn] = ws.ptr();
            S.s[2 * tn] = int64_t(tn * chunk);
        }
        PtrTableUse ptu(ds, stream);
        PtrTable *pt = nullptr;
        if (!affine) {
            std::vector<uint8_t *> tab(ns * kMaxBases, nullptr);
            for (size_t s = 0; s < ns; s++) {
                uint8_t **t = &tab[s * kMaxBases];
                for (size_t i = 0; i < c.k; i++) t[i] = const_cast<uint8_t *>(data[(s0 + s) * c.k + i]);
                for (size_t i = 0; i < c.m; i++) t[c.k + c.nu + i] = par[(s0 + s) * c.m + i];
                if (ws.l) t[2 * tn] = ws.ptr() + s * tn * chunk;
            }
            e = ptr_table(ds, tab, stream, &pt);
            if (e) return e;
            ptu.t = pt;
        }
        for (size_t st = 0; st + 1 < pl.gstage_begin.size(); st++) {
            uint32_t b = pl.gstage_begin[st], end = pl.gstage_begin[st + 1];
            while (b < end) {
                uint32_t n = std::min<uint32_t>(end - b, uint32_t(0x7fffffffu / tiles));
                launch_gexec<16>(pl.gstage_maxd[st], dim3(n * tiles), stream, P, g, ds.d_tabs, b, tiles, sc, 0, sc, n,
                                 affine ? kBatchAffine : kBatchTable,
                                 pt ? static_cast<uint8_t *const *>(pt->d) : nullptr, &S, uint32_t(ns), lps);
                CLAY_HIP(hipGetLastError());
                launches++;
                b += n;
            }
        }
        ptu.launched = true;
        e = ptu.done();
        if (e) return e;
    }
    t_last_launches += launches;
    t_last_path = "staged-batch";
    return Error{};
}

// Batched bit-sliced encode (k_bs_encode over nstripes x ntiles flattened tiles, one
// launch): stripe s = stripe 0's node pointers + s * a uniform data / parity stride.
template <int KD, int M, int PG>
static Error launch_bs_batch(CodeState &cs, int dev, const uint8_t *const *data0, uint8_t *const *par0,
                             int64_t sdata, int64_t spar, size_t ns, size_t sc, hipStream_t stream, bool *done) {
    using Kn = bs::BsKernel<KD, M, PG>;
    using S = typename Kn::S;
    for (int p = 0; p < M; p++)
        for (int i = 0; i < S::K; i++)
            if (S::RS.g[p][i] != cs.rs.gen[(S::K + p) * S::K + i])
                return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "bit-sliced RS table mismatch");
    const uint64_t ntiles = (sc + Kn::W - 1) / Kn::W;
    // sub-chunks well under a tile would leave most lanes idle: the staged batch packs them
    if (sc < uint64_t(Kn::W) / 2 || ntiles * ns >= 0xFFFFFFFFull) return Error{};
    if constexpr (KD == 4 && M == 2) {
        // (4,2,5): the line-local kernel (bitslice_line.hpp), same 2048-position tiles
        bs::Enc1Args e{};
        for (int i = 0; i < KD; i++) e.data[i] = data0[i];
        for (int x = 0; x < M; x++) e.par[x] = par0[x];
        e.sc = sc;
        e.ntiles = uint32_t(ntiles);
        e.nstripes = uint32_t(ns);
        e.sdata = sdata;
        e.spar = spar;
        e.tiles_per_xcd = uint32_t((ntiles * ns + 7) / 8);
        e.nslots = std::min(e.tiles_per_xcd, uint32_t(std::max(1, dev_props(dev).cus / 8) * 8));
        bool bt1 = sc % 8 != 0 || (sdata & 7) != 0 || (spar & 7) != 0;
        for (int i = 0; i < KD; i++) bt1 |= (reinterpret_cast<uintptr_t>(e.data[i]) & 7u) != 0;
        for (int x = 0; x < M; x++) bt1 |= (reinterpret_cast<uintptr_t>(e.par[x]) & 7u) != 0;
        CLAY_HIP(launch_bs_encode1_kernel(KD, M, bt1, e, stream));
        t_last_launches++;
        char buf1[64];
        std::snprintf(buf1, sizeof(buf1), "bitsliced-batch-line-k%dm%d-w%d", KD, M, Kn::W);
        t_last_path = buf1;
        *done = true;
        return Error{};
    }
    const int per_cu = std::max(1, int((160 * 1024) / (Kn::LDS_WORDS * 4)));
    bs::BsArgs a{};
    for (int i = 0; i < S::K; i++) a.data[i] = i < KD ? data0[i] : nullptr;
    for (int x = 0; x < M; x++) a.par[x] = par0[x];
    a.sc = sc;
    a.ntiles = uint32_t(ntiles);
    a.nstripes = uint32_t(ns);
    a.sdata = sdata;
    a.spar = spar;
    a.tiles_per_xcd = uint32_t((ntiles * ns + 7) / 8);
    const uint32_t max_slots = uint32_t(std::max(1, dev_props(dev).raw.multiProcessorCount / 8) * per_cu);
    a.nslots = std::min(max_slots, a.tiles_per_xcd);
    bool bt = sc % 8 != 0 || (sdata & 7) != 0 || (spar & 7) != 0;  // byte tails
    for (int i = 0; i < KD; i++) bt |= (reinterpret_cast<uintptr_t>(a.data[i]) & 7u) != 0;
    for (int x = 0; x < M; x++) bt |= (reinterpret_cast<uintptr_t>(a.par[x]) & 7u) != 0;
    if (bt) bs::k_bs_encode<KD, M, PG, true><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), 0, stream>>>(a);
    else bs::k_bs_encode<KD, M, PG><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), 0, stream>>>(a);
    CLAY_HIP(hipGetLastError());
    t_last_launches++;
    char buf[64];
    std::snprintf(buf, sizeof(buf), "bitsliced-batch-k%dm%d-w%d", KD, M, Kn::W);
    t_last_path = buf;
    *done = true;
    return Error{};
}
static Error encode_bs_batch(CodeState &cs, int dev, const uint8_t *const *data, uint8_t *const *par, size_t ns,
                             size_t chunk, hipStream_t stream, const Strided *sd, bool *done) {
    *done = false;
    const clay_code_t &c = cs.code;
    const size_t sc = chunk / c.sub_chunk_no;
    const int key = int(c.k * 100 + c.m);
    if (c.d != c.k + c.m - 1 || !(key == 402 || key == 804 || key == 903 || key == 603)) return Error{};
    // stripe-0 pointers and one stride for all data nodes, one for all parity nodes
    std::vector<const uint8_t *> d0(c.k);
    std::vector<uint8_t *> p0(c.m);
    int64_t sdata = 0, spar = 0;
    auto dptr = [&](size_t s, size_t i) -> const uint8_t * {
        return sd ? sd->data + int64_t(s) * sd->dstripe + int64_t(i) * sd->dnode : data[s * c.k + i];
    };
    auto pptr = [&](size_t s, size_t i) -> uint8_t * {
        return sd ? sd->par + int64_t(s) * sd->pstripe + int64_t(i) * sd->pnode : par[s * c.m + i];
    };
    sdata = int64_t(dptr(1, 0) - dptr(0, 0));
    spar = int64_t(pptr(1, 0) - pptr(0, 0));
    for (size_t i = 0; i < c.k; i++) d0[i] = dptr(0, i);
    for (size_t i = 0; i < c.m; i++) p0[i] = pptr(0, i);
    if (!sd) {
        for (size_t s = 0; s < ns; s++) {
            for (size_t i = 0; i < c.k; i++)
                if (dptr(s, i) != d0[i] + int64_t(s) * sdata) return Error{};
            for (size_t i = 0; i < c.m; i++)
                if (pptr(s, i) != p0[i] + int64_t(s) * spar) return Error{};
        }
    }
    switch (key) {
    case 402: return launch_bs_batch<4, 2, 64>(cs, dev, d0.data(), p0.data(), sdata, spar, ns, sc, stream, done);
    case 804: return launch_bs_batch<8, 4, 8>(cs, dev, d0.data(), p0.data(), sdata, spar, ns, sc, stream, done);
    case 903: return launch_bs_batch<9, 3, 6>(cs, dev, d0.data(), p0.data(), sdata, spar, ns, sc, stream, done);
    default: return launch_bs_batch<6, 3, 16>(cs, dev, d0.data(), p0.data(), sdata, spar, ns, sc, stream, done);
    }
}

static Error encode_device_impl(const clay_code_t *code, const uint8_t *const *data, uint8_t *const *par,
                                size_t n_stripes, size_t chunk, int dev, void *stream, const Strided *sd = nullptr) {
    Error e = check_code(code);
    if (e) return e;
    if (sd ? (!sd->data || !sd->par) : (!data || !par))
        return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null chunk array");
    if (chunk == 0 || chunk % code->sub_chunk_no != 0)
        return make_error(CLAY_ERR_INVALID_CHUNK_SIZE, code->sub_chunk_no, chunk, 0,
                          "Invalid chunk size: expected divisible by %zu, got %zu", code->sub_chunk_no, chunk);
    if (!sd) {
        for (size_t i = 0; i < n_stripes * code->k; i++)
            if (!data[i]) return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null data chunk");
        for (size_t i = 0; i < n_stripes * code->m; i++)
            if (!par[i]) return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null parity chunk");
    }
    if (n_stripes == 0) return Error{};
    t_last_launches = 0;
    DevState *ds;
    e = dev_state(dev, &ds);
    if (e) return e;
    DeviceGuard g(dev);
    CodeState &cs = *code_state(*code);
    if (cs.rs.init_err)
        return make_error(CLAY_ERR_RECONSTRUCTION_FAILED, 0, 0, 0, "RS reconstruction failed: RS init failed: %s",
                          rs_error_name(cs.rs.init_err));
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int mode = g_encode_mode.load(std::memory_order_relaxed), tile = g_encode_tile.load(std::memory_order_relaxed);
    // many small stripes: one launch for the whole batch instead of one per stripe
    // (launch-bound below ~4 MiB of data per stripe) -- the bit-sliced kernel where the
    // code has one and the stripes sit at uniform strides, else one launch per plan level
    if (mode == kModeAuto && n_stripes >= 4 && code->k * chunk <= (size_t(4) << 20) &&
        code->q * code->t <= size_t(kMaxTn)) {
        bool done = false;
        e = encode_bs_batch(cs, dev, data, par, n_stripes, chunk, st, sd, &done);
        if (e || done) return e;
        return encode_staged_batch(cs, *ds, dev, data, par, n_stripes, chunk, st, sd);
    }
    std::vector<const uint8_t *> dv;
    std::vector<uint8_t *> pv;
    if (sd) {  // per-stripe kernels below take pointer arrays
        for (size_t s = 0; s < n_stripes; s++) {
            for (size_t i = 0; i < code->k; i++) dv.push_back(sd->data + int64_t(s) * sd->dstripe + int64_t(i) * sd->dnode);
            for (size_t i = 0; i < code->m; i++) pv.push_back(sd->par + int64_t(s) * sd->pstripe + int64_t(i) * sd->pnode);
        }
        data = dv.data();
        par = pv.data();
    }
    if (mode == kModeAuto || mode >= kModeBs) {
        bool done = false;
        e = encode_bitsliced(cs, dev, data, par, n_stripes, chunk, st, mode, tile, &done);
        if (e || done) return e;
        if (mode >= kModeBs)
            return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "bit-sliced encode kernel does not support this code/alignment");
    }
    if (mode == kModeAuto || mode == kModeFused) {
        bool done = false;
        e = encode_fused(cs, *ds, dev, data, par, n_stripes, chunk, st, &done);
        if (e || done) return e;
        if (mode == kModeFused)
            return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "fused encode kernel does not support this code/alignment");
    }
    return encode_staged(cs, *ds, dev, data, par, n_stripes, chunk, st);
}

// ---------------------------------------------------------------------------
// Decode / repair on device
// ---------------------------------------------------------------------------
// The streaming decodes (stream_decode.hpp phase A + stream_local.hpp / stream_fused2.hpp) for
// q = 4, t = 4 codes with k = 9 / 10.  `cin` / `cout`: internal node pointers (inputs of present
// nodes, outputs of erased nodes, nullptr if not wanted).
// Shared by the streaming decodes: pattern checks, RS rows used, H_K^-1, the v_perm tables of
// its rows and of A_i = H_K^-1 gamma H_i, the node loads of a tile.  *ok = false: not eligible
// (per_sec_max: the most erasures one y-section may hold).
template <int KD>
static Error dec_setup(CodeState &cs, const uint8_t *const *cin, uint8_t *const *cout, const std::vector<uint8_t> &erased,
                       size_t sc, int per_sec_max, bs::DecArgs &a, std::vector<uint32_t> &tabs, bool *ok,
                       bool any_sc = false) {
    *ok = false;
    const clay_code_t &c = cs.code;
    using S = bs::Shape<KD, 4>;
    if (int(c.k) != KD || c.m != 4 || c.q != 4 || c.t != 4 || c.q * c.t != 16) return Error{};
    // any_sc (k_stream_local256: LDS-DMA and 16-byte stores at any byte alignment, partial pieces
    // patched / stored byte by byte): any sub-chunk >= 512 and any chunk alignment; the other
    // streaming decodes need 8-byte rows
    if ((!any_sc && sc % 8) || sc < 512 || double(S::ALPHA) * double(sc) >= 4294967296.0) return Error{};
    const GF &gf = GF::get();
    std::vector<int> E;
    int per_sec[4] = {0, 0, 0, 0};
    for (int i = 0; i < 16; i++)
        if (erased[i]) {
            E.push_back(i);
            per_sec[i / 4]++;
        }
    if (E.empty() || E.size() > 4) return Error{};
    for (int y = 0; y < 4; y++)
        if (per_sec[y] > per_sec_max) return Error{};
    for (int i = 0; i < 16; i++) {
        if (any_sc) continue;
        if (cin[i] && reinterpret_cast<uintptr_t>(cin[i]) % 8) return Error{};
        if (cout[i] && reinterpret_cast<uintptr_t>(cout[i]) % 8) return Error{};
    }
    for (int p = 0; p < 4; p++)
        for (int i = 0; i < S::K; i++)
            if (S::RS.g[p][i] != cs.rs.gen[(S::K + p) * S::K + i])
                return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "bit-sliced RS table mismatch");
    a = bs::DecArgs{};
    a.g2 = -1;
    // RS rows used: the first 12 present shards (reconstruct, decode.rs:374); K = the rest
    uint32_t used = 0;
    int nused = 0;
    std::vector<int> Kset;
    for (int i = 0; i < 16; i++) {
        if (!erased[i] && nused < S::K) {
            used |= 1u << i;
            nused++;
        } else {
            Kset.push_back(i);
        }
    }
    if (nused != S::K || Kset.size() != 4) return Error{};
    auto Hc = [&](int pchk, int i) -> uint8_t {
        return i < S::K ? cs.rs.gen[(S::K + pchk) * S::K + i] : uint8_t(i - S::K == pchk ? 1 : 0);
    };
    std::vector<uint8_t> hk(16), hinv;
    for (int pchk = 0; pchk < 4; pchk++)
        for (int j = 0; j < 4; j++) hk[pchk * 4 + j] = Hc(pchk, Kset[j]);
    if (!gf_invert(hk, 4, hinv)) return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "singular RS check submatrix");
    a.ne = uint32_t(E.size());
    tabs.assign(bs::kDecTabWords, 0);
    for (int i = 0; i < 16; i++) a.rix[i] = -1;
    for (size_t r = 0; r < E.size(); r++) {
        const int e = E[r];
        a.rix[e] = int(r);
        a.emask[e / 4] |= 1u << (e % 4);
        a.out[r] = cout[e];
        const int row = int(std::find(Kset.begin(), Kset.end(), e) - Kset.begin());
        for (int j = 0; j < 4; j++) perm_table(hinv[row * 4 + j], &tabs[(r * 4 + j) * 8]);
        for (int i = 0; i < 16; i++) {  // A_(y,x)[e_r] = (H_K^-1 gamma H_i)[row of e_r], i = 4y + x
            uint8_t v = 0;
            for (int j = 0; j < 4; j++) v ^= gf.mul(hinv[row * 4 + j], gf.mul(kGamma, Hc(j, i)));
            perm_table(v, &tabs[(16 + i * 4 + r) * 8]);
        }
    }
    a.used = used;
    const uint32_t R = tuning().decode_ring;  // 10 unless a measurement sets CLAY_DECODE_RING
    uint32_t n[4] = {0, 0, 0, 0}, nt = 0;
    for (int y = 0; y < 4; y++) {
        a.sec_off[y] = nt;
        for (int x = 0; x < 4; x++) {
            const int i = 4 * y + x;
            a.node[i] = cin[i];
            if (cin[i]) {
                a.alive |= 1u << i;
                a.load_node[nt++] = uint32_t(i);
                n[y]++;
            }
        }
    }
    a.sec_off[4] = nt;
    a.nt = nt;
    // k_stream_fused2's compile-time phase-A copies: section y with at most one erased node x,
    // every other node used and every node alive but that one and the shortened ones (i in [KD, 12))
    for (int y = 0; y < 4; y++) {
        uint32_t shortn = 0;
        for (int x = 0; x < 4; x++)
            if (4 * y + x >= KD && 4 * y + x < S::K) shortn |= 1u << x;
        const uint32_t em = a.emask[y], un = (used >> (4 * y)) & 15u, al = (a.alive >> (4 * y)) & 15u;
        const bool ok1 = __builtin_popcount(em) <= 1 && un == (~em & 15u) && al == (~em & ~shortn & 15u);
        a.scase[y] = ok1 ? (em ? __builtin_ctz(em) : 4) : -1;
        // k_stream_local256 (one erased row): no erasure, every node alive and only node 0 / nodes
        // 0-1 used (the ignored nodes of one erasure: the last present ones); the fused decode
        // takes the run-time copy for these
        if (!ok1 && em == 0 && al == (~shortn & 15u) && (un == 1u || un == 3u)) a.scase[y] = un == 1u ? 5 : 6;
    }
    if (nt == 0) return Error{};
    // the local kernel streams through R - 1 buffers (the last holds tables): a step's
    // loads are issued during the step before it, across tiles too (section 3 -> section 0)
    for (int y = 0; y < 4; y++)
        if (n[y] > R - 1 || n[y] + n[(y + 1) % 4] > R - 1) return Error{};
    if (R < 5) return Error{};  // S/C region (4 buffers) + the phase-B table buffer
    a.ring = R;
    a.sc = sc;
    a.region = uint32_t(((sc + 7) / 8 + 63) / 64 * 64);
    *ok = true;
    return Error{};
}

// the pattern's tables: uploaded once per (table contents, device), cached with the code
static Error dec_tables(CodeState &cs, const DevProps &prop, const std::vector<uint32_t> &tabs, hipStream_t stream,
                        const uint32_t **out) {
    std::lock_guard<std::mutex> lk(cs.mu);
    auto key = std::make_pair(std::vector<uint32_t>(tabs), prop.dev);
    auto it = cs.dtabs.find(key);
    if (it == cs.dtabs.end()) {
        if (capturing(stream)) return not_prepared("streaming-decode pattern table");
        const uint32_t *d = nullptr;
        Error ue = upload_vec(tabs, &d);
        if (ue) return ue;
        it = cs.dtabs.emplace(key, d).first;
    }
    *out = it->second;
    return Error{};
}

hipError_t launch_stream_local_kernel(int kd, int g, const bs::DecArgs &a, hipStream_t stream, int dev);  // decode_stream.hip
hipError_t launch_stream_local256_kernel(int kd, int g, const bs::DecArgs &a, hipStream_t stream, int dev);  // decode_local256.hip
hipError_t launch_stream_local256_any_kernel(int kd, int g, const bs::DecArgs &a, hipStream_t stream,
                                             int dev);  // decode_local256_any.hip

// Local decode (stream_local.hpp): erasures in one y-section G (any number) plus at most one
// erasure in one other section g2 -- every iscore dependency inside a wave, one launch, no
// workspace.  G = the section with the most erasures; section g2's digit goes to bits 0-1 of
// the lane column.
template <int KD>
static Error launch_stream_local(CodeState &cs, const DevProps &prop, const uint8_t *const *cin, uint8_t *const *cout,
                                 const std::vector<uint8_t> &erased, size_t sc, hipStream_t stream, bool *done) {
    *done = false;
    int per_sec[4] = {0, 0, 0, 0};
    for (int i = 0; i < 16 && i < int(erased.size()); i++) per_sec[i / 4] += erased[i] ? 1 : 0;
    int G = 0, nsec = 0;
    for (int y = 0; y < 4; y++) {
        if (per_sec[y] > per_sec[G]) G = y;
        nsec += per_sec[y] ? 1 : 0;
    }
    if (nsec == 0 || nsec > 2) return Error{};
    int g2 = -1;
    for (int y = 0; y < 4; y++)
        if (y != G && per_sec[y]) {
            if (per_sec[y] > 1) return Error{};  // two sections with several erasures: rounds needed
            g2 = y;
        }
    // one erasure in section G plus at most one in g2, or two in G and none elsewhere: the
    // 256-byte-run kernel (stream_local256.hpp), which also takes sub-chunks that are not a
    // multiple of 8
    const bool w256 = (per_sec[G] == 1 || (per_sec[G] == 2 && g2 < 0)) && !tuning().local_w64;
    bs::DecArgs a;
    std::vector<uint32_t> tabs;
    bool ok = false;
    Error e = dec_setup<KD>(cs, cin, cout, erased, sc, 4, a, tabs, &ok, w256);
    if (e || !ok) return e;
    // column digits: section g2 (if any) at bits 0-1, the others above in section order
    {
        uint32_t sh = 4;
        for (int y = 0; y < 4; y++)
            if (y != G) a.csh[y] = y == g2 ? 0u : (sh -= 2) + 2;
    }
    a.g2 = g2;
    if (g2 >= 0) a.x2 = uint32_t(__builtin_ctz(a.emask[g2]));
    perm_table(gamma_det_inv(), &tabs[bs::kDecDetInv * 8]);  // (1 + gamma^2)^-1, transforms.rs:108-125
    const uint32_t per_xcd = uint32_t(std::max(1, prop.cus / 8));
    // the 256-byte-run kernel: XCD regions of whole 32-byte units and 256-byte tiles as the encode's
    if (w256) {
        a.region = uint32_t(((sc + 7) / 8 + 31) / 32 * 32);
        a.nslots = std::min(per_xcd, std::max(1u, (a.region + 255u) / 256u));
    } else {
        a.nslots = std::min(per_xcd, std::max(1u, a.region / 64u));
    }
    e = dec_tables(cs, prop, tabs, stream, &a.tabs);
    if (e) return e;
    if (w256) {
        // rows of 8-byte multiples at 8-byte-aligned chunks: the 8-byte kernel; else the ANY one
        bool any = sc % 8 != 0;
        for (int i = 0; i < 16; i++) {
            any = any || (cin[i] && reinterpret_cast<uintptr_t>(cin[i]) % 8);
            any = any || (cout[i] && reinterpret_cast<uintptr_t>(cout[i]) % 8);
        }
        if (any) CLAY_HIP(launch_stream_local256_any_kernel(KD, G, a, stream, prop.dev));
        else CLAY_HIP(launch_stream_local256_kernel(KD, G, a, stream, prop.dev));
        t_last_exec = "stream-local256";
    } else {
        CLAY_HIP(launch_stream_local_kernel(KD, G, a, stream, prop.dev));
        t_last_exec = "stream-local";
    }
    t_last_launches += 1;
    *done = true;
    return Error{};
}

hipError_t launch_stream_fused2_kernel(int kd, const bs::DecArgs &a, hipStream_t stream, int dev,
                                       bool two);  // decode_stream.hip

// Rounds of k_stream_fused2 (stream_fused2.hpp): per section Y with an erasure and iscore level L,
// the targets are the layers z with z_Y in E_Y and exactly L - 1 other sections y with z_y in E_y,
// P(Y, L) = ceil(targets x 8 / 64) passes of 64 lanes x (8-byte piece).  The four loader waves share
// them: each section with an erasure gets at least one wave, the spare waves go where they cut
// the sum over levels of the busiest wave's passes most, and a section's nw waves take every
// nw-th pass.  f2_plan packs, per loader wave li, byte li of a.lwave: bits 0-1 its section, 2-3 its
// part, 4-5 nw - 1, bit 6 set (no section: 0); false when a wave would hold more than the kernel's
// kF2Iters (TWO) / kF2Iters1 passes of some level.
static uint32_t f2_targets(const uint32_t (&emask)[4], int Y, int L) {
    uint32_t n = 0;
    for (uint32_t z = 0; z < 256; z++) {
        int red = 0;
        bool ty = false;
        for (int y = 0; y < 4; y++) {
            const uint32_t d = (z >> (2 * (3 - y))) & 3u;
            const bool in = (emask[y] >> d) & 1u;
            red += in ? 1 : 0;
            if (y == Y) ty = in;
        }
        n += (ty && red == L) ? 1u : 0u;
    }
    return n;
}
static bool f2_plan(const uint32_t (&emask)[4], bool two, uint32_t *lwave) {
    uint32_t P[4][4] = {}, nw[4] = {};
    int nact = 0;
    for (int Y = 0; Y < 4; Y++) {
        if (!emask[Y]) continue;
        nact++;
        nw[Y] = 1;
        for (int L = 1; L <= 4; L++) P[Y][L - 1] = (f2_targets(emask, Y, L) * 8u + 63u) / 64u;
    }
    const int *cap = two ? bs::kF2Iters : bs::kF2Iters1;
    // the spare waves: the split (every active section >= 1 wave, 4 in all) with the smallest sum
    // over levels of the busiest wave's passes (each level's round is one step) among those within
    // the kernel's item registers, first in lexicographic order of (nw[0], .., nw[3]) among equals
    if (nact > 0 && nact < 4) {
        uint32_t best[4] = {0, 0, 0, 0}, bcost = ~0u;
        for (uint32_t n0 = 0; n0 <= 4; n0++)
            for (uint32_t n1 = 0; n1 <= 4; n1++)
                for (uint32_t n2 = 0; n2 <= 4; n2++)
                    for (uint32_t n3 = 0; n3 <= 4; n3++) {
                        const uint32_t n[4] = {n0, n1, n2, n3};
                        if (n0 + n1 + n2 + n3 != 4) continue;
                        bool ok = true;
                        for (int Y = 0; Y < 4; Y++) ok = ok && ((n[Y] > 0) == (nw[Y] > 0));
                        if (!ok) continue;
                        uint32_t cost = 0;
                        for (int L = 0; L < 4; L++) {
                            uint32_t mx = 0;
                            for (int Y = 0; Y < 4; Y++)
                                if (n[Y]) mx = std::max(mx, (P[Y][L] + n[Y] - 1u) / n[Y]);
                            if (mx > uint32_t(cap[L])) ok = false;  // over the kernel's item registers
                            cost += mx;
                        }
                        if (!ok) continue;
                        if (cost < bcost) {
                            bcost = cost;
                            for (int Y = 0; Y < 4; Y++) best[Y] = n[Y];
                        }
                    }
        if (bcost == ~0u) return false;  // no split within the item registers
        for (int Y = 0; Y < 4; Y++) nw[Y] = best[Y];
    }
    uint32_t pack = 0;
    int li = 0;
    for (int Y = 0; Y < 4; Y++) {
        for (uint32_t part = 0; part < nw[Y]; part++, li++)
            pack |= (uint32_t(Y) | part << 2 | (nw[Y] - 1u) << 4 | 64u) << (8 * li);
        for (int L = 0; L < 4 && nw[Y]; L++)
            if ((P[Y][L] + nw[Y] - 1u) / nw[Y] > uint32_t(cap[L])) return false;
        if (two && P[Y][3]) return false;  // the TWO kernel inverts the pairs during the level-4 round's slot
    }
    *lwave = pack;
    return true;
}

// Fused decode v2 (stream_fused2.hpp): erasures in at least two y-sections with at most two per
// section (round 6: two in a section -- both-erased PFT pairs inverted after the rounds), one launch,
// rounds of tile k-1 on the loader waves while tile k streams.  Ring of 10 - ne node buffers + the
// S/C region.
template <int KD>
static Error launch_stream_fused2(CodeState &cs, const DevProps &prop, const uint8_t *const *cin, uint8_t *const *cout,
                                  const std::vector<uint8_t> &erased, size_t sc, hipStream_t stream, bool *done) {
    *done = false;
    bs::DecArgs a;
    std::vector<uint32_t> tabs;
    bool ok = false;
    Error e = dec_setup<KD>(cs, cin, cout, erased, sc, 2, a, tabs, &ok);
    if (e || !ok) return e;
    if (a.ne < 2) return Error{};
    bool two = false;
    for (int y = 0; y < 4; y++) two = two || __builtin_popcount(a.emask[y]) > 1;
    if (!f2_plan(a.emask, two, &a.lwave)) return Error{};  // more round targets than the kernel's item registers
    // both-erased pairs: per erased row, the other erased row of its section
    a.npair = 0;
    for (int r = 0; r < 4; r++) a.pinfo[r] = 0;
    for (int y = 0; y < 4; y++) {
        if (__builtin_popcount(a.emask[y]) != 2) continue;
        const uint32_t x1 = uint32_t(__builtin_ctz(a.emask[y])), x2 = 31u - uint32_t(__builtin_clz(a.emask[y]));
        const int r1 = a.rix[4 * y + int(x1)], r2 = a.rix[4 * y + int(x2)];
        a.pinfo[r1] = 1u | uint32_t(r2) << 1 | uint32_t(y) << 3 | x1 << 5 | x2 << 7;
        a.pinfo[r2] = 1u | uint32_t(r1) << 1 | uint32_t(y) << 3 | x2 << 5 | x1 << 7;
        a.npair += 2;
    }
    if (a.npair) perm_table(gamma_det_inv(), &tabs[bs::kDecDetInv * 8]);  // (1 + gamma^2)^-1
    const uint32_t RB = 10 - a.ne;  // the S/C region takes ne of the 10 node buffers of LDS
    // the loads of a step are issued during the step before it when the ring holds both; else
    // (round 6: two neighbouring sections with 7-8 alive nodes and RB = 6) the step is split: the
    // rest of its loads after its barrier, behind a second one.  Section 0 of tile k + 1 needs no
    // split: every ring buffer is free at B_r(k), before its barrier.
    a.split = 0;
    for (int y = 0; y < 4; y++) {
        const uint32_t ny = a.sec_off[y + 1] - a.sec_off[y];
        if (ny > RB) return Error{};
        if (y > 0 && (a.sec_off[y] - a.sec_off[y - 1]) + ny > RB) a.split |= 1u << y;
    }
    a.ring = RB;
    const uint32_t per_xcd = uint32_t(std::max(1, prop.cus / 8));
    a.nslots = std::min(per_xcd, std::max(1u, a.region / 64u));
    e = dec_tables(cs, prop, tabs, stream, &a.tabs);
    if (e) return e;
    if (!two) a.split = 0;  // (no pattern with one erasure per section overflows the ring)
    CLAY_HIP(launch_stream_fused2_kernel(KD, a, stream, prop.dev, two));
    t_last_launches += 1;
    t_last_exec = "stream-fused2";
    *done = true;
    return Error{};
}

// repair_stream.hip: bit-sliced repair kernel (repair_kernel.hpp); 1 launched, 0 no
// instantiation for (k, m), < 0 HIP error
int launch_bs_repair_kernel(int k, int m, int y0, const bs::RepArgs &a, hipStream_t stream, int dev, int cus,
                            int stream_mode, int *launches);

// One erased node with every other node present, in a q = m code (d = n - 1), through
// clay_decode_device_codeword: when the chunks are one codeword, the erased chunk is the one a repair from all
// n - 1 helpers rebuilds (the codeword through the k data chunks is unique: decode.rs:31-161 and
// repair.rs:140-421 return the same bytes; on inputs that are NOT a codeword the two differ, so
// auto keeps the decode), and the repair reads only
// the beta = alpha / q layers of its repair plane from each helper (repair.rs:61-126) instead of
// every layer: (10,4,13) 1 GiB {0}: 0.16 ms vs 0.39 on the local decode.  Runs the streaming
// bit-sliced repair kernel on the whole chunks (full = 1) when it has an instantiation for the
// code and every CU gets a tile; *done = false otherwise.
static Error decode_by_repair(const clay_code_t &c, const uint8_t *const *chunks, size_t lost, uint8_t *out,
                              size_t chunk, int dev, hipStream_t stream, bool *done) {
    *done = false;
    const size_t tn = c.q * c.t;
    if (c.q != c.m || tn > 16 || !out) return Error{};
    bs::RepArgs ra{};
    const size_t lost_int = internal_of(c, lost);
    for (size_t i = 0; i < c.n; i++) {
        if (i == lost) continue;
        if (!chunks[i]) return Error{};
        ra.h[internal_of(c, i)] = chunks[i];
    }
    ra.out = out;
    ra.sc = chunk / c.sub_chunk_no;
    ra.x0 = uint32_t(lost_int % c.q);
    ra.full = 1u;
    int nl = 0;
    const int r = launch_bs_repair_kernel(int(c.k), int(c.m), int(lost_int / c.q), ra, stream, dev, dev_props(dev).cus, 3,
                                          &nl);
    if (r < 0) return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "HIP error: %s", hipGetErrorString(hipError_t(-r)));
    if (r > 0) {
        t_last_launches += nl;
        t_last_exec = "bs-repair-stream";
        *done = true;
    }
    return Error{};
}

// Single erasure of a small q = m code without shortened nodes ((4,2,5), BASELINE config 2) with
// every other chunk present: k_bs_decode1 (bitslice_line.hpp), the erased node's whole
// decode_layered as compile-time XOR networks, one launch.
static Error launch_bs_decode1(CodeState &cs, const DevProps &prop, const uint8_t *const *chunks, size_t e,
                               uint8_t *out, size_t chunk, hipStream_t stream, bool *done) {
    *done = false;
    const clay_code_t &c = cs.code;
    const int W = bs_decode1_tile(int(c.k), int(c.m));
    if (!W || c.d != c.k + c.m - 1 || c.nu != 0 || !out || c.q * c.t > 8) return Error{};
    const size_t sc = chunk / c.sub_chunk_no;
    if (sc == 0 || chunk % c.sub_chunk_no) return Error{};
    using S = bs::Shape<4, 2>;  // the only instantiation (bs_decode1_tile)
    for (int p = 0; p < 2; p++)
        for (int i = 0; i < S::K; i++)
            if (S::RS.g[p][i] != cs.rs.gen[(S::K + p) * S::K + i])
                return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "bit-sliced RS table mismatch");
    bs::Dec1Args a{};
    bool bt = sc % 8 != 0 || (reinterpret_cast<uintptr_t>(out) & 7u) != 0;
    for (size_t i = 0; i < c.n; i++) {
        if (i == e) continue;
        if (!chunks[i]) return Error{};
        a.node[internal_of(c, i)] = chunks[i];
        bt |= (reinterpret_cast<uintptr_t>(chunks[i]) & 7u) != 0;
    }
    a.out = out;
    a.sc = sc;
    a.ntiles = uint32_t((sc + size_t(W) - 1) / size_t(W));
    a.tiles_per_xcd = (a.ntiles + 7) / 8;
    a.nslots = std::min(a.tiles_per_xcd, uint32_t(std::max(1, prop.cus / 8) * 8));
    CLAY_HIP(launch_bs_decode1_kernel(int(c.k), int(c.m), int(internal_of(c, e)), bt, a, stream));
    t_last_launches += 1;
    t_last_exec = "bs-decode1";
    *done = true;
    return Error{};
}

static Error decode_device_impl(const clay_code_t *code, const uint8_t *const *chunks, const size_t *er, size_t ner,
                                uint8_t *const *outs, size_t chunk, int dev, void *stream, bool codeword = false) {
    Error e = check_code(code);
    if (e) return e;
    const clay_code_t &c = *code;
    if (!chunks || !outs) return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null chunk array");
    std::vector<size_t> ids, lens;
    for (size_t i = 0; i < c.n; i++)
        if (chunks[i]) {
            ids.push_back(i);
            lens.push_back(chunk);
        }
    if (ids.empty() && ner == 0) return Error{};
    size_t cs_sz = 0;
    std::vector<uint8_t> erased;
    e = validate_decode(c, AvailView{ids.data(), lens.data(), ids.size()}, er, ner, &cs_sz, erased);
    if (e) return e;
    const size_t tn = c.q * c.t;
    std::vector<uint8_t> want(tn, 0);
    for (size_t i = 0; i < ner; i++) {
        size_t in = internal_of(c, er[i]);
        if (er[i] < c.k && !outs[er[i]])
            return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: no output buffer for erased node %zu",
                              er[i]);
        want[in] = outs[er[i]] ? 1 : 0;
    }
    t_last_launches = 0;
    DevState *ds;
    e = dev_state(dev, &ds);
    if (e) return e;
    DeviceGuard g(dev);
    CodeState &cs = *code_state(c);
    if (tn > size_t(kMaxTn))
        return make_error(CLAY_ERR_DEVICE, tn, 0, 0, "device engine supports at most %d internal nodes", kMaxTn);
    std::vector<uint8_t> key(erased);
    key.insert(key.end(), want.begin(), want.end());
    const Plan *plan = nullptr;
    e = cached_plan(cs, cs.dec, key, [&](std::unique_ptr<Plan> &p) { return plan_decode(c, cs.rs, erased, want, p); },
                    &plan);
    if (e) return e;
    ExecPtrs P{};
    for (size_t i = 0; i < c.n; i++) {
        size_t in = internal_of(c, i);
        P.p[in] = chunks[i] ? const_cast<uint8_t *>(chunks[i]) : (want[in] ? outs[i] : nullptr);
    }
    const int xmode = g_exec_mode.load(std::memory_order_relaxed);
    size_t n_erased = 0;
    for (size_t in = 0; in < tn; in++) n_erased += erased[in] && !(in >= c.k && in < c.k + c.nu) ? 1 : 0;
    // clay_decode_device_codeword (the caller vouches, for this call only, that the chunks are one
    // codeword): a single erasure is rebuilt by the repair kernel under the exec modes that pick
    // the bit-sliced repair kernels (auto, "stream": as repair_device_impl); every other decode,
    // and every decode under "grouped" / "tile" (A/B runs), runs as clay_decode_device does
    if (codeword && (xmode == kExecAuto || xmode == kExecStream) && n_erased == 1 && ner == 1 && ids.size() + 1 == c.n) {
        bool done = false;
        e = decode_by_repair(c, chunks, er[0], outs[er[0]], chunk, dev, static_cast<hipStream_t>(stream), &done);
        if (e || done) return e;
    }
    // one erasure of (4,2,5) with every other chunk present: the bit-sliced single-erasure decode
    if ((xmode == kExecAuto || xmode == kExecStream) && n_erased == 1 && ner == 1 && ids.size() + 1 == c.n) {
        bool done = false;
        e = launch_bs_decode1(cs, dev_props(dev), chunks, er[0], outs[er[0]], chunk, static_cast<hipStream_t>(stream),
                              &done);
        if (e || done) return e;
    }
    // streaming decodes of q = 4, t = 4 codes (sc % 8 == 0, sc >= 512):
    //  * the local decode (erasures in one section plus at most one other, stream_local.hpp):
    //    auto, "stream" and "stream-local";
    //  * the fused decode v2 (2-4 erasures in distinct sections, stream_fused2.hpp): auto from 3
    //    erasures, "stream" and "stream-fused2" from 2 ((10,4,13) 1 GiB: {0,4,8,12} 0.52 ms vs 0.92
    //    on the grouped executor, {0,4,8} 0.48 vs 0.79; {0,4} 0.458 vs 0.452 on the local decode;
    //    profiles/r04/fused2/)
    const bool stream_all = xmode == kExecStream;
    const bool try_local = xmode == kExecAuto || stream_all || xmode == kExecStreamLocal;
    const bool try_f2 = xmode == kExecStreamFused2 || stream_all || (xmode == kExecAuto && n_erased >= 3);
    // (2,1) sections (two erasures in one section, one in another): the fused decode v2 first --
    // 0.48-0.53 ms vs 0.50-0.54 on the 64-byte local decode (profiles/r06/decode/two_small_*)
    bool f2_first = false;
    if (try_f2 && try_local && n_erased == 3 && tn == 16) {
        int per[4] = {0, 0, 0, 0};
        for (size_t in = 0; in < tn; in++) per[in / 4] += erased[in] ? 1 : 0;
        int nsec = 0, mx = 0;
        for (int y = 0; y < 4; y++) {
            nsec += per[y] ? 1 : 0;
            mx = std::max(mx, per[y]);
        }
        f2_first = nsec == 2 && mx == 2;
    }
    if ((try_local || try_f2) && tn == 16) {
        const uint8_t *cin[16] = {};
        uint8_t *cout[16] = {};
        for (size_t i = 0; i < c.n; i++) {
            const size_t in = internal_of(c, i);
            if (erased[in]) cout[in] = want[in] ? outs[i] : nullptr;
            else cin[in] = chunks[i];
        }
        bool done = false;
        const DevProps &prop = dev_props(dev);
        const size_t sc = chunk / c.sub_chunk_no;
        hipStream_t st = static_cast<hipStream_t>(stream);
        if (f2_first) {
            if (c.k == 10) e = launch_stream_fused2<10>(cs, prop, cin, cout, erased, sc, st, &done);
            else if (c.k == 9) e = launch_stream_fused2<9>(cs, prop, cin, cout, erased, sc, st, &done);
            if (e || done) return e;
        }
        if (try_local) {
            if (c.k == 10) e = launch_stream_local<10>(cs, prop, cin, cout, erased, sc, st, &done);
            else if (c.k == 9) e = launch_stream_local<9>(cs, prop, cin, cout, erased, sc, st, &done);
            if (e || done) return e;
        }
        if (try_f2 && !f2_first) {
            if (c.k == 10) e = launch_stream_fused2<10>(cs, prop, cin, cout, erased, sc, st, &done);
            else if (c.k == 9) e = launch_stream_fused2<9>(cs, prop, cin, cout, erased, sc, st, &done);
            if (e || done) return e;
        }
    }
    return run_plan(cs, *plan, dev, *ds, static_cast<hipStream_t>(stream), P, chunk / c.sub_chunk_no, chunk);
}

static Error repair_device_impl(const clay_code_t *code, size_t lost, const size_t *ids, const uint8_t *const *bufs,
                                const size_t *lens, size_t nh, size_t chunk, uint8_t *out, int dev, void *stream,
                                bool full = false) {
    Error e = check_code(code);
    if (e) return e;
    const clay_code_t &c = *code;
    std::vector<uint8_t> hin;
    std::vector<long> slot_of;
    std::vector<size_t> sub;
    e = validate_repair(c, lost, ids, lens, nh, chunk, hin, slot_of, sub);
    if (e) return e;
    if (!out) return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null output");
    t_last_launches = 0;
    DevState *ds;
    e = dev_state(dev, &ds);
    if (e) return e;
    DeviceGuard g(dev);
    const size_t tn = c.q * c.t;
    if (tn > size_t(kMaxTn))
        return make_error(CLAY_ERR_DEVICE, tn, 0, 0, "device engine supports at most %d internal nodes", kMaxTn);
    CodeState &cs = *code_state(c);
    // bit-sliced single-launch repair (repair_kernel.hpp): q = m codes with every other node a
    // helper (no aloof nodes); auto and "stream" exec modes ((9,3,11) 256 MiB chunks: 0.345-0.357
    // vs 0.39-0.41 ms grouped on the same boxes, profiles/r03/)
    const int xm = g_exec_mode.load(std::memory_order_relaxed);
    const bool xauto = xm == kExecAuto;
    if ((xauto || xm == kExecStream) && c.q == c.m && tn <= 16 && nh + 1 == c.n) {
        bs::RepArgs ra{};
        const size_t lost_int = internal_of(c, lost);
        bool ok = true;
        for (size_t in = 0; in < tn; in++) {
            if (in == lost_int || (in >= c.k && in < c.k + c.nu)) continue;
            if (slot_of[in] < 0) ok = false;
            else ra.h[in] = bufs[slot_of[in]];
        }
        if (ok) {
            ra.out = out;
            ra.sc = chunk / c.sub_chunk_no;
            ra.x0 = uint32_t(lost_int % c.q);
            ra.full = full ? 1u : 0u;
            // streaming variant (LDS-DMA, one workgroup per CU): auto when every CU gets a tile,
            // always in exec mode "stream"
            int nl = 0;
            const int r = launch_bs_repair_kernel(int(c.k), int(c.m), int(lost_int / c.q), ra, static_cast<hipStream_t>(stream),
                                                  dev, dev_props(dev).cus, xauto ? 1 : 2, &nl);
            if (r < 0) return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "HIP error: %s", hipGetErrorString(hipError_t(-r)));
            if (r > 0) {
                t_last_launches += nl;
                t_last_exec = r == 2 ? "bs-repair-stream" : "bs-repair";
                return Error{};
            }
        }
    }
    std::vector<uint8_t> key(hin);
    key.push_back(uint8_t(lost & 0xFF));
    key.push_back(uint8_t(lost >> 8));
    key.push_back(uint8_t(full));
    const Plan *plan = nullptr;
    e = cached_plan(cs, cs.rep, key,
                    [&](std::unique_ptr<Plan> &p) { return plan_repair(c, cs.rs, lost, hin, slot_of, sub, p, full); },
                    &plan);
    if (e) return e;
    ExecPtrs P{};
    for (size_t in = 0; in < tn; in++)
        if (slot_of[in] >= 0) P.p[tn + in] = const_cast<uint8_t *>(bufs[slot_of[in]]);
    P.p[2 * tn + 1] = out;
    return run_plan(cs, *plan, dev, *ds, static_cast<hipStream_t>(stream), P, chunk / c.sub_chunk_no, chunk);
}

// ---------------------------------------------------------------------------
// Host-side copies the API's semantics require (the returned data chunks, encode.rs:44-55 /
// decode.rs:155-158), split over a few threads and run beside the GPU pipeline.
struct CopyJob {
    uint8_t *dst;
    const uint8_t *src;  // nullptr: zero fill
    size_t n;
};
class HostCopier {
  public:
    explicit HostCopier(std::vector<CopyJob> jobs) : jobs_(std::move(jobs)) {
        size_t total = 0;
        for (auto &j : jobs_) total += j.n;
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        const size_t nt = std::min<size_t>({8, hw, std::max<size_t>(1, total >> 24)});  // >= 16 MiB per thread
        const size_t per = (total + nt - 1) / std::max<size_t>(1, nt);
        for (size_t t = 0; t < nt && total; t++)
            th_.emplace_back([this, t, per] { run(t * per, (t + 1) * per); });
    }
    ~HostCopier() { join(); }
    void join() {
        for (auto &t : th_)
            if (t.joinable()) t.join();
    }

  private:
    void run(size_t lo, size_t hi) {  // byte range [lo, hi) of the concatenated jobs
        size_t at = 0;
        for (auto &j : jobs_) {
            const size_t a = std::max(lo, at), b = std::min(hi, at + j.n);
            if (a < b) {
                if (j.src) std::memcpy(j.dst + (a - at), j.src + (a - at), b - a);
                else std::memset(j.dst + (a - at), 0, b - a);
            }
            at += j.n;
        }
    }
    std::vector<CopyJob> jobs_;
    std::vector<std::thread> th_;
};

// Host-streaming pipeline.  Each byte offset of the sub-chunks
// is an independent codeword, so an operation on host chunks is cut into pieces of `w`
// bytes of every sub-chunk row.  Piece p of a host buffer of R rows (pitch sc) is one
// hipMemcpy2DAsync into a compact device buffer (R rows of wp bytes); the device
// operation runs on the pieces; outputs go back by 2D copies.  Pieces round-robin over
// the device's pipeline streams, so the H2D of piece p+1, the kernels of piece p and the
// D2H of piece p-1 overlap (PCIe is full duplex).  Used by clay_encode_host_pipelined and
// by the host-buffer API (clay_encode / clay_decode / clay_repair).
struct HostIn {
    const uint8_t *p;
    size_t rows;
};
struct HostOut {
    uint8_t *p;
    size_t rows;
};
template <class Op>
static Error host_pipeline(int device, size_t sc, const std::vector<HostIn> &ins, const std::vector<HostOut> &outs,
                           size_t piece_bytes, int n_streams, Op &&op, size_t *launches_out) {
    size_t in_rows = 0, all_rows = 0;
    for (auto &i : ins) in_rows += i.rows;
    all_rows = in_rows;
    for (auto &o : outs) all_rows += o.rows;
    if (sc == 0 || all_rows == 0) return Error{};
    // default: 256 MiB of input per piece over 2 streams (scripts/sweep_host_api.sh), whole
    // 256-byte tiles; CLAY_HOST_PIECE_MB / CLAY_HOST_STREAMS override the defaults
    const size_t def_piece = tuning().host_piece;
    const int def_streams = tuning().host_streams;
    if (n_streams <= 0) n_streams = def_streams;
    size_t w = piece_bytes ? piece_bytes : def_piece / std::max<size_t>(1, in_rows);
    w = w >= 256 ? w / 256 * 256 : (w + 7) / 8 * 8;
    w = std::max<size_t>(8, std::min(w, sc));
    const size_t np = (sc + w - 1) / w;
    const int ns = int(std::max<size_t>(1, std::min<size_t>(np, n_streams > 0 ? size_t(n_streams) : 2)));
    DevState *ds;
    Error e = dev_state(device, &ds);
    if (e) return e;
    DeviceGuard g(device);
    // streams and piece buffers of this call: from the device's pools (no device-wide
    // lock across the call, so pipelined calls from several threads run concurrently)
    struct Res {
        DevState &ds;
        std::vector<hipStream_t> st;
        std::vector<Lease *> buf;
        ~Res() {
            // every exit path, errors included: copies to / from the caller's host buffers
            // may still be queued, and the caller may free those buffers once we return
            for (auto x : st) (void)hipStreamSynchronize(x);
            for (size_t i = 0; i < buf.size(); i++) lease_release(ds, buf[i], st[i]);
            std::lock_guard<std::mutex> lk(ds.mu);
            for (auto x : st) ds.host_streams.push_back(x);
        }
    } r{*ds, {}, {}};
    {
        std::lock_guard<std::mutex> lk(ds->mu);
        while (int(r.st.size()) < ns) {
            hipStream_t st;
            if (!ds->host_streams.empty()) {
                st = ds->host_streams.back();
                ds->host_streams.pop_back();
            } else {
                CLAY_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            }
            r.st.push_back(st);
        }
    }
    const size_t need = all_rows * w;
    for (int s = 0; s < ns; s++) {
        Lease *l = nullptr;
        e = lease_acquire(*ds, need, r.st[s], &l);
        if (e) return e;
        r.buf.push_back(l);
    }
    std::vector<const uint8_t *> din(ins.size());
    std::vector<uint8_t *> dout(outs.size());
    size_t launches = 0;
    for (size_t p = 0; p < np; p++) {
        const int s = int(p % size_t(ns));
        hipStream_t st = r.st[s];
        uint8_t *buf = static_cast<uint8_t *>(r.buf[s]->d);
        const size_t off = p * w, wp = std::min(w, sc - off);
        size_t at = 0;
        for (size_t i = 0; i < ins.size(); i++) {
            uint8_t *dst = buf + at * wp;
            if (ins[i].p)
                CLAY_HIP(hipMemcpy2DAsync(dst, wp, ins[i].p + off, sc, wp, ins[i].rows, hipMemcpyHostToDevice, st));
            din[i] = ins[i].p ? dst : nullptr;
            at += ins[i].rows;
        }
        for (size_t j = 0; j < outs.size(); j++) {
            dout[j] = outs[j].p ? buf + at * wp : nullptr;
            at += outs[j].rows;
        }
        e = op(din, dout, wp, st);
        if (e) return e;
        launches += t_last_launches;
        for (size_t j = 0; j < outs.size(); j++)
            if (outs[j].p)
                CLAY_HIP(hipMemcpy2DAsync(outs[j].p + off, sc, dout[j], wp, wp, outs[j].rows, hipMemcpyDeviceToHost, st));
    }
    for (int s = 0; s < ns; s++) CLAY_HIP(hipStreamSynchronize(r.st[s]));
    if (launches_out) *launches_out = launches;
    return Error{};
}

static int current_device(Error *e) {
    int ndev = 0, d = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        *e = make_error(CLAY_ERR_DEVICE, 0, 0, 0, "HIP error: no GPU device available (no CPU fallback)");
        return -1;
    }
    (void)hipGetDevice(&d);
    return d;
}

}  // namespace clay

// ===========================================================================
// C ABI
// ===========================================================================
using namespace clay;

extern "C" {

int clay_abi_version(void) { return CLAY_ABI_VERSION; }
const char *clay_build_info(void) { return "clay_amd " __DATE__ " gfx950 HIP"; }
int clay_set_encode_path(int mode) {
    // low byte: path; next byte: variant.  Only paths that produce the reference's parity
    // exist; unknown paths or variants are rejected (-1) and leave the setting unchanged.
    const int path = mode & 0xFF, tile = (mode >> 8) & 0xFF;
    if (mode < 0 || (mode >> 16) != 0) return -1;
    bool ok = false;
    switch (path) {
    case kModeAuto: case kModeStaged: case kModeFused: ok = tile == 0; break;
    case kModeBs: ok = tile == 0 || tile == 1 || tile == 4; break;     // v1 lanes of 32 B per column group
    case kModeStream: ok = tile == 0 || tile == 1 || tile == 2 || tile == 4 || tile == 7; break;  // loader waves
    default: ok = false;
    }
    if (!ok) return -1;
    const int prev = g_encode_mode.load() | (g_encode_tile.load() << 8);
    g_encode_tile.store(tile);
    g_encode_mode.store(path);
    return prev;
}
int clay_set_exec_mode(int mode) {
    if (mode != kExecAuto && mode != kExecGrouped && mode != kExecTile && mode != kExecStream &&
        mode != kExecStreamLocal && mode != kExecStreamFused2)
        return -1;
    return g_exec_mode.exchange(mode);
}
const char *clay_last_encode_path(void) { return t_last_path.c_str(); }
const char *clay_last_exec_path(void) { return t_last_exec; }
size_t clay_last_launch_count(void) { return t_last_launches; }

int clay_new(size_t k, size_t m, size_t d, clay_code_t *out, clay_error_t *err) {
    if (!out) return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null output"), err);
    Error e = code_new(k, m, d, out);
    if (err) std::memset(err, 0, sizeof(*err));
    return e ? report(e, err) : 0;
}
int clay_new_default(size_t k, size_t m, clay_code_t *out, clay_error_t *err) {
    return clay_new(k, m, k + m - 1, out, err);
}
double clay_normalized_repair_bandwidth(const clay_code_t *c) {
    return double(c->d) / (double(c->k) * double(c->d - c->k + 1));
}
size_t clay_encoded_chunk_size(const clay_code_t *c, size_t len) { return encoded_chunk_size(*c, len); }

int clay_minimum_to_repair(const clay_code_t *code, size_t lost, const size_t *avail, size_t nav, size_t *helpers_out,
                           size_t *n_helpers, size_t *sub_out, size_t *n_sub, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = check_code(code);
    if (e) return report(e, err);
    std::vector<size_t> h, s;
    e = minimum_to_repair(*code, lost, avail, nav, h, s);
    if (n_helpers) *n_helpers = h.size();
    if (n_sub) *n_sub = e ? 0 : s.size();
    if (e) return report(e, err);
    if (helpers_out) std::copy(h.begin(), h.end(), helpers_out);
    if (sub_out) std::copy(s.begin(), s.end(), sub_out);
    return 0;
}

int clay_encode_device(const clay_code_t *code, const uint8_t *const *data, uint8_t *const *par, size_t chunk,
                       int device, void *stream, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = encode_device_impl(code, data, par, 1, chunk, device, stream);
    return e ? report(e, err) : 0;
}

int clay_encode_device_batch(const clay_code_t *code, const uint8_t *const *data, uint8_t *const *par, size_t ns,
                             size_t chunk, int device, void *stream, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = encode_device_impl(code, data, par, ns, chunk, device, stream);
    return e ? report(e, err) : 0;
}

int clay_encode_device_strided(const clay_code_t *code, const uint8_t *data, int64_t data_node_stride,
                               int64_t data_stripe_stride, uint8_t *parity, int64_t parity_node_stride,
                               int64_t parity_stripe_stride, size_t n_stripes, size_t chunk, int device, void *stream,
                               clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    const Strided sd{data, data_node_stride, data_stripe_stride, parity, parity_node_stride, parity_stripe_stride};
    Error e = encode_device_impl(code, nullptr, nullptr, n_stripes, chunk, device, stream, &sd);
    return e ? report(e, err) : 0;
}

static Error ygroup_impl(const clay_code_t *code, size_t y, const uint8_t *src, uint8_t *dst, size_t chunk, int dev,
                         void *stream, bool to_group) {
    Error e = check_code(code);
    if (e) return e;
    if (!src || !dst) return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null chunk");
    if (y >= code->t)
        return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: y-section %zu >= t = %zu", y,
                          code->t);
    if (chunk == 0 || chunk % code->sub_chunk_no != 0)
        return make_error(CLAY_ERR_INVALID_CHUNK_SIZE, code->sub_chunk_no, chunk, 0,
                          "Invalid chunk size: expected divisible by %zu, got %zu", code->sub_chunk_no, chunk);
    if (src == dst) return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: in-place regroup");
    DevState *ds;
    e = dev_state(dev, &ds);
    if (e) return e;
    DeviceGuard g(dev);
    const uint64_t sc = chunk / code->sub_chunk_no;
    size_t pw = 1;
    for (size_t j = y + 1; j < code->t; j++) pw *= code->q;
    const uint64_t pieces = (sc + 4095) / 4096;
    const uint64_t blocks = uint64_t(code->sub_chunk_no) * pieces;
    if (blocks > 0x7fffffffull) return make_error(CLAY_ERR_DEVICE, 0, 0, 0, "chunk too large for one regroup launch");
    auto k = to_group ? k_ygroup<true> : k_ygroup<false>;
    k<<<dim3(uint32_t(blocks)), dim3(256), 0, static_cast<hipStream_t>(stream)>>>(
        src, dst, sc, uint32_t(code->beta), uint32_t(code->q), uint32_t(pw), uint32_t(pieces));
    CLAY_HIP(hipGetLastError());
    t_last_launches = 1;
    return Error{};
}

int clay_chunk_to_ygroup(const clay_code_t *code, size_t y, const uint8_t *chunk, uint8_t *group, size_t chunk_size,
                         int device, void *stream, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = ygroup_impl(code, y, chunk, group, chunk_size, device, stream, true);
    return e ? report(e, err) : 0;
}

int clay_ygroup_to_chunk(const clay_code_t *code, size_t y, const uint8_t *group, uint8_t *chunk, size_t chunk_size,
                         int device, void *stream, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = ygroup_impl(code, y, group, chunk, chunk_size, device, stream, false);
    return e ? report(e, err) : 0;
}

int clay_decode_device(const clay_code_t *code, const uint8_t *const *chunks, const size_t *er, size_t ner,
                       uint8_t *const *outs, size_t chunk, int device, void *stream, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = decode_device_impl(code, chunks, er, ner, outs, chunk, device, stream);
    return e ? report(e, err) : 0;
}

int clay_decode_device_codeword(const clay_code_t *code, const uint8_t *const *chunks, const size_t *er, size_t ner,
                                uint8_t *const *outs, size_t chunk, int device, void *stream, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = decode_device_impl(code, chunks, er, ner, outs, chunk, device, stream, true);
    return e ? report(e, err) : 0;
}

int clay_repair_device(const clay_code_t *code, size_t lost, const size_t *ids, const uint8_t *const *bufs, size_t nh,
                       size_t chunk, uint8_t *out, int device, void *stream, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = repair_device_impl(code, lost, ids, bufs, nullptr, nh, chunk, out, device, stream);
    return e ? report(e, err) : 0;
}

int clay_repair_device_full_chunks(const clay_code_t *code, size_t lost, const size_t *ids,
                                   const uint8_t *const *chunks, size_t nh, size_t chunk, uint8_t *out, int device,
                                   void *stream, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = repair_device_impl(code, lost, ids, chunks, nullptr, nh, chunk, out, device, stream, true);
    return e ? report(e, err) : 0;
}

int clay_reserve_workspace(const clay_code_t *code, size_t chunk, int device, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = check_code(code);
    if (e) return report(e, err);
    DevState *ds;
    e = dev_state(device, &ds);
    if (e) return report(e, err);
    DeviceGuard g(device);
    // an idle workspace lease any stream can take, plus the encode plan on the device
    Lease *l = nullptr;
    e = lease_acquire(*ds, code->q * code->t * chunk, nullptr, &l);
    if (e) return report(e, err);
    {   // nothing was enqueued on it: hand it back unused, so that any stream -- also one that is
        // capturing a graph (no event query or allocation while capturing) -- may take it
        std::lock_guard<std::mutex> lk(ds->mu);
        l->busy = false;
    }
    CodeState &cs = *code_state(*code);
    const Plan *pl = nullptr;
    CodeState::DevGrouped gp{};
    if (!cs.rs.init_err && code->q * code->t <= size_t(kMaxTn)) {
        e = encode_plan(cs, &pl);
        if (!e) e = upload_groups(cs, *pl, device, &gp);
    }
    return e ? report(e, err) : 0;
}

int clay_release_workspace(int device, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    DevState *ds;
    Error e = dev_state(device, &ds);
    if (e) return report(e, err);
    DeviceGuard g(device);
    std::lock_guard<std::mutex> lk(ds->mu);
    for (auto it = ds->pool.begin(); it != ds->pool.end();) {
        Lease &l = **it;
        if (!l.busy && !l.pinned && hipEventSynchronize(l.ev) == hipSuccess) {
            (void)hipFree(l.d);
            (void)hipEventDestroy(l.ev);
            it = ds->pool.erase(it);
        } else {
            ++it;
        }
    }
    for (auto it = ds->tables.begin(); it != ds->tables.end();) {
        if (it->second.users > 0) {  // a call between lookup and launch holds it
            ++it;
            continue;
        }
        free_table(it->second);
        it = ds->tables.erase(it);
    }
    return 0;
}

int clay_release_captured(int device, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    DevState *ds;
    Error e = dev_state(device, &ds);
    if (e) return report(e, err);
    // No device-wide synchronize here: hipDeviceSynchronize while another thread captures (global
    // capture mode, torch.cuda.graph's default) would invalidate that capture.  The caller has
    // waited for every replay of the graphs and destroyed them (clay.h); refuse while one of this
    // library's calls is inside a capture right now (its table or lease is in use).
    // A lease taken inside a capture is refused back while that call runs (busy) or while the
    // capture it was taken in is still open (its graph does not exist yet, so the caller cannot
    // have destroyed it): unpinning it then would hand a graph-owned workspace to the next eager
    // call.  Pointer tables likewise, by their capture's stream and id.
    std::lock_guard<std::mutex> lk(ds->mu);
    for (auto &t : ds->captured)
        if (t->users > 0 || (t->cap_id && capture_id(t->cap_st) == t->cap_id))
            return report(make_error(CLAY_ERR_DEVICE, 0, 0, 0, "a stream capture is using the pointer-table arena"), err);
    for (auto &l : ds->pool)
        if (l->captured && (l->busy || (l->cap_id && capture_id(l->cap_st) == l->cap_id)))
            return report(make_error(CLAY_ERR_DEVICE, 0, 0, 0, "a stream capture is using a pooled workspace"), err);
    ds->captured.clear();
    ds->cap_used = 0;
    for (auto &l : ds->pool)
        if (l->pinned) {
            // the caller has waited for every replay (clay.h): no event guards this buffer now
            l->pinned = l->captured = false;
            l->used = false;
            l->cap_st = nullptr;
            l->cap_id = 0;
        }
    return 0;
}

size_t clay_workspace_bytes(int device) {
    DevState *ds;
    if (dev_state(device, &ds)) return 0;
    std::lock_guard<std::mutex> lk(ds->mu);
    size_t b = 0;
    for (auto &l : ds->pool) b += l->bytes;
    return b;
}

int clay_plan_export(const clay_code_t *code, int kind, const uint8_t *mask, const uint8_t *want, size_t lost,
                     uint32_t *ops_out, size_t ops_cap, uint32_t *srcs_out, size_t srcs_cap, uint32_t *stages_out,
                     size_t stages_cap, size_t counts[3], clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = check_code(code);
    if (e) return report(e, err);
    const clay_code_t &c = *code;
    const size_t tn = c.q * c.t;
    RsCtx rs(c);
    std::unique_ptr<Plan> p;
    if (kind == 0) {
        e = plan_encode(c, rs, p);
    } else if (kind == 1) {
        if (!mask || !want) return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null mask"), err);
        e = plan_decode(c, rs, std::vector<uint8_t>(mask, mask + tn), std::vector<uint8_t>(want, want + tn), p);
    } else if (kind == 2) {
        if (!mask) return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null mask"), err);
        std::vector<uint8_t> hin(mask, mask + tn);
        std::vector<long> so(tn, -1);
        std::vector<size_t> sub;
        if (lost >= c.n)
            return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: Invalid lost node index: %zu >= %zu", lost, c.n), err);
        e = repair_subchunk_indices(c, internal_of(c, lost), sub);
        if (!e) e = plan_repair(c, rs, lost, hin, so, sub, p);
    } else {
        e = make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: plan kind %d", kind);
    }
    if (e) return report(e, err);
    if (counts) {
        counts[0] = p->ops.size();
        counts[1] = p->srcs.size();
        counts[2] = p->stage_begin.size();
    }
    if (ops_out && ops_cap >= p->ops.size() * 4 && srcs_out && srcs_cap >= p->srcs.size() * 4 && stages_out &&
        stages_cap >= p->stage_begin.size()) {
        for (size_t i = 0; i < p->ops.size(); i++) {
            ops_out[4 * i] = p->ops[i].base;
            ops_out[4 * i + 1] = p->ops[i].slot;
            ops_out[4 * i + 2] = p->ops[i].src_begin;
            ops_out[4 * i + 3] = p->ops[i].nsrc;
        }
        for (size_t i = 0; i < p->srcs.size(); i++) {
            srcs_out[4 * i] = p->srcs[i].base;
            srcs_out[4 * i + 1] = p->srcs[i].slot;
            srcs_out[4 * i + 2] = p->srcs[i].coef;
            srcs_out[4 * i + 3] = 0;
        }
        std::copy(p->stage_begin.begin(), p->stage_begin.end(), stages_out);
    }
    return 0;
}

int clay_encode_host_pipelined(const clay_code_t *code, const uint8_t *const *data_chunks,
                               uint8_t *const *parity_chunks, size_t chunk, int device, size_t piece_bytes,
                               int n_streams, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = check_code(code);
    if (e) return report(e, err);
    const clay_code_t &c = *code;
    if (!data_chunks || !parity_chunks)
        return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null chunk array"), err);
    if (chunk == 0 || chunk % c.sub_chunk_no != 0)
        return report(make_error(CLAY_ERR_INVALID_CHUNK_SIZE, c.sub_chunk_no, chunk, 0,
                                 "Invalid chunk size: expected divisible by %zu, got %zu", c.sub_chunk_no, chunk),
                      err);
    for (size_t i = 0; i < c.k; i++)
        if (!data_chunks[i]) return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null data chunk"), err);
    for (size_t i = 0; i < c.m; i++)
        if (!parity_chunks[i]) return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null parity chunk"), err);
    const size_t alpha = c.sub_chunk_no, sc = chunk / alpha;
    std::vector<HostIn> ins;
    std::vector<HostOut> outs;
    for (size_t i = 0; i < c.k; i++) ins.push_back({data_chunks[i], alpha});
    for (size_t j = 0; j < c.m; j++) outs.push_back({parity_chunks[j], alpha});
    size_t launches = 0;
    e = host_pipeline(device, sc, ins, outs, piece_bytes, n_streams,
                      [&](const std::vector<const uint8_t *> &din, const std::vector<uint8_t *> &dout, size_t wp,
                          hipStream_t st) {
                          return encode_device_impl(code, din.data(), dout.data(), 1, alpha * wp, device, st);
                      },
                      &launches);
    if (e) return report(e, err);
    t_last_launches = launches;
    return 0;
}

int clay_encode(const clay_code_t *code, const uint8_t *data, size_t len, uint8_t *const *out, size_t chunk,
                clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = check_code(code);
    if (e) return report(e, err);
    const clay_code_t &c = *code;
    if (!out) return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null output"), err);
    size_t expect = encoded_chunk_size(c, len);
    if (chunk != expect)
        return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0,
                                 "Invalid parameters: chunk_size %zu does not match encoded chunk size %zu", chunk,
                                 expect),
                      err);
    for (size_t i = 0; i < c.n; i++)
        if (!out[i]) return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null output chunk"), err);
    const int dev = current_device(&e);
    if (e) return report(e, err);
    // data chunks: zero-padded copy of the input (encode.rs:44-55).  Chunks wholly inside
    // the input feed the GPU straight from `data` while host threads copy them into
    // out[i]; a chunk that needs padding is built first and fed from out[i].
    const size_t alpha = c.sub_chunk_no, sc = chunk / alpha;
    std::vector<HostIn> ins;
    std::vector<CopyJob> jobs;
    for (size_t i = 0; i < c.k; i++) {
        const size_t lo = i * chunk, n = lo < len ? std::min(chunk, len - lo) : 0;
        if (n == chunk) {
            jobs.push_back({out[i], data + lo, chunk});
            ins.push_back({data + lo, alpha});
        } else {
            if (n) std::memcpy(out[i], data + lo, n);
            std::memset(out[i] + n, 0, chunk - n);
            ins.push_back({out[i], alpha});
        }
    }
    HostCopier copier(std::move(jobs));
    // parity: the host-streaming pipeline
    std::vector<HostOut> outs;
    for (size_t j = 0; j < c.m; j++) outs.push_back({out[c.k + j], alpha});
    size_t launches = 0;
    e = host_pipeline(dev, sc, ins, outs, 0, 0,
                      [&](const std::vector<const uint8_t *> &din, const std::vector<uint8_t *> &dout, size_t wp,
                          hipStream_t st) {
                          return encode_device_impl(code, din.data(), dout.data(), 1, alpha * wp, dev, st);
                      },
                      &launches);
    copier.join();
    if (e) return report(e, err);
    t_last_launches = launches;
    return 0;
}

int clay_decode(const clay_code_t *code, const size_t *ids, const uint8_t *const *bufs, const size_t *lens,
                size_t n_avail, const size_t *er, size_t ner, uint8_t *out, size_t out_cap, size_t *out_len,
                clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    if (out_len) *out_len = 0;
    Error e = check_code(code);
    if (e) return report(e, err);
    const clay_code_t &c = *code;
    if (n_avail == 0 && ner == 0) return 0;
    size_t chunk = 0;
    std::vector<uint8_t> erased;
    e = validate_decode(c, AvailView{ids, lens, n_avail}, er, ner, &chunk, erased);
    if (e) return report(e, err);
    const size_t need = c.k * chunk;
    if (!out || out_cap < need)
        return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: output buffer too small"), err);
    std::vector<const uint8_t *> host_of(c.n, nullptr);
    for (size_t i = 0; i < n_avail; i++) host_of[ids[i]] = bufs[i];
    std::vector<CopyJob> jobs;  // available data chunks into the output, beside the GPU work
    for (size_t i = 0; i < c.k; i++)
        if (host_of[i]) jobs.push_back({out + i * chunk, host_of[i], chunk});
    HostCopier copier(std::move(jobs));
    bool any_data_erased = false;
    for (size_t i = 0; i < ner; i++) any_data_erased |= er[i] < c.k;
    if (any_data_erased) {
        const int dev = current_device(&e);
        if (e) return report(e, err);
        // pieces of every sub-chunk row: inputs = the available chunks (in internal-node
        // order), outputs = the erased data chunks straight into `out`
        const size_t alpha = c.sub_chunk_no, sc = chunk / alpha;
        std::vector<HostIn> ins(c.n, HostIn{nullptr, alpha});
        std::vector<HostOut> outs(c.n, HostOut{nullptr, alpha});
        for (size_t i = 0; i < n_avail; i++) ins[ids[i]].p = bufs[i];
        for (size_t i = 0; i < ner; i++)
            if (er[i] < c.k) outs[er[i]].p = out + er[i] * chunk;
        // the device decode sees chunks[] with nullptr = absent, outs[] for erased data nodes
        size_t launches = 0;
        e = host_pipeline(dev, sc, ins, outs, 0, 0,
                          [&](const std::vector<const uint8_t *> &din, const std::vector<uint8_t *> &dout, size_t wp,
                              hipStream_t st) {
                              return decode_device_impl(code, din.data(), er, ner, dout.data(), alpha * wp, dev, st);
                          },
                          &launches);
        if (e) return report(e, err);
        t_last_launches = launches;
    }
    if (out_len) *out_len = need;
    return 0;
}

int clay_repair(const clay_code_t *code, size_t lost, const size_t *ids, const uint8_t *const *bufs, const size_t *lens,
                size_t nh, size_t chunk, uint8_t *out, clay_error_t *err) {
    if (err) std::memset(err, 0, sizeof(*err));
    Error e = check_code(code);
    if (e) return report(e, err);
    const clay_code_t &c = *code;
    {
        std::vector<uint8_t> hin;
        std::vector<long> so;
        std::vector<size_t> sub;
        e = validate_repair(c, lost, ids, lens, nh, chunk, hin, so, sub);
        if (e) return report(e, err);
    }
    if (!out) return report(make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: null output"), err);
    const int dev = current_device(&e);
    if (e) return report(e, err);
    // pieces of every sub-chunk row: each helper holds beta rows (its repair layers, in
    // index order), the output alpha rows
    const size_t alpha = c.sub_chunk_no, sc = chunk / alpha, beta = nh ? lens[0] / sc : 0;
    std::vector<HostIn> ins;
    for (size_t i = 0; i < nh; i++) ins.push_back({bufs[i], beta});
    std::vector<HostOut> outs{{out, alpha}};
    std::vector<size_t> plens(nh);
    size_t launches = 0;
    e = host_pipeline(dev, sc, ins, outs, 0, 0,
                      [&](const std::vector<const uint8_t *> &din, const std::vector<uint8_t *> &dout, size_t wp,
                          hipStream_t st) {
                          for (auto &l : plens) l = beta * wp;
                          return repair_device_impl(code, lost, ids, din.data(), plens.data(), nh, alpha * wp, dout[0],
                                                    dev, st);
                      },
                      &launches);
    if (e) return report(e, err);
    t_last_launches = launches;
    return 0;
}

}  // extern "C"
