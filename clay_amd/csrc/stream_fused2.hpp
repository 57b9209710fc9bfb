// stream_fused2.hpp -- single-launch decode for q = 4, t = 4 codes with 2-4 erasures in distinct
// y-sections (the BASELINE worst case {0,4,8,12} among them): every survivor byte read from HBM
// once, every output byte written once, and the latency-bound iscore rounds (decode.rs:196-254)
// of tile k-1 run on other waves while tile k streams.
//
// Why not k_stream_decode (the fused kernel of stream_decode.hpp)?  There the compute waves run
// phase B themselves and its S/C region aliases ring buffers, so every tile drains the load
// pipeline (measured: memory + phase A 0.51 ms, full 1.05 ms).  Here:
//   * LDS = a ring of RB = 10 - ne node buffers (16 KiB: one node x 256 layers x 64 B) that
//     streams continuously across tiles + a separate S/C region (ne x 16 KiB, [row r][z][64 B]);
//   * 8 compute waves: phase A of tile k (StreamDec::phase_a, one barrier per section; each
//     step a copy with the section's erasure structure at compile time, DecArgs::scase), the
//     presolve S' = H_K^-1 S in registers (check j outer: its row tables through scalar loads
//     once per tile), then S'(k) into the S/C region (below);
//   * 4 loader waves issue every LDS-DMA (as in k_stream_syn; the next tile's first loads once
//     phase A freed the ring) AND solve tile k-1 meanwhile: the round of iscore level y + 1
//     during section step y of tile k (term-parallel: one item per (target layer, 8 bytes); a
//     wave owns one section Y and sums the three X != x_e(Y) terms A_(Y,X) C(e_Y, z[Y:=X]) of a
//     target in registers (tables loaded once per kernel), one 64-bit LDS atomic XOR per row;
//     every lane's target offsets are enumerated once per kernel and kept in registers);
//   * after the last round each compute lane reads C(k-1) from, and writes S'(k) to, the same
//     bytes of the region (no hand-over barrier), then stores C(k-1) (8-byte pieces, 64-byte row
//     runs): stores come from waves that never wait on vmcnt, so the loaders' counted DMA waits
//     see loads only;
//   * five workgroup barriers per tile (four section steps, rounds done), all waves.
// Tables live in global memory (scalar loads; the solver's in registers): the ring and the S/C
// region take all 160 KiB of LDS.
#pragma once

#include "stream_decode.hpp"

namespace clay {
namespace bs {

// solver work items per lane and round (passes of 64 lanes over targets x 8 pieces), the most over
// the eligible patterns.  One erasure per section, 2-4 erasures: level 1 has 27 / 36 / 48 targets
// for 4 / 3 / 2 erasures (4 / 5 / 6 passes), level 2 27 / 24 / 16 (4 / 3 / 2), level 3 9 / 4
// (2 / 1), level 4 1 (1).  Four erasures with two in a section (round 6: (2,1,1) and (2,2)
// sections): level 1 72 / 64 targets (9 / 8 passes), level 2 48 / 64 (6 / 8), level 3 8 (1)
// (tests/test_gpu_stream_decode.py::f2_fits and engine.hip f2_fits count them).
// (kF2Iters / kF2Off / kF2Items: decode_args.hpp, shared with the host's eligibility check)
template <int N>
using IC = std::integral_constant<int, N>;

// S/C region layout: row of layer z of an erased row's 16 KiB block at 64 z.  (Round 6 measured a
// swizzled layout -- quarter = XOR of the layer's base-4 digits, bench_tools/lds_conflicts_fused2.py:
// SQ_LDS_BANK_CONFLICT 13.5 M -> 3.2 M per decode -- at 0.58 vs 0.51 ms for {0,4,8,12}: the extra
// address arithmetic in the loader waves' rounds, which bound the kernel, costs more than the
// conflicts; profiles/r06/decode/.)

// PROBE (bench_tools only; the library instantiates 0): 1 = loader waves skip the rounds,
// 2 = no output stores, 4 = no phase-A math, 8 = no presolve, 16 = s_memtime segment timing
// (workgroup 0 prints the totals of compute wave 0 and loader wave 0), 64 = rounds at priority 0,
// 128 = phase A without the per-section compile-time copies (StreamDec::phase_a)
// TWO: the instantiation for two erasures in a section (both-erased pairs, split steps, the larger
// round item sets); patterns with at most one erasure per section run TWO = false, whose hot code
// is the round-5 kernel's (the larger TWO kernel ran {0,4,8,12} 15 % slower: 0.58 vs 0.51 ms)
template <int KD, int G, int PROBE = 0, bool TWO = false>
__global__ __launch_bounds__((StreamDec<KD, G>::BLOCK)) void k_stream_fused2(DecArgs a) {
    using Kn = StreamDec<KD, G>;
    // round work items per lane and level (decode_args.hpp)
    static constexpr int IT[4] = {TWO ? kF2Iters[0] : kF2Iters1[0], TWO ? kF2Iters[1] : kF2Iters1[1],
                                  TWO ? kF2Iters[2] : kF2Iters1[2], TWO ? kF2Iters[3] : kF2Iters1[3]};
    static constexpr int OFF[4] = {0, IT[0], IT[0] + IT[1], IT[0] + IT[1] + IT[2]};
    static constexpr int NIT = IT[0] + IT[1] + IT[2] + IT[3];
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t xcd = blockIdx.x & 7u, wslot = blockIdx.x >> 3, ns = a.nslots;
    const uint32_t sc = uint32_t(a.sc);
    const typename Kn::Map tm(sc, a.region, ns, xcd, wslot);
    const uint32_t ntile = tm.n;
    if (ntile == 0) return;  // uniform per workgroup
    const uint32_t RB = a.ring, NT = a.nt;
    constexpr uint32_t BUF = uint32_t(Kn::BUF);
    uint8_t *const scr = smem + RB * BUF;  // S/C region
    const cu32p tabc = (cu32p)(a.tabs);  // constant address space: uniform loads become s_load

    if (wave >= Kn::CWAVES) {
        // ---------------- loader + solver waves ----------------
        __builtin_amdgcn_s_setprio(3);
        const int li = wave - Kn::CWAVES;
        typename Kn::Loader L;
        Kn::template loader_init<true>(L, sc, li, lane);
        const uint32_t lds0 = lds_addr_of(smem);
        const uint32_t nloads = ntile * NT;
        uint32_t issued = 0;
        auto issue_upto = [&](uint32_t lim) {
            if (lim > nloads) lim = nloads;
            for (; issued < lim; issued++) {
                const uint32_t k = issued / NT, q = issued % NT;
                Kn::issue(a, L, lds0 + (issued % RB) * BUF, a.node[a.load_node[q]], tm.tile(k, wslot, ns), li);
            }
        };
        issue_upto(RB);
        // the rounds' work of this wave (a.lwave, engine.hip f2_plan): every nw-th pass, from pass
        // `part`, over the targets red in section Y (one to four waves per section with an erasure;
        // a wave without a section only loads); the A_(Y,X) tables of its X outside E_Y, loaded
        // once into registers (tile-invariant; zero for an X outside the used shards: no dropped
        // term, decode.rs:374)
        const uint32_t ne = a.ne;
        const uint32_t lw = (a.lwave >> (8 * li)) & 0xffu;
        const bool lact = (lw >> 6) & 1u;
        const uint32_t part = (lw >> 2) & 3u, nw = ((lw >> 4) & 3u) + 1u;
        // the round tables (tg), the lane's work items (rb) and the section's erased digits:
        // the round-5 enumeration for one erasure per section (!TWO), the general one for up to two
        GfTab tg[3][4];
        uint32_t rb[NIT];
        uint32_t Y = lw & 3u, x1 = 0, x2 = 0, nY = 0, Xj[3] = {0, 0, 0};
        uint32_t src1 = 0, src2 = 0, wy64 = 0;
        auto setup_one = [&]() BS_INL {
        uint32_t xe[4], esec = 0;
#pragma unroll
        for (int y = 0; y < 4; y++) {
            xe[y] = a.emask[y] ? uint32_t(__builtin_ctz(a.emask[y])) : 0u;
            esec |= (a.emask[y] ? 1u : 0u) << y;
        }
        const uint32_t xY = xe[Y];
        const bool wact = lact && ((esec >> Y) & 1u);
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const uint32_t X = uint32_t(j) + (uint32_t(j) >= xY ? 1u : 0u);
            const bool use = wact && ((a.used >> (4u * Y + X)) & 1u);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                // loaded unconditionally (every table exists), then masked: zero = no term
                const uint32_t keep = (use && uint32_t(r) < ne) ? ~0u : 0u;
                const GfTab t = load_tab_c(tabc + (16u + (4u * Y + X) * 4u + uint32_t(r)) * 8u);
                tg[j][r] = GfTab{t.w0 & keep, t.w1 & keep, t.w2 & keep, t.w3 & keep, t.w4 & keep};
                asm volatile("" : "+v"(tg[j][r].w0), "+v"(tg[j][r].w1), "+v"(tg[j][r].w2), "+v"(tg[j][r].w3),
                             "+v"(tg[j][r].w4));
            }
        }
        // C(e_Y, .): rix read unconditionally (xY = 0 for a section without an erasure), then the
        // value selected -- a select between loads would become a load through a selected pointer
        // and move the kernel arguments to scratch memory
        const uint32_t rY = opq(uint32_t(a.rix[4u * Y + xY]));
        const uint8_t *src5 = scr + (wact ? rY : 0u) * BUF;
        wy64 = Kn::wt(int(Y)) * 64u;
        // the lane's work items of every round, tile-invariant: byte offset (layer without section
        // Y's digit) x 64 + 8-byte piece, ~0 = none.  Level L's targets: z_Y = x_e(Y), L - 1 of the
        // other erased sections red (subset `sub`), base-3 digits for the other erased sections,
        // base-4 digits for the sections without an erasure; the lowest-weight section's digit
        // varies fastest (neighbouring items on different LDS banks)
        const uint32_t no = uint32_t(__builtin_popcount(esec)) - (wact ? 1u : 0u);  // other erased sections
        const uint32_t n4 = 4u - uint32_t(__builtin_popcount(esec));                // sections without one
        sfor<4>([&](auto yc) BS_INL {
            constexpr int y = decltype(yc)::value;
            constexpr uint32_t L = uint32_t(y) + 1u;
            uint32_t c3 = 1, c4 = 1, nsub = 0;
            for (uint32_t i = 0; i + (L - 1u) < no; i++) c3 *= 3u;
            for (uint32_t i = 0; i < n4; i++) c4 *= 4u;
            for (uint32_t m = 0; m < (1u << no); m++) nsub += uint32_t(__builtin_popcount(m)) == L - 1u ? 1u : 0u;
            const uint32_t per = c3 * c4, total = (wact && L - 1u <= no) ? nsub * per : 0u;
#pragma unroll
            for (int i = 0; i < IT[y]; i++) {
                const uint32_t it = uint32_t(lane) + 64u * (uint32_t(i) * nw + part);
                const uint32_t ci = it >> 3, d8 = (it & 7u) * 8u;
                if (ci >= total) {
                    rb[OFF[y] + i] = ~0u;
                    continue;
                }
                const uint32_t sub = ci / per;
                uint32_t v = ci % per, mask = 0, cnt = 0;
                for (uint32_t m = 0; m < (1u << no); m++)
                    if (uint32_t(__builtin_popcount(m)) == L - 1u) {
                        if (cnt == sub) mask = m;
                        cnt++;
                    }
                uint32_t zb = 0, o = 0;  // o: index among the other erased sections (descending)
                sfor<4>([&](auto qc) BS_INL {
                    constexpr int yy = 3 - decltype(qc)::value;
                    if (uint32_t(yy) == Y) return;
                    const uint32_t xy = xe[yy];
                    uint32_t dgt;
                    if ((esec >> yy) & 1u) {
                        if ((mask >> o) & 1u) {
                            dgt = xy;
                        } else {
                            const uint32_t u = v % 3u;
                            v /= 3u;
                            dgt = u + (u >= xy ? 1u : 0u);
                        }
                        o++;
                    } else {
                        dgt = v & 3u;
                        v >>= 2;
                    }
                    zb += dgt * Kn::wt(yy);
                });
                rb[OFF[y] + i] = zb * 64u + d8;
            }
        });
            x1 = x2 = xY;
            nY = 1;
            src1 = src2 = uint32_t(src5 - scr);
#pragma unroll
            for (int j = 0; j < 3; j++) Xj[j] = uint32_t(j) + (uint32_t(j) >= xY ? 1u : 0u);
        };
        auto setup_two = [&]() BS_INL {
        // erased nodes per section: em[y] (one or two bits: round 6 takes two in a section)
        uint32_t em[4], esec = 0;
#pragma unroll
        for (int y = 0; y < 4; y++) {
            em[y] = a.emask[y];
            esec |= (em[y] ? 1u : 0u) << y;
        }
        const uint32_t emY = em[Y];
        const bool wact = lact && ((esec >> Y) & 1u);
        // the section's erased digits x1 <= x2 (x2 = x1 for one erasure) and its used digits X_j:
        // the three (one erasure) or two (two erasures) X outside E_Y
        x1 = emY ? uint32_t(__builtin_ctz(emY)) : 0u, x2 = emY ? 31u - uint32_t(__builtin_clz(emY)) : 0u;
        {
            uint32_t pool = ~emY & 15u;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                Xj[j] = pool ? uint32_t(__builtin_ctz(pool)) : 4u;  // 4: none (two erasures: 2 terms)
                pool &= pool - 1u;
            }
        }
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const uint32_t X = Xj[j] & 3u;
            const bool use = wact && Xj[j] < 4u && ((a.used >> (4u * Y + X)) & 1u);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                // loaded unconditionally (every table exists), then masked: zero = no term
                const uint32_t keep = (use && uint32_t(r) < ne) ? ~0u : 0u;
                const GfTab t = load_tab_c(tabc + (16u + (4u * Y + X) * 4u + uint32_t(r)) * 8u);
                tg[j][r] = GfTab{t.w0 & keep, t.w1 & keep, t.w2 & keep, t.w3 & keep, t.w4 & keep};
                asm volatile("" : "+v"(tg[j][r].w0), "+v"(tg[j][r].w1), "+v"(tg[j][r].w2), "+v"(tg[j][r].w3),
                             "+v"(tg[j][r].w4));
            }
        }
        // C(e, .) of the section's erased rows: rix read unconditionally (x = 0 for a section without
        // an erasure), then the values selected -- a select between loads would become a load
        // through a selected pointer and move the kernel arguments to scratch memory
        const uint32_t r1 = opq(uint32_t(a.rix[4u * Y + x1])), r2 = opq(uint32_t(a.rix[4u * Y + x2]));
        src1 = (wact ? r1 : 0u) * BUF, src2 = (wact ? r2 : 0u) * BUF;
        wy64 = Kn::wt(int(Y)) * 64u;
        // the lane's work items of every round, tile-invariant: (target layer without section Y's
        // digit) x 64 + 8-byte piece, bit 0 = the target's red erased node of section Y is x2 (else
        // x1); ~0 = none.  Level L's targets:
        // z_Y in E_Y, L - 1 of the other erased sections red (subset `sub`: z_y in E_y), the other
        // erased sections non-red (z_y outside E_y), free digits for the sections without an
        // erasure; the lowest-weight section's digit varies fastest (neighbouring items on
        // different LDS banks), the choice of z_Y slowest
        nY = uint32_t(__builtin_popcount(emY));
        sfor<4>([&](auto yc) BS_INL {
            constexpr int y = decltype(yc)::value;
            constexpr uint32_t L = uint32_t(y) + 1u;
            // per subset m (bit yy = section yy red) of the other erased sections with L - 1 red:
            // the number of targets (no arrays indexed at run time: they would live in scratch)
            const uint32_t others = esec & ~(1u << Y);
            const uint32_t n4 = 4u - uint32_t(__builtin_popcount(esec));
            uint32_t c4 = 1;
            for (uint32_t i = 0; i < n4; i++) c4 *= 4u;
            auto per_sub = [&](uint32_t m) {
                uint32_t c = c4;
                sfor<4>([&](auto qc) BS_INL {
                    constexpr int yy = decltype(qc)::value;
                    if (!((others >> yy) & 1u)) return;
                    const uint32_t ne_y = uint32_t(__builtin_popcount(em[yy]));
                    c *= ((m >> yy) & 1u) ? ne_y : 4u - ne_y;
                });
                return c;
            };
            uint32_t total = 0;
            if (wact)
                for (uint32_t m = 0; m < 16u; m++)
                    if (!(m & ~others) && uint32_t(__builtin_popcount(m)) == L - 1u) total += per_sub(m);
            total *= nY;
#pragma unroll
            for (int i = 0; i < IT[y]; i++) {
                const uint32_t it = uint32_t(lane) + 64u * (uint32_t(i) * nw + part);
                uint32_t ci = it >> 3;
                const uint32_t d8 = (it & 7u) * 8u;
                if (ci >= total) {
                    rb[OFF[y] + i] = ~0u;
                    continue;
                }
                const uint32_t tsel = ci / (total / nY);  // 0: z_Y = x1, 1: z_Y = x2
                ci -= tsel * (total / nY);
                uint32_t mask = 0;
                for (uint32_t m = 0; m < 16u; m++)
                    if (!(m & ~others) && uint32_t(__builtin_popcount(m)) == L - 1u) {
                        const uint32_t c = per_sub(m);
                        if (ci < c) {
                            mask = m;
                            break;
                        }
                        ci -= c;
                    }
                uint32_t v = ci, zb = 0;
                sfor<4>([&](auto qc) BS_INL {
                    constexpr int yy = 3 - decltype(qc)::value;
                    if (uint32_t(yy) == Y) return;
                    const uint32_t e = em[yy];
                    uint32_t dgt;
                    if ((esec >> yy) & 1u) {
                        // the (v mod n)-th digit inside (red) or outside (non-red) E_yy
                        const bool red = (mask >> yy) & 1u;
                        const uint32_t pool = red ? e : (~e & 15u), n = uint32_t(__builtin_popcount(pool));
                        uint32_t u = v % n, pl = pool;
                        v /= n;
                        for (; u; u--) pl &= pl - 1u;
                        dgt = uint32_t(__builtin_ctz(pl));
                    } else {
                        dgt = v & 3u;
                        v >>= 2;
                    }
                    zb += dgt * Kn::wt(yy);
                });
                rb[OFF[y] + i] = zb * 64u + d8 + tsel;
            }
        });
        };
        GfTab dinv{0, 0, 0, 0, 0};
        if constexpr (!TWO) {
            setup_one();
        } else {
            setup_two();
            dinv = load_tab_c(tabc + kDecDetInv * 8);  // (1 + gamma^2)^-1; unset unless a.npair (unused then)
        }
        // ---- the round of iscore level LV + 1 of tile k - 1 (passes [I0, I1) of the lane's items):
        // every target layer z of the level red in section Y adds sum over X != x_e(Y) of
        // A_(Y,X) C(e_Y, z[Y := X]) (the three terms summed in registers, one 64-bit LDS atomic per
        // row)
        auto round = [&](auto lvc) BS_INL {
            constexpr int LV = decltype(lvc)::value;
#pragma unroll
            for (int i = 0; i < IT[LV]; i++) {
                const uint32_t ob = rb[OFF[LV] + i];
                if (ob == ~0u) continue;
                const uint32_t obb = TWO ? ob & ~7u : ob;
                const bool t2 = TWO && (ob & 1u);  // the target's red erased node: x2 (else x1)
                const uint8_t *src = scr + (t2 ? src2 : src1);
                uint32_t acc[4][2] = {};
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    if (TWO && j == 2 && nY == 2u) break;  // two erasures in the section: two used X
                    const uint32_t X = Xj[j];
                    const uint2 cv = *reinterpret_cast<const uint2 *>(src + obb + X * wy64);
                    const GfIdx i0 = gf_idx(cv.x), i1 = gf_idx(cv.y);
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        acc[r][0] ^= gf_mul_idx(i0, tg[j][r]);
                        acc[r][1] ^= gf_mul_idx(i1, tg[j][r]);
                    }
                }
                const uint32_t xt = t2 ? x2 : x1;
                const uint32_t oz = obb + xt * wy64;
#pragma unroll
                for (int r = 0; r < 4; r++)
                    if (uint32_t(r) < ne)  // the region holds ne rows
                        __hip_atomic_fetch_xor(reinterpret_cast<uint64_t *>(scr + uint32_t(r) * BUF + oz),
                                               uint64_t(acc[r][0]) | (uint64_t(acc[r][1]) << 32), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        };
        // ---- the both-erased pairs (two erasures in a section, TWO only): row r at a layer z whose
        // digit of r's section is its partner's digit holds U after the rounds (the phase-A Out term
        // needs the erased partner), so C(r, z) = det^-1 (U(r, z) + gamma U(r', z')) and C(r', z') =
        // det^-1 (U(r', z') + gamma U(r, z)), z' = z with r's digit (get_coupled_from_uncoupled,
        // decode.rs:228-232, transforms.rs:108-125): 64 layer pairs x 8 pieces per section, both
        // entries of a pair by one lane (no hand-over between lanes)
        auto pairs = [&]() BS_INL {
            const uint32_t gl = uint32_t(li) * 64u + uint32_t(lane);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const uint32_t pi = a.pinfo[r];
                const uint32_t pr = (pi >> 1) & 3u;
                if (!(pi & 1u) || pr < uint32_t(r)) continue;  // uniform: each pair once
                const uint32_t sh = 2u * (3u - ((pi >> 3) & 3u)), xr = (pi >> 5) & 3u, xo = (pi >> 7) & 3u;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const uint32_t it = gl + 256u * uint32_t(h);
                    const uint32_t zi = it >> 3, d8 = (it & 7u) * 8u;
                    // zi: the three other digits; insert the section's digit at bit sh
                    const uint32_t lo = zi & ((1u << sh) - 1u), hi = (zi >> sh) << (sh + 2u);
                    const uint32_t z = hi | (xo << sh) | lo, zp = hi | (xr << sh) | lo;
                    uint2 *q1 = reinterpret_cast<uint2 *>(scr + uint32_t(r) * BUF + z * 64u + d8);
                    uint2 *q2 = reinterpret_cast<uint2 *>(scr + pr * BUF + zp * 64u + d8);
                    const uint2 u1 = *q1, u2 = *q2;
                    *q1 = make_uint2(gf_mul(u1.x ^ gf_xt(u2.x), dinv), gf_mul(u1.y ^ gf_xt(u2.y), dinv));
                    *q2 = make_uint2(gf_mul(u2.x ^ gf_xt(u1.x), dinv), gf_mul(u2.y ^ gf_xt(u1.y), dinv));
                }
            }
        };
        constexpr bool TM = (PROBE & 16) != 0;
        uint64_t tm_vm = 0, tm_bar = 0, tm_rnd = 0, tm_end = 0, t0 = 0;
        const uint64_t tm_start = TM ? __builtin_amdgcn_s_memtime() : 0;
        for (uint32_t k = 0; k <= ntile; k++) {
            sfor<4>([&](auto yc) BS_INL {
                constexpr int y = decltype(yc)::value;
                if constexpr (TM) t0 = __builtin_amdgcn_s_memtime();
                if (k < ntile) {
                    // loads of step (k, y) landed; the loads issued after them may stay in flight
                    const uint32_t qend = k * NT + a.sec_off[y + 1];
                    wait_vm_rt(int((issued - qend) * uint32_t(Kn::BPL)));
                }
                if constexpr (TM) {
                    const uint64_t t1 = __builtin_amdgcn_s_memtime();
                    tm_vm += t1 - t0;
                    t0 = t1;
                }
                lds_barrier();  // B_y(k): step (k, y) landed; C(k-1) of level y visible
                if constexpr (TM) {
                    const uint64_t t1 = __builtin_amdgcn_s_memtime();
                    tm_bar += t1 - t0;
                    t0 = t1;
                }
                if (k < ntile) issue_upto(k * NT + a.sec_off[y] + RB);
                if (TWO && ((a.split >> y) & 1u)) {  // the rest of step (k, y)'s loads, then a second barrier
                    if (k < ntile) wait_vm_rt(int((issued - (k * NT + a.sec_off[y + 1])) * uint32_t(Kn::BPL)));
                    lds_barrier();
                }
                if (k == 0 || (PROBE & 1)) return;
                // PROBE 64: the round at the compute waves' priority (the DMA issue above stays at 3)
                if constexpr ((PROBE & 64) != 0) __builtin_amdgcn_s_setprio(0);
                round(IC<y>{});
                // TWO: every round of tile k - 1 is done (the last, level 4, has no targets with two
                // erasures in a section: at most three sections hold erasures), so the loaders
                // invert the both-erased pairs in place before B_r(k)
                if constexpr (TWO && y == 3) pairs();
                if constexpr ((PROBE & 64) != 0) __builtin_amdgcn_s_setprio(3);
                if constexpr (TM) tm_rnd += __builtin_amdgcn_s_memtime() - t0;
            });
            if constexpr (TM) t0 = __builtin_amdgcn_s_memtime();
            lds_barrier();  // B_r(k): every atomic of tile k-1 done (lgkmcnt(0) before the barrier)
            // the compute waves are past phase A(k): every ring buffer is free, so the next tile's
            // first RB loads stream during the presolve, the region hand-over and the stores
            if (k + 1u < ntile) issue_upto((k + 1u) * NT + RB);
            if constexpr (TM) tm_end += __builtin_amdgcn_s_memtime() - t0;
        }
        wait_vm0();
        if constexpr (TM) {
            if (blockIdx.x == 0 && li == 0 && lane == 0)
                printf("f2-timing loader tiles %u total %lu vmwait %lu barrier %lu rounds %lu br %lu\n", ntile,
                       (unsigned long)(__builtin_amdgcn_s_memtime() - tm_start), (unsigned long)tm_vm,
                       (unsigned long)tm_bar, (unsigned long)tm_rnd, (unsigned long)tm_end);
        }
        return;
    }

    // ---------------- compute waves ----------------
    // lane map (round 6): part p = lane & 7; column c = d0 d1 d2 with digit 2 from the wave (waves
    // 4-7: d2 in {2, 3}, whose section-2 companions are the shortened nodes -- the light steps of
    // StreamDec::section), digit 1 from lane bits 3-4 (the 32-lane ds_read_b64 groups see four
    // digit-1 values: read4's SWZ row swizzle keeps own and companion reads conflict free), digit 0
    // from wave bit 1 and lane bit 5
    const uint32_t cw = uint32_t(wave), ck = (uint32_t(threadIdx.x) >> 3) & 7u;
    const uint32_t c0 = ((((cw >> 1) & 1u) | (((ck >> 2) & 1u) << 1)) << 4) | ((ck & 3u) << 2) |
                        ((cw & 1u) | (((cw >> 2) & 1u) << 1));
    const uint32_t p = uint32_t(threadIdx.x) & 7u;
    const uint32_t emG = a.emask[G];
    const int xeG = emG ? __builtin_ctz(emG) : -1;
    constexpr bool TM = (PROBE & 16) != 0;
    uint64_t tm_pa = 0, tm_pabar = 0, tm_pre = 0, tm_br = 0, tm_rd = 0, tm_bw = 0, tm_st = 0, t0 = 0;
    const uint64_t tm_start = TM ? __builtin_amdgcn_s_memtime() : 0;
    for (uint32_t k = 0; k <= ntile; k++) {
        uint32_t S[32];
        if constexpr (TM) t0 = __builtin_amdgcn_s_memtime();
        if (k < ntile) {
            const typename Kn::Tile t = tm.tile(k, wslot, ns);
            const bool straddle = t.vend < t.b0 + uint32_t(Kn::W) && ((t.vend - t.b0) & 15u) == 8u;
            const uint32_t pcs = (t.vend - t.b0) >> 4;
            const uint32_t poff0 = 8u * p + ((straddle && p == 2u * pcs) ? 8u : 0u);
#pragma unroll
            for (int w = 0; w < 32; w++) S[w] = 0;
            Kn::template phase_a<((PROBE & 4) ? 2 : 0) | (PROBE & 128), false, false, TWO, true>(a, smem, k * NT, c0, poff0, xeG, S,
                                                                                    RB, TM ? &tm_pabar : nullptr);
            // bit planes -> bytes
#pragma unroll
            for (int j = 0; j < 4; j++) {
                uint32_t v[8];
#pragma unroll
                for (int w = 0; w < 8; w++) v[w] = S[j * 8 + w];
                transpose8(v);
#pragma unroll
                for (int w = 0; w < 8; w++) S[j * 8 + w] = v[w];
            }
        } else {
#pragma unroll
            for (int y = 0; y < 4; y++) {  // B_y(ntile): the last tile's rounds (+ the split steps' second barriers)
                lds_barrier();
                if (TWO && ((a.split >> y) & 1u)) lds_barrier();
            }
        }
        if constexpr (TM) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            tm_pa += t1 - t0;
            t0 = t1;
        }
        lds_barrier();  // B_r(k): C(k-1) complete in the region
        if constexpr (TM) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            tm_br += t1 - t0;
            t0 = t1;
        }
        // S' = H_K^-1 S per slot (tables: scalar loads), after B_r(k) so the loaders stream
        if (k < ntile && !(PROBE & 8)) {
            // check j outer: its 4 tables (rows r) are loaded once per tile and serve the 4 slots
            // (16 table loads per tile instead of 64; an opaque base per j keeps them from being
            // hoisted out of the tile loop into SGPRs that spill)
            uint32_t U[4][4][2] = {};  // [slot g][row r][word]
            sfor<4>([&](auto jc) BS_INL {
                constexpr int j = decltype(jc)::value;
                uint32_t zoff = 0;
                asm volatile("" : "+s"(zoff));
                const cu32p tj = tabc + zoff;
                GfTab tb[4];
                sfor<4>([&](auto rc) BS_INL {
                    constexpr int r = decltype(rc)::value;
                    if (uint32_t(r) < a.ne) tb[r] = load_tab_c(tj + (r * 4 + j) * 8);  // erased rows only
                });
                sfor<4>([&](auto gc) BS_INL {
                    constexpr int g = decltype(gc)::value;
                    const GfIdx i0 = gf_idx(S[j * 8 + 2 * g]), i1 = gf_idx(S[j * 8 + 2 * g + 1]);
                    sfor<4>([&](auto rc) BS_INL {
                        constexpr int r = decltype(rc)::value;
                        if (uint32_t(r) < a.ne) {  // uniform
                            U[g][r][0] ^= gf_mul_idx(i0, tb[r]);
                            U[g][r][1] ^= gf_mul_idx(i1, tb[r]);
                        }
                    });
                });
            });
#pragma unroll
            for (int g = 0; g < 4; g++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    S[r * 8 + 2 * g] = U[g][r][0];
                    S[r * 8 + 2 * g + 1] = U[g][r][1];
                }
        }
        if constexpr (TM) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            tm_pre += t1 - t0;
            t0 = t1;
        }
        // C(k-1) out of the region and S'(k) in: each lane reads, then overwrites, the same 16 x 8
        // bytes (rows r, its four slots' layers, its 8-byte piece), so no lane can overwrite a
        // byte another lane has yet to read -- no hand-over barrier (the both-erased pairs of TWO
        // were inverted in place by the loaders before B_r(k))
        uint2 ov[16];  // [row r][slot g]
        {
            const uint32_t z0 = Kn::layer0(opq(c0));
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if (uint32_t(r) >= a.ne) continue;
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    uint2 *q = reinterpret_cast<uint2 *>(scr + uint32_t(r) * BUF + (z0 + uint32_t(g) * Kn::wt(G)) * 64u + 8u * p);
                    if (k >= 1) ov[r * 4 + g] = *q;
                    if (k < ntile) *q = make_uint2(S[r * 8 + 2 * g], S[r * 8 + 2 * g + 1]);
                }
            }
        }
        if constexpr (TM) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            tm_rd += t1 - t0;
            t0 = t1;
        }
        if (k >= 1 && !(PROBE & 2)) {
            // 8-byte stores: eight lanes (p) write each layer's 64-byte row run of the tile
            const typename Kn::Tile t = tm.tile(k - 1, wslot, ns);
            const uint32_t pp = opq(p);  // opaque per tile: dst_r + 8 p is not hoisted into 4 x 64-bit registers
            if (t.b0 + 8u * pp + 8u <= t.vend) {
                const uint32_t z0 = Kn::layer0(opq(c0));
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    uint8_t *dst = a.out[r];
                    if (uint32_t(r) >= a.ne || !dst) continue;
#pragma unroll
                    for (int g = 0; g < 4; g++)
                        *reinterpret_cast<uint2 *>(dst + uint64_t(z0 + uint32_t(g) * Kn::wt(G)) * sc + t.b0 + 8u * pp) =
                            ov[r * 4 + g];
                }
            }
        }
        if constexpr (TM) tm_st += __builtin_amdgcn_s_memtime() - t0;
    }
    if constexpr (TM) {
        if (blockIdx.x == 0 && (threadIdx.x == 0 || threadIdx.x == 256))  // compute waves 0 and 4 (one SIMD)
            printf("f2-timing compute w%u tiles %u total %lu phaseA %lu (barriers %lu) B_r %lu presolve %lu Cread+Swrite %lu - %lu "
                   "stores %lu\n",
                   unsigned(threadIdx.x >> 6), ntile, (unsigned long)(__builtin_amdgcn_s_memtime() - tm_start), (unsigned long)tm_pa,
                   (unsigned long)tm_pabar, (unsigned long)tm_br, (unsigned long)tm_pre, (unsigned long)tm_rd,
                   (unsigned long)tm_bw, (unsigned long)tm_st);
    }
}

}  // namespace bs
}  // namespace clay
