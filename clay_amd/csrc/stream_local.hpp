// stream_local.hpp -- single-launch decode for q = 4, t = 4 codes ((10,4,13), (9,4,12)) whose
// erasures lie in one y-section G, plus at most one erasure in one other section g2:
// {0}, {0,4}, {0,1}, {0,1,4}, {0,1,2,3}, ...  Every survivor byte is read from HBM once, every
// output byte written once, and no workgroup barrier separates the iscore levels: all of the
// reference's layered decode (decode.rs:196-329) after the RS syndromes happens in registers.
//
// Why the dependencies stay inside a wave.  Phase A (StreamDec::phase_a, RT mode) gives every
// lane the syndromes S(z) of its four layers z = (column c, slot g = digit G) x 8 positions, with
// the terms gamma * C(e, z') of erased companions dropped (stream_decode.hpp).  The dropped term of
// layer z in section Y is C of section Y's erased node at z[Y := X] -- a layer on the same Y-line:
//   * Y = G: the same lane (another slot);
//   * Y = g2: the host puts section g2's digit at bits 0-1 of c, so the Y-line is the four lanes
//     l, l ^ 8, l ^ 16, l ^ 24 of one wave: their terms are XOR-reduced by two lane shuffles.
// Per position the solve is then (syndrome form, stream_decode.hpp; A_i = H_K^-1 gamma H_i):
//   presolve   C_r(g) = row e_r of H_K^-1 S(g), every slot          (level 0 done)
//   (i)   g2-lines of the slots g outside E_G: red lanes (digit g2 = x2) add
//         sum over the line's other lanes X of A_(g2,X)[r] C_e2(X, g)
//   (ii)  slots g in E_G: add sum over used (G, A), A not in E_G, of A_(G,A)[r] C_(G,g)(slot A)
//   (iii) slots g in E_G, red lanes: the g2-line terms of (i) from the now final C_e2
//   (iv)  both-erased pairs of section G ((G, x) at slot g <-> (G, g) at slot x, x, g in E_G):
//         C = det^-1 (U + gamma U*) (get_coupled_from_uncoupled, transforms.rs:108-125)
// Each step only reads values the previous steps finished, which is the reference's iscore order.
#pragma once

#include "stream_decode.hpp"

namespace clay {
namespace bs {

template <int KD, int G>
struct StreamLocal {
    using D = StreamDec<KD, G>;
    static constexpr int BLOCK = D::BLOCK;

    // 2 dwords (8 positions) of C_r at slot g, r uniform at run time.  Opaque masks instead of
    // selects: a select between loads of S becomes a load through a selected pointer, i.e. a
    // dynamic index, and S would move to scratch memory.
    __device__ static uint2 get(const uint32_t (&C)[32], uint32_t r, int g) {
        uint2 v = make_uint2(0u, 0u);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t m = opq(r == uint32_t(k) ? 0xffffffffu : 0u);
            v.x |= C[k * 8 + 2 * g] & m;
            v.y |= C[k * 8 + 2 * g + 1] & m;
        }
        return v;
    }
    __device__ static void put(uint32_t (&C)[32], uint32_t r, int g, uint2 v) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t m = opq(r == uint32_t(k) ? 0xffffffffu : 0u);
            C[k * 8 + 2 * g] = (C[k * 8 + 2 * g] & ~m) | (v.x & m);
            C[k * 8 + 2 * g + 1] = (C[k * 8 + 2 * g + 1] & ~m) | (v.y & m);
        }
    }
    // C_r(g) ^= A_i[r] * v for the ne erased rows (tables 16 + 4 i + r)
    __device__ static void add_term(uint32_t (&C)[32], const uint8_t *tl, uint32_t i, uint2 v, int g, uint32_t ne) {
        const GfIdx i0 = gf_idx(v.x), i1 = gf_idx(v.y);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            if (uint32_t(r) < ne) {
                const GfTab t = D::tab_at(tl, int(16u + i * 4u + uint32_t(r)));
                C[r * 8 + 2 * g] ^= gf_mul_idx(i0, t);
                C[r * 8 + 2 * g + 1] ^= gf_mul_idx(i1, t);
            }
        }
    }
    // steps (i) / (iii): slots g of mask `slots`, terms of the g2-line (lanes differing in bits 3-4)
    __device__ static void line_g2(const DecArgs &a, uint32_t (&C)[32], const uint8_t *tl, uint32_t c, uint32_t slots) {
        const uint32_t ne = a.ne, g2 = uint32_t(a.g2), x2 = a.x2;
        const uint32_t d2 = c & 3u;  // this lane's digit of section g2
        const uint32_t r2 = uint32_t(a.rix[4 * g2 + x2]);
        const bool red = d2 == x2;
        const bool src = !red && ((a.used >> (4u * g2 + d2)) & 1u);
        const uint32_t ti = 16u + (4u * g2 + d2) * 4u;  // per-lane table row (d2 varies over the line)
#pragma unroll
        for (int g = 0; g < 4; g++) {
            if (!((slots >> g) & 1u)) continue;
            uint2 v = get(C, r2, g);
            if (!src) v = make_uint2(0u, 0u);
            const GfIdx i0 = gf_idx(v.x), i1 = gf_idx(v.y);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if (uint32_t(r) >= ne) continue;
                const GfTab t = D::tab_at(tl, int(ti + uint32_t(r)));
                uint32_t w0 = gf_mul_idx(i0, t), w1 = gf_mul_idx(i1, t);
                w0 ^= uint32_t(__shfl_xor(int(w0), 8));
                w1 ^= uint32_t(__shfl_xor(int(w1), 8));
                w0 ^= uint32_t(__shfl_xor(int(w0), 16));
                w1 ^= uint32_t(__shfl_xor(int(w1), 16));
                if (red) {
                    C[r * 8 + 2 * g] ^= w0;
                    C[r * 8 + 2 * g + 1] ^= w1;
                }
            }
        }
    }
};

// grid = 8 * nslots (one workgroup per CU, 64-byte tiles as k_stream_syn); LDS = 10 x 16 KiB:
// a ring of a.ring - 1 node buffers and the tables (presolve, A_i, det^-1) in the last buffer.
template <int KD, int G>
__global__ __launch_bounds__((StreamDec<KD, G>::BLOCK)) void k_stream_local(DecArgs a) {
    using Kn = StreamDec<KD, G>;
    using Lc = StreamLocal<KD, G>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t xcd = blockIdx.x & 7u, wslot = blockIdx.x >> 3, ns = a.nslots;
    const uint32_t sc = uint32_t(a.sc);
    const typename Kn::Map tm(sc, a.region, ns, xcd, wslot);
    const uint32_t ntile = tm.n;
    if (ntile == 0) return;  // uniform per workgroup
    const uint32_t R = a.ring - 1u, NT = a.nt;
    constexpr uint32_t BUF = uint32_t(Kn::BUF);

    if (wave >= Kn::CWAVES) {
        // ---------------- loader waves: global ring, load g -> buffer g % R (k_stream_syn) ----------------
        __builtin_amdgcn_s_setprio(3);
        const int li = wave - Kn::CWAVES;
        typename Kn::Loader L;
        Kn::loader_init_rt(L, a, li, lane);
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
                Kn::issue(a, L, lds0 + (issued % R) * BUF, a.node[a.load_node[q]], tm.tile(k, wslot, ns), li);
            }
        };
        issue_upto(R);
        for (uint32_t k = 0; k < ntile; k++) {
            for (int y = 0; y < 4; y++) {
                const uint32_t qend = k * NT + a.sec_off[y + 1];
                wait_vm_rt(int((issued - qend) * uint32_t(Kn::BPL)));
                lds_barrier();
                issue_upto(k * NT + a.sec_off[y] + R);
            }
        }
        wait_vm0();
        return;
    }

    // ---------------- compute waves ----------------
    const uint32_t c0 = uint32_t(threadIdx.x) >> 3, p = uint32_t(threadIdx.x) & 7u;
    const uint32_t eG = a.emask[G], ne = a.ne;
    const bool has2 = a.g2 >= 0;
    for (uint32_t k = 0; k < ntile; k++) {
        const typename Kn::Tile t = tm.tile(k, wslot, ns);
        const bool straddle = t.vend < t.b0 + uint32_t(Kn::W) && ((t.vend - t.b0) & 15u) == 8u;
        const uint32_t pcs = (t.vend - t.b0) >> 4;
        const uint32_t poff0 = 8u * p + ((straddle && p == 2u * pcs) ? 8u : 0u);
        uint32_t S[32];
#pragma unroll
        for (int w = 0; w < 32; w++) S[w] = 0;
        Kn::template phase_a<0, true>(a, smem, k * NT, c0, poff0, -1, S, R);
        // bit planes -> bytes: S[j * 8 + 2g .. +1] = check j at slot g
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t v[8];
#pragma unroll
            for (int w = 0; w < 8; w++) v[w] = S[j * 8 + w];
            transpose8(v);
#pragma unroll
            for (int w = 0; w < 8; w++) S[j * 8 + w] = v[w];
        }
        // presolve, in place: S[r * 8 + 2g ..] = row e_r of H_K^-1 S(g) (C where level 0); sfor, so
        // every index into S is a constant from the start (S stays in registers)
        sfor<4>([&](auto gc) BS_INL {
            constexpr int g = decltype(gc)::value;
            uint32_t U[4][2] = {};
            sfor<4>([&](auto jc) BS_INL {
                constexpr int j = decltype(jc)::value;
                const uint8_t *tl = smem + R * BUF + opq(0u);  // tables re-read, not hoisted
                const GfIdx i0 = gf_idx(S[j * 8 + 2 * g]), i1 = gf_idx(S[j * 8 + 2 * g + 1]);
                sfor<4>([&](auto rc) BS_INL {
                    constexpr int r = decltype(rc)::value;
                    if (uint32_t(r) < ne) {  // the erased rows only (uniform)
                        const GfTab tb = Kn::tab_at(tl, r * 4 + j);
                        U[r][0] ^= gf_mul_idx(i0, tb);
                        U[r][1] ^= gf_mul_idx(i1, tb);
                    }
                });
                __builtin_amdgcn_sched_barrier(0);
            });
            sfor<4>([&](auto rc) BS_INL {
                constexpr int r = decltype(rc)::value;
                S[r * 8 + 2 * g] = U[r][0];
                S[r * 8 + 2 * g + 1] = U[r][1];
            });
        });
        const uint8_t *tl = smem + R * BUF + opq(0u);
        const uint32_t c = opq(c0);
        // (i) g2-lines of the slots outside E_G (sources: level-0 values)
        if (has2) Lc::line_g2(a, S, tl, c, ~eG & 15u);
        // (ii) slots g in E_G: the in-lane terms of the used nodes (G, A), A not in E_G
#pragma unroll
        for (int g = 0; g < 4; g++) {
            if (!((eG >> g) & 1u)) continue;
            const uint32_t rg = uint32_t(a.rix[4 * G + g]);
#pragma unroll
            for (int A = 0; A < 4; A++) {
                if (((eG >> A) & 1u) || !((a.used >> (4 * G + A)) & 1u)) continue;
                Lc::add_term(S, tl, uint32_t(4 * G + A), Lc::get(S, rg, A), g, ne);
            }
        }
        // (iii) red lanes of the g2-lines: the terms of slots in E_G (sources final after (ii))
        if (has2) Lc::line_g2(a, S, tl, c, eG);
        // (iv) both-erased pairs of section G: C = det^-1 (U + gamma U*)
        if (__builtin_popcount(eG) >= 2) {
            const GfTab dinv = Kn::tab_at(tl, kDecDetInv);
#pragma unroll
            for (int g = 0; g < 4; g++) {
#pragma unroll
                for (int x = g + 1; x < 4; x++) {
                    if (!((eG >> g) & 1u) || !((eG >> x) & 1u)) continue;
                    const uint32_t rx = uint32_t(a.rix[4 * G + x]), rg = uint32_t(a.rix[4 * G + g]);
                    const uint2 u1 = Lc::get(S, rx, g), u2 = Lc::get(S, rg, x);  // (G,x)@g, (G,g)@x
                    const uint2 c1 = make_uint2(gf_mul(u1.x ^ gf_xt(u2.x), dinv), gf_mul(u1.y ^ gf_xt(u2.y), dinv));
                    const uint2 c2 = make_uint2(gf_mul(u2.x ^ gf_xt(u1.x), dinv), gf_mul(u2.y ^ gf_xt(u1.y), dinv));
                    Lc::put(S, rx, g, c1);
                    Lc::put(S, rg, x, c2);
                }
            }
        }
        // outputs: 8 bytes per lane, slot and erased row (64-byte row runs per 8 lanes)
        const uint32_t z0 = Kn::layer0_rt(a, c);
        const bool valid = t.b0 + 8u * p + 8u <= t.vend;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            uint8_t *dst = a.out[r];
            if (uint32_t(r) >= ne || !dst || !valid) continue;
#pragma unroll
            for (int g = 0; g < 4; g++)
                *reinterpret_cast<uint2 *>(dst + (uint64_t(z0 + uint32_t(g) * Kn::wt(G)) * sc + t.b0 + 8u * p)) =
                    make_uint2(S[r * 8 + 2 * g], S[r * 8 + 2 * g + 1]);
        }
    }
}

}  // namespace bs
}  // namespace clay
