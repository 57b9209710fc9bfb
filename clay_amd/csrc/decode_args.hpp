// decode_args.hpp -- kernel arguments of the streaming decode (stream_decode.hpp), shared by
// the host planner (engine.hip) and the kernel translation unit (decode_stream.hip).
#pragma once
#include <stdint.h>

namespace clay {
namespace bs {

constexpr int kDecBuf = 16384;  // one LDS node buffer: 256 layers x 64 B

struct DecArgs {
    const uint8_t *node[16];  // internal nodes with data (alive real nodes), else nullptr
    uint8_t *out[4];          // per erased index r: output chunk (nullptr: not wanted)
    uint64_t sc;
    uint32_t region, nslots;  // XCD region bytes (multiple of 64), workgroups per XCD
    uint32_t alive;           // bit i: internal node i has data
    uint32_t used;            // bit i: node i is among the first 12 present (the RS rows used)
    uint32_t ne;              // erased count (1..4)
    int32_t rix[16];          // erased index r of internal node i, else -1
    uint32_t emask[4];        // per section y: bit x set if node (y, x) is erased
    uint32_t ring;            // staging ring buffers R = 10
    uint32_t nt;              // loads per tile (alive nodes)
    uint32_t sec_off[5];      // first load of section y's step within a tile
    uint32_t load_node[16];   // internal node of each load of a tile
    // device buffer (kDecTabWords dwords) of v_perm tables, 8 dwords each (5 used): table
    // t = r * 4 + j: row e_r of H_K^-1, check j; table 16 + i * 4 + r: A_i[e_r] =
    // (H_K^-1 gamma H_i)[e_r] for node i; table kDecDetInv: det^-1 (local decode only)
    const uint32_t *tabs;
    // local decode (k_stream_local): bit position of section y's layer digit in the column c
    // (a permutation of 0, 2, 4 over the sections != G; section g2's digit at 0, so its lines
    // are lanes l, l ^ 8, l ^ 16, l ^ 24 of one wave); g2 = the section of the one erasure
    // outside section G (-1: none), x2 its digit
    uint32_t csh[4];
    int32_t g2;
    uint32_t x2;
    // per section y, the phase-A copy (StreamDec::phase_a of k_stream_fused2, Local256::step):
    // x (0..3) = node (y, x) erased and every other node used, 4 = none erased and all used,
    // 5 / 6 = none erased, all alive and only node 0 / nodes 0-1 used (k_stream_local256 only),
    // -1 = the run-time copy
    int32_t scase[4];
    // k_stream_fused2 with two erasures in a section (round 6): per erased row r, pinfo[r] = bit 0:
    // r has a partner (the other erased node of its section), bits 1-2 the partner's row, 3-4 the
    // section, 5-6 r's digit, 7-8 the partner's digit (packed: few scalar registers); npair = rows
    // with a partner (both-erased PFT pairs, transforms.rs:108-125, inverted after the rounds)
    uint32_t pinfo[4];
    uint32_t npair;
    // k_stream_fused2: bit y = section y's loads do not all fit the ring during step y - 1 (two
    // neighbouring sections with more alive nodes than the ring holds): the rest is issued after
    // B_y and waited for behind a second barrier
    uint32_t split;
    // k_stream_fused2: byte li = loader wave li's share of the rounds (engine.hip f2_plan): bits
    // 0-1 its section, 2-3 its part, 4-5 the section's wave count - 1, bit 6 set (0: no rounds)
    uint32_t lwave;
};
// k_stream_fused2: solver work items per lane and round (passes of 64 lanes over targets x 8
// pieces, per iscore level) of the TWO instantiation (two erasures in a section) and of the other;
// the host declines patterns whose target counts exceed them (engine.hip f2_plan)
constexpr int kF2Iters[4] = {5, 4, 2, 1};
constexpr int kF2Iters1[4] = {6, 4, 2, 1};
// local decode: v_perm table of det^-1 = (1 + gamma^2)^-1 (pair inversion, transforms.rs:108-125)
constexpr int kDecDetInv = 80;
// 3 KiB: k_stream_local copies them into LDS with three 1 KiB LDS-DMA instructions
constexpr int kDecTabWords = 768;
static_assert((kDecDetInv + 1) * 8 <= kDecTabWords, "every table inside the block the kernels copy");

}  // namespace bs
}  // namespace clay
