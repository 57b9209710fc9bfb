// line_args.hpp -- kernel arguments of the line-local bit-sliced kernels (bitslice_line.hpp: the
// (4,2,5) encode and single-erasure decode), shared by the host (engine.hip) and the kernel
// translation unit (line_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace clay {
namespace bs {

struct Dec1Args {
    const uint8_t *node[8];  // internal nodes (the erased one: unused)
    uint8_t *out;            // the erased node's chunk
    uint64_t sc;             // sub-chunk bytes
    uint32_t ntiles, tiles_per_xcd, nslots;
};

struct Enc1Args {
    const uint8_t *data[8];  // data nodes
    uint8_t *par[4];         // parity nodes (the last y-section)
    uint64_t sc;             // sub-chunk bytes
    uint32_t ntiles, tiles_per_xcd, nslots;
    // batches: stripe s's nodes at data[i] + s * sdata, par[x] + s * spar (ntiles tiles per
    // stripe, tiles_per_xcd over all nstripes * ntiles); nstripes = 0: one stripe
    uint32_t nstripes;
    int64_t sdata, spar;
};

}  // namespace bs

// line_kernels.hip: k_bs_encode1 for code (k, m); bt = byte tails.  hipErrorInvalidValue: no
// instantiation
hipError_t launch_bs_encode1_kernel(int k, int m, bool bt, const bs::Enc1Args &a, hipStream_t stream);
// line_kernels.hip: k_bs_decode1 for code (k, m) and erased internal node e; bt = byte tails
// (unaligned chunks or sc % 8 != 0).  hipErrorInvalidValue: no instantiation
hipError_t launch_bs_decode1_kernel(int k, int m, int e, bool bt, const bs::Dec1Args &a, hipStream_t stream);
// positions per tile and threads per workgroup of that instantiation (0: none)
int bs_decode1_tile(int k, int m);

}  // namespace clay
