// decode1_args.hpp -- kernel arguments of the single-erasure bit-sliced decode (bitslice_decode1.hpp),
// shared by the host (engine.hip) and the kernel translation unit (decode_bs1.hip).
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

}  // namespace bs

// decode_bs1.hip: k_bs_decode1 for code (k, m) and erased internal node e; bt = byte tails
// (unaligned chunks or sc % 8 != 0).  hipErrorInvalidValue: no instantiation
hipError_t launch_bs_decode1_kernel(int k, int m, int e, bool bt, const bs::Dec1Args &a, hipStream_t stream);
// positions per tile and threads per workgroup of that instantiation (0: none)
int bs_decode1_tile(int k, int m);

}  // namespace clay
