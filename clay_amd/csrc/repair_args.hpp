// repair_args.hpp -- kernel arguments of the bit-sliced repair kernels (repair_kernel.hpp),
// shared by the host runtime (engine.hip) and the kernel translation unit (repair_stream.hip)
// so the struct passed by value across the two has one definition.
#pragma once
#include <stdint.h>

namespace clay {
namespace bs {

struct RepArgs {
    const uint8_t *h[16];  // internal node -> its helper buffer (nullptr: shortened, zero)
    uint8_t *out;          // the lost node's chunk
    uint64_t sc;
    uint32_t x0;           // lost node = (Y0, x0)
    uint32_t full;         // 1: helper buffers are whole chunks (layer z at z * sc);
                           // 0: the beta plane layers in ascending order (layer j at j * sc)
    uint32_t ntiles, per_xcd;
    uint64_t b_start;      // first byte position (k_bs_repair: tiles of [b_start, sc))
};

}  // namespace bs
}  // namespace clay
