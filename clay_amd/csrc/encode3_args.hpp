// encode3_args.hpp -- kernel arguments of the (9,3) streaming encode (stream_encode3.hpp), shared
// by the host (engine.hip) and the kernel translation unit (encode_stream3.hip).
#pragma once
#include <stdint.h>

namespace clay {
namespace bs {

struct Enc3Args {
    const uint8_t *data[9];
    uint8_t *par[3];
    uint64_t sc;
    uint32_t region;   // XCD region bytes (StreamMap: full tiles round robin, the remainder split)
    uint32_t ns;       // workgroups per XCD
};

}  // namespace bs
}  // namespace clay
