// repair_stream.hip -- instantiations and launcher of the bit-sliced repair kernel
// (repair_kernel.hpp), in their own translation unit; the host-side checks are in engine.hip.
#include <hip/hip_runtime.h>

#include "repair_kernel.hpp"

namespace clay {

template <int KD, int M, int Y0>
static hipError_t launch_one(bs::RepArgs a, hipStream_t stream, uint32_t *w_out) {
    using Kn = bs::BsRepair<KD, M, Y0>;
    *w_out = Kn::W;
    a.ntiles = uint32_t((a.sc + Kn::W - 1) / Kn::W);
    a.per_xcd = (a.ntiles + 7) / 8;
    bs::k_bs_repair<KD, M, Y0><<<dim3(a.per_xcd * 8), dim3(Kn::BLOCK), 0, stream>>>(a);
    return hipGetLastError();
}

template <int KD, int M>
static hipError_t launch_km(int y0, const bs::RepArgs &a, hipStream_t stream, uint32_t *w) {
    switch (y0) {
    case 0: return launch_one<KD, M, 0>(a, stream, w);
    case 1: return launch_one<KD, M, 1>(a, stream, w);
    case 2: return launch_one<KD, M, 2>(a, stream, w);
    default:
        if constexpr (bs::Shape<KD, M>::T > 3) return launch_one<KD, M, 3>(a, stream, w);
        return hipErrorInvalidValue;
    }
}

// 1 = launched, 0 = no instantiation for (k, m), < 0 = HIP error
int launch_bs_repair_kernel(int k, int m, int y0, const bs::RepArgs &a, hipStream_t stream) {
    uint32_t w = 0;
    hipError_t e;
    if (k == 9 && m == 3) e = launch_km<9, 3>(y0, a, stream, &w);
    else if (k == 10 && m == 4) e = launch_km<10, 4>(y0, a, stream, &w);
    else if (k == 4 && m == 2) e = launch_km<4, 2>(y0, a, stream, &w);
    else return 0;
    return e == hipSuccess ? 1 : -int(e);
}

}  // namespace clay
